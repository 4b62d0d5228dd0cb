#!/bin/bash
# Round 4: parity of the reworked PersonalizedFedAVG kernel (golden + geometry), the one-process
# multi-device bench rehearsal (--procs 1, aliased entries on cuda:0) and smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_personalized.py "tests/test_gpu_geometry.py::test_personalized_kernel_edges_bit_identical" > $O/pytest_pers.log 2>&1 || { echo "pers tests failed"; tail -40 $O/pytest_pers.log; exit 1; }
tail -2 $O/pytest_pers.log
timeout -k 10 300 python bench.py --procs 1 --gpus 4 --alias --steps 5 --warmup 2 --no-cpu-baseline > $O/multi_alias.jsonl 2> $O/multi_alias.err || { echo "multi alias failed"; tail -20 $O/multi_alias.err; exit 1; }
tail -c 1500 $O/multi_alias.jsonl
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo done
