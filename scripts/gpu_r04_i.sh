#!/bin/bash
# Round 4: the fused own-window peer exchange — multi-device tests (bit-identical to the host
# composition), the aliased one-process bench, and the headline bench line (no regression).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multi_device.py > $O/pytest_multi.log 2>&1 || { echo "multi tests failed"; grep -E "FAILED|Error" $O/pytest_multi.log | head; tail -40 $O/pytest_multi.log; exit 1; }
tail -2 $O/pytest_multi.log
timeout -k 10 300 python bench.py --procs 1 --gpus 4 --alias --steps 5 --warmup 2 --no-cpu-baseline > $O/multi_alias.jsonl 2> $O/multi_alias.err || { echo "multi alias failed"; tail -20 $O/multi_alias.err; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.jsonl 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.jsonl | head -c 700
echo done
