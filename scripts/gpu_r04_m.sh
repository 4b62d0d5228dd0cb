#!/bin/bash
# Round 4: the new mixed-entry multi-device test first, then the whole -m gpu suite on the final
# kernels, smoke() and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multi_device.py -k "quantised_and_mixed or plans_outliving" > $O/pytest_new.log 2>&1 || { echo "new tests failed"; tail -40 $O/pytest_new.log; exit 1; }
tail -2 $O/pytest_new.log
timeout -k 10 1000 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo done
