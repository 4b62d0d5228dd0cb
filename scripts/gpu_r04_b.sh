#!/bin/bash
# Round 4: the new multi-device tests first, then the whole -m gpu suite on the cleaned kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_multi_device.py "tests/test_gpu_staging.py::test_delta_first_round_then_reordered_full_update" > $O/pytest_multi.log 2>&1 || { echo "multi tests failed rc=$?"; grep -E "FAILED|Error|error" $O/pytest_multi.log | head -20; tail -40 $O/pytest_multi.log; exit 1; }
tail -3 $O/pytest_multi.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu --deselect tests/test_gpu_multi_device.py > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed rc=$?"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
