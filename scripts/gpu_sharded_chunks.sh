#!/bin/bash
# Sharded-path GPU tests, the chunk sweep and a kernel timeline (one GPU, forced 1-rank RCCL).
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sharded.log 2>&1 && \
tail -3 gpurun_out/pytest_sharded.log && bash scripts/gpu_chunks.sh "${1:-1 2 4 8}" && bash scripts/gpu_sharded_trace.sh 4 native
