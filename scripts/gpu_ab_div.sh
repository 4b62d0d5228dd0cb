set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
VARIANTS="fast ieee" CMD="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh
VARIANTS="fast ieee" CMD="python bench.py --workload personalized --steps 10 --warmup 3 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh
VARIANTS="fast ieee" CMD="python bench.py --workload personalized --pers-weights int --steps 10 --warmup 3 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh
VARIANTS="fast ieee" CMD="python bench.py --workload qsgd --steps 20 --warmup 5 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh
VARIANTS="fast ieee" CMD="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-probe" bash scripts/gpu_ab.sh
