set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "banded or c3" > gpurun_out/t_band.log 2>&1 || { echo "band tests failed"; tail -40 gpurun_out/t_band.log; exit 1; }
tail -3 gpurun_out/t_band.log
VARIANTS="prod" ARGS="--workload c3 --reps 5 --check" bash scripts/gpu_variants.sh
VARIANTS="prod" ARGS="--workload c3syn --reps 5" bash scripts/gpu_variants.sh
VARIANTS="prod" ARGS="--workload c3d --reps 3 --check" bash scripts/gpu_variants.sh
