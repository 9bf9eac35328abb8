set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
VARIANTS="prod d53e87d fbval prod d53e87d fbval" ARGS="--workload c2 --reps 10" bash scripts/gpu_variants.sh
VARIANTS="prod fbval" ARGS="--workload c5 --reps 5" bash scripts/gpu_variants.sh
VARIANTS="prod fbval" ARGS="--workload ref --reps 5" bash scripts/gpu_variants.sh
