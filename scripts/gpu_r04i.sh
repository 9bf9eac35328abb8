set -o pipefail
mkdir -p gpurun_out
VARIANTS="prod grpblk d53e87d prod grpblk d53e87d" ARGS="--workload c2 --reps 10" bash scripts/gpu_variants.sh
