set -o pipefail
VARIANTS="prod wpe2 wpe3p2x2" ARGS="--ref-pair 3,4 --ref-len 0" bash scripts/gpu_variants.sh && \
VARIANTS="prod wpe2" ARGS="--ref-len 10000" bash scripts/gpu_variants.sh && \
VARIANTS="prod wpe2" ARGS="--workload c5" bash scripts/gpu_variants.sh && \
VARIANTS="prod wpe2" ARGS="--workload c2" bash scripts/gpu_variants.sh
