set -o pipefail
TESTS=1 BENCHES="c2_fused:--steps 20 --no-c4-strong;c2_unfused:MSA_FUSED_REDUCE=0 --steps 20 --no-c4-strong;c2_fused2:--steps 20 --no-c4-strong;c2_unfused2:MSA_FUSED_REDUCE=0 --steps 20 --no-c4-strong;c5_fused:--workload c5 --steps 10;c5_unfused:MSA_FUSED_REDUCE=0 --workload c5 --steps 10" bash scripts/gpu_check.sh r6e
