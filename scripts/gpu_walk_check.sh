# device walk: walk parity tests, walk stats (diagnostic build vlib/libmsa_tbstats.so), c5 / ref / 97k benches
# (build the diagnostic library first, on the CPU: scripts/build_variant.sh tbstats -DMSA_TB_STATS)
set -o pipefail
mkdir -p gpurun_out
K="traceback or walk or gotoh or ref or c5 or affine or capped" TESTS= bash scripts/gpu_check.sh walk || exit 2
bash scripts/gpu_tbstats.sh || exit 2
BENCHES="c5:--workload c5 --steps 20 --warmup 3;ref:--workload ref --steps 20 --warmup 3;refwhole:--workload ref --ref-len 0 --steps 3 --warmup 1" bash scripts/gpu_check.sh walk
