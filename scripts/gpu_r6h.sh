set -o pipefail
TESTS=1 BENCHES="rw:--workload ref --ref-len 0 --ref-pair 3,4 --steps 3 --warmup 1;ref:--workload ref --steps 20;c5:--workload c5 --steps 10;c2:--steps 20 --no-c4-strong" bash scripts/gpu_check.sh r6h && bash scripts/prof_round.sh "refwhole"
