# same-box A/B: the current library against the round-5 sources (vlib/libmsa_r05.so)
set -o pipefail
R5=MSA_LIB_PATH=vlib/libmsa_r05.so
BENCHES="c3:--workload c3 --steps 20;c3_r5:$R5 --workload c3 --steps 20;c3b:--workload c3 --steps 20;c3b_r5:$R5 --workload c3 --steps 20;c2:--steps 20 --no-c4-strong;c2_r5:$R5 --steps 20 --no-c4-strong;c4:--workload c4 --steps 20;c4_r5:$R5 --workload c4 --steps 20;c5:--workload c5 --steps 10;c5_r5:$R5 --workload c5 --steps 10;ref:--workload ref --steps 20;ref_r5:$R5 --workload ref --steps 20" bash scripts/gpu_check.sh r6i
