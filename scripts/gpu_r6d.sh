# full GPU suite on the tree's build, then: fused block reduction A/B (C2, C5), FL_PS_FILL=32 and a
# 3-wave fill budget on the whole-sequence reference pair
set -o pipefail
TESTS=1 BENCHES="c2_fused:--steps 20 --no-c4-strong;c2_unfused:MSA_FUSED_REDUCE=0 --steps 20 --no-c4-strong;c2_fused2:--steps 20 --no-c4-strong;c2_unfused2:MSA_FUSED_REDUCE=0 --steps 20 --no-c4-strong;c5_fused:--workload c5 --steps 10;c5_unfused:MSA_FUSED_REDUCE=0 --workload c5 --steps 10;rw_prod:--workload ref --ref-len 0 --ref-pair 3,4 --steps 3 --warmup 1;rw_fw3:MSA_LIB_PATH=vlib/libmsa_fw3.so --workload ref --ref-len 0 --ref-pair 3,4 --steps 3 --warmup 1;ref_prod:--workload ref --steps 20" bash scripts/gpu_check.sh r6d
