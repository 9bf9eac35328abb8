# FL_PS / fill-launch register budget A/B on the whole-sequence reference pair (and ref 10k, C5 for PS=32)
set -o pipefail
B=""
for v in ps16 ps32 ps16fw3 ps16fw2; do
  B="$B;rw_$v:MSA_LIB_PATH=vlib/libmsa_$v.so --workload ref --ref-len 0 --ref-pair 3,4 --steps 3 --warmup 1"
done
B="$B;rw_prod:--workload ref --ref-len 0 --ref-pair 3,4 --steps 3 --warmup 1"
B="$B;ref_ps32:MSA_LIB_PATH=vlib/libmsa_ps32.so --workload ref --steps 20;c5_ps32:MSA_LIB_PATH=vlib/libmsa_ps32.so --workload c5 --steps 10;c2_ps32:MSA_LIB_PATH=vlib/libmsa_ps32.so --steps 20 --no-c4-strong"
BENCHES="${B#;}" bash scripts/gpu_check.sh r6c
