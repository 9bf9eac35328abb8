set -o pipefail
mkdir -p gpurun_out
for cfg in "prod:cse305_parallel_sequence_alignment_amd/libmsa.so:4:4000" "prod:cse305_parallel_sequence_alignment_amd/libmsa.so:64:4000" "wpe5:vlib/libmsa_wpe5.so:4:4000" "wpe5:vlib/libmsa_wpe5.so:4:1000" "wpe5:vlib/libmsa_wpe5.so:16:4000"; do
  IFS=: read nm lib np ln <<< "$cfg"
  MSA_LIB_PATH=$lib MSA_C4_KERNEL=cflow timeout -k 10 150 python scripts/dbg_cflow.py --pairs $np --len $ln --reps 4 > gpurun_out/r6b_dbg_${nm}_${np}_${ln}.json
  rc=$?; [ $rc -eq 0 ] || { echo "dbg $cfg status $rc"; exit 2; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r6b_dbg_${nm}_${np}_${ln}.json')); print('$cfg', [(r['n_bad'], r['bad'][:4], r['err']) for r in d['runs']])"
done
BENCHES="c2_prod:--steps 20 --no-c4-strong;c2_ps16:MSA_LIB_PATH=vlib/libmsa_ps16.so --steps 20 --no-c4-strong;c5_prod:--workload c5 --steps 10;c5_ps16:MSA_LIB_PATH=vlib/libmsa_ps16.so --workload c5 --steps 10;ref_prod:--workload ref --steps 20;ref_ps16:MSA_LIB_PATH=vlib/libmsa_ps16.so --workload ref --steps 20;ref20_prod:--workload ref --ref-len 20000 --steps 10;ref20_ps16:MSA_LIB_PATH=vlib/libmsa_ps16.so --workload ref --ref-len 20000 --steps 10;rw_prod:--workload ref --ref-len 0 --ref-pair 3,4 --steps 3 --warmup 1;rw_ps16:MSA_LIB_PATH=vlib/libmsa_ps16.so --workload ref --ref-len 0 --ref-pair 3,4 --steps 3 --warmup 1" bash scripts/gpu_check.sh r6b
