# decoder batching variant (vlib/libmsa_decb.so): walk tests + c5/ref/refwhole benches against the in-tree build
set -o pipefail
mkdir -p gpurun_out
MSA_LIB_PATH=vlib/libmsa_decb.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "traceback or walk or gotoh or c5 or capped" > gpurun_out/r6k_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r6k_tests.log; [ $rc -eq 0 ] || exit 2
for v in prod decb; do
  if [ $v = prod ]; then L=cse305_parallel_sequence_alignment_amd/libmsa.so; else L=vlib/libmsa_$v.so; fi
  for b in "c5:--workload c5 --steps 20 --warmup 3" "ref:--workload ref --steps 20 --warmup 3" "refwhole:--workload ref --ref-len 0 --ref-pair 3,4 --steps 3 --warmup 1"; do
    n=${b%%:*}; a=${b#*:}
    MSA_LIB_PATH=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline $a > gpurun_out/r6k_${v}_$n.json 2> gpurun_out/r6k_${v}_$n.err || { echo "bench $v $n failed"; exit 2; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r6k_${v}_$n.json').read().strip().splitlines()[-1]); print('$v $n', d['value'], d['config'].get('traceback_ms'))"
  done
done
