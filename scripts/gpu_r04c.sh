set -o pipefail
mkdir -p gpurun_out
for v in stprod std53 st911 stbdd; do
  MSA_LIB_PATH=variants/libmsa_$v.so timeout -k 10 120 python scripts/stamps_flow.py --workload c2 --tag $v > gpurun_out/sf_$v.json 2> gpurun_out/sf_$v.err || { echo "stamps $v failed"; tail -5 gpurun_out/sf_$v.err; exit 1; }
  cat gpurun_out/sf_$v.json
done
MSA_LIB_PATH=variants/libmsa_cb8.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "couple or packed or c4" > gpurun_out/t_cb8.log 2>&1 || { echo "cb8 tests failed"; tail -30 gpurun_out/t_cb8.log; exit 1; }
tail -2 gpurun_out/t_cb8.log
for pr in 1024 128 512; do
  MSA_LIB_PATH=variants/libmsa_cb8.so timeout -k 10 200 python -u bench.py --workload c4 --pairs $pr --no-cpu-baseline --steps 10 > gpurun_out/cb8_$pr.json 2> gpurun_out/cb8_$pr.err || { echo "cb8 bench failed"; tail -5 gpurun_out/cb8_$pr.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/cb8_$pr.json').read().strip().splitlines()[-1]); print('cb8 $pr', d['value'], d['config'].get('dp_kernel_ms'))"
done
VARIANTS="prod ws8" ARGS="--workload c3d --reps 3" bash scripts/gpu_variants.sh
VARIANTS="prod" ARGS="--workload c3 --reps 5" bash scripts/gpu_variants.sh
