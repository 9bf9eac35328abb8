set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "couple or packed or c4 or split or sharded" > gpurun_out/t_couple.log 2>&1 || { echo "couple tests failed"; tail -40 gpurun_out/t_couple.log; exit 1; }
tail -3 gpurun_out/t_couple.log
for spec in "c4:--workload c4" "c4_128:--workload c4 --pairs 128" "c4_256:--workload c4 --pairs 256" "c4_512:--workload c4 --pairs 512"; do
  name="${spec%%:*}"; args="${spec#*:}"
  timeout -k 10 200 python -u bench.py $args --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/cb_$name.json 2> gpurun_out/cb_$name.err || { echo "bench $name failed"; tail -20 gpurun_out/cb_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/cb_$name.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['config'].get('dp_kernel_ms'), d['roofline']['frac'], d['config'].get('dp_launch'), {k:v for k,v in d['config'].items() if 'match' in k})"
done
MSA_COUPLE=4 timeout -k 10 200 python -u bench.py --workload c4 --no-cpu-baseline --steps 20 > gpurun_out/cb_c4_g4.json 2> gpurun_out/cb_c4_g4.err && python -c "import json; d=json.loads(open('gpurun_out/cb_c4_g4.json').read().strip().splitlines()[-1]); print('c4 G4', d['value'], d['config'].get('dp_kernel_ms'))"
VARIANTS="prod d53e87d 9114fa2 bdd8bfa 8f6bea8 ho3 prod" ARGS="--workload c2 --reps 10" bash scripts/gpu_variants.sh
