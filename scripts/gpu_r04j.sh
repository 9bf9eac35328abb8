set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
VARIANTS="prod grpblk d53e87d prod grpblk d53e87d" ARGS="--workload c2 --reps 10" bash scripts/gpu_variants.sh
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bj_c2.json 2> gpurun_out/bj_c2.err || { tail -20 gpurun_out/bj_c2.err; exit 1; }
cut -c 1-400 gpurun_out/bj_c2.json
timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline --steps 20 > gpurun_out/bj_c5.json 2> gpurun_out/bj_c5.err || { tail -20 gpurun_out/bj_c5.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bj_c5.json').read().strip().splitlines()[-1]); print('c5', d['value'], d['ms_per_step'], d['config'].get('dp_kernel_ms'))"
timeout -k 10 200 python -u bench.py --workload ref --no-cpu-baseline --steps 20 > gpurun_out/bj_ref.json 2> gpurun_out/bj_ref.err || { tail -20 gpurun_out/bj_ref.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bj_ref.json').read().strip().splitlines()[-1]); print('ref', d['value'], d['ms_per_step'], d['config'].get('dp_kernel_ms'))"
MSA_LIB_PATH=variants/libmsa_bkstage.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "banded or c3" > gpurun_out/t_bkstage.log 2>&1 || { echo "bkstage tests failed"; tail -30 gpurun_out/t_bkstage.log; exit 1; }
tail -2 gpurun_out/t_bkstage.log
VARIANTS="prod bkstage" ARGS="--workload c3 --reps 5" bash scripts/gpu_variants.sh
VARIANTS="prod bkstage" ARGS="--workload c3d --reps 3" bash scripts/gpu_variants.sh
MSA_FLOW_BATCH=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "packed or c4 or split or sharded" > gpurun_out/t_fb.log 2>&1 || { echo "flow batch tests failed"; tail -30 gpurun_out/t_fb.log; exit 1; }
tail -2 gpurun_out/t_fb.log
for pr in 128 256 512 1024; do
  for fb in 0 1; do
    MSA_FLOW_BATCH=$fb timeout -k 10 200 python -u bench.py --workload c4 --pairs $pr --no-cpu-baseline --steps 10 > gpurun_out/fb_${pr}_$fb.json 2> gpurun_out/fb_${pr}_$fb.err || { echo "bench failed"; tail -5 gpurun_out/fb_${pr}_$fb.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/fb_${pr}_$fb.json').read().strip().splitlines()[-1]); print('pairs $pr flowbatch $fb', d['value'], d['config'].get('dp_kernel_ms'), {k:v for k,v in d['config'].items() if 'match' in k})"
  done
done
