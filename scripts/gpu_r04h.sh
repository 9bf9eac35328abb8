set -o pipefail
mkdir -p gpurun_out
MSA_FLOW_BATCH=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "packed or c4 or split or sharded or linear" > gpurun_out/t_fb.log 2>&1 || { echo "flow batch tests failed"; tail -40 gpurun_out/t_fb.log; exit 1; }
tail -2 gpurun_out/t_fb.log
for pr in 128 256 512 1024; do
  for fb in 0 1; do
    MSA_FLOW_BATCH=$fb timeout -k 10 200 python -u bench.py --workload c4 --pairs $pr --no-cpu-baseline --steps 10 > gpurun_out/fb_${pr}_$fb.json 2> gpurun_out/fb_${pr}_$fb.err || { echo "bench failed"; tail -5 gpurun_out/fb_${pr}_$fb.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/fb_${pr}_$fb.json').read().strip().splitlines()[-1]); print('pairs $pr flowbatch $fb', d['value'], d['config'].get('dp_kernel_ms'), {k:v for k,v in d['config'].items() if 'match' in k})"
  done
done
