# round-4 variant checks: the flow-batch build (no in-kernel staging/reduction) and the band H-staging build
set -o pipefail
mkdir -p gpurun_out
FB=variants/libmsa_fbatch.so
MSA_LIB_PATH=$FB timeout -k 10 150 python -u -m pytest tests -m gpu -x -v --timeout 60 --timeout-method thread -k "sw_linear_H_small" > gpurun_out/k_first.log 2>&1 || { echo "fbatch first test failed"; tail -30 gpurun_out/k_first.log; exit 1; }
tail -2 gpurun_out/k_first.log
MSA_LIB_PATH=$FB timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k_fb_all.log 2>&1 || { echo "fbatch suite failed"; tail -30 gpurun_out/k_fb_all.log; exit 1; }
tail -2 gpurun_out/k_fb_all.log
MSA_LIB_PATH=$FB MSA_FLOW_BATCH=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "packed or c4 or split or sharded or batch" > gpurun_out/k_fb_on.log 2>&1 || { echo "flow batch tests failed"; tail -30 gpurun_out/k_fb_on.log; exit 1; }
tail -2 gpurun_out/k_fb_on.log
for pr in 128 512; do
  for fb in 0 1; do
    MSA_LIB_PATH=$FB MSA_FLOW_BATCH=$fb timeout -k 10 200 python -u bench.py --workload c4 --pairs $pr --no-cpu-baseline --steps 10 > gpurun_out/k_fb_${pr}_$fb.json 2> gpurun_out/k_fb_${pr}_$fb.err || { echo "bench failed"; tail -5 gpurun_out/k_fb_${pr}_$fb.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/k_fb_${pr}_$fb.json').read().strip().splitlines()[-1]); print('pairs $pr flowbatch $fb', d['value'], d['config'].get('dp_kernel_ms'))"
  done
done
MSA_LIB_PATH=variants/libmsa_bkstage.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "banded or c3" > gpurun_out/k_bkstage.log 2>&1 || { echo "bkstage tests failed"; tail -30 gpurun_out/k_bkstage.log; exit 1; }
tail -2 gpurun_out/k_bkstage.log
VARIANTS="prod bkstage prod bkstage" ARGS="--workload c3 --reps 5" bash scripts/gpu_variants.sh
VARIANTS="prod bkstage" ARGS="--workload c3d --reps 3" bash scripts/gpu_variants.sh
VARIANTS="prod grpblk prod grpblk" ARGS="--workload c2 --reps 10" bash scripts/gpu_variants.sh
