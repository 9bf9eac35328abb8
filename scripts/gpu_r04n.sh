# production tree: GPU suite, smoke, default bench; then the reduce-only fold variant (variants/libmsa_red.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { echo "bench failed"; tail -20 gpurun_out/final_bench.err; exit 1; }
cut -c 1-700 gpurun_out/final_bench.json
V=variants/libmsa_red.so
MSA_LIB_PATH=$V timeout -k 10 60 python -u -m pytest tests -m gpu -x -v --timeout 30 --timeout-method thread -k "sw_linear_H_small" > gpurun_out/n_first.log 2>&1 || { echo "red first test failed"; tail -20 gpurun_out/n_first.log; exit 1; }
MSA_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 60 --timeout-method thread > gpurun_out/n_all.log 2>&1 || { echo "red suite failed"; tail -30 gpurun_out/n_all.log; exit 1; }
tail -1 gpurun_out/n_all.log
VARIANTS="prod red prod red" ARGS="--workload c2 --reps 10" bash scripts/gpu_variants.sh || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/n_bp$i.json 2>/dev/null || exit 1
  MSA_LIB_PATH=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/n_br$i.json 2>/dev/null || exit 1
  python -c "import json; f=lambda p: json.loads(open(p).read().strip().splitlines()[-1]); a=f('gpurun_out/n_bp$i.json'); b=f('gpurun_out/n_br$i.json'); print('prod', a['value'], a['ms_per_step'], a['config'].get('h_matches_cpu'), '| red', b['value'], b['ms_per_step'], b['config'].get('h_matches_cpu'))"
done
