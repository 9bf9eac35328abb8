set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "wide or ref1_stripe or whole or at_size or sharded" > gpurun_out/t_new.log 2>&1 || { echo "new tests failed"; tail -40 gpurun_out/t_new.log; exit 1; }
tail -12 gpurun_out/t_new.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/t_all.log; exit 1; }
tail -3 gpurun_out/t_all.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || { tail -20 gpurun_out/b_c2.err; exit 1; }
cat gpurun_out/b_c2.json
timeout -k 10 200 python -u bench.py --workload ref --no-cpu-baseline --steps 20 > gpurun_out/b_ref10k.json 2> gpurun_out/b_ref10k.err || { tail -20 gpurun_out/b_ref10k.err; exit 1; }
MSA_FLOW_LDS_MIN=0 timeout -k 10 200 python -u bench.py --workload ref --no-cpu-baseline --steps 20 > gpurun_out/b_ref10k_lds0.json 2> gpurun_out/b_ref10k_lds0.err || { tail -20 gpurun_out/b_ref10k_lds0.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload ref --ref-pair 3,4 --ref-len 0 --no-cpu-baseline --steps 10 > gpurun_out/b_refwhole.json 2> gpurun_out/b_refwhole.err || { tail -20 gpurun_out/b_refwhole.err; exit 1; }
timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline --steps 20 > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err || { tail -20 gpurun_out/b_c5.err; exit 1; }
python - <<'PY'
import json
for f in ["b_ref10k", "b_ref10k_lds0", "b_refwhole", "b_c5"]:
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    c = d["config"]
    print(f, d["value"], d["ms_per_step"], c.get("dp_kernel_ms"), c.get("traceback_ms"), {k: v for k, v in c.items() if "match" in k or "ok" in k})
PY
