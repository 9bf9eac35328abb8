#!/bin/bash
# usage: scripts/gpu_state.sh   (run on the GPU box): full GPU suite, then one bench line per config
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for spec in "c2:--workload c2" "c3:--workload c3" "c3syn:--workload c3 --synthetic" "c4:--workload c4" "c4_128:--workload c4 --pairs 128" "c5:--workload c5" "ref:--workload ref" "ref20k:--workload ref --ref-len 20000" "refwhole:--workload ref --ref-pair 3,4 --ref-len 0"; do
  name="${spec%%:*}"; args="${spec#*:}"
  timeout -k 10 300 python -u bench.py $args --steps 20 --warmup 3 > gpurun_out/st_$name.json 2> gpurun_out/st_$name.err || { echo "bench $name failed"; tail -20 gpurun_out/st_$name.err; exit 1; }
  python - "$name" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads(open(f"gpurun_out/st_{n}.json").read().strip().splitlines()[-1])
c = d["config"]
print(n, d["value"], d["ms_per_step"], c.get("dp_kernel_ms"), c.get("traceback_ms"), d.get("roofline", {}).get("frac"), {k: v for k, v in c.items() if "match" in k or "ok" in k or k in ("dp_launch", "converged")})
PY
done
