#!/bin/bash
# usage: scripts/gpu_round4.sh <round> (on the GPU box): GPU suite, one bench line per config, then
# rocprofv3 kernel stats + PMC passes (scripts/prof.sh) for c2 c3 c4 c5 ref
set -o pipefail
RND=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${RND}_gpu_tests.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${RND}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${RND}_gpu_tests.txt
for spec in "c2:--workload c2" "c3:--workload c3" "c3syn:--workload c3 --synthetic" "c4:--workload c4" "c4_128:--workload c4 --pairs 128" "c5:--workload c5" "ref:--workload ref" "ref20k:--workload ref --ref-len 20000" "refwhole:--workload ref --ref-pair 3,4 --ref-len 0"; do
  name="${spec%%:*}"; args="${spec#*:}"
  timeout -k 10 300 python -u bench.py $args --steps 20 --warmup 3 > gpurun_out/${RND}_${name}_bench.json 2> gpurun_out/${RND}_${name}_bench.err || { echo "bench $name failed"; tail -20 gpurun_out/${RND}_${name}_bench.err; exit 1; }
  python - "$RND" "$name" <<'PY'
import json, sys
r, n = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/{r}_{n}_bench.json").read().strip().splitlines()[-1])
c = d["config"]
print(n, d["value"], d["ms_per_step"], c.get("dp_kernel_ms"), c.get("traceback_ms"), d.get("roofline", {}).get("frac"), {k: v for k, v in c.items() if "match" in k or "ok" in k or k in ("dp_launch",)})
PY
done
for wl in c2 c3 c4 c5 ref; do
  bash scripts/prof.sh $wl gpurun_out/prof_$wl > gpurun_out/prof_$wl.log 2>&1 || { echo "prof $wl failed"; tail -20 gpurun_out/prof_$wl.log; exit 1; }
  echo "profiled $wl"
done
