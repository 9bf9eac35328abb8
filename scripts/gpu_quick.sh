# quick GPU check: selected tests (K=pytest -k expr), then bench lines (BENCHES="name:[VAR=val ...] args;...")
set -o pipefail
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/t_quick.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_quick.log; exit 1; }
  tail -2 gpurun_out/t_quick.log
fi
IFS=';' read -ra BL <<< "$BENCHES"
for b in "${BL[@]}"; do
  name="${b%%:*}"; args="${b#*:}"
  pre=""; rest=""
  for tok in $args; do if [ -z "$rest" ] && [[ "$tok" == *=* ]] && [[ "$tok" != --* ]]; then pre="$pre $tok"; else rest="$rest $tok"; fi; done
  timeout -k 10 300 env $pre python -u bench.py --no-cpu-baseline $rest > gpurun_out/bq_$name.json 2> gpurun_out/bq_$name.err || { echo "bench $name failed"; tail -20 gpurun_out/bq_$name.err; exit 1; }
  python - "$name" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads(open(f"gpurun_out/bq_{n}.json").read().strip().splitlines()[-1])
c = d["config"]
print(n, d["value"], d["ms_per_step"], c.get("dp_kernel_ms"), c.get("traceback_ms"), {k: v for k, v in c.items() if "match" in k or "ok" in k or k == "dp_launch"})
PY
done
