#!/bin/bash
# usage (on the GPU box): [TESTS=1] [K=expr] BENCHES="name:[VAR=val ...] bench args;..." bash scripts/gpu_check.sh <tag>
# GPU tests (whole -m gpu suite, or -k K) then one bench line per entry, under gpurun_out/<tag>_*.
# A test or result-check failure (exit 1) is reported and the next step runs; a fault, abort, or time
# limit (any other status) ends the script there.
set -o pipefail
TAG=${1:-chk}
mkdir -p gpurun_out
stop() { echo "STOP after $1 (status $2)"; exit 2; }
if [ -n "$TESTS" ] || [ -n "$K" ]; then
  kx=(); [ -n "$K" ] && kx=(-k "$K")
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${kx[@]}" \
    > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || stop tests $rc
  # a per-test time limit (pytest-timeout, thread method) also exits 1: a hung GPU test ends the script
  grep -q "+++ Timeout +++" gpurun_out/${TAG}_tests.log && stop "tests (a test hit its time limit)" $rc
  [ $rc -eq 1 ] && grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_tests.log | head -20
fi
IFS=';' read -ra BL <<< "$BENCHES"
for b in "${BL[@]}"; do
  [ -z "$b" ] && continue
  name="${b%%:*}"; args="${b#*:}"
  pre=""; rest=""
  for tok in $args; do if [ -z "$rest" ] && [[ "$tok" == *=* ]] && [[ "$tok" != --* ]]; then pre="$pre $tok"; else rest="$rest $tok"; fi; done
  timeout -k 10 300 env $pre python -u bench.py --no-cpu-baseline $rest > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "bench $name failed (status $rc)"; tail -4 gpurun_out/${TAG}_$name.err
    [ $rc -eq 1 ] || stop "bench $name" $rc
    continue
  fi
  python - "gpurun_out/${TAG}_$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[2], d["value"], d["ms_per_step"], c.get("dp_kernel_ms"), c.get("traceback_ms"),
      {k: v for k, v in c.items() if "match" in k or "ok" in k or k in ("dp_launch", "kernel_errors")})
PY
done
