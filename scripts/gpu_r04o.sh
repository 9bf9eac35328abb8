# C3 band kernel: chunk length (stripes) x warm-up (stripes) sweep on the production library
set -o pipefail
mkdir -p gpurun_out
for wl in c3 c3syn; do
  for ch in 8 12 16 24; do
    for wm in 14 16 20; do
      MSA_BAND_CHUNK=$ch MSA_BAND_WARM=$wm timeout -k 10 120 python scripts/time_plan.py --workload $wl --reps 5 > gpurun_out/o_${wl}_${ch}_${wm}.txt 2>&1 || { echo "run failed"; tail -5 gpurun_out/o_${wl}_${ch}_${wm}.txt; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/o_${wl}_${ch}_${wm}.txt').read().strip().splitlines()[-1]); print('$wl chunk $ch warm $wm', round(d['median_ms'], 4), d['error'], d.get('run_info'))"
    done
  done
done
