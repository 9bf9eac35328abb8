set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "banded or c3" > gpurun_out/t_band.log 2>&1 || { echo "band tests failed"; tail -40 gpurun_out/t_band.log; exit 1; }
tail -3 gpurun_out/t_band.log
VARIANTS="prod bknost" ARGS="--workload c3d --reps 3" bash scripts/gpu_variants.sh
for cw in "12 20" "16 20" "12 16" "16 16" "20 16" "24 16" "16 12"; do set -- $cw
  MSA_BAND_CHUNK=$1 MSA_BAND_WARM=$2 timeout -k 10 120 python scripts/time_plan.py --workload c3 --reps 5 > gpurun_out/tb_$1_$2.txt 2>&1 || { echo "tune $cw failed"; tail -5 gpurun_out/tb_$1_$2.txt; exit 1; }
  echo "C=$1 W=$2 $(python -c "import json; d=json.loads(open('gpurun_out/tb_$1_$2.txt').read().strip().splitlines()[-1]); print(d['median_ms'], d['run_info'])")"
done
for cw in "16 16" "12 16"; do set -- $cw
  MSA_BAND_CHUNK=$1 MSA_BAND_WARM=$2 MSA_LIB_PATH=variants/libmsa_bknost.so timeout -k 10 120 python scripts/time_plan.py --workload c3 --reps 5 > gpurun_out/tbn_$1_$2.txt 2>&1 || exit 1
  echo "nostore C=$1 W=$2 $(python -c "import json; d=json.loads(open('gpurun_out/tbn_$1_$2.txt').read().strip().splitlines()[-1]); print(d['median_ms'], d['run_info'])")"
done
