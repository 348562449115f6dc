set -o pipefail
mkdir -p gpurun_out
for m in 0 1 2 3 4 7; do
  G2OHIP_SCHUR_MODE=$m timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$m.json 2>/dev/null || { echo FAIL $m; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$m.json')); print('mode $m', round(d['stages_ms_avg']['schur_rows']*1e3,1), 'us')"
done
