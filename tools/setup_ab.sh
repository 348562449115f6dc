set -o pipefail
mkdir -p gpurun_out
for cfg in C5 C4; do
for bal in 1 0 1; do
  G2OHIP_SCHUR_BALANCE=$bal timeout -k 10 300 python bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline --no-posegraph --no-c5 > gpurun_out/r06_setup_${cfg}_$bal.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r06_setup_${cfg}_$bal.json').read().strip().splitlines()[-1]);print('$cfg bal=$bal', round(d['value'],1), 'schur_rows', round(d['stages_ms_avg']['schur_rows'],4), 'setup', d['setup_s'])"
done; done
