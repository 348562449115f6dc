# dev A/B helper for gpurun: a list of "CONFIG SETTINGS..." lines for tools/ab_bench.py, one bench process per setting
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
TAG=${1:-ab}
shift
i=0
for spec in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python tools/ab_bench.py $spec > $O/${TAG}_$i.log 2>&1 || { echo AB_FAIL $spec; tail -20 $O/${TAG}_$i.log; exit 1; }
  cat $O/${TAG}_$i.log
done
