set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=r04x
timeout -k 10 1000 env G2OHIP_ND_ABSORB=8 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/${T}_tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
bash tools/gpu_ab.sh ${T} "C4 - G2OHIP_ND_ABSORB=8 - G2OHIP_ND_ABSORB=8" "C5 - G2OHIP_ND_ABSORB=8 --steps 6" "C3 - G2OHIP_ND_ABSORB=8 --steps 3 --warmup 1"
