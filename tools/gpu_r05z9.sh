# chi2 partial sums with the four-edge group loop kept rolled (a quarter of the code): full GPU suite, smoke, A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/r05z9_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05z9_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05z9_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/r05z9_smoke.log; exit 1; }
tail -1 $O/r05z9_smoke.log
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
bash tools/gpu_ab.sh r05z9_ab "C4 - $B - $B --steps 20 --warmup 3" "C5 - $B --steps 8 --warmup 2" "C3 - $B --steps 3 --warmup 1" || exit 1
