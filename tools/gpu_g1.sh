set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/sh_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/sh_tests.log; exit 1; }
tail -12 gpurun_out/sh_tests.log
G2OHIP_LIB=g2o_amd/libg2o_hip_phases.so timeout -k 10 200 python tools/phase_probe.py C4 > gpurun_out/phase_c4.log 2>&1 || { echo PHASE_FAIL; tail -20 gpurun_out/phase_c4.log; exit 1; }
head -30 gpurun_out/phase_c4.log
