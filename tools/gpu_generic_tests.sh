set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_generic.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r02c_pytest.log 2>&1; rc=$?; tail -30 gpurun_out/r02c_pytest.log; exit $rc
