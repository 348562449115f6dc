set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver_contract.py tests/test_gpu_marginals.py tests/test_host.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/g1_pytest.log 2>&1; rc=$?
tail -30 gpurun_out/g1_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-posegraph > gpurun_out/g1_bench.json 2> gpurun_out/g1_bench.err || { tail -20 gpurun_out/g1_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/g1_bench.json')); print('C4', round(d['value'],1), d['runtime'], json.dumps(d.get('c5'))[:600])"
