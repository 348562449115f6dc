set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_marginals.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w64_t2.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/w64_t2.log; exit 1; }
tail -2 gpurun_out/w64_t2.log
timeout -k 10 900 python -u tools/dist_factor_time.py --config C5 --ranks 8,2 > gpurun_out/dist_c5_rs.json 2> gpurun_out/dist_c5_rs.err || { echo DIST_FAIL; tail -20 gpurun_out/dist_c5_rs.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/dist_c5_rs.json"))
print("single", d["single"]["factor_ms"], d["single"]["solve_ms"])
for n, v in d["by_ranks"].items():
    for r, x in enumerate(v["per_rank"]):
        i = x["info"]
        print(n, r, "factor %.3f solve %.3f" % (x["factor_ms"], x["solve_ms"]), "rs", i.get("reduce_scatter"), "seg", i.get("rs_segment_doubles"), "tail", i.get("rs_tail_doubles"), "model_in %.3g allred %.3g" % (i.get("model_input_s", 0), i.get("model_input_allreduce_s", 0)), "owned", i["owned_fronts"], "shared", i["shared_fronts"])
PY
