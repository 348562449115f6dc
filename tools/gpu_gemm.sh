#!/bin/bash
# Dev: GEMM tile micro-benchmark at two shapes + one PMC pass (MFMA busy / waits) of the 64x64 tile kernel
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 120 ./tools/ubench_gemm 4096 2048 > gpurun_out/ubg1.log 2>&1 || { echo UB1_FAIL; tail -5 gpurun_out/ubg1.log; exit 1; }
timeout -k 5 120 ./tools/ubench_gemm 3072 384 > gpurun_out/ubg2.log 2>&1 || { echo UB2_FAIL; tail -5 gpurun_out/ubg2.log; exit 1; }
cat gpurun_out/ubg1.log gpurun_out/ubg2.log
timeout -k 5 120 ./tools/ubench_gemm 0 > gpurun_out/ubg0.log 2>&1 && cat gpurun_out/ubg0.log
rm -rf gpurun_out/pmcg
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "k_tri<64, 64" --output-format csv -d gpurun_out/pmcg -o run -- ./tools/ubench_gemm 4096 2048 > gpurun_out/pmcg.log 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/pmcg.log; exit 1; }
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmcg/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
by = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    by[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in by.items():
    print(k, {c: round(x) for c, x in v.items()})
PY
