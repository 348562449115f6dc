set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=r04t
BA="--config C4 --steps 2 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 --no-kernel-timing"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES --kernel-include-regex "k_step|k_syrk|k_extend_add" --output-format csv -d $O/${T}_pmc_sq -o run -- python bench.py $BA > $O/${T}_pmc_sq.log 2>&1 || { echo PMC1_FAIL; tail -20 $O/${T}_pmc_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "k_step|k_syrk|k_extend_add" --output-format csv -d $O/${T}_pmc_tcc -o run -- python bench.py $BA > $O/${T}_pmc_tcc.log 2>&1 || { echo PMC2_FAIL; tail -20 $O/${T}_pmc_tcc.log; exit 1; }
echo PMC_OK
