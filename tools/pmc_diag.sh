#!/bin/bash
# Dev: PMC passes over the memory-bound kernels of one short bench run; tools/pmc_table.py summarises.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmcd
rm -rf $O; mkdir -p $O
RX='k_schur|k_linearize|k_backsub|k_vertex_reduce|k_syrk|k_error_partial'
k=0
for P in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR" \
         "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv -d $O/p$k -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/p$k.log 2>&1 || { echo PMC_FAIL $k; tail -5 $O/p$k.log; exit 1; }
done
echo PMC_OK
python tools/pmc_table.py $O
