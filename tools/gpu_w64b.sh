#!/bin/bash
# Dev: tools/gpu_w64.sh then the phase probe of the W64 build
set -o pipefail
bash tools/gpu_w64.sh "$@" || exit 1
G2OHIP_LIB=g2o_amd/libg2o_hip_phases.so timeout -k 10 200 python tools/phase_probe.py C4 > gpurun_out/phase_c4_w64.log 2>&1 || { echo PHASE_FAIL; tail -5 gpurun_out/phase_c4_w64.log; exit 1; }
grep -A3 "diag chain\|diag task\|block-0" gpurun_out/phase_c4_w64.log | head -30
