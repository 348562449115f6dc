set -o pipefail
mkdir -p gpurun_out
true && \
G2OHIP_LIB=g2o_amd/libg2o_hip_phases.so timeout -k 10 300 python tools/phase_probe.py C4 > gpurun_out/phase_c4.log 2>&1
rc=$?; cat gpurun_out/ub_chol32.log gpurun_out/phase_c4.log; exit $rc
