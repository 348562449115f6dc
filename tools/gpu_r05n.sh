# phase probe of the Cholesky chain (dev library): C4 and C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
export G2OHIP_LIB=$PWD/g2o_amd/libg2o_hip_phases.so
timeout -k 10 200 python tools/phase_probe.py C4 > $O/r05n_phase_c4.log 2>&1; cat $O/r05n_phase_c4.log | tail -40
