# Schur row pass mode split on the dev library (G2OHIP_SCHUR_MODE: 1 no products, 2 no staging, 3 neither)
set -o pipefail
export TMPDIR=/tmp
export G2OHIP_LIB=$PWD/g2o_amd/libg2o_hip_phases.so
bash tools/gpu_ab.sh r05l_ab "C4 - G2OHIP_SCHUR_MODE=1 G2OHIP_SCHUR_MODE=2 G2OHIP_SCHUR_MODE=3 G2OHIP_SCHUR_SB_KX=256 G2OHIP_SCHUR_SB_KX=256,G2OHIP_SCHUR_MODE=3 --steps 10 --warmup 2" "C5 - G2OHIP_SCHUR_MODE=1 G2OHIP_SCHUR_MODE=2 G2OHIP_SCHUR_MODE=3 --steps 4 --warmup 2"
