# blocked fronts (big panels + GEMM trailing updates) on the tile-bound levels, after the GEMM loop fix
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_ab.sh r05i_ab "C4 - G2OHIP_CHOL_WIDE_FRONTS=8 G2OHIP_CHOL_WIDE_FRONTS=4 G2OHIP_CHOL_WIDE_FRONTS=8,G2OHIP_CHOL_WIDE_PB=256 - --steps 20 --warmup 3" "C5 - G2OHIP_CHOL_WIDE_FRONTS=32 G2OHIP_CHOL_WIDE_FRONTS=8 G2OHIP_CHOL_WIDE_FRONTS=32,G2OHIP_CHOL_WIDE_PB=256 - --steps 8 --warmup 2"
