# per-launch GEMM ring choice (G2OHIP_SYRK_BIG_K): large k_syrk passes on the (32, 2) ring
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_ab.sh r05j_ab "C3 - G2OHIP_SYRK_BIG_K=1024 G2OHIP_SYRK_BIG_K=512 G2OHIP_SYRK_BIG_K=2048 G2OHIP_SYRK_BIG_K=1024,G2OHIP_SYRK_BIG_TILES=2048 - --steps 3 --warmup 1" "C5 - G2OHIP_SYRK_BIG_K=256 G2OHIP_SYRK_BIG_K=256,G2OHIP_SYRK_BIG_TILES=2048 - --steps 8 --warmup 2"
