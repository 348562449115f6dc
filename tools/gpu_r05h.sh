# GEMM: MFMA issue-rate peaks, and the k_syrk ring variants in situ after the single-path chunk loop
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 60 ./tools/ubench_gemm 0 > $O/r05h_peaks.log 2>&1 && cat $O/r05h_peaks.log || exit 1
bash tools/gpu_ab.sh r05h_ab "C3 - G2OHIP_SYRK_DMA=1 G2OHIP_SYRK_DMA=5 G2OHIP_SYRK_DMA=6 G2OHIP_SYRK_DMA=3 - --steps 3 --warmup 1" "C5 - G2OHIP_SYRK_DMA=1 G2OHIP_SYRK_DMA=5 - --steps 8 --warmup 2"
