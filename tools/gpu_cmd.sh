set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=r04ai
bash tools/gpu_ab.sh ${T} "C4 - G2OHIP_ZERO_PER_WG=4 G2OHIP_ZERO_PER_WG=16 - G2OHIP_ZERO_PER_WG=4 G2OHIP_ZERO_PER_WG=16" "C5 - G2OHIP_ZERO_PER_WG=4 G2OHIP_ZERO_PER_WG=16 - --steps 6"
