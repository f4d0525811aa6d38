# round 6: proposal-launch variants (N2 dev libraries): base, F1 cache blocks by LDS-DMA (glds), SLP vectorisation (slp)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_bitwise.sh ${VARS:-base lpf} 2>&1 | tee gpurun_out/r6c_ab.txt
