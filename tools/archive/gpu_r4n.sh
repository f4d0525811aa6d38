# round 4: local energy of iteration k on a side stream (positions snapshot) overlapping iteration
# k+1's mc_step, vs sequential; N2 fp32 at 4096 and 512 walkers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/pipe_r4n.txt
: > $out
for B in 4096 512; do
  timeout -k 10 180 python tools/pipe_probe.py 20 $B | tee -a $out || exit 1
done
