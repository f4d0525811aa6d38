# round 4: proposal-launch occupancy / workgroup shape re-checked on the final code: 6 waves/SIMD
# (-DAQ_PROP_WAVES=6, 15 VGPRs spilled), 2 and 8 configurations per workgroup (AQ_PROP_WPB), against
# the shipped 5 waves / 4 per workgroup; N2 loop at 4096 and 512 walkers, events on (per-launch
# averages), three interleaved reps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_r4zz.txt
: > $out
for B in 4096 512; do
  for rep in 1 2 3; do
    for t in base mv2 mv8 wk2; do
      r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
      echo "$t rep$rep $r" | tee -a $out
      r=$(AIQMC_NOPROF=1 AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
      echo "$t noprof rep$rep $r" | tee -a $out
    done
  done
done
