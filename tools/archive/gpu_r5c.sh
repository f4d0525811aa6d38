# round 5: proposal launch at 6 waves/SIMD (80 VGPRs, 9 spilled) vs 5, interleaved N2 loop A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_r5c.txt
: > $out
for B in 4096 512; do
  for rep in 1 2 3; do
    for v in new w6 w6w4; do
      r=$(AIQMC_LIB_VARIANT=$v AIQMC_NOPROF=1 timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
      echo "$v rep$rep $r" | tee -a $out
    done
  done
  for v in new w6 w6w4; do
    r=$(AIQMC_LIB_VARIANT=$v timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
    echo "$v events $r" | tee -a $out
  done
done
