# round 4: number of fused limdrift accumulator slots (1024 = base / 256 / 128) with the fused
# integer reduction forced at 4096 walkers (AIQMC_FUSE_REDUCE=2) against the default partial-sum
# launches, and at 512 walkers (fused by default); N2 loop, interleaved reps, no events
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_r4t.txt
: > $out
for rep in 1 2 3; do
  r=$(AIQMC_NOPROF=1 AIQMC_LIB_VARIANT=base timeout -k 10 120 python tools/mc_loop.py 20 N2 4096) || exit 1
  echo "base launches rep$rep $r" | tee -a $out
  for t in base s256 s128; do
    r=$(AIQMC_NOPROF=1 AIQMC_FUSE_REDUCE=2 AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 4096) || exit 1
    echo "$t fused rep$rep $r" | tee -a $out
  done
done
for rep in 1 2 3; do
  for t in base s256 s128; do
    r=$(AIQMC_NOPROF=1 AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 512) || exit 1
    echo "$t rep$rep $r" | tee -a $out
  done
done
