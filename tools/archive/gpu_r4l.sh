# round 4: compiler scheduling strategies on the N2 dev library (base / max-ilp / max-memory-clause),
# N2 loop at 4096 and 512 walkers, two interleaved reps without HIP events + one with; then the fused
# integer limdrift reduction forced at 4096 walkers (AIQMC_FUSE_REDUCE=2) vs the partial-sum launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_r4l.txt
: > $out
for B in 4096 512; do
  for rep in 1 2; do
    for t in base ilp mclause; do
      r=$(AIQMC_NOPROF=1 AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || { echo "$t FAILED" >> $out; exit 1; }
      echo "$t rep$rep $r" | tee -a $out
    done
  done
  for t in base ilp mclause; do
    r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
    echo "$t events $r" | tee -a $out
  done
done
for rep in 1 2; do
  for f in 1 2; do
    r=$(AIQMC_NOPROF=1 AIQMC_FUSE_REDUCE=$f timeout -k 10 120 python tools/mc_loop.py 20 N2 4096) || exit 1
    echo "fuse_reduce=$f rep$rep $r" | tee -a $out
  done
done
