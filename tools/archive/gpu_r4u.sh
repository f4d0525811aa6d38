# round 4: ILP in the first-derivative pass at its 2-waves/SIMD register budget (256): E4's (r, s)
# loop unrolled 2 / 4, the h-stream column loop unrolled 2; N2 loop at 4096 and 512 walkers, per-
# launch averages from HIP events, three interleaved reps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_r4w.txt
: > $out
for B in 4096 512; do
  for rep in 1 2 3; do
    for t in base e4r2 e4r2s2; do
      r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
      echo "$t rep$rep $r" | tee -a $out
    done
  done
done
