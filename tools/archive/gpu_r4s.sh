# round 4: acceptance / moved-electron inputs loaded before the limdrift factors' memory round trip
# (old = before, base = after); the whole -m gpu suite, then dev-library A/B
#
# at 512, 1024, 4096 walkers (three reps without events, one with)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/tests_tail.txt | tail -12
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/ab_r4s.txt
: > $out
for B in 512 1024 4096; do
  for rep in 1 2 3; do
    for t in old base; do
      r=$(AIQMC_NOPROF=1 AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
      echo "$t rep$rep $r" | tee -a $out
    done
  done
  for t in old base; do
    r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
    echo "$t events $r" | tee -a $out
  done
done
