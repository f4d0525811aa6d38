# round 4: packed walker launches for 5 <= N <= 8 (two per wave).  The whole -m gpu suite (ECP, DMC,
# T-moves and the C / C2 goldens run these walker launches), then the C and C2-ccECP loops with
# AIQMC_PACKW=0 (one wave per walker) vs default, three interleaved reps + one with events
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/tests_tail.txt | tail -12
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/ab_r4o.txt
: > $out
for sysn in C2_ecp C; do
  for rep in 1 2 3; do
    for t in 0 1; do
      r=$(AIQMC_NOPROF=1 AIQMC_PACKW=$t timeout -k 10 120 python tools/mc_loop.py 20 $sysn 4096) || exit 1
      echo "packw=$t rep$rep $r" | tee -a $out
    done
  done
  for t in 0 1; do
    r=$(AIQMC_PACKW=$t timeout -k 10 120 python tools/mc_loop.py 20 $sysn 4096) || exit 1
    echo "packw=$t events $r" | tee -a $out
  done
done
