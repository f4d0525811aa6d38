# round 4: packed proposals for 5 <= N <= 8 (k_quad_grad, two per wave): the -m gpu suite, then the
# C2 / C loops packed vs one-wave (AIQMC_QUAD_GRAD=0) at 4096 walkers, the HIP-event overhead in the N2
# loop (profile on/off), and a rocprofv3 kernel trace of the C2 loop (both paths)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; rc=$?; echo "suite rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/tests_tail.txt | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for sys in C2 C; do for rep in 1 2; do
  echo "packed $(timeout -k 10 120 python tools/mc_loop.py 10 $sys 4096)" || exit 1
  echo "onewave $(AIQMC_QUAD_GRAD=0 timeout -k 10 120 python tools/mc_loop.py 10 $sys 4096)" || exit 1
done; done
for B in 4096 512; do for rep in 1 2; do
  echo "events   $(timeout -k 10 120 python tools/mc_loop.py 20 N2 $B)" || exit 1
  echo "noevents $(AIQMC_NOPROF=1 timeout -k 10 120 python tools/mc_loop.py 20 N2 $B)" || exit 1
done; done
cd /tmp
for v in 1 0; do
  rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_c2_$v
  AIQMC_QUAD_GRAD=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c2_$v -o run -- python3 $GRAFT_REPO_ROOT/tools/mc_loop.py 5 C2 4096 > /dev/null 2>&1 || { echo PROF_FAIL; exit 1; }
  python3 $GRAFT_REPO_ROOT/profiles/summarize.py $GRAFT_REPO_ROOT/gpurun_out/prof_c2_$v > $GRAFT_REPO_ROOT/gpurun_out/prof_c2_$v.json
done
echo PROF_OK
