# round 4: the walker launch's pair adjoints (B3) software-pipelined over the walker-cache reads
# (base) vs one cache round trip per iteration (old, -DAQ_WALK_B3_PIPE); parity subset on the main
# library, then the N2 loop at 4096 / 512 walkers, three interleaved reps + one with events
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mc_fp32.py tests/test_gpu_fullsize.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/parity_r4x.log 2>&1; rc=$?
echo "parity rc=$rc"; tail -2 gpurun_out/parity_r4x.log
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/ab_r4x.txt
: > $out
for B in 4096 512; do
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
