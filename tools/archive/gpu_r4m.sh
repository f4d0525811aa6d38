# round 4: walker launches re-using the previous sweep's pivot order.  Parity first (the new
# trajectory test, host-draw parity, fp32 Metropolis vs the oracle, sharded), then the N2 loop
# with AIQMC_WPIV=0 (partial pivoting every sweep) vs default at 4096 and 512 walkers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_mc_fp32.py tests/test_gpu_sharded.py -m gpu -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/parity_r4m.log 2>&1; rc=$?
echo "parity rc=$rc"; tail -4 gpurun_out/parity_r4m.log
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/ab_r4m.txt
: > $out
for B in 4096 512; do
  for rep in 1 2 3; do
    for t in 0 1; do
      r=$(AIQMC_NOPROF=1 AIQMC_WPIV=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
      echo "wpiv=$t rep$rep $r" | tee -a $out
    done
  done
  for t in 0 1; do
    r=$(AIQMC_WPIV=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
    echo "wpiv=$t events $r" | tee -a $out
  done
done
