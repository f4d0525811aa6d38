# round 4: the 7-waves/SIMD compact proposal instantiation (PW7) vs the 5-wave one, N2 loop without HIP
# events at 512 / 1024 / 2048 walkers (AIQMC_PW7=0/1, three interleaved reps), then the N2 fp32 parity
# tests and the sharded tests with PW7 forced on
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_r4k.txt
: > $out
for B in 512 1024 2048; do
  for rep in 1 2 3; do
    for t in 0 1; do
      r=$(AIQMC_NOPROF=1 AIQMC_PW7=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || { echo "$t FAILED" >> $out; exit 1; }
      echo "pw7=$t rep$rep $r" | tee -a $out
    done
  done
  for t in 0 1; do
    r=$(AIQMC_PW7=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
    echo "pw7=$t events $r" | tee -a $out
  done
done
for rep in 1 2; do
  echo "philox $(AIQMC_NOPROF=1 timeout -k 10 120 python tools/mc_loop.py 20 N2 512)" | tee -a $out || exit 1
  echo "host   $(AIQMC_NOPROF=1 AIQMC_HOST_DRAWS=1 timeout -k 10 120 python tools/mc_loop.py 20 N2 512)" | tee -a $out || exit 1
done
AIQMC_PW7=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_mc_fp32.py tests/test_precision_fp32.py tests/test_gpu_parity.py -m gpu -q -rf --timeout 180 --timeout-method thread > gpurun_out/parity_pw7.log 2>&1; echo "parity rc=$?"; tail -3 gpurun_out/parity_pw7.log
