# round 4: compact proposal LDS (5.6 KB/wave) at 5 and 7 waves/SIMD vs the shipped layout, N2 loop
# without HIP events at 512 / 1024 / 4096 walkers (three interleaved reps), kernel times from a second
# pass with events; then the N2 fp32 parity tests on c7
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_r4k.txt
: > $out
for B in 512 1024 4096; do
  for rep in 1 2 3; do
    for t in base c5 c7; do
      r=$(AIQMC_NOPROF=1 AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || { echo "$t FAILED" >> $out; exit 1; }
      echo "$t rep$rep $r" | tee -a $out
    done
  done
  for t in base c5 c7; do
    r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
    echo "$t events $r" | tee -a $out
  done
done
AIQMC_LIB_VARIANT=c7 timeout -k 10 300 python -u -m pytest tests/test_gpu_mc_fp32.py tests/test_precision_fp32.py -m gpu -q -rf --timeout 180 --timeout-method thread > gpurun_out/parity_c7.log 2>&1; echo "parity rc=$?"; tail -3 gpurun_out/parity_c7.log
