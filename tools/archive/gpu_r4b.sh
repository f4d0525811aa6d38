# round 4: MFMA on the proposal path (Phi formation, B1): interleaved A/B of dev libraries
# (base = round-3 kernel, phi = Phi on MFMA, both = Phi + B1 on MFMA) at 4096 and 512 walkers,
# then the N2 fp32 parity tests on the 'both' library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_mfma.txt
: > $out
for B in 4096 512; do
  for rep in 1 2 3; do
    for t in base phi both; do
      r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || { echo "$t FAILED" >> $out; exit 1; }
      echo "$t rep$rep $r" | tee -a $out
    done
  done
done
AIQMC_LIB_VARIANT=both timeout -k 10 300 python -u -m pytest tests/test_gpu_mc_fp32.py tests/test_precision_fp32.py -m gpu -q -rf --timeout 180 --timeout-method thread > gpurun_out/parity_both.log 2>&1; echo "parity rc=$?"; tail -5 gpurun_out/parity_both.log
