# round 4: A/B of dev libraries given as arguments (N2 loop at 4096 and 512 walkers, three
# interleaved reps), then the N2 fp32 parity tests on the last one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_r4d.txt
: > $out
for B in 4096 512; do
  for rep in 1 2 3; do
    for t in "$@"; do
      r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || { echo "$t FAILED" >> $out; exit 1; }
      echo "$t rep$rep $r" | tee -a $out
    done
  done
done
last=${@: -1}
AIQMC_LIB_VARIANT=$last timeout -k 10 300 python -u -m pytest tests/test_gpu_mc_fp32.py tests/test_precision_fp32.py tests/test_gpu_parity.py -k "N2 or fp32 or mc" -m gpu -q -rf --timeout 180 --timeout-method thread > gpurun_out/parity_r4d.log 2>&1; echo "parity rc=$?"; tail -5 gpurun_out/parity_r4d.log
