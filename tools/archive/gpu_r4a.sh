# round 4: new fp32 Metropolis / limdrift tests, then the whole -m gpu suite, then the N2 loop at
# 4096 and 512 walkers (no-regression check of the guarded reduction)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mc_fp32.py -m gpu -q -s -rf --timeout 180 --timeout-method thread > gpurun_out/mc_fp32.log 2>&1; rc=$?
grep -E "reference|flips|vs float64|oracle fp32|two sweeps|x_hip|passed|failed|Error" gpurun_out/mc_fp32.log | head -80
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; echo "suite rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/tests_tail.txt | tail -8
for B in 4096 512; do timeout -k 10 120 python tools/mc_loop.py 20 N2 $B || exit 1; done
