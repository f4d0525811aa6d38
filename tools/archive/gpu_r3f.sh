set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 120 python tools/mc_loop.py 20 2>&1 | grep -v amdgpu.ids | sed "s/^/fused rep$rep /"
  AIQMC_NOFUSE_REDUCE=1 timeout -k 10 120 python tools/mc_loop.py 20 2>&1 | grep -v amdgpu.ids | sed "s/^/launches rep$rep /"
done
for W in 512 1024; do
  timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | sed "s/^/fused /"
  AIQMC_NOFUSE_REDUCE=1 timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | sed "s/^/launches /"
done
PYTEST_K="fused" bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; echo "tests rc=$?"; grep -E "passed|failed|FAILED|Error" gpurun_out/tests_tail.txt | tail -8
