set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pgrad.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_pgrad.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|^E " gpurun_out/pytest_pgrad.log | head -40
exit $rc
