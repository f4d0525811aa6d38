set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dmc.py tests/test_ecp.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tm.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_tm.log; exit 1; }
tail -25 gpurun_out/pytest_tm.log
