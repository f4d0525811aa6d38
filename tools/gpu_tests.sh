# GPU: the -m gpu suite (optionally filtered: PYTEST_K), log under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${SUITE_TIMEOUT:-900} python -u -m pytest tests -m gpu -q -rf --timeout 180 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
exit $rc
