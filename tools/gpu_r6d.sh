# round 6: local-energy stage prefetch A/B (dev libraries base / lpf), then the RCCL / fused-loss tests on the
# in-tree library (F1 LDS-DMA on by default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
VARS="base lpf" bash tools/gpu_r6c.sh && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_mc_fp32.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r6d_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6d_tests.log; exit $rc
