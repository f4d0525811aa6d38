# round 4: (1) the cost of the HIP events around the launches (profile on/off), N2 loop at 4096 and 512;
# (2) tests/test_gpu_sharded.py (two and eight gloo ranks, 32,768 walkers in 8 blocks, bench N=8 line)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 4096 512; do for rep in 1 2 3; do
  echo "events   $(timeout -k 10 120 python tools/mc_loop.py 20 N2 $B)" || exit 1
  echo "noevents $(AIQMC_NOPROF=1 timeout -k 10 120 python tools/mc_loop.py 20 N2 $B)" || exit 1
done; done
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/sharded.log 2>&1; rc=$?; tail -5 gpurun_out/sharded.log; exit $rc
