# round 4: the -m gpu suite on the in-tree library, then the N2 loop at 4096 and 512 walkers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; rc=$?; echo "suite rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/tests_tail.txt | tail -8
[ $rc -eq 0 ] || exit $rc
for B in 4096 512; do for rep in 1 2; do timeout -k 10 120 python tools/mc_loop.py 20 N2 $B || exit 1; done; done
