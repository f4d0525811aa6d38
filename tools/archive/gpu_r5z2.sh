# round 5, after the packed-F2 change (library 4fbb6bf3): the -m gpu suite, smoke, PMC passes
# stamped for the library, then the default bench (which reads them)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/tests_tail.txt | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.txt 2>&1 || { tail -20 gpurun_out/smoke.txt; exit 1; }
grep SMOKE_OK gpurun_out/smoke.txt
bash tools/gpu_r5u.sh
