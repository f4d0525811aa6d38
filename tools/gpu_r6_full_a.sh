# round 6 measurement pass, part A (shipped library): -m gpu suite, smoke, PMC passes of the N2 loop
# (profiles/pmc_r06.json) and of the side configurations (profiles/pmc_side_r06.json), both stamped
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SUITE_TIMEOUT=900 bash tools/gpu_tests.sh > gpurun_out/r6f_suite_tail.txt 2>&1; rc=$?; tail -4 gpurun_out/r6f_suite_tail.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6f_smoke.txt 2>&1 || { echo SMOKE_FAIL; tail gpurun_out/r6f_smoke.txt; exit 1; }
tail -1 gpurun_out/r6f_smoke.txt
PMC_ROUND=r06 bash tools/gpu_pmc3.sh > gpurun_out/r6f_pmc.txt 2>&1 || { echo PMC_FAIL; tail -5 gpurun_out/r6f_pmc.txt; exit 1; }
tail -2 gpurun_out/r6f_pmc.txt
PMC_ROUND=r06 bash tools/gpu_side_prof.sh > gpurun_out/r6f_side.txt 2>&1 || { echo SIDE_FAIL; tail -5 gpurun_out/r6f_side.txt; exit 1; }
tail -3 gpurun_out/r6f_side.txt
