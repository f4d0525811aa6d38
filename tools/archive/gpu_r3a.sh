set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/tests_tail.txt
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r3a.json 2> gpurun_out/bench_r3a.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_r3a.err; exit 1; }
head -c 1500 gpurun_out/bench_r3a.json; echo
for v in lapvalu lapmfma; do AIQMC_LIB_VARIANT=$v timeout -k 10 120 python tools/lap_parity.py 2>&1 | grep -v amdgpu.ids || exit 1; done
bash tools/ab_variants.sh lapvalu lapmfma
bash tools/gpu_pmc3.sh 4096
