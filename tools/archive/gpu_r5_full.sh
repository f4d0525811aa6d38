# round-5 measurement pass: GPU suite, fp32 tail, default bench, rocprofv3 kernel stats of the
# bench, PMC passes stamped with the library hash (gpurun_out/pmc_r04.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/tests_tail.txt | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python tools/fp32_tail.py > gpurun_out/fp32_tail.txt 2>&1; grep -v amdgpu.ids gpurun_out/fp32_tail.txt | head -14
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline_local_energy']['avg_launch_ms'], {k: v['ms_per_step'] for k, v in d.get('strong_scaling_per_rank', {}).items()})"
rm -rf gpurun_out/prof
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err || { echo PROF_FAIL; exit 1; }
cd $GRAFT_REPO_ROOT && python3 profiles/summarize.py gpurun_out/prof > gpurun_out/prof_summary.json && echo PROF_OK
PMC_ROUND=r05 bash tools/gpu_pmc3.sh 4096
