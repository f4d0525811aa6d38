# tests + fp32 tail + mc loop + bench + kernel-trace profile + PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/tests_tail.txt
timeout -k 10 120 python tools/fp32_tail.py > gpurun_out/fp32_tail.txt 2>&1 && cat gpurun_out/fp32_tail.txt | head -14
timeout -k 10 120 python tools/mc_loop.py 5 > gpurun_out/mc_loop.txt 2>&1 && cat gpurun_out/mc_loop.txt
timeout -k 10 120 python tools/graph_probe.py > gpurun_out/graph_probe.txt 2>&1; cat gpurun_out/graph_probe.txt | tail -3
timeout -k 10 120 python -m pytest tests/test_gpu_fullsize.py -q -s -k float32_matches_float64 > gpurun_out/f32_vs_f64.txt 2>&1; grep "fp32 vs fp64" gpurun_out/f32_vs_f64.txt
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json | head -c 1500; echo
rm -rf gpurun_out/prof
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err || { echo PROF_FAIL; exit 1; }
cd $GRAFT_REPO_ROOT && python3 profiles/summarize.py gpurun_out/prof > gpurun_out/prof_summary.json && echo PROF_OK
bash tools/gpu_pmc2.sh
