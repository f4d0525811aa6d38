# round 5: range-safe pivots (both sides), anchored walker pivot order, bench --gpus spawn
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32_pivot_range.py tests/test_gpu_fp32_statistics.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "pivot or far_electron or spawns_ranks" > gpurun_out/r5a_tests.log 2>&1
rc=$?; tail -30 gpurun_out/r5a_tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ecp --no-adam --no-dmc > gpurun_out/r5a_bench.json 2> gpurun_out/r5a_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r5a_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5a_bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline_local_energy']['avg_launch_ms'], d['walker_grad_avg_ms'], {k: v['ms_per_step'] for k, v in d.get('strong_scaling_per_rank', {}).items()})"
