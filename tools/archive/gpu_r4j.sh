# round 4: C parity + packed-vs-one-wave tests, the C2-with-ccECP (8, 2) loop packed vs one-wave,
# and the default bench with the HIP events confined to the last timed iteration
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "C or packed" -m gpu -q -rf --timeout 180 --timeout-method thread > gpurun_out/packed.log 2>&1; rc=$?; tail -4 gpurun_out/packed.log
[ $rc -eq 0 ] || exit $rc
for sys in C2_ecp C; do for rep in 1 2; do
  echo "packed $(timeout -k 10 120 python tools/mc_loop.py 10 $sys 4096)" || exit 1
  echo "onewave $(AIQMC_QUAD_GRAD=0 timeout -k 10 120 python tools/mc_loop.py 10 $sys 4096)" || exit 1
done; done
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['local_energy_evals_per_s'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline_local_energy']['avg_launch_ms'], {k: v['ms_per_step'] for k, v in d.get('strong_scaling_per_rank', {}).items()})"
