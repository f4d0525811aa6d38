set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh > gpurun_out/tests_tail.txt 2>&1; echo "tests rc=$?"; grep -E "passed|failed|FAILED|Error" gpurun_out/tests_tail.txt | tail -8
for rep in 1 2; do
  timeout -k 10 120 python tools/mc_loop.py 20 2>&1 | grep -v amdgpu.ids | sed "s/^/fused rep$rep /"
  AIQMC_NOFUSE_REDUCE=1 timeout -k 10 120 python tools/mc_loop.py 20 2>&1 | grep -v amdgpu.ids | sed "s/^/launches rep$rep /"
done
for W in 512 1024; do
  timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | sed "s/^/fused /"
  AIQMC_NOFUSE_REDUCE=1 timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | sed "s/^/launches /"
done
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r3e.json 2> gpurun_out/bench_r3e.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_r3e.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r3e.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], {k: v['ms_per_step'] for k, v in d.get('strong_scaling_per_rank', {}).items()})"
PMC_TAG=lapmfma AIQMC_LIB_VARIANT=lapmfma bash tools/gpu_pmc3.sh 4096
