# round 5: PMC passes stamped for the shipped library, then the default bench (which reads them)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PMC_ROUND=r05 bash tools/gpu_pmc3.sh 4096 && cp gpurun_out/pmc_r05.json profiles/pmc_r05.json || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_final.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['pmc_null_reason'])"
