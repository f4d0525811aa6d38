set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ecp --no-adam --no-dmc --no-per-rank > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_q.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_q.json')); print('BENCH', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
