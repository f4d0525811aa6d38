# round 5: does the headline depend on how long the GPU has been busy before the timed region
# (clock ramp)?  bench.py head only, --warmup 5 vs 100, interleaved, and --steps 20 vs 200
set -o pipefail
cd $GRAFT_REPO_ROOT
F="--no-ecp --no-adam --no-dmc --no-cpu-baseline --no-per-rank"
for rep in 1 2; do
  for spec in "20 5" "20 100" "200 5"; do
    set -- $spec
    r=$(timeout -k 10 200 python bench.py --steps $1 --warmup $2 $F 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms']*1e3,1), round(d['roofline_local_energy']['avg_launch_ms']*1e3,1))") || { echo FAIL; exit 1; }
    echo "steps=$1 warmup=$2 rep$rep: ms_per_step proposal_us el_pair_us = $r"
  done
done
