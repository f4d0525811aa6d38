#!/bin/bash
# rocprofv3 kernel-trace summary of a short N2 loop (tools/mc_loop.py; AIQMC_LIB_VARIANT selects a dev library):
# per-kernel calls and average µs.  usage: tools/kstats.sh TAG [mc_loop args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
rm -rf gpurun_out/ks_$TAG
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ks_$TAG -o run -- python3 $GRAFT_REPO_ROOT/tools/mc_loop.py "$@" > $GRAFT_REPO_ROOT/gpurun_out/ks_$TAG.log 2>&1 || { echo KS_FAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/ks_$TAG.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/ks_$TAG -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY' | tee gpurun_out/ks_$TAG.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:86]:86s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:9.2f} us')
PY
