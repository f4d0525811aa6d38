#!/bin/bash
# Local-energy occupancy probe: N2 dev libraries `base` and `w3` (k_walker_lap compiled for 3 waves/SIMD,
# -DAQ_LAP_WPE=3) at 1 and 2 waves per walker (AIQMC_LAPW), interleaved, plus a kernel trace of the
# base library's loop (prep / lap split at 4096 walkers).  Output under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/lap_occ_ab.txt
: > $out
for rep in 1 2; do
  for t in base w3; do
    for w in 1 2; do
      r=$(AIQMC_LIB_VARIANT=$t AIQMC_LAPW=$w timeout -k 10 120 python tools/mc_loop.py 20) || { echo "$t lapw$w FAILED" >> $out; exit 1; }
      echo "$t lapw$w rep$rep $r" | tee -a $out
    done
  done
done
AIQMC_LIB_VARIANT=base timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/lapprof -o run -- python tools/mc_loop.py 5 > gpurun_out/lapprof.log 2>&1 || exit 1
find gpurun_out/lapprof -name '*kernel_stats.csv' -exec cp {} gpurun_out/lap_kernel_stats.csv \;
python - <<'EOF'
import csv
rows = list(csv.DictReader(open("gpurun_out/lap_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
EOF
