# round 4: texture-address / vector-L1 pressure of the N2 kernels (rocprofv3 --pmc, one pass each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_ta
rm -rf $OUT; mkdir -p $OUT
cd /tmp
passes=(
 "ta=SQ_WAVES TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
 "tcp=SQ_WAVES TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
 "tad=SQ_WAVES TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE"
)
for spec in "${passes[@]}"; do
  name=${spec%%=*}; ctrs=${spec#*=}
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "k_walker" -d "$OUT/$name" -o "$name" -f csv -- python3 $GRAFT_REPO_ROOT/tools/mc_loop.py 2 N2 4096 > "$OUT/$name.log" 2>&1 || { echo "PASS $name FAILED"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name done"
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, collections, os
root = "gpurun_out/pmc_ta"
for name in ("ta", "tcp", "tad"):
    for f in glob.glob(os.path.join(root, name, "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:48] + " g" + r.get("Grid_Size", r.get("Grid_Size_X", "?"))
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
        for k in sorted(acc):
            d = {c: v / len(n[k]) for c, v in acc[k].items()}
            print(name, k, {c: round(v, 1) for c, v in d.items()})
PY
