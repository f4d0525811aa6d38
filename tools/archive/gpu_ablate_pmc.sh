# per-ablation instruction counts of the proposal kernel (dev build, -DAQ_ABLATE)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp AIQMC_LIB_VARIANT=dev
OUT=$GRAFT_REPO_ROOT/gpurun_out/abl
rm -rf $OUT; mkdir -p $OUT
cd /tmp
for m in 0 1 2 4 8 16 32 64 127; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 \
    --kernel-include-regex "k_walker_rev" -d $OUT/m$m -o m$m -f csv -- python3 $GRAFT_REPO_ROOT/tools/ablate_one.py $m > $OUT/m$m.log 2>&1 || { echo "mask $m failed"; tail -3 $OUT/m$m.log; exit 1; }
done
cd $GRAFT_REPO_ROOT && python3 - <<'PY'
import csv, glob, collections
rows = {}
for m in [0, 1, 2, 4, 8, 16, 32, 64, 127]:
    agg = collections.defaultdict(float); waves = 0
    for f in glob.glob(f"gpurun_out/abl/m{m}/*/*counter_collection.csv") + glob.glob(f"gpurun_out/abl/m{m}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if int(r["Grid_Size"]) // int(r["Workgroup_Size"]) != 57344: continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    w = agg["SQ_WAVES"]
    rows[m] = {k: v / w for k, v in agg.items() if k != "SQ_WAVES"} if w else {}
keys = ["SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_SALU", "SQ_INSTS_LDS"]
print("mask   " + " ".join(f"{k[9:]:>10s}" for k in keys))
for m, r in rows.items():
    print(f"{m:4d}   " + " ".join(f"{r.get(k, 0):10.1f}" for k in keys))
PY
