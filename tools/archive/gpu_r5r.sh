# round 5: counters of the ccECP quadrature launch (k_quad_value<float,4,1>, BASELINE config 3;
# ECP_SYSTEM=C2_ecp: k_quad_value<float,8,2>; PMC_TAG names the output directory)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_ecp${PMC_TAG:-}
rm -rf $OUT; mkdir -p $OUT
passes=(
 "mix=SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
 "stall=SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
 "misc=SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
)
cd /tmp
for spec in "${passes[@]}"; do
  name=${spec%%=*}; ctrs=${spec#*=}
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "k_quad_value|k_ecp|k_moved_value" \
    -d "$OUT/$name" -o "$name" -f csv -- python3 $GRAFT_REPO_ROOT/tools/ecp_only.py > "$OUT/$name.log" 2>&1 || { echo "PASS $name FAILED"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name done"
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, collections
import os
root = "gpurun_out/pmc_ecp" + os.environ.get("PMC_TAG", "")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    w = sum(d["SQ_WAVES"]) / max(1, len(d["SQ_WAVES"]))
    print(k, {c: round(sum(v) / len(v) / max(w, 1), 1) for c, v in d.items() if c != "SQ_WAVES"}, "waves", w)
PY
