# PMC passes (one rocprofv3 process per pass, counters only) over tools/mc_loop.py, summarised by
# profiles/pmc_r03.py into gpurun_out/pmc_r03.json, stamped with the loaded library's hash.
# usage: bash tools/gpu_pmc3.sh [walkers]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W=${1:-4096}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc3${PMC_TAG:+_$PMC_TAG}
rm -rf $OUT; mkdir -p $OUT
passes=(
 "mix=SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
 "stall=SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
 "misc=SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM"
 "mem=SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
 "fetch=SQ_WAVES FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
 "write=SQ_WAVES WRITE_SIZE"
)
SHA=$(python3 -c "import sys; sys.path.insert(0,'ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd'); import aiqmc._lib as l; print(l.library_sha16())")
cd /tmp
for spec in "${passes[@]}"; do
  name=${spec%%=*}; ctrs=${spec#*=}
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "k_walker|k_moved" \
    -d "$OUT/$name" -o "$name" -f csv -- python3 $GRAFT_REPO_ROOT/tools/mc_loop.py 2 N2 $W > "$OUT/$name.log" 2>&1 || { echo "PASS $name FAILED"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name done"
done
cd $GRAFT_REPO_ROOT && python3 profiles/pmc_r03.py $OUT $SHA $W > gpurun_out/pmc_${PMC_ROUND:-r04}${PMC_TAG:+_$PMC_TAG}.json && echo PMC_OK
