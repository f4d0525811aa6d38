# PMC passes (one rocprofv3 process per pass, counters only) over tools/mc_loop.py, summarised.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
rm -rf $OUT; mkdir -p $OUT
passes=(
 "mix=SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
 "stall=SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_THREAD_CYCLES_VALU"
 "misc=SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS"
 "mem=SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VALU2"
 "fetch=SQ_WAVES FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
 "write=SQ_WAVES WRITE_SIZE"
 "noreuse_mix=SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_LDS"
 "noreuse_fetch=SQ_WAVES FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
 "noreuse_write=SQ_WAVES WRITE_SIZE"
)
cd /tmp
for spec in "${passes[@]}"; do
  name=${spec%%=*}; ctrs=${spec#*=}
  nr=""; [[ $name == noreuse_* ]] && nr=1
  AIQMC_NOREUSE=$nr timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "k_walker|k_moved|k_accept|k_taueff" \
    -d "$OUT/$name" -o "$name" -f csv -- python3 $GRAFT_REPO_ROOT/tools/mc_loop.py 2 > "$OUT/$name.log" 2>&1 || { echo "PASS $name FAILED"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "pass $name done"
done
cd $GRAFT_REPO_ROOT && python3 profiles/pmc_summary.py $OUT > gpurun_out/pmc_summary.txt && \
  python3 profiles/pmc_r02.py $OUT > gpurun_out/pmc_r02.json && echo PMC_OK
