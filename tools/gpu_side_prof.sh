# Side measurements of the bench (ccECP C / C2 E_L, Be Adam, Ne DMC): rocprofv3 kernel-trace summary of
# tools/side_loop.py, then PMC passes (one process per side configuration and counter group),
# summarised by profiles/pmc_side.py into gpurun_out/pmc_side_${PMC_ROUND:-r06}.json (library-stamped)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_side
rm -rf $OUT gpurun_out/side_prof; mkdir -p $OUT
SHA=$(python3 -c "import sys; sys.path.insert(0,'ab-initio-flexible-gaussian-basis-neural-network-quantum-monte-carlo_amd'); import aiqmc._lib as l; print(l.library_sha16())")
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/side_prof -o side -- python3 $GRAFT_REPO_ROOT/tools/side_loop.py > $GRAFT_REPO_ROOT/gpurun_out/side_prof.log 2>&1 || { echo SIDE_TRACE_FAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/side_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 profiles/summarize.py gpurun_out/side_prof > gpurun_out/side_prof_summary.json && echo SIDE_TRACE_OK
passes=(
 "fetch=SQ_WAVES FETCH_SIZE"
 "write=SQ_WAVES WRITE_SIZE"
 "mix=SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32"
)
cd /tmp
for side in ecp_c ecp_c2 adam_be dmc_ne; do
  for spec in "${passes[@]}"; do
    name=${spec%%=*}; ctrs=${spec#*=}
    mkdir -p $OUT/$side
    timeout -s KILL 180 rocprofv3 --pmc $ctrs --kernel-include-regex "k_quad|k_walker" \
      -d "$OUT/$side/$name" -o "$name" -f csv -- python3 $GRAFT_REPO_ROOT/tools/side_loop.py $side > "$OUT/$side/$name.log" 2>&1 || { echo "PASS $side $name FAILED"; tail -5 "$OUT/$side/$name.log"; exit 1; }
    echo "pass $side $name done"
  done
done
cd $GRAFT_REPO_ROOT && python3 profiles/pmc_side.py $OUT $SHA > gpurun_out/pmc_side_${PMC_ROUND:-r06}.json && echo PMC_SIDE_OK
