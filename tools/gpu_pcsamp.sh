# PC sampling of the N2 MC loop (which instructions the proposal kernel's waves sit on)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pcs
rm -rf $OUT; mkdir -p $OUT
cd /tmp
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-stochastic} --pc-sampling-unit ${PCS_UNIT:-cycles} --pc-sampling-interval ${PCS_INTERVAL:-65536} -d $OUT -o pcs -f csv -- python3 $GRAFT_REPO_ROOT/tools/mc_loop.py 2 > $OUT/run.log 2>&1
rc=$?
echo "rc=$rc"; tail -5 $OUT/run.log; find $OUT -type f | head; 
