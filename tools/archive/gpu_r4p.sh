# round 4: rocprofv3 kernel trace of the N2 loop (no HIP events) at 4096 and 512 walkers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 4096 512; do
  AIQMC_NOPROF=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_loop_$B -o run -- python tools/mc_loop.py 10 N2 $B > gpurun_out/prof_loop_$B.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_loop_$B -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/loop_kernel_stats_$B.csv
  head -12 gpurun_out/loop_kernel_stats_$B.csv | cut -c1-160
done
