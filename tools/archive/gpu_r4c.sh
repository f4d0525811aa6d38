# round 4: per-phase cycles of the walker and proposal launches (N2, 4096 and 512 walkers)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 4096 512; do
  WALKERS=$B AIQMC_LIB_VARIANT=phaseprof timeout -k 10 120 python profiles/phase_prof.py > gpurun_out/phase_$B.json 2> gpurun_out/phase_$B.err || { tail -5 gpurun_out/phase_$B.err; exit 1; }
  echo "B=$B"; cat gpurun_out/phase_$B.json
done
