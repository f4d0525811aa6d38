# round 4 probe: the fused limdrift reduction's read (taueff_wave) removed (-DAQ_ABL_TE, wrong
# results, timing only) vs the dev base, N2 loop at 512 / 1024 walkers, per-kernel rocprof
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/ab_r4q.txt
: > $out
for B in 512 1024; do
  for rep in 1 2; do
    for t in base note; do
      r=$(AIQMC_NOPROF=1 AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $B) || exit 1
      echo "$t rep$rep $r" | tee -a $out
    done
  done
done
for t in base note; do
  AIQMC_NOPROF=1 AIQMC_LIB_VARIANT=$t timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q_$t -o run -- python tools/mc_loop.py 10 N2 512 > gpurun_out/prof_q_$t.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_q_$t -name "*kernel_stats.csv" | head -1)
  echo "== $t" | tee -a $out; head -6 "$f" | cut -d, -f1-4 | tee -a $out
done
