# round 5: per-phase cycles of the walker / proposal waves at 512 and 4096 walkers (phaseprof
# library), and a rocprofv3 kernel trace of the N2 loop at 512 walkers on the shipped library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp32_statistics.py -k early -m gpu -q -rf -s --timeout 200 --timeout-method thread > gpurun_out/r5e_tests.log 2>&1
rc=$?; grep -E "^it |passed|failed" gpurun_out/r5e_tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for B in 512 4096; do
  AIQMC_LIB_VARIANT=phaseprof WALKERS=$B timeout -k 10 120 python profiles/phase_prof.py > gpurun_out/r5e_phase_$B.json 2> gpurun_out/r5e_phase_$B.err || { tail -5 gpurun_out/r5e_phase_$B.err; exit 1; }
done
python3 - <<'PY'
import json
for B in (512, 4096):
    d = json.load(open(f"gpurun_out/r5e_phase_{B}.json"))["reuse"]
    for kind in ("walker", "proposal"):
        t = d[kind]["total"]
        print(B, kind, {k: round(100 * v / t, 1) for k, v in d[kind].items() if k != "total"}, "total", t)
PY
rm -rf gpurun_out/prof512
cd /tmp
AIQMC_NOPROF=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof512 -o run -- python3 $GRAFT_REPO_ROOT/tools/mc_loop.py 10 N2 512 > $GRAFT_REPO_ROOT/gpurun_out/r5e_loop512.txt 2>&1 || { echo PROF_FAIL; exit 1; }
cd $GRAFT_REPO_ROOT && python3 profiles/summarize.py gpurun_out/prof512 > gpurun_out/r5e_loop512_summary.json && echo PROF_OK
python3 -c "
import json; d=json.load(open('gpurun_out/r5e_loop512_summary.json'))
for r in d[:12]: print(r['kernel'][:70], r['workgroups'], r['launches'], round(r['avg_us'],1), r.get('vgpr'), r.get('occupancy_waves_per_simd'))
"
