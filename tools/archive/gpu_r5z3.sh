# round 5: N <= 4 packed LU / Gauss-Jordan: the pivot row entry A[p][c] by DPP row rotations + select
# instead of two lane permutes per elimination step (k_quad_value, k_quad_grad), qvold = HEAD vs
# qvnew dev libraries (shapes 4_1, 8_2).  Outputs bitwise (pp E_L,
# T-moves, Metropolis positions), then ms per pp E_L batch / T-move step and per VMC iteration.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
out=gpurun_out/ab_r5z3.txt
: > $out
export ECP_SYSTEMS="C_ecp C2_ecp"
for t in qvold qvnew; do
  export AIQMC_LIB_VARIANT=$t
  for s in Be C_ecp C2_ecp; do
    timeout -k 10 120 python tools/pos_dump.py gpurun_out/ab/pos_${t}_$s.npy $s > /dev/null 2>&1 || { echo "pos_dump $t $s FAILED"; exit 1; }
  done
done
for rep in 1 2 3; do for t in qvold qvnew; do
  export AIQMC_LIB_VARIANT=$t
  r=$(timeout -k 10 180 python tools/ecp_tm_ab.py gpurun_out/ab/ecp_$t.npz 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo "$t FAILED: $r"; exit 1; }
  echo "$t rep$rep $r" | tee -a $out
done; done
for s in Be C_ecp C2_ecp; do
  for rep in 1 2; do for t in qvold qvnew; do
    r=$(AIQMC_LIB_VARIANT=$t AIQMC_NOPROF=1 timeout -k 10 120 python tools/mc_loop.py 20 $s 4096 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo "$t $s FAILED: $r"; exit 1; }
    echo "$t rep$rep $r" | tee -a $out
  done; done
  for t in qvold qvnew; do
    r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 $s 4096 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo "$t $s FAILED: $r"; exit 1; }
    echo "$t events $r" | tee -a $out
  done
done
python3 - <<'PY' | tee -a $out
import numpy as np
a, b = np.load("gpurun_out/ab/ecp_qvold.npz"), np.load("gpurun_out/ab/ecp_qvnew.npz")
for k in a.files:
    print(k, "bitwise", np.array_equal(a[k], b[k]), "max|d|", float(np.nanmax(np.abs(a[k] - b[k]))))
for s in ("Be", "C_ecp", "C2_ecp"):
    x, y = np.load(f"gpurun_out/ab/pos_qvold_{s}.npy"), np.load(f"gpurun_out/ab/pos_qvnew_{s}.npy")
    print(s, "positions bitwise", np.array_equal(x, y), "max|d|", float(np.abs(x - y).max()))
PY
# rocprofv3 kernel stats of the default bench on the shipped library (this step failed here: the
# variant stayed exported; tools/gpu_r5z4.sh runs it)
unset AIQMC_LIB_VARIANT
rm -rf gpurun_out/prof
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof.err || { echo PROF_FAIL; exit 1; }
cd $GRAFT_REPO_ROOT && python3 profiles/summarize.py gpurun_out/prof > gpurun_out/prof_summary.json && echo PROF_OK
