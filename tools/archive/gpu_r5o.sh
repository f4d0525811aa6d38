# round 5: the fixed-order Gauss-Jordan's pivot-row broadcast across row groups by gfx950 row swaps
# (v_permlane16/32_swap, AQ_GJ_PERMLANE) instead of ds_bpermute: positions bitwise, N2 loop timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
VARS="${VARS:-base gjpl}"
for t in $VARS; do
  AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/pos_dump.py gpurun_out/ab/pos_$t.npy > /dev/null 2>&1 || { echo "$t pos_dump FAILED"; exit 1; }
done
python3 - $VARS <<'PY'
import sys, numpy as np
ref = np.load(f"gpurun_out/ab/pos_{sys.argv[1]}.npy")
for t in sys.argv[2:]:
    x = np.load(f"gpurun_out/ab/pos_{t}.npy")
    print(f"{t} vs {sys.argv[1]}: bitwise equal {np.array_equal(x, ref)}, max |diff| {np.max(np.abs(x - ref)):.3e}")
PY
for rep in 1 2 3; do for W in 4096 512; do for t in $VARS; do
  r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo "$t FAILED"; exit 1; }
  echo "$t W=$W rep$rep $r"
done; done; done
