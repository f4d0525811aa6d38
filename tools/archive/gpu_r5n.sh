# round 5: proposal workgroups of 10 / 4 waves with the F4/B2 lane-order weights staged once per
# workgroup in LDS (AQ_XW_LDS) vs the 2-wave default: positions bitwise, N2 loop at 4096 / 512 walkers
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for t in base w10 w10x w4x; do
  AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/pos_dump.py gpurun_out/ab/pos_$t.npy > /dev/null 2>&1 || { echo "$t pos_dump FAILED"; exit 1; }
done
python3 - base w10 w10x w4x <<'PY'
import sys, numpy as np
ref = np.load(f"gpurun_out/ab/pos_{sys.argv[1]}.npy")
for t in sys.argv[2:]:
    x = np.load(f"gpurun_out/ab/pos_{t}.npy")
    print(f"{t} vs {sys.argv[1]}: bitwise equal {np.array_equal(x, ref)}, max |diff| {np.max(np.abs(x - ref)):.3e}")
PY
for rep in 1 2 3; do for W in 4096 512; do for t in base w10 w10x w4x; do
  r=$(AIQMC_LIB_VARIANT=$t timeout -k 10 120 python tools/mc_loop.py 20 N2 $W 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo "$t FAILED"; exit 1; }
  echo "$t W=$W rep$rep $r"
done; done; done
