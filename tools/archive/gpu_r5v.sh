# round 5: k_quad_value with 1 / 2 / 4 independent waves per workgroup (C and C2 ccECP dev libraries):
# pp E_L and T-move outputs bitwise, ms per call
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export ECP_SYSTEMS="C_ecp C2_ecp"
for rep in 1 2 3; do for t in qv1 qv2 qv4; do
  export AIQMC_LIB_VARIANT=$t
  r=$(timeout -k 10 180 python tools/ecp_tm_ab.py gpurun_out/ab/ecp_$t.npz 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo "$t FAILED: $r"; exit 1; }
  echo "$t rep$rep $r"
done; done
python3 - <<'PY'
import numpy as np
a = np.load("gpurun_out/ab/ecp_qv1.npz")
for t in ("qv2", "qv4"):
    b = np.load(f"gpurun_out/ab/ecp_{t}.npz")
    print(t, "vs qv1 bitwise:", all(np.array_equal(a[k], b[k]) for k in a.files))
PY
