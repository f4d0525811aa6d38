# round 5: ECP A/B of the in-tree library (main) against a saved copy (old): per-pair radial factors,
# then the T-move cdf once per row in LDS; outputs bitwise, ms per pp E_L batch and per T-move step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2; do for t in old main; do
  if [ $t = main ]; then unset AIQMC_LIB_VARIANT; else export AIQMC_LIB_VARIANT=$t; fi
  r=$(timeout -k 10 180 python tools/ecp_tm_ab.py gpurun_out/ab/ecp_$t.npz 2>&1 | grep -v amdgpu.ids | tail -n 1) || { echo "$t FAILED: $r"; exit 1; }
  echo "$t rep$rep $r"
done; done
unset AIQMC_LIB_VARIANT
python3 - <<'PY'
import numpy as np
a = np.load("gpurun_out/ab/ecp_old.npz"); b = np.load("gpurun_out/ab/ecp_main.npz")
for k in a.files:
    print(k, "bitwise", np.array_equal(a[k], b[k]), "max|d|", float(np.max(np.abs(a[k] - b[k]))) if a[k].size else 0.0)
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_ecp.py tests/test_dmc.py tests/test_gpu_pgrad.py > gpurun_out/r5s_tests.txt 2>&1 || { tail -30 gpurun_out/r5s_tests.txt; exit 1; }
tail -1 gpurun_out/r5s_tests.txt
