# round 5: k_quad_value / k_quad_grad F2 without the [SW][12] pair-value block (new - old by a DPP
# row shift; LDS per wave 5,632 -> 3,328 B for the C atom's quadrature launch, 8,384 -> 6,080 B for
# its proposals): qvold (HEAD) vs qvnew dev libraries (shapes 4_1, 8_2).  Outputs bitwise (pp E_L,
# T-moves, Metropolis positions), then ms per pp E_L batch / T-move step and per VMC iteration.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
out=gpurun_out/ab_r5z.txt
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
