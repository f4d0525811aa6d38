#!/bin/bash
# k_quad_value fixed-order LU (walker pivot record) vs per-configuration partial pivoting:
# interleaved timing of the C / C2 ccECP pp local energy and T-moves on two dev libraries
# (tools/build_variant.sh qfix "" / qpiv -DAQ_QUAD_PIVOTED, DEVSHAPES="8_2 4_1"), then the
# outputs compared (not bitwise: the pivot order differs, the determinant ratios agree to rounding).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export ECP_SYSTEMS="C_ecp C2_ecp"
for r in 1 2 3; do
  for v in qfix qpiv; do
    AIQMC_LIB_VARIANT=$v timeout -k 10 240 python tools/ecp_tm_ab.py gpurun_out/q_$v.npz | sed "s/^/$v /"
  done
done
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/q_qfix.npz"), np.load("gpurun_out/q_qpiv.npz")
for k in a.files:
    x, y = a[k].astype(np.float64), b[k].astype(np.float64)
    d = np.abs(x - y); s = np.maximum(np.abs(y), 1.0)
    print(k, "max_abs", float(d.max()), "max_rel", float((d / s).max()), "bitwise", bool((a[k] == b[k]).all()))
PY
