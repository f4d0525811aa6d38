"""Run only the ccECP side measurement of bench.py (for PMC passes on the packed kernels);
ECP_SYSTEM=C2_ecp for the C2 batch (default C_ecp)."""
import json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
sys.path.insert(0, bench.PKG)
print(json.dumps(bench.ecp_side_bench(torch.float32, torch.device("cuda", 0), 4096, 3, False,
                                      name=os.environ.get("ECP_SYSTEM", "C_ecp"))))
