"""Run only the C-atom ECP side measurement of bench.py (for PMC passes on the N=4 kernels)."""
import json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
sys.path.insert(0, bench.PKG)
print(json.dumps(bench.ecp_side_bench(torch.float32, torch.device("cuda", 0), 4096, 3, False)))
