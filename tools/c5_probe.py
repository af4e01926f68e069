"""C5 elastodynamics step timing (bench.elastodynamics_c5) in one process;
run it twice with different AFEM_* settings to compare.
usage: python tools/c5_probe.py [n] [steps] [mg]   (mg: the multigrid-preconditioned run only)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = af.Context(0)
pcs = ("multigrid",) if len(sys.argv) > 3 and sys.argv[3] == "mg" else ("multigrid", "jacobi")
out = bench.elastodynamics_c5(ctx, af, n, steps, preconditioners=pcs)
out["AFEM_SPMV"] = os.environ.get("AFEM_SPMV", "")
print(json.dumps(out), flush=True)
