"""C5 Newmark steps with one preconditioner (for profiling):
python tools/c5_mg_only.py [n] [steps] [multigrid|jacobi]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
pc = sys.argv[3] if len(sys.argv) > 3 else "multigrid"
ctx = af.Context(0)
print(json.dumps(bench.elastodynamics_c5(ctx, af, n, steps, preconditioners=(pc,))), flush=True)
