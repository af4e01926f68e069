"""The C4 leg alone (bench.py poisson_c4: n=463 Poisson box on one GPU,
assembly warmup 2 + `reps` timed, then 50 fixed Jacobi-PCG iterations), so a
rocprofv3 trace or PMC pass sees only C4's dispatches.
usage: python tools/c4_probe.py [n=463] [cg_iters=50] [reps=5]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 463
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
ctx = af.Context(0)
print(json.dumps(bench.poisson_c4(ctx, af, n, reps=reps, cg_iters=iters)), flush=True)
