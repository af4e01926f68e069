"""C3 block-3 elasticity assembly leg alone (bench.elasticity_c3), for
profiling: python tools/c3_probe.py [n] [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 170
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctx = af.Context(0)
print(json.dumps(bench.elasticity_c3(ctx, af, n, reps=reps)), flush=True)
