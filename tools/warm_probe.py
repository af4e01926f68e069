"""Where the cube kernel's slow first launches come from (C2): 60 launches of
the stencil kernel back to back, then the cube kernel (per-launch HIP event
times, in groups of 10), then a 2 s pause, then the cube kernel again.
usage: python tools/warm_probe.py [n=215]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 215
ctx = af.Context(0)
mesh, bsr, ls, bottom, dbottom, _ = bench.poisson_setup(ctx, af, n, None, 1, 0)
rhs = ls.rhsVariable()


def run(cubes, reps):
    af.set_variant("AFEM_ASSEMBLY_CUBES", cubes)
    for i in range(reps):
        ctx.event_record(2 * i)
        bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set")
        ctx.event_record(2 * i + 1)
    ctx.synchronize()
    t = [ctx.event_elapsed(2 * i, 2 * i + 1) for i in range(reps)]
    return " ".join(f"{np.median(t[k:k + 10]):.3f}" for k in range(0, reps, 10))


print("cubes first   ", run("1", 60), flush=True)
print("stencil       ", run("0", 60), flush=True)
print("cubes again   ", run("1", 60), flush=True)
time.sleep(2.0)
print("cubes after 2s", run("1", 60), flush=True)
print("stencil       ", run("0", 60), flush=True)
