"""Cube kernel at C2: the same assembly timed (HIP events) three ways in one
process -- back to back with no synchronisation, with a synchronisation after
each launch, and inside the bench's step (assembly + penalty list + forced
values) -- to tell sustained-load clocks from the step's other kernels.
usage: python tools/b2b_probe.py [n=215] [reps=30]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 215
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ctx = af.Context(0)
mesh, bsr, ls, bottom, dbottom, _ = bench.poisson_setup(ctx, af, n, None, 1, 0)
step = bench.make_step(ctx, bsr, ls, bottom, dbottom)
rhs = ls.rhsVariable()


def run(mode):
    for _ in range(5):
        step()
    ctx.synchronize()
    for i in range(reps):
        if mode == "step":
            step(2 * i)
        else:
            ctx.event_record(2 * i)
            bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set")
            ctx.event_record(2 * i + 1)
            if mode == "sync":
                ctx.synchronize()
    ctx.synchronize()
    t = [ctx.event_elapsed(2 * i, 2 * i + 1) for i in range(reps)]
    return float(np.median(t)), float(np.median(t[-10:]))


for mode in ("b2b", "sync", "step", "b2b", "sync", "step"):
    m, l10 = run(mode)
    print(f"{mode:5s} median {m:.4f} ms  last10 {l10:.4f}", flush=True)
