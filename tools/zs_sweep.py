"""Cube kernel z-segment length at settled clocks: 150 ms of launches first,
then for each zs the median of `reps` back-to-back launches (HIP events),
interleaved over `rounds` rounds.
usage: python tools/zs_sweep.py n reps rounds zs [zs ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
import bench  # noqa: E402

n, reps, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
zss = sys.argv[4:]
ctx = af.Context(0)
mesh, bsr, ls, bottom, dbottom, _ = bench.poisson_setup(ctx, af, n, None, 1, 0)
rhs = ls.rhsVariable()
asm = lambda: bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set")  # noqa: E731
t = time.perf_counter()
while time.perf_counter() - t < 0.15:
    asm()
    ctx.synchronize()
res = {z: [] for z in zss}
for _ in range(rounds):
    for z in zss:
        af.set_variant("AFEM_CUBES_ZS", z)
        asm()
        for i in range(reps):
            ctx.event_record(2 * i)
            asm()
            ctx.event_record(2 * i + 1)
        ctx.synchronize()
        res[z] += [ctx.event_elapsed(2 * i, 2 * i + 1) for i in range(reps)]
for z in zss:
    print(f"n {n} zs {z:>3s} median {np.median(res[z]):.4f} ms", flush=True)
