"""Prints the strip signatures (shift/swap pattern, steps, width, slot stream)
of the uniform slices of Kuhn boxes (AFEM_DEBUG_PATTERNS diagnostic of the
structure build).  usage: AFEM_DEBUG_PATTERNS=1 python tools/pattern_probe.py [n ...]"""
import os
import sys

sys.path.insert(0, os.getcwd())
import arcanefem_amd as af  # noqa: E402

ctx = af.Context(0)
for n in [int(a) for a in sys.argv[1:]] or [60, 215]:
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    print(n, bsr.stats()["uniform_slices"], bsr.stats()["n_slices"], flush=True)
