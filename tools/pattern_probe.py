import sys, os
sys.path.insert(0, os.getcwd())
import arcanefem_amd as af
ctx = af.Context(0)
for n in (60, 215):
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    print(n, bsr.stats()["uniform_slices"], bsr.stats()["n_slices"], flush=True)
