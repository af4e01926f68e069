"""GPU probe of the generic element-functor path (examples/generic_example.py):
correctness on a small box against the oracle / the atomic path / the
fixed-physics kernel, bitwise reproducibility, then C2-size timings of the
cell-unit kernel, the atomic kernel and the fixed-physics strip kernels.
usage: python tools/generic_probe.py [n_small] [n_big] [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples"))
import arcanefem_amd as af  # noqa: E402
import generic_example as gx  # noqa: E402
from oracle import oracle as O  # noqa: E402

n_small = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n_big = int(sys.argv[2]) if len(sys.argv) > 2 else 215
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
ctx = af.Context(0)


def vals(bsr):
    return bsr.download()[2].copy()


# ---- small box, k = 1 and 3, both layouts
for k in (1, 3):
    for per_row in (False, True):
        mesh = af.Mesh.structured(ctx, 3, n_small, jitter=0.2, seed=20250220)
        bsr = af.BSRFormat(mesh, k).initialize(per_row)
        bsr.computeSparsity()
        E, nu = 21.0e5, 0.28
        lam, mu = E * nu / ((1 + nu) * (1 - 2 * nu)), E / (2 * (1 + nu))
        kind = gx.POISSON if k == 1 else gx.ELASTICITY
        gx.assemble(bsr, kind, gx.UNITS, overwrite=True, lam=lam, mu=mu)
        a = vals(bsr)
        gx.assemble(bsr, kind, gx.UNITS, overwrite=True, lam=lam, mu=mu)
        a2 = vals(bsr)
        gx.assemble(bsr, kind, gx.UNITS, overwrite=False, lam=lam, mu=mu)
        acc2 = vals(bsr)
        gx.assemble(bsr, kind, gx.ATOMIC, overwrite=True, lam=lam, mu=mu)
        b = vals(bsr)
        if k == 1:
            bsr.assemblePoissonP1(1.0, 0.0)
        else:
            bsr.assembleElasticityP1Ex(lam, 2 * mu)
        c = vals(bsr)
        cells, coords, _ = mesh.download()
        orp, ocols = O.sparsity(mesh.n_nodes, mesh.n_own_nodes, cells)
        if k == 1:
            ov, _ = O.assemble_poisson(mesh.n_own_nodes, cells, coords, orp, ocols, 0.0)
        else:
            ov, _ = O.assemble_elasticity_tet(mesh.n_own_nodes, cells, coords, orp, ocols, lam, 2 * mu)
            if per_row:
                ov = O.blocks_to_row_order_k(orp, ov, 3)
        sc = np.abs(ov).max()
        print(f"k={k} per_row={per_row} plan={bsr.functor_plan()} "
              f"units-oracle {np.abs(a - ov).max() / sc:.2e} atomic-oracle {np.abs(b - ov).max() / sc:.2e} "
              f"builtin-oracle {np.abs(c - ov).max() / sc:.2e} repro {np.array_equal(a, a2)} "
              f"accumulate {np.abs(acc2 - 2 * a).max() / sc:.2e}", flush=True)
        bsr.close()
        mesh.close()

# ---- C2 timing
mesh = af.Mesh.structured(ctx, 3, n_big, jitter=0.2, seed=20250220)
bsr = af.BSRFormat(mesh, 1).initialize(True)
bsr.computeSparsity()
ctx.synchronize()
t0 = time.perf_counter()
plan = bsr.functor_plan()
ctx.synchronize()
print(f"n={n_big} plan build {1e3 * (time.perf_counter() - t0):.1f} ms: {plan}", flush=True)
st = bsr.stats()
nnz = bsr.view().nnz_blocks
ab = 4 * st["n_incidences"] + 24 * mesh.n_nodes + 8 * (mesh.n_own_nodes + 1) + 12 * nnz


def timeit(fn, base, r):
    fn()
    ctx.synchronize()
    for i in range(r):
        ctx.event_record(base + 2 * i)
        fn()
        ctx.event_record(base + 2 * i + 1)
    ctx.synchronize()
    return float(np.median([ctx.event_elapsed(base + 2 * i, base + 2 * i + 1) for i in range(r)]))


t_units = timeit(lambda: gx.assemble(bsr, gx.POISSON, gx.UNITS, overwrite=True), 0, reps)
u = vals(bsr)
t_units_acc = timeit(lambda: gx.assemble(bsr, gx.POISSON, gx.UNITS, overwrite=False), 40, 3)
t_atomic = timeit(lambda: gx.assemble(bsr, gx.POISSON, gx.ATOMIC, overwrite=True), 60, 3)
t_fixed = timeit(lambda: bsr.assemblePoissonP1(1.0, 0.0), 80, reps)
f = vals(bsr)
print(f"n={n_big} dof={mesh.n_own_nodes} B_alg={ab / 1e9:.3f} GB units(overwrite) {t_units:.3f} ms "
      f"frac {ab / (t_units * 1e-3) / 8e12:.3f} | units(accumulate) {t_units_acc:.3f} | atomic {t_atomic:.3f} ms "
      f"frac {ab / (t_atomic * 1e-3) / 8e12:.3f} | fixed {t_fixed:.3f} ms | max|units-fixed|/max "
      f"{np.abs(u - f).max() / np.abs(f).max():.2e}", flush=True)

# ---- lean element physics (cofactor form, one reciprocal per cell) on the same box
t_lean = timeit(lambda: gx.assemble(bsr, gx.POISSON_LEAN, gx.UNITS, overwrite=True), 100, reps)
ln = vals(bsr)
print(f"n={n_big} units(lean cofactor functor) {t_lean:.3f} ms frac {ab / (t_lean * 1e-3) / 8e12:.3f} "
      f"max|lean-fixed|/max {np.abs(ln - f).max() / np.abs(f).max():.2e}", flush=True)
bsr.close()
mesh.close()

# ---- unstructured: the bench's L-shape-3D refined `levels` times (argv[4], 0 = skip)
levels = int(sys.argv[4]) if len(sys.argv) > 4 else 0
if levels > 0:
    import bench
    from arcanefem_amd.gmsh import read_gmsh

    gm = read_gmsh(os.path.join(ROOT, "tests", "golden", "L-shape-3D.msh"))
    cells, coords = bench.refine_tets(gm.cells, gm.coords, levels, "cpu")
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    del cells, coords
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ctx.synchronize()
    t0 = time.perf_counter()
    plan = bsr.functor_plan()
    ctx.synchronize()
    print(f"unstructured levels={levels} dof={mesh.n_own_nodes} plan build {1e3 * (time.perf_counter() - t0):.1f} ms: "
          f"{plan}", flush=True)
    st = bsr.stats()
    nnz = bsr.view().nnz_blocks
    ab = 4 * st["n_incidences"] + 24 * mesh.n_nodes + 8 * (mesh.n_own_nodes + 1) + 12 * nnz
    t_fixed = timeit(lambda: bsr.assemblePoissonP1(1.0, 0.0), 120, reps)
    f = vals(bsr)
    t_lean = timeit(lambda: gx.assemble(bsr, gx.POISSON_LEAN, gx.UNITS, overwrite=True), 160, reps)
    ln = vals(bsr)
    t_mod = timeit(lambda: gx.assemble(bsr, gx.POISSON, gx.UNITS, overwrite=True), 200, reps)
    print(f"unstructured: fixed strip {t_fixed:.3f} ms frac {ab / (t_fixed * 1e-3) / 8e12:.3f} | units(lean) "
          f"{t_lean:.3f} ms frac {ab / (t_lean * 1e-3) / 8e12:.3f} | units(module) {t_mod:.3f} ms frac "
          f"{ab / (t_mod * 1e-3) / 8e12:.3f} | max|lean-fixed|/max {np.abs(ln - f).max() / np.abs(f).max():.2e}",
          flush=True)
