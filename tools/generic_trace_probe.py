"""Round-6 probe of the r05j SIGSEGV: the generic_unstructured
leg aborted under `rocprofv3 --kernel-trace` at the launch of the wide
k_assemble_units instance from examples/libafem_generic_example.so.  Runs the
leg's steps with the library loaded before / after torch (whose wheel bundles
a second HIP + HSA runtime and rocprofiler-register, ROCm 7.0) or without torch
at all.  Usage: python tools/generic_trace_probe.py {torch_first,gx_first,no_torch} LEVELS"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples"))


def refine_np(cells, coords, levels):
    c = np.asarray(cells, dtype=np.int64)
    x = np.asarray(coords, dtype=np.float64)
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    for _ in range(levels):
        n = x.shape[0]
        e = np.stack([np.stack([c[:, i], c[:, j]], -1) for i, j in pairs], 1)
        key = e.min(-1) * n + e.max(-1)
        uk, inv = np.unique(key.reshape(-1), return_inverse=True)
        mid = n + inv.reshape(-1, 6)
        x = np.concatenate([x, 0.5 * (x[uk // n] + x[uk % n])])
        v0, v1, v2, v3 = c.T
        m01, m02, m03, m12, m13, m23 = mid.T
        ch = [(v0, m01, m02, m03), (m01, v1, m12, m13), (m02, m12, v2, m23), (m03, m13, m23, v3),
              (m01, m02, m03, m13), (m01, m02, m12, m13), (m02, m03, m13, m23), (m02, m12, m13, m23)]
        c = np.stack([np.stack(t, 1) for t in ch], 1).reshape(-1, 4)
    return c.astype(np.int32), x


def main():
    mode, levels = sys.argv[1], int(sys.argv[2])
    import arcanefem_amd as af
    import generic_example as gx
    from arcanefem_amd.gmsh import read_gmsh

    ctx = af.Context(0)
    if mode == "gx_first":
        gx.load()
    gm = read_gmsh(os.path.join(ROOT, "tests", "golden", "L-shape-3D.msh"))
    if mode == "no_torch":
        cells, coords = refine_np(gm.cells, gm.coords, levels)
    else:
        import bench
        cells, coords = bench.refine_tets(gm.cells, gm.coords, levels, "cpu")
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    plan = bsr.functor_plan()
    print(mode, "plan wide", plan["wide"], "units", plan["n_units"], flush=True)
    for _ in range(3):
        gx.assemble(bsr, gx.POISSON, gx.UNITS, overwrite=True)
    ctx.synchronize()
    print(mode, "ok", "torch loaded:", "torch" in sys.modules, flush=True)
    bsr.close()
    mesh.close()


if __name__ == "__main__":
    main()
