"""A/B of two builds of libafem on the same box: runs this script's timing
part in two child processes (AFEM_LIB=libA, AFEM_LIB=libB) alternately.
usage: python tools/ab_lib.py libA.so libB.so [n] [reps] [rounds] [mode]
mode: poisson (C2-style scalar assembly, default) | c3 (block-3 elasticity) |
      unstructured (L-shape-3D refined n times, Poisson: the general strip instances)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, ROOT)
    import numpy as np
    import arcanefem_amd as af
    n, reps, mode = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    ctx = af.Context(0)
    if mode == "unstructured":
        import bench
        from arcanefem_amd.gmsh import read_gmsh
        gm = read_gmsh(os.path.join(ROOT, "tests", "golden", "L-shape-3D.msh"))
        cells, coords = bench.refine_tets(gm.cells, gm.coords, n, "cpu")
        mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    else:
        mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
    k = 3 if mode == "c3" else 1
    bsr = af.BSRFormat(mesh, k).initialize(False if k == 3 else True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, k * mesh.n_own_nodes)
    ts = []
    for r in range(reps + 3):
        ctx.event_record(0)
        if k == 3:
            bsr.assembleElasticityP1Ex(1.4e6, 1.6e6, 0.0, (0.0, 0.0, -1.0), ls.rhsVariable(), rhs_mode="set")
        else:
            bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
        ctx.event_record(1)
        ctx.synchronize()
        if r >= 3:
            ts.append(ctx.event_elapsed(0, 1))
    _, _, vals = bsr.download()
    print(f"{np.median(ts):.4f} {np.min(ts):.4f} {float(np.sum(np.abs(vals))):.17g} {bsr.stats()['last_kernel']}",
          flush=True)
    sys.exit(0)
a, b = sys.argv[1], sys.argv[2]
n = sys.argv[3] if len(sys.argv) > 3 else "215"
reps = sys.argv[4] if len(sys.argv) > 4 else "30"
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 2
mode = sys.argv[6] if len(sys.argv) > 6 else "poisson"
res = {a: [], b: []}
for _ in range(rounds):
    for lib in (a, b):
        env = dict(os.environ, AFEM_LIB=os.path.abspath(lib))
        out = subprocess.run([sys.executable, __file__, "--child", n, reps, mode], env=env, capture_output=True,
                             text=True, timeout=300)
        if out.returncode != 0:
            print(out.stdout, out.stderr)
            sys.exit(1)
        res[lib].append(out.stdout.split())
        print(lib, out.stdout.strip(), flush=True)
