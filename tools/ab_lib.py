"""A/B of two builds of libafem on the same box: runs this script's timing
part in two child processes (AFEM_LIB=libA, AFEM_LIB=libB) alternately.
usage: python tools/ab_lib.py libA.so libB.so [n] [reps] [rounds]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, ROOT)
    import numpy as np
    import arcanefem_amd as af
    n, reps = int(sys.argv[2]), int(sys.argv[3])
    ctx = af.Context(0)
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes)
    ts = []
    for r in range(reps + 3):
        ctx.event_record(0)
        bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
        ctx.event_record(1)
        ctx.synchronize()
        if r >= 3:
            ts.append(ctx.event_elapsed(0, 1))
    _, _, vals = bsr.download()
    print(f"{np.median(ts):.4f} {np.min(ts):.4f} {float(np.sum(vals)):.17g} {bsr.stats()['uniform_slices']}", flush=True)
    sys.exit(0)
a, b = sys.argv[1], sys.argv[2]
n = sys.argv[3] if len(sys.argv) > 3 else "215"
reps = sys.argv[4] if len(sys.argv) > 4 else "30"
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 2
res = {a: [], b: []}
for _ in range(rounds):
    for lib in (a, b):
        env = dict(os.environ, AFEM_LIB=os.path.abspath(lib))
        out = subprocess.run([sys.executable, __file__, "--child", n, reps], env=env, capture_output=True, text=True,
                             timeout=300)
        if out.returncode != 0:
            print(out.stdout, out.stderr)
            sys.exit(1)
        res[lib].append(out.stdout.split())
        print(lib, out.stdout.strip(), flush=True)
