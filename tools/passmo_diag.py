import sys, os, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import arcanefem_amd as af
from oracle import oracle as O
import test_oracle_passmo as T
from test_gpu_passmo import _replay_gpu
from arcanefem_amd.gmsh import read_gmsh
bar = read_gmsh(os.path.join(T.GOLDEN, T.BAR3D["mesh"]))
ctx = af.Context(0)
dts = O.passmo_time_steps(T.BAR3D["start"], T.BAR3D["final"], T.BAR3D["dt"])
Uo, Vo, Ao = O.passmo_newmark(bar.cells, bar.coords, T.BAR3D["lam"], T.BAR3D["mu"], T.BAR3D["rho"], dts, T.bar3d_imposed(bar), T.BAR3D["penalty"])
print("oracle vs golden", T.check_golden(bar, Uo))
for pc in ("jacobi", "block3"):
    U, V, A, it = _replay_gpu(ctx, bar, pc)
    print(pc, "golden", T.check_golden(bar, U), "vs oracle U %.3g V %.3g A %.3g" % tuple(np.abs(g - o).max() / np.abs(o).max() for g, o in ((U, Uo), (V, Vo), (A, Ao))), "iters", it)
