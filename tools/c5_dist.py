"""C5 (3D Newmark elastodynamics, re-assembly every step, multigrid PCG) over
several ranks on ONE GPU through the host transport: the rehearsal of the
8-GPU run (RCCL needs one GPU per rank).  Weak scaling: an n^3 box per rank
stacked in z (n = 128: the config's ~2e6 nodes per GPU).  The global V-cycle
runs with distributed coarse levels (libafem multigrid.hip).
usage: python tools/c5_dist.py <world> [n] [steps] [out.json]
Spawns the ranks itself (one process per rank, gloo control plane)."""
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main(rank, world, port, n, steps, out):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = port
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    import arcanefem_amd as af
    from arcanefem_amd.elastodynamics import Elastodynamics3D
    from arcanefem_amd.parallel import HostCommunicator

    ctx = af.Context(0)
    comm = HostCommunicator(ctx, async_exchange=True)
    mesh = af.Mesh.structured(ctx, 3, n, nz=n * world, jitter=0.2, seed=20250220, nranks=world, rank=rank)
    _, coords, _ = mesh.download()
    fixed = np.nonzero(coords[:, 0] < 0.5 / n)[0].astype(np.int32)  # the x = 0 face, ghosts included
    dyn = Elastodynamics3D(ctx, mesh, E=21.0e5, nu=0.28, rho=1.0, dt=1.0e-3, body_force=(0.0, 0.0, -1.0),
                           fixed_nodes=fixed, rtol=1e-8, comm=comm, preconditioner="multigrid")
    t0 = time.perf_counter()
    dyn.step()
    ctx.synchronize()
    first = time.perf_counter() - t0
    dist.barrier()
    its, conv = [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        st = dyn.step()
        its.append(int(st["iterations"]))
        conv.append(bool(st["converged"]))
    ctx.synchronize()
    dist.barrier()
    dt = (time.perf_counter() - t0) / steps
    import torch

    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    nodes = torch.tensor([float(mesh.n_own_nodes)], dtype=torch.float64)
    dist.all_reduce(nodes)
    if rank == 0:
        res = {"config": f"C5 elastodynamics 3D Newmark, {world} rank(s) on one GPU over the host transport, "
                         f"weak: n={n} per rank stacked in z ({int(nodes[0])} nodes, {3 * int(nodes[0])} DoF), "
                         f"x = 0 face clamped, multigrid PCG rtol 1e-8 (distributed coarse levels)",
               "world": world, "ms_per_step": round(float(t[0]) * 1e3, 2), "first_step_ms": round(first * 1e3, 1),
               "cg_iterations": its, "converged": conv, "steps": steps}
        print(json.dumps(res), flush=True)
        if out:
            with open(out, "w") as f:
                json.dump(res, f)
    assert not comm.errors, comm.errors
    dyn.close()
    comm.close()
    dist.barrier()
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--rank":
        rank_main(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5]), int(sys.argv[6]),
                  sys.argv[7] if len(sys.argv) > 7 else "")
        return
    world = int(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    out = sys.argv[4] if len(sys.argv) > 4 else ""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = [subprocess.Popen([sys.executable, __file__, "--rank", str(r), str(world), port, str(n), str(steps), out])
             for r in range(world)]
    rc = 0
    for p in procs:
        p.wait()
        rc = rc or p.returncode
    sys.exit(rc)


if __name__ == "__main__":
    main()
