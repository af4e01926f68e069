"""One rank of the distributed GPU tests (tests/test_gpu_distributed.py).

Run as a child process per rank: python tests/dist_worker.py <case> <rank> <world> <port> <out.npz>.
The rank runs the PRODUCT's distributed path on its own z-slab -- libafem's
halo plan, halo packing/unpacking, distributed Jacobi-PCG and its reductions
-- with the halo bytes and the dot-product sums moved by the host transport
(arcanefem_amd.parallel.HostCommunicator over torch.distributed gloo), since
RCCL does not run several ranks on one GPU.  Results go to out.npz.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

# case parameters shared with the test
POISSON = dict(n=5, nz=8)
POISSON_PAT = dict(n=12, nz=16)  # slabs whose rows are mostly interior stencil rows: the pattern SpMV
POISSON_PAT8 = dict(n=16, nz=71)  # the same over 8 slabs (9 node layers each; a middle slab's rows next to
# either ghost layer miss the pattern: 7 of 9 layers x 15^2/17^2 interior in-layer rows = 61 % >= 1/2)
DYN = dict(n=3, nz=5, E=21e5, nu=0.28, rho=1.0, dt=1e-3, f=(0.0, -9.81, 1.0), steps=4)
# slabs whose owned boxes coarsen (even n; 2 ranks: 8 and 9 owned layers -> 7 (padded) and 8 cells in z)
POISSON_MG = dict(n=8, nz=16)
# large enough for distributed coarse levels (level 1: 9 x 9 x 17 nodes over the slabs, then the gathered box)
POISSON_MG2 = dict(n=16, nz=32)
DYN_MG = dict(n=8, nz=12, E=21e5, nu=0.28, rho=1.0, dt=1e-3, f=(0.0, -9.81, 1.0), steps=3)
# BASELINE config C5 at its per-GPU size: n = 128 per rank (2.15 M nodes, the config's ~2e6 nodes per
# GPU), 2 ranks stacked in z, the bench's material / step / clamp
DYN_C5 = dict(n=128, nz=256, E=21e5, nu=0.28, rho=1.0, dt=1e-3, f=(0.0, 0.0, -1.0), steps=3)
# generalized alpha with Rayleigh damping: the RHS's stiffness SpMVs exchange their operand's ghosts too
DYN_DAMP = dict(etam=0.3, etak=1e-3, alpm=0.2, alpf=0.4, time_discretization="generalized-alpha")


def main():
    case, rank, world, port, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = port
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    import arcanefem_amd as af
    from arcanefem_amd.parallel import HostCommunicator

    ctx = af.Context(0)
    # "*_async" / "lists:*": the exchange callback on libafem's worker thread
    # (afem_comm_host_async): the CG's interior SpMV runs with the halo in flight
    asy = case.endswith("_async") or case.startswith("lists:")
    comm = HostCommunicator(ctx, async_exchange=asy)
    res = {}
    if case.endswith("_async"):
        case = case[:-len("_async")]
    if case in ("poisson", "poisson_pat", "poisson_pat8", "poisson_mg", "poisson_mg2"):
        prm = {"poisson": POISSON, "poisson_pat": POISSON_PAT, "poisson_pat8": POISSON_PAT8, "poisson_mg": POISSON_MG,
               "poisson_mg2": POISSON_MG2}[case]
        n, nz = prm["n"], prm["nz"]
        mesh = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=0.2, seed=20250220, nranks=world, rank=rank)
        bsr = af.BSRFormat(mesh, 1).initialize(True)
        bsr.computeSparsity()
        ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
        bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
        bsr.toLinearSystem(ls)
        ls.applyDirichletViaPenalty(mesh.bottom_nodes(), 0.5, 1e30)
        ls.set_halo_structured(comm, mesh)
        if case in ("poisson_mg", "poisson_mg2"):
            # point Jacobi, then the block-Jacobi V-cycles on the slabs' owned boxes,
            # then (below) the global V-cycle: fine level distributed, coarse levels replicated
            ls.setSolverOptions(rtol=1e-14, max_iter=20000, preconditioner="jacobi")
            it_j = ls.solve()["iterations"]
            af.set_variant("AFEM_MG_MULTI", "block")
            ls.setSolverOptions(preconditioner="multigrid")
            it_b = ls.solve()["iterations"]
            af.set_variant("AFEM_MG_MULTI", None)
            ls.setSolverOptions(preconditioner="multigrid")
        ls.setSolverOptions(rtol=1e-14, max_iter=20000)
        st = ls.solve()
        _, _, l2g = mesh.download()
        res = dict(l2g=l2g, n_own=mesh.n_own_nodes, x=ls.solution_host(with_ghosts=True), iters=st["iterations"],
                   converged=int(st["converged"]), rel=st["rel_residual"], spmv=st["spmv_kernel"])
        if case in ("poisson_mg", "poisson_mg2"):
            res["iters_jacobi"] = it_j
            res["iters_block"] = it_b
            if rank == 0:  # the same global box on ONE rank: the multigrid solve the slabs must reproduce
                m1 = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=0.2, seed=20250220)
                b1 = af.BSRFormat(m1, 1).initialize(True)
                b1.computeSparsity()
                l1 = af.DoFLinearSystem().initialize(ctx, m1.n_own_nodes, m1.n_nodes)
                b1.assemblePoissonP1(1.0, 5.5, l1.rhsVariable(), rhs_mode="set")
                b1.toLinearSystem(l1)
                l1.applyDirichletViaPenalty(m1.bottom_nodes(), 0.5, 1e30)
                l1.setSolverOptions(rtol=1e-14, max_iter=20000, preconditioner="multigrid")
                res["iters_single"] = l1.solve()["iterations"]
        # CG iter/s with the halo attached (fixed iterations)
        ls.setSolverOptions(fixed_iterations=20)
        ls.solve()
    elif case.startswith("lists:"):
        # the halo from the caller's own synchronisation lists (afem_ls_set_halo:
        # what the Arcane shim builds from IVariableSynchronizer), then
        # afem_ls_synchronize of a ghosted vector (m_u.synchronize())
        from golden_cases import CASES
        from arcanefem_amd.gmsh import read_gmsh

        mfile, f, bcs, _, P = CASES[case[6:]]
        gm = read_gmsh(os.path.join(ROOT, "tests", "golden", mfile))
        part = af.partition_rcb(gm.dim, gm.coords, world)
        plan = af.subdomain_plan(gm.cells, part, world, rank)
        l2g = plan["local_to_global"]
        g2l = np.full(gm.n_nodes, -1, dtype=np.int64)
        g2l[l2g] = np.arange(l2g.size)
        lcells = g2l[gm.cells[plan["cells"]]].astype(np.int32)
        assert (lcells >= 0).all()
        mesh = af.Mesh.from_arrays(ctx, gm.dim, lcells, gm.coords[l2g], n_own=plan["n_own"])
        bsr = af.BSRFormat(mesh, 1).initialize(True)
        bsr.computeSparsity()
        ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
        bsr.assemblePoissonP1(1.0, f, ls.rhsVariable(), rhs_mode="set")
        bsr.toLinearSystem(ls)
        for g, v in bcs:
            loc = g2l[gm.group_nodes(g)]
            own = loc[(loc >= 0) & (loc < mesh.n_own_nodes)].astype(np.int32)
            if own.size:
                ls.applyDirichletViaPenalty(own, v, P)
        nbr = plan["neighbors"]
        ls.set_halo(comm, nbr, [plan["send"][int(r)] for r in nbr], [plan["recv"][int(r)] for r in nbr])
        # synchronize(): owners' values land in the ghosts
        xs = np.where(np.arange(l2g.size) < mesh.n_own_nodes, l2g + 0.25, -1.0)
        dx = ctx.malloc(8 * xs.size)
        ctx.to_device(dx, xs)
        ls.synchronize(dx)
        synced = ctx.to_host(dx, xs.size, np.float64)
        ctx.free(dx)
        ls.setSolverOptions(rtol=1e-14, max_iter=20000)
        st = ls.solve()
        res = dict(l2g=l2g, n_own=mesh.n_own_nodes, x=ls.solution_host(with_ghosts=True), iters=st["iterations"],
                   converged=int(st["converged"]), rel=st["rel_residual"], synced=synced, spmv=st["spmv_kernel"])
    elif case.startswith("amg:"):
        # the algebraic multigrid PCG over RCB subdomains (amg.hip: per-rank
        # aggregation, distributed coarse levels, then one gathered level):
        # "amg:<golden case>" (coarsest level held to 16 rows, as the one-rank
        # AMG tests do) or "amg:refined<k>" (L-shape-3D refined k times, z-min
        # nodes clamped by penalty)
        from golden_cases import CASES
        from arcanefem_amd.gmsh import read_gmsh

        name = case[4:]
        if name.endswith("_dist"):
            # distributed coarse levels (per-rank aggregation of a distributed
            # operator, coarse ghosts and halo) down to 200 global rows, then the gather
            af.set_variant("AFEM_AMG_GATHER", "200")
            name = name[:-len("_dist")]
        if name.startswith("refined"):
            import bench

            gm = read_gmsh(os.path.join(ROOT, "tests", "golden", "L-shape-3D.msh"))
            cells, coords = bench.refine_tets(gm.cells, gm.coords, int(name[7:]), "cpu")
            dim, f, P = 3, 5.5, 1e30
            z = coords[:, 2]
            bcs = [(np.nonzero(z <= z.min() + 1e-9)[0], 0.5)]
        else:
            af.set_variant("AFEM_AMG_DENSE", "16")
            mfile, f, bcs0, _, P = CASES[name]
            gm = read_gmsh(os.path.join(ROOT, "tests", "golden", mfile))
            cells, coords, dim = gm.cells, gm.coords, gm.dim
            bcs = [(gm.group_nodes(g), v) for g, v in bcs0]
        part = af.partition_rcb(dim, coords, world)
        mesh = af.Mesh.subdomain(ctx, dim, cells, coords, part, world, rank)
        _, _, l2g = mesh.download()
        g2l = np.full(coords.shape[0], -1, dtype=np.int64)
        g2l[l2g] = np.arange(l2g.size)
        bsr = af.BSRFormat(mesh, 1).initialize(True)
        bsr.computeSparsity()
        ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
        bsr.assemblePoissonP1(1.0, f, ls.rhsVariable(), rhs_mode="set")
        bsr.toLinearSystem(ls)
        for nodes, v in bcs:
            loc = g2l[nodes]
            own = loc[(loc >= 0) & (loc < mesh.n_own_nodes)].astype(np.int32)
            if own.size:
                ls.applyDirichletViaPenalty(own, v, P)
        if world > 1:
            ls.set_halo_mesh(comm, mesh)
        ls.setSolverOptions(rtol=1e-14, max_iter=20000, method="pcg", preconditioner="amg")
        st = ls.solve()
        res = dict(l2g=l2g, n_own=mesh.n_own_nodes, x=ls.solution_host(with_ghosts=True), iters=st["iterations"],
                   converged=int(st["converged"]), rel=st["rel_residual"], levels=st["amg_levels"],
                   coarse=st["amg_coarse_rows"])
    elif case.startswith("gmsh:"):
        # a reference Gmsh mesh partitioned by libafem's RCB into `world`
        # ghosted subdomains (afem_mesh_create_subdomain), Poisson + penalty
        # Dirichlet as the golden case, halo plan from the subdomain
        from golden_cases import CASES
        from arcanefem_amd.gmsh import read_gmsh

        mfile, f, bcs, _, P = CASES[case[5:]]
        gm = read_gmsh(os.path.join(ROOT, "tests", "golden", mfile))
        part = af.partition_rcb(gm.dim, gm.coords, world)
        mesh = af.Mesh.subdomain(ctx, gm.dim, gm.cells, gm.coords, part, world, rank)
        _, _, l2g = mesh.download()
        g2l = np.full(gm.n_nodes, -1, dtype=np.int64)
        g2l[l2g] = np.arange(l2g.size)
        bsr = af.BSRFormat(mesh, 1).initialize(True)
        bsr.computeSparsity()
        ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
        bsr.assemblePoissonP1(1.0, f, ls.rhsVariable(), rhs_mode="set")
        bsr.toLinearSystem(ls)
        for g, v in bcs:
            loc = g2l[gm.group_nodes(g)]
            own = loc[(loc >= 0) & (loc < mesh.n_own_nodes)].astype(np.int32)
            if own.size:
                ls.applyDirichletViaPenalty(own, v, P)
        ls.set_halo_mesh(comm, mesh)
        ls.setSolverOptions(rtol=1e-14, max_iter=20000)
        st = ls.solve()
        res = dict(l2g=l2g, n_own=mesh.n_own_nodes, x=ls.solution_host(with_ghosts=True), iters=st["iterations"],
                   converged=int(st["converged"]), rel=st["rel_residual"], part=part)
    elif case == "elastodynamics_c5":
        # C5 at its configured per-GPU size over 2 slabs (host transport), multigrid PCG; rank 0 also runs
        # the single-domain loop of the same global mesh (decomposition invariance at size)
        from arcanefem_amd.elastodynamics import Elastodynamics3D

        p = DYN_C5
        n, nz = p["n"], p["nz"]

        def run(mesh, cm):
            ids = np.arange(mesh.n_nodes)
            _, _, l2g_ = mesh.download()
            fixed = ids[l2g_ % (n + 1) == 0].astype(np.int32)  # node x-index 0, as the bench's c5 leg
            sim = Elastodynamics3D(ctx, mesh, p["E"], p["nu"], p["rho"], p["dt"], body_force=p["f"],
                                   fixed_nodes=fixed, rtol=1e-10, comm=cm, preconditioner="multigrid")
            its = []
            for _ in range(p["steps"]):
                st = sim.step()
                assert st["converged"], st
                its.append(st["iterations"])
            U = sim.state_host()[0]
            sim.close()
            return U, l2g_, its

        mesh = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=0.2, seed=20250220, nranks=world, rank=rank)
        U, l2g, its = run(mesh, comm)
        res = dict(l2g=l2g, n_own=mesh.n_own_nodes, U=U, iters=np.array(its))
        mesh.close()
        dist.barrier()
        if rank == 0:
            m1 = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=0.2, seed=20250220)
            U1, _, its1 = run(m1, None)
            res["U_single"] = U1
            res["iters_single"] = np.array(its1)
            m1.close()
        dist.barrier()
    elif case in ("elastodynamics", "elastodynamics_mg", "elastodynamics_damped"):
        from arcanefem_amd.elastodynamics import Elastodynamics3D

        p = DYN_MG if case == "elastodynamics_mg" else DYN
        pc = "multigrid" if case == "elastodynamics_mg" else "jacobi"
        kw = DYN_DAMP if case == "elastodynamics_damped" else {}
        mesh = af.Mesh.structured(ctx, 3, p["n"], nz=p["nz"], jitter=0.2, seed=20250220, nranks=world, rank=rank)
        _, coords, l2g = mesh.download()
        fixed = np.nonzero(coords[:, 0] < 0.5 / p["n"])[0].astype(np.int32)  # the x = 0 layer, ghosts included
        sim = Elastodynamics3D(ctx, mesh, p["E"], p["nu"], p["rho"], p["dt"], body_force=p["f"], fixed_nodes=fixed,
                               rtol=1e-14, comm=comm, preconditioner=pc, **kw)
        its = []
        for _ in range(p["steps"]):
            st = sim.step()
            its.append(st["iterations"])
            assert st["converged"], st
        U, V, A = sim.state_host()
        res = dict(l2g=l2g, n_own=mesh.n_own_nodes, U=U, V=V, A=A, iters=np.array(its))
        sim.close()
        if case == "elastodynamics_mg" and rank == 0:  # the one-rank multigrid loop's iterations
            m1 = af.Mesh.structured(ctx, 3, p["n"], nz=p["nz"], jitter=0.2, seed=20250220)
            _, c1, _ = m1.download()
            f1 = np.nonzero(c1[:, 0] < 0.5 / p["n"])[0].astype(np.int32)
            s1 = Elastodynamics3D(ctx, m1, p["E"], p["nu"], p["rho"], p["dt"], body_force=p["f"], fixed_nodes=f1,
                                  rtol=1e-14, preconditioner="multigrid")
            res["iters_single"] = np.array([s1.step()["iterations"] for _ in range(p["steps"])])
            s1.close()
    else:
        raise SystemExit(f"unknown case {case}")
    assert not comm.errors, comm.errors
    np.savez(out, **res)
    dist.barrier()
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
