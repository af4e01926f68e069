"""Benchmark of the MI355X FEM assembly + CG path (BASELINE.json metric).

A step = one numeric assembly of the Poisson-3D P1 system on a fixed sparsity:
matrix values + constant-source RHS (one fused kernel; the module's
rhs.fill(0) + applyConstantSourceToRhs, modules/poisson/FemModule.cc:163-169),
the penalty Dirichlet list (forced info/value, rhs = P g) and the forced
values written into the CSR (the reference's K14/K8/K16/K19 sequence).
Inputs (mesh, structure) are resident in HBM before the timed region.
Afterwards a fixed number of Jacobi-PCG iterations on the assembled CSR is
timed for the CG iter/s half of the metric.

Timing: before the W untimed warmup steps the step runs back to back for
--settle-ms (150) of wall time, untimed, so the GPU clocks have left their
post-idle ramp (settle(); reported as settle_ms / settle_steps).  `value` = DoF
assembled per second over the K timed steps (wall clock between barriers, max
over ranks).  The roofline of the assembly kernels uses
the MEDIAN of the per-step kernel durations (HIP events recorded on the
context stream around each assembly launch; BASELINE.md §4 asks for medians);
the committed rocprofv3 kernel-stats summary of the same command is in
profiles/.

Multi-GPU (torchrun): one process per GPU; the mesh is a z-slab per rank with
one ghost layer and the same per-rank size (weak scaling); assembly needs no
communication, the CG exchanges ghost values and sums dot products through
RCCL (libafem's own communicator; torch.distributed/gloo is only the control
plane: bootstrap of the RCCL id, barriers, max-over-ranks of the timings).

Side measurements at N=1 (rank 0): C4 (Poisson-3D at 10^8 DoF on one GPU:
assembly + CG), C3 (block-3 elasticity), C5 (elastodynamics step), and the
CPU baselines of BASELINE.md §4 (assembly cell loop, OpenMP Jacobi-PCG over 50
fixed iterations, the C1 dense SequentialBasic end to end).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MDoF/s assembly + CG iter/s, Poisson-3D P1 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# the CG's SpMV by afem_solve_stats.spmv_kernel (include/arcanefem_amd.h AFEM_SPMV_*)
SPMV_KERNELS = {0: "k_spmv_stream4u", 1: "k_spmv_pat", 2: "k_spmv_v16", 3: "k_spmv_blk", 4: "other"}
# block-3 assembly kernels by afem_bsr_stats.last_kernel (include/arcanefem_amd.h AFEM_KERNEL_*)
ELAST3_KERNELS = {4: "k_assemble_elast_strip", 5: "k_assemble_elast_tet", 6: "k_assemble_elast_tet_global",
                  8: "k_assemble_elast_wg", 9: "k_assemble_elast_strip<..,BIG>"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU).  Under torch.distributed.run WORLD_SIZE decides; without a launcher "
                         "bench.py spawns the N rank processes itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="untimed back-to-back steps before the warmup, until the GPU clocks settle (0: none)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: an n x n x n box per GPU stacked in z (C2 per GPU; n = 231 is BASELINE.md's C4 weak "
                         "size); strong: ONE n x n x n box cut into N z-slabs (C4, n = 463)")
    ap.add_argument("--n", type=int, default=None,
                    help="cells per unit length (default: weak 215 -> 10.08M DoF per GPU, strong 463 -> 99.9M DoF)")
    ap.add_argument("--cg-iters", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="skip the CPU baselines (the oracle timed at the C2 size on the host cores, N = 1 only)")
    ap.add_argument("--no-extras", action="store_true", help="skip the side measurements (N = 1 only anyway)")
    ap.add_argument("--legs", default="c4,c3,c2_generic,c2_arrays,c2_arrays_natural,unstructured,unstructured_solve,"
                                      "generic_unstructured,c5",
                    help="the side measurements to run (comma list of c4, c3, c2_generic, c2_arrays, "
                         "c2_arrays_natural, unstructured, unstructured_solve (the unstructured leg's system solved "
                         "by the Jacobi- and the AMG-PCG), generic_unstructured, c5)")
    ap.add_argument("--no-headline", action="store_true",
                    help="N = 1: skip the headline C2 step (and the CPU baselines), run only --legs (per-leg "
                         "rocprofv3 runs, tools/profile_legs.sh)")
    ap.add_argument("--c3-n", type=int, default=170, help="C3 block-3 elasticity box (170 -> 5.0M nodes)")
    ap.add_argument("--c4-n", type=int, default=463, help="C4 Poisson box on one GPU (463 -> 99.9M DoF); 0: skip")
    ap.add_argument("--c5-n", type=int, default=128,
                    help="C5 elastodynamics box (128 -> 2.15M nodes, the config's ~2e6 per GPU; 2^7 cells: 5 coarse grids)")
    ap.add_argument("--c5-steps", type=int, default=5)
    ap.add_argument("--comm", choices=("rccl", "host"), default="rccl",
                    help="N > 1: the CG's transport (host: gloo callbacks, for rehearsing several ranks on one GPU)")
    ap.add_argument("--unstructured-levels", type=int, default=6,
                    help="refinements of L-shape-3D.msh for the unstructured leg (6 -> 12 M DoF); 0: skip")
    args = ap.parse_args(argv)
    if args.n is None:
        args.n = 215 if args.scaling == "weak" else 463
    return args


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(nranks):
    """`--gpus N` without a launcher: start the N rank processes the way
    torch.distributed.run would (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*;
    the same command line), wait for them, exit with the first failure.  This
    process touches no GPU API (the ranks do).  A rank that fails ends the
    others (they would wait in the rendezvous or a barrier forever)."""
    import subprocess

    port = str(_free_port())
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks), LOCAL_WORLD_SIZE=str(nranks),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    code, t_fail = 0, None
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and code == 0:
                code = rc if rc > 0 else 1
                t_fail = time.time()
                for q in live:  # the PIDs this launcher started, nothing else
                    q.terminate()
        if t_fail is not None and time.time() - t_fail > 20:
            for q in live:
                q.kill()
        time.sleep(0.05)
    return code


def algorithmic_bytes(n_inc, n_local, n_own, nnz):
    """Per assembly launch: incidence table 4 B per (owned
    row, incident cell) = the connectivity bytes 4*nv*Ncell, node coordinates
    24 B, row offsets 8 B, columns 4 B + values 8 B per non-zero, RHS 8 B per
    owned DoF (written once: the fused fill(0) + source)."""
    return 4 * n_inc + 24 * n_local + 8 * (n_own + 1) + 12 * nnz + 8 * n_own


def cg_bytes(nnz, n_own):
    """Per Jacobi-PCG iteration: SpMV on the CSR 12 nnz + 8 (N+1)
    + 8 N gathers + 8 N store; the two vector passes between the reductions
    (r, z and r.z: 40 N; x and the new direction: 40 N)."""
    return 12 * nnz + 8 * (n_own + 1) + 96 * n_own


def poisson_setup(ctx, af, n, nz, world, rank):
    mesh = af.Mesh.structured(ctx, 3, n, nz=nz, jitter=0.2, seed=20250220, nranks=world, rank=rank)
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    ctx.synchronize()
    t0 = time.perf_counter()
    bsr.computeSparsity()
    ctx.synchronize()
    sparsity_ms = (time.perf_counter() - t0) * 1e3
    ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
    bsr.toLinearSystem(ls)
    bottom = mesh.bottom_nodes()
    dbottom = ctx.malloc(max(4 * bottom.size, 4))
    ctx.to_device(dbottom, bottom)
    return mesh, bsr, ls, bottom, dbottom, sparsity_ms


def make_step(ctx, bsr, ls, bottom, dbottom):
    rhs = ls.rhsVariable()

    def step(ev=None):
        if ev is not None:
            ctx.event_record(ev)
        bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set")  # rhs.fill(0) + applyConstantSourceToRhs, fused
        if ev is not None:
            ctx.event_record(ev + 1)
        ls.applyDirichletViaPenaltyDevice(dbottom, bottom.size, 0.5, 1.0e30)
        ls.applyBoundaryConditions()

    return step


def roofline(bsr, mesh, kernel_ms):
    st = bsr.stats()
    # the instances the assembly launches: uniform slices, compact general
    # slices, big general slices (> 16 slots / > 352 nodes, assembly.hip);
    # generator boxes under the cell-first kernel: k_assemble_cubes alone
    names = ["k_assemble_stencil<kSigKuhn3D>"] if st["stencil_slices"] > 0 else []
    if st["uniform_instance_slices"] > 0 or (st["stencil_slices"] == 0 and st["uniform_slices"] > 0):
        names.append("k_assemble_strip<4,2,16,uniform>")
    if st["general_slices"] > 0:
        names.append("k_assemble_strip<4,2,16,general>")
    if st["max_slice_width"] > 16 or st["max_slice_nodes"] > 352:
        names.append("k_assemble_strip<4,4,32,general>")
    if st.get("last_kernel") == 10:  # AFEM_KERNEL_CUBES (cubes.hip)
        # canonical lattices (cube_lattice 3): the staged path's two passes
        names = ["k_assemble_cubes", "k_cube_unstage"] if st.get("cube_lattice") == 3 else ["k_assemble_cubes"]
    kname = " + ".join(names)
    nnz = bsr.view().nnz_blocks
    ab = algorithmic_bytes(int(st["n_incidences"]), mesh.n_nodes, mesh.n_own_nodes, nnz)
    achieved = ab / (kernel_ms * 1e-3) / 1e9
    if st.get("last_kernel") == 10:
        kmin = cube_min_bytes(st, mesh.n_nodes, mesh.n_own_nodes, nnz)
        kmin_note = ("cube kernel: coordinates + row offsets + values + RHS" if st.get("cube_lattice") != 3 else
                     "staged canonical path: coordinates + caller ids + the 128-B lattice lines written and read "
                     "back + row maps and offsets + values + RHS")
    else:
        kmin = ab
        kmin_note = ("strip kernels: per-row strips and slice node lists replace the incidence table; "
                     "taken as the algorithmic bytes")
    return {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": int(ab),
            "bytes_kernel_min": int(kmin), "bytes_kernel_min_note": kmin_note,
            "frac_kernel_min": round(kmin / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "kernel_ms": round(kernel_ms, 4),
            "cube_lattice": int(st.get("cube_lattice", 0)),
            "inc_padding": round(st["inc_table_entries"] / max(int(st["n_incidences"]), 1) - 1.0, 4),
            "uniform_slice_frac": round(st["uniform_slices"] / max(st["n_slices"], 1), 4),
            "stencil_slice_frac": round(st["stencil_slices"] / max(st["n_slices"], 1), 4),
            "shared_strip_frac": round(st.get("shared_strip_slices", 0) / max(st["n_slices"], 1), 4)}


def cube_min_bytes(st, n_local, n_own, nnz, rhs_read=False):
    """What the cube kernel (cubes.hip) must move per launch: it derives the
    connectivity from the lattice, so it reads the node coordinates (24 B),
    the row offsets (8 B per row) and writes every value (8 B per non-zero)
    and the RHS (8 B per row; + 8 B read when it adds).  Canonical lattices
    (the caller's random numbering, cube_lattice 3) run staged: per row the
    caller id (4 B), its 128-B lattice line written and read back, the lattice
    index and position map (12 B) and the row offset (8 B).  VERDICT r4 #1:
    the algorithmic bytes count the incidence table and the columns, which
    this kernel never reads."""
    rows = (4 + 256 + 12 + 8) * n_own if st.get("cube_lattice") == 3 else 8 * (n_own + 1)
    return 24 * n_local + rows + 8 * nnz + (16 if rhs_read else 8) * n_own


def leg_profile(leg, size):
    """profiles/pmc_<leg>.json (tools/collect_leg.py) when it was taken at this
    size on one GPU: the HBM bytes per launch of the leg's kernels from the
    rocprofv3 PMC passes (2 FETCH_SIZE + WRITE_SIZE) and their rocprofv3
    kernel-trace mean duration."""
    try:
        with open(os.path.join(ROOT, "profiles", f"pmc_{leg}.json")) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None
    return pm if pm.get("size") == size and pm.get("world") in (None, 1) else None


def with_traffic(rf, leg, size, kernel_ms):
    """roofline.traffic / frac_traffic: the PMC bytes per
    launch of the committed profile of this leg at this size, over this run's
    kernel time; the same two fractions recomputed from the profile's own
    rocprofv3 mean (frac_profile, frac_traffic_profile) so the line can be
    checked against profiles/ alone."""
    pm = leg_profile(leg, size)
    rf["traffic"] = rf["frac_traffic"] = None
    if pm is None:
        return rf
    b = pm["hbm_bytes_per_launch"]
    rf["traffic"] = int(b)
    rf["frac_traffic"] = round(b / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    rf["traffic_profile"] = pm.get("tag")
    pk = pm.get("kernel_mean_ms")
    if pk:
        rf["profile_kernel_ms"] = round(pk, 4)
        rf["frac_profile"] = round(rf["algorithmic_bytes_per_launch"] / (pk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        rf["frac_traffic_profile"] = round(b / (pk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if rf.get("bytes_kernel_min"):
        rf["traffic_over_min"] = round(b / rf["bytes_kernel_min"], 3)
    return rf


def cg_traffic(leg, size, n_own, iter_per_s):
    """CG fraction in bytes actually moved: the SpMV's PMC
    bytes per call from the committed profile (profiles/pmc_<leg>.json: the
    pattern SpMV does not read the column indices cg_bytes counts) + the two
    vector passes of an iteration (80 B per row, cg_bytes), times this run's
    iterations per second; and the SpMV's own moved-byte fraction at the
    profile's kernel mean."""
    pm = leg_profile(leg, size)
    if pm is None:
        return {}
    b = pm["hbm_bytes_per_launch"] + 80 * n_own
    out = {"cg_traffic_per_iter": int(b), "cg_frac_traffic": round(b * iter_per_s / 1e9 / HBM_PEAK_GBS, 4),
           "spmv_traffic": int(pm["hbm_bytes_per_launch"]), "spmv_profile": pm.get("tag")}
    if pm.get("kernel_mean_ms"):
        out["spmv_kernel_ms"] = round(pm["kernel_mean_ms"], 4)
        out["spmv_frac_traffic"] = round(pm["hbm_bytes_per_launch"] / (pm["kernel_mean_ms"] * 1e-3) / 1e9
                                         / HBM_PEAK_GBS, 4)
    return out


def _pick(d, keys):
    return {k: d[k] for k in keys if d is not None and k in d}


def compact_line(out):
    """The LAST stdout line (the driver keeps ~8 KB of stdout
    and only the contract keys of the parsed line): the contract keys, the
    headline's roofline and CPU baseline without their notes, the CG half of
    the metric with its moved-byte fraction, and one summary per side leg
    (kernel ms, frac, frac_traffic ...).  The full record is the preceding
    {"bench_detail": ...} line."""
    keys = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    c = _pick(out, keys)
    cfg = out["config"]
    c["config"] = {"workload": cfg["workload"].split(",")[0], **_pick(cfg, ("n", "dof_total", "nnz_rank0",
                                                                           "parallelism"))}
    c["roofline"] = _pick(out["roofline"], ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic",
                                            "frac_traffic", "kernel_ms", "algorithmic_bytes_per_launch",
                                            "bytes_kernel_min", "frac_kernel_min", "profile_kernel_ms",
                                            "frac_profile", "traffic_profile"))
    cpu = out.get("cpu_baseline")
    if cpu:
        c["cpu_baseline"] = {**_pick(cpu, ("value", "unit", "cores", "kind", "value_single_thread")),
                             "sample": "C2 itself, oracle cell loop (OpenMP, atomic adds), median of 5"}
    c.update(_pick(out, ("value_unsettled", "ms_per_step_unsettled", "cg_iter_per_s", "cg_roofline_frac",
                         "cg_frac_traffic", "spmv_frac_traffic", "cg_ms_per_iter")))
    if out.get("cpu_baseline_cg"):
        c["cpu_cg_iter_per_s"] = out["cpu_baseline_cg"]["value"]

    def leg(e, extra=()):
        r = e.get("roofline", {})
        s = {"ms": e.get("kernel_ms", e.get("kernel_ms_median")), "frac": r.get("frac"),
             "frac_traffic": r.get("frac_traffic"), "frac_kernel_min": r.get("frac_kernel_min")}
        s.update(_pick(e, extra))
        return {k: v for k, v in s.items() if v is not None}

    legs = {}
    if "c4" in out:
        legs["c4"] = leg(out["c4"], ("cg_iter_per_s", "cg_roofline_frac", "cg_frac_traffic"))
    for k in ("c3", "c2_generic", "generic_unstructured", "c2_arrays", "c2_arrays_natural", "unstructured"):
        if k in out:
            legs[k] = leg(out[k], ("evaluations_per_cell",))
    u = out.get("unstructured", {}).get("solve")
    if u:
        legs["unstructured"]["solve_ms"] = {"jacobi": u["jacobi"]["solve_ms"], "amg": u["amg"]["solve_ms"],
                                            "amg_iterations": u["amg"]["iterations"]}
    if "c5" in out:
        c5 = out["c5"]
        b = c5.get("breakdown", {})
        legs["c5"] = {"ms_per_step": c5.get("ms_per_step"), "cg_iterations": c5.get("cg_iterations_per_step"),
                      "converged": all(c5.get("converged", [False])),
                      **_pick(b, ("assemble_ms", "rhs_ms", "solve_ms", "precond_ms", "pcg_spmv_vectors_ms",
                                  "vcycle_ms_per_iteration")),
                      "assembly_frac": b.get("assembly_roofline", {}).get("frac"),
                      "jacobi_ms_per_step": c5.get("jacobi_ms_per_step")}
    if legs:
        c["legs"] = legs
    if out.get("per_rank"):
        c["per_rank"] = [_pick(p, ("rank", "assembly_kernel_ms", "step_ms_own", "cg_ms_per_iter_own",
                                   "halo_wait_ms_per_iter", "allreduce_ms_per_iter")) for p in out["per_rank"]]
    c["detail"] = "the bench_detail line above"
    return c


def settle(ctx, step, ms):
    """GPU clocks ramp over the first tens of milliseconds of load after an
    idle spell (tools/warm_probe.py, DESIGN.md section 5: the cube kernel's
    first C2 launches 0.71 ms, 0.55 ms after ~50 launches, 0.69 again after a
    2 s pause; the stencil kernel likewise): the step runs back to back for
    `ms` of wall time before the warmup steps, so the timed steps see the
    clocks a sustained loop runs at.  Untimed; reported as settle_ms /
    settle_steps.  Returns the step count."""
    k = 0
    if ms <= 0:
        return k
    t = time.perf_counter()
    while (time.perf_counter() - t) * 1e3 < ms:
        for _ in range(8):
            step()
        ctx.synchronize()
        k += 8
    return k


def time_launches(ctx, fn, reps, warmup, settle_ms, base=200):
    """A side leg's kernel timing, like the headline's: `fn` back to back for
    settle_ms (untimed, the clocks' ramp), `warmup` untimed launches, then
    `reps` launches each bracketed by HIP events on the context stream.
    Returns (the per-launch ms, settle launches)."""
    steps = settle(ctx, fn, settle_ms)
    for _ in range(warmup):
        fn()
    ctx.synchronize()
    for i in range(reps):
        ctx.event_record(base + 2 * i)
        fn()
        ctx.event_record(base + 2 * i + 1)
    ctx.synchronize()
    return [ctx.event_elapsed(base + 2 * i, base + 2 * i + 1) for i in range(reps)], steps


def poisson_c4(ctx, af, n, reps=5, warmup=2, cg_iters=50, settle_ms=150.0):
    """BASELINE config C4's problem (Poisson-3D at ~10^8 DoF) on ONE GPU: the
    north-star size.  Assembly kernel time = median of `reps` launches after
    `warmup` (HIP events), CG = `cg_iters` fixed Jacobi-PCG iterations."""
    mesh, bsr, ls, bottom, dbottom, sp_ms = poisson_setup(ctx, af, n, None, 1, 0)
    step = make_step(ctx, bsr, ls, bottom, dbottom)
    settle_steps = settle(ctx, step, settle_ms)
    for _ in range(warmup):
        step()
    ctx.synchronize()
    for i in range(reps):
        step(210 + 2 * i)
    ctx.synchronize()
    ks = [ctx.event_elapsed(210 + 2 * i, 211 + 2 * i) for i in range(reps)]
    kms = float(np.median(ks))
    nnz = bsr.view().nnz_blocks
    ls.setSolverOptions(fixed_iterations=cg_iters)
    ctx.synchronize()
    t0 = time.perf_counter()
    st = ls.solve()
    ctx.synchronize()
    cg_s = time.perf_counter() - t0
    ips = cg_iters / cg_s
    out = {"config": f"C4 problem on 1 GPU: Poisson-3D P1 jittered Kuhn box n={n} ({mesh.n_own_nodes} DoF, "
                     f"{mesh.n_cells} tets, {nnz} nnz), CSR assembly + penalty Dirichlet; CG = {cg_iters} fixed "
                     f"Jacobi-PCG iterations",
           "dof": int(mesh.n_own_nodes), "nnz": int(nnz),
           "value": round(mesh.n_own_nodes / (kms * 1e-3) / 1e6, 1), "unit": "MDoF/s (assembly kernels)",
           "kernel_ms_median": round(kms, 4), "kernel_ms_all": [round(x, 4) for x in ks],
           "roofline": roofline(bsr, mesh, kms),
           "cg_iter_per_s": round(ips, 2), "cg_roofline_frac": round(cg_bytes(nnz, mesh.n_own_nodes) * ips / 1e9
                                                                       / HBM_PEAK_GBS, 4),
           "cg_device_ms": round(st["solve_ms"], 2), "cg_spmv": SPMV_KERNELS.get(st["spmv_kernel"]),
           "cg_iterations": cg_iters,
           "sparsity_ms": round(sp_ms, 1), "settle_ms": settle_ms, "settle_steps": settle_steps}
    out.update(cg_traffic("c4_spmv", n, mesh.n_own_nodes, ips))
    with_traffic(out["roofline"], "c4", n, kms)
    ctx.free(dbottom)
    ls.reset()
    bsr.close()
    mesh.close()
    return out


def elasticity_c3(ctx, af, n, reps=10, warmup=2, settle_ms=150.0):
    """BASELINE config C3: block-3 P1 elasticity on tetrahedra (BSR, ordered per
    block), stiffness + body force fused, on fixed sparsity; kernel time = median
    of HIP-event launch times.  Algorithmic bytes per launch: incidence
    table 4*nv*Ncell, coordinates 24 N, row offsets 8 (N+1), block columns
    4 nnz_b, block values 72 nnz_b, RHS 24 N."""
    E, nu = 21.0e5, 0.28
    lam = E * nu / ((1 + nu) * (1 - 2 * nu))
    mu2 = E / (1 + nu)
    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
    bsr = af.BSRFormat(mesh, 3).initialize(False)
    t0 = time.perf_counter()
    bsr.computeSparsity()
    ctx.synchronize()
    sp_ms = (time.perf_counter() - t0) * 1e3
    rhs = ctx.malloc(8 * 3 * mesh.n_own_nodes)
    f = (0.0, 0.0, -1.0)
    ks, settle_steps = time_launches(ctx, lambda: bsr.assembleElasticityP1Ex(lam, mu2, 0.0, f, rhs, rhs_mode="set"),
                                     reps, warmup, settle_ms)
    kms = float(np.median(ks))
    st = bsr.stats()
    v = bsr.view()
    nnz_b = v.nnz_blocks
    n_own, n_loc = mesh.n_own_nodes, mesh.n_nodes
    ab = 4 * int(st["n_incidences"]) + 24 * n_loc + 8 * (n_own + 1) + 76 * nnz_b + 24 * n_own
    out = {"config": f"C3 elasticity block-3 P1 tets, Kuhn box n={n} ({n_own} nodes, {3 * n_own} DoF, "
                     f"{mesh.n_cells} tets), BSR per-block, stiffness + body force",
           "value": round(3 * n_own / (kms * 1e-3) / 1e6, 1), "unit": "MDoF/s", "kernel_ms": round(kms, 4),
           "kernel": ELAST3_KERNELS.get(int(st["last_kernel"]), str(int(st["last_kernel"]))),
           "roofline": {"bound": "hbm", "achieved": round(ab / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ab / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "algorithmic_bytes_per_launch": int(ab), "bytes_kernel_min": int(ab),
                        "bytes_kernel_min_note": "strip kernels: per-row strips and slice node lists replace the "
                                                 "incidence table; taken as the algorithmic bytes",
                        "kernel_ms": round(kms, 4)},
           "kernel_ms_all": [round(x, 4) for x in ks], "settle_steps": settle_steps,
           "sparsity_ms": round(sp_ms, 1)}
    with_traffic(out["roofline"], "c3", n, kms)
    ctx.free(rhs)
    bsr.close()
    mesh.close()
    return out


def refine_tets(cells, coords, levels, device):
    """Uniform (red) refinement of a tetrahedral mesh, `levels` times: every
    tet -> 4 corner tets + the inner octahedron cut along one diagonal (8
    children of bounded shape; node valences stay irregular).  Synthetic input
    generation with torch on the host (edge midpoints deduplicated by
    torch.unique; torch's own HIP runtime is not used next to libafem's); not
    on the measured path."""
    import torch

    c = torch.as_tensor(np.asarray(cells, dtype=np.int64), device=device)
    x = torch.as_tensor(np.asarray(coords, dtype=np.float64), device=device)
    pairs = [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)]
    for _ in range(levels):
        n = x.shape[0]
        e = torch.stack([torch.stack([c[:, i], c[:, j]], -1) for i, j in pairs], 1)
        key = e.min(-1).values * n + e.max(-1).values
        uk, inv = torch.unique(key.reshape(-1), return_inverse=True)
        mid = n + inv.reshape(-1, 6)
        x = torch.cat([x, 0.5 * (x[uk // n] + x[uk % n])])
        v0, v1, v2, v3 = c.unbind(1)
        m01, m02, m03, m12, m13, m23 = mid.unbind(1)
        ch = [(v0, m01, m02, m03), (m01, v1, m12, m13), (m02, m12, v2, m23), (m03, m13, m23, v3),
              (m01, m02, m03, m13), (m01, m02, m12, m13), (m02, m03, m13, m23), (m02, m12, m13, m23)]
        c = torch.stack([torch.stack(t, 1) for t in ch], 1).reshape(-1, 4)
        del e, key, uk, inv, mid
    return c.to(torch.int32).cpu().numpy(), x.cpu().numpy()


def unstructured_leg(ctx, af, mesh_file, levels, reps=7, warmup=2, settle_ms=150.0, solve=False, rtol=1e-8):
    """An unstructured mesh at the C2 scale: the reference's L-shape-3D Gmsh
    mesh refined `levels` times (levels = 6: 68 M tets, 12 M DoF).  No brick
    order, no uniform slices: Hilbert-curve slices and the general strip
    instance.  Poisson assembly (+ source) on fixed sparsity, median kernel
    time, roofline as C2's.  solve=True (`unstructured_solve` in --legs): the
    assembled system with the z-min nodes clamped by penalty, solved to rtol
    by the Jacobi-PCG and by the PCG with the algebraic multigrid V-cycle
    (amg.hip; the reference's solve on such meshes is Hypre PCG + BoomerAMG,
    femutils/HypreDoFLinearSystem.cc:686-742): iterations, setup and solve
    times, and the two solutions' difference."""
    from arcanefem_amd.gmsh import read_gmsh

    gm = read_gmsh(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", mesh_file))
    cells, coords = refine_tets(gm.cells, gm.coords, levels, "cpu")
    mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
    z = coords[:, 2]
    dn = np.nonzero(z <= z.min() + 1e-9 * max(1.0, abs(z.min())))[0].astype(np.int32) if solve else None
    del cells, coords, z
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    ctx.synchronize()
    t0 = time.perf_counter()
    bsr.computeSparsity()
    ctx.synchronize()
    sp_ms = (time.perf_counter() - t0) * 1e3
    rhs = ctx.malloc(8 * mesh.n_own_nodes)
    ks, settle_steps = time_launches(ctx, lambda: bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set"), reps, warmup,
                                     settle_ms)
    kms = float(np.median(ks))
    st = bsr.stats()
    out = {"config": f"{mesh_file} refined {levels}x ({mesh.n_own_nodes} DoF, {mesh.n_cells} tets, "
                     f"max row length {st['max_row_len']}), Hilbert-ordered slices, Poisson assembly + source",
           "dof": int(mesh.n_own_nodes), "value": round(mesh.n_own_nodes / (kms * 1e-3) / 1e6, 1),
           "unit": "MDoF/s (assembly kernels)", "kernel_ms": round(kms, 4),
           "roofline": with_traffic(roofline(bsr, mesh, kms), "unstructured", levels, kms),
           "kernel_ms_all": [round(x, 4) for x in ks], "settle_steps": settle_steps,
           "last_kernel": int(st["last_kernel"]), "max_slice_nodes": int(st["max_slice_nodes"]),
           "max_slice_width": int(st["max_slice_width"]), "sparsity_ms": round(sp_ms, 1)}
    ctx.free(rhs)
    if solve:
        ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes, mesh.n_nodes)
        bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable())
        bsr.toLinearSystem(ls)
        sols, res = {}, {}
        for pc in ("jacobi", "amg"):
            ls.applyDirichletViaPenalty(dn, 0.5, 1.0e30)
            ls.setSolverOptions(rtol=rtol, max_iter=100000, method="pcg", preconditioner=pc)
            t0 = time.perf_counter()
            sst = ls.solve()
            wall = (time.perf_counter() - t0) * 1e3
            sols[pc] = ls.solution_host().copy()
            r = {"iterations": int(sst["iterations"]), "converged": bool(sst["converged"]),
                 "rel_residual": sst["rel_residual"], "solve_ms": round(sst["solve_ms"], 1),
                 "wall_ms": round(wall, 1)}
            if pc == "amg":
                r.update(cycle="V(1,1) damped Jacobi, K-cycle (two flexible-CG steps) on levels 1-2 "
                               "(AFEM_AMG_KCYCLE)",
                         levels=int(sst["amg_levels"]), coarse_rows=int(sst["amg_coarse_rows"]),
                         operator_complexity=round(sst["amg_complexity"], 3),
                         setup_ms=round(sst["amg_setup_ms"], 1),
                         ms_per_iteration=round((sst["solve_ms"] - sst["amg_setup_ms"]) / max(1, sst["iterations"]),
                                                4))
            else:
                r["ms_per_iteration"] = round(sst["solve_ms"] / max(1, sst["iterations"]), 4)
            res[pc] = r
        res["rtol"] = rtol
        res["dirichlet_nodes"] = int(dn.size)
        res["max_rel_diff_amg_vs_jacobi"] = float(np.abs(sols["amg"] - sols["jacobi"]).max() /
                                                  np.abs(sols["jacobi"]).max())
        res["speedup_amg_vs_jacobi"] = round(res["jacobi"]["solve_ms"] / max(1e-9, res["amg"]["solve_ms"]), 2)
        out["solve"] = res
        del sols
    bsr.close()
    mesh.close()
    return out


def c2_arrays_leg(ctx, af, n, natural=False, reps=10, warmup=2, settle_ms=150.0):
    """C2 handed over the way a caller's mesh arrives: the generator's box
    downloaded and uploaded with afem_mesh_create.
    * natural=False (`c2_arrays`): nodes and cells renumbered by a seeded
      random permutation (seed 1234, SURVEY §8d's robustness variant); the
      structure build recovers the lattice from the coordinates and the cube
      kernel runs through the caller-numbering maps (cube_lattice 3);
    * natural=True (`c2_arrays_natural`): the nodes in the
      lexicographic order of a cartesian Arcane mesh (x fastest: the
      generator's own numbering), the cells in a random order with their
      vertices rotated; the structure build recognises the natural lattice and
      runs the headline cube kernel on the caller's arrays with no map
      (cube_lattice 2).
    Poisson assembly + source, median kernel time, roofline as C2's."""
    m0 = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
    cells, coords, _ = m0.download()
    m0.close()
    rng = np.random.default_rng(1234)
    if natural:
        cells = np.ascontiguousarray(np.roll(cells[rng.permutation(cells.shape[0])], 1, axis=1))
        pc = coords
    else:
        p = rng.permutation(coords.shape[0]).astype(np.int32)
        cells = p[cells][rng.permutation(cells.shape[0])]
        pc = np.empty_like(coords)
        pc[p] = coords
    del coords
    mesh = af.Mesh.from_arrays(ctx, 3, cells, pc)
    del cells, pc
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    ctx.synchronize()
    t0 = time.perf_counter()
    bsr.computeSparsity()
    ctx.synchronize()
    sp_ms = (time.perf_counter() - t0) * 1e3
    rhs = ctx.malloc(8 * mesh.n_own_nodes)
    ks, settle_steps = time_launches(ctx, lambda: bsr.assemblePoissonP1(1.0, 5.5, rhs, rhs_mode="set"), reps, warmup,
                                     settle_ms)
    kms = float(np.median(ks))
    st = bsr.stats()
    order = "lexicographic (x fastest) node order, cells in a random order" if natural else \
        "nodes and cells in a random order (seed 1234)"
    out = {"config": f"C2 box n={n} via afem_mesh_create, {order}: "
                     f"{mesh.n_own_nodes} DoF, {mesh.n_cells} tets, Poisson assembly + source",
           "dof": int(mesh.n_own_nodes), "value": round(mesh.n_own_nodes / (kms * 1e-3) / 1e6, 1),
           "unit": "MDoF/s (assembly kernels)", "kernel_ms": round(kms, 4),
           "roofline": with_traffic(roofline(bsr, mesh, kms), "c2_arrays_natural" if natural else "c2_arrays", n,
                                    kms),
           "kernel_ms_all": [round(x, 4) for x in ks], "settle_steps": settle_steps,
           "brick_order": int(st["brick_order"]), "cube_lattice": int(st["cube_lattice"]),
           "sparsity_ms": round(sp_ms, 1)}
    ctx.free(rhs)
    bsr.close()
    mesh.close()
    return out


def c2_generic_leg(ctx, af, n, reps=10, warmup=6, atomic_reps=2, settle_ms=150.0, unstructured_levels=0):
    """C2 through the path an UNCHANGED module takes: BSRFormat::assembleBilinear
    with the module's own element lambda (_computeElementMatrixTetra4Gpu,
    modules/poisson/FemModule.h:177-186: examples/elements.hpp PoissonTet4,
    compiled into examples/libafem_generic_example.so) on libafem's cell-unit
    kernel (include/arcanefem_amd_generic.hpp k_assemble_units), values
    written once (Mode::Overwrite = resetMatrixValues + assembleBilinear).
    The roofline's algorithmic bytes are the headline's without the RHS (no
    source term in assembleBilinear).  Also timed: the reference's algorithm
    (one lane per cell, f64 atomics into HBM: assemble_bilinear_atomic) on the
    same structure, and the values against the fixed-physics strip kernel.
    unstructured_levels > 0 (`generic_unstructured`): the same
    functor on the reference's L-shape-3D mesh refined that many times (the
    unstructured leg's mesh: slice-piece units of the Hilbert order)."""
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import generic_example as gx

    # the functor library is loaded (its code object registered) BEFORE the
    # refinement imports torch: torch's wheel carries a second HIP + HSA runtime
    # and rocprofiler-register (ROCm 7.0), and a code object first loaded after
    # those under rocprofv3 --kernel-trace faults in the tool's launch hook
    # (r05j; reproduced and isolated in r06c: tools/generic_trace_probe.py --
    # torch first: SIGSEGV at the first k_assemble_units launch; library first,
    # or no torch: clean; without the profiler all three run)
    gx.load()
    if unstructured_levels > 0:
        from arcanefem_amd.gmsh import read_gmsh

        gm = read_gmsh(os.path.join(ROOT, "tests", "golden", "L-shape-3D.msh"))
        cells, coords = refine_tets(gm.cells, gm.coords, unstructured_levels, "cpu")
        mesh = af.Mesh.from_arrays(ctx, 3, cells, coords)
        del cells, coords
        what = f"L-shape-3D.msh refined {unstructured_levels}x"
    else:
        mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
        what = f"C2 box n={n}"
    bsr = af.BSRFormat(mesh, 1).initialize(True)
    bsr.computeSparsity()
    ctx.synchronize()
    t0 = time.perf_counter()
    plan = bsr.functor_plan()
    ctx.synchronize()
    plan_ms = (time.perf_counter() - t0) * 1e3

    ks, settle_steps = time_launches(ctx, lambda: gx.assemble(bsr, gx.POISSON, gx.UNITS, overwrite=True), reps,
                                     warmup, settle_ms, base=150)
    kms = float(np.median(ks))
    vals_u = bsr.download()[2]
    ka, _ = time_launches(ctx, lambda: gx.assemble(bsr, gx.POISSON, gx.ATOMIC, overwrite=True), atomic_reps, 1, 0.0,
                          base=190)
    kam = float(np.median(ka))
    bsr.assemblePoissonP1(1.0, 0.0, None)
    vals_f = bsr.download()[2]
    st = bsr.stats()
    nnz = bsr.view().nnz_blocks
    ab = 4 * int(st["n_incidences"]) + 24 * mesh.n_nodes + 8 * (mesh.n_own_nodes + 1) + 12 * nnz
    ach = ab / (kms * 1e-3) / 1e9
    # what k_assemble_units must move: its plan entries, the functor's own
    # connectivity read per evaluation (4 x i32: the module's lambda reads
    # cn_cv itself), coordinates, row offsets, values
    ent_b = 24 if plan["wide"] else 8 if plan["packed"] else 16
    kmin = ((ent_b + 16) * plan["n_entries"] + 16 * plan["n_patterns"] * plan["packed"] + 24 * mesh.n_nodes
            + 8 * (mesh.n_own_nodes + 1) + 8 * nnz)
    fmt = "wide" if plan["wide"] else "packed" if plan["packed"] else "compact"
    out = {"config": f"{what} ({mesh.n_own_nodes} DoF, {mesh.n_cells} tets): assembleBilinear(the Poisson "
                     f"module's tet4 element lambda) through the generic element-functor entry, values overwritten",
           "dof": int(mesh.n_own_nodes), "value": round(mesh.n_own_nodes / (kms * 1e-3) / 1e6, 1),
           "unit": "MDoF/s (assembly kernel)", "kernel_ms": round(kms, 4), "kernel_ms_all": [round(x, 4) for x in ks],
           "roofline": {"bound": "hbm", "kernel": f"k_assemble_units<4,1,{fmt},PoissonTet4>",
                        "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": int(ab),
                        "bytes_kernel_min": int(kmin),
                        "bytes_kernel_min_note": "plan entries (+ pattern table when packed) + the functor's "
                                                 "connectivity reads per evaluation + coordinates + row offsets "
                                                 "+ values",
                        "frac_kernel_min": round(kmin / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "kernel_ms": round(kms, 4)},
           "settle_steps": settle_steps,
           "evaluations_per_cell": round(plan["n_entries"] / mesh.n_cells, 4),
           "plan": {k: int(plan[k]) for k in ("n_units", "n_stages", "n_entries", "rows_per_layer", "width", "nbuf",
                                              "wide", "lattice", "packed", "n_patterns")},
           "plan_build_ms": round(plan_ms, 1),
           "atomic_kernel_ms": round(kam, 4), "atomic_frac": round(ab / (kam * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "vs_fixed_physics_max_rel": float(np.abs(vals_u - vals_f).max() / np.abs(vals_f).max())}
    if unstructured_levels > 0:
        with_traffic(out["roofline"], "generic_unstructured", unstructured_levels, kms)
    else:
        with_traffic(out["roofline"], "c2_generic", n, kms)
    bsr.close()
    mesh.close()
    return out


def c5_breakdown(dyn, steps):
    """Where a C5 step goes: `steps` more steps with the
    per-phase HIP events of afem_elastodynamics_profile (outside the timed
    steps above: the events and the per-cycle pairs would perturb them), the
    median of each phase, and the block-3 roofline of the re-assembly kernel:
    c0 M + K and the body-force RHS on the fixed structure, algorithmic bytes as
    C3's (incidence table 4 B per (row, cell), coordinates 24 B per node, row
    offsets 8 B, block columns 4 B + 72 B of values per block, RHS 24 B per
    node)."""
    dyn.profile(True)
    ts = []
    for _ in range(steps):
        dyn.step()
        ts.append(dyn.step_timing())
    dyn.profile(False)
    med = {k: float(np.median([t[k] for t in ts])) for k in ("assemble_ms", "rhs_ms", "bc_ms", "solve_ms",
                                                              "precond_ms", "update_ms", "total_ms", "iterations")}
    t0 = ts[0]
    n_own, n_loc, nnz_b, n_inc = t0["n_own_nodes"], t0["n_nodes"], t0["nnz_blocks"], t0["n_incidences"]
    ab = 4 * n_inc + 24 * n_loc + 8 * (n_own + 1) + 76 * nnz_b + 24 * n_own
    ka = med["assemble_ms"]
    it = max(med["iterations"], 1.0)
    pcg_other = med["solve_ms"] - med["precond_ms"]
    return {"steps": steps, "assemble_ms": round(ka, 4), "rhs_ms": round(med["rhs_ms"], 4),
            "bc_ms": round(med["bc_ms"], 4), "solve_ms": round(med["solve_ms"], 3),
            "precond_ms": round(med["precond_ms"], 3), "pcg_spmv_vectors_ms": round(pcg_other, 3),
            "update_ms": round(med["update_ms"], 4), "total_ms": round(med["total_ms"], 3),
            "iterations": med["iterations"], "vcycle_ms_per_iteration": round(med["precond_ms"] / it, 4),
            "pcg_spmv_vectors_ms_per_iteration": round(pcg_other / it, 4),
            "assembly_roofline": {"bound": "hbm", "kernel": "k_assemble_elast_strip (c0 M + K + body force)",
                                  "algorithmic_bytes_per_launch": int(ab),
                                  "achieved": round(ab / (ka * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(ab / (ka * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}


def elastodynamics_c5(ctx, af, n, steps, preconditioners=("multigrid", "jacobi"), profile_steps=3):
    """BASELINE config C5 on one GPU: 3D Newmark elastodynamics, every step
    re-assembles c0 M + K and the body-force RHS on the fixed block-3
    structure, adds M (c0 U + c3 V + c4 A), clamps the x = 0 face by penalty,
    solves by PCG (rtol 1e-8) and updates U, V, A on the device.  One line per
    preconditioner: the geometric multigrid V-cycle (built at the first step,
    reused) and point Jacobi."""
    from arcanefem_amd.elastodynamics import Elastodynamics3D

    mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
    ids = np.arange(mesh.n_own_nodes)
    fixed = ids[ids % (n + 1) == 0].astype(np.int32)  # node x-index 0 (the jittered x is not exactly 0)
    out = {"config": f"C5 elastodynamics 3D Newmark, Kuhn box n={n} ({mesh.n_own_nodes} nodes, "
                     f"{3 * mesh.n_own_nodes} DoF, x = 0 face clamped), reassembly every step + PCG rtol 1e-8"}
    for pc in preconditioners:
        dyn = Elastodynamics3D(ctx, mesh, E=21.0e5, nu=0.28, rho=1.0, dt=1.0e-3, body_force=(0.0, 0.0, -1.0),
                               fixed_nodes=fixed, rtol=1e-8, preconditioner=pc)
        t0 = time.perf_counter()
        dyn.step()
        ctx.synchronize()
        first_ms = (time.perf_counter() - t0) * 1e3
        iters, conv = [], []
        t0 = time.perf_counter()
        for _ in range(steps):
            st = dyn.step()
            iters.append(int(st["iterations"]))
            conv.append(bool(st["converged"]))
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / steps
        key = "" if pc == preconditioners[0] else f"{pc}_"
        out[f"{key}preconditioner"] = pc
        out[f"{key}steps_per_s"] = round(1.0 / dt, 2)
        out[f"{key}ms_per_step"] = round(dt * 1e3, 2)
        out[f"{key}cg_iterations_per_step"] = float(np.mean(iters))
        out[f"{key}iterations"] = iters
        out[f"{key}converged"] = conv
        out[f"{key}first_step_ms"] = round(first_ms, 1)
        if pc == preconditioners[0]:
            out["breakdown"] = c5_breakdown(dyn, profile_steps)
        dyn.close()
    mesh.close()
    return out


def host_cores():
    """(the lease's thread count, cores this process may run on, nproc): the
    lease's OMP_NUM_THREADS (16 per GPU on the MI355X boxes) capped by the
    affinity mask, and the affinity mask itself -- the node's host cores the CPU
    baseline is stated on."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    lim = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(aff, lim) if lim > 0 else aff), aff, nproc


def cgroup_cpu_limit():
    """The cgroup v2 CPU quota of this job (cpu.max: quota / period), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def download_c2(ctx, mesh, bsr, ls, bottom):
    """The headline's input and output, copied to the host for the CPU
    baseline: cells, coordinates, structure (bit-equal to the oracle's own
    sparsity, tests/test_gpu_parity.py) and the GPU's assembled values / RHS
    (compared with the oracle's below, a parity check at the C2 size)."""
    cells, coords, _ = mesh.download()
    rp, cols, vals = bsr.download()
    return dict(cells=cells, coords=coords, n_own=mesh.n_own_nodes, rp=rp, cols=cols, gpu_vals=vals,
                gpu_rhs=ls.rhs_host(), dirichlet=bottom)


def cpu_baseline(c2, runs=5):
    """the oracle (C restatement of the reference's cell
    loop with linear column search, femutils/BSRFormat.h:807-836, + RHS +
    penalty) at the headline's C2 size on this host: one single-threaded
    assembly, then the median of `runs` on every core this job may use
    (OpenMP, atomic adds: the reference's multi-core loop) after one warm-up.
    `value` is the multi-core rate.  The oracle's values are also compared with
    the GPU's (max relative difference in `sample`)."""
    from oracle import oracle as O

    cells, coords, n_own, rp, cols = c2["cells"], c2["coords"], c2["n_own"], c2["rp"], c2["cols"]

    def one(fn):
        t0 = time.perf_counter()
        vals, rhs = fn(n_own, cells, coords, rp, cols, 5.5)
        O.dirichlet_penalty(c2["dirichlet"], 0.5, 1e30, rp, cols, vals, rhs)
        return time.perf_counter() - t0, vals, rhs

    t1, _, _ = one(O.assemble_poisson)
    lease, aff, nproc = host_cores()

    def median_on(threads):
        O.omp_threads(threads)
        one(O.assemble_poisson_omp)  # thread-pool warm-up
        ts = []
        for _ in range(runs):
            t, v, r = one(O.assemble_poisson_omp)
            ts.append(t)
        return float(np.median(ts)), v, r

    t_lease, _, _ = median_on(lease)
    # every core of the affinity mask too; under a cgroup CPU
    # quota smaller than the mask (16 CPUs on the MI355X boxes) the extra threads
    # only time-share, so `value` is the faster of the two thread counts
    t_aff, vals, rhs = median_on(aff) if aff != lease else (t_lease, None, None)
    if vals is None:
        _, vals, rhs = median_on(lease)
    tm, threads = (t_lease, lease) if t_lease <= t_aff else (t_aff, aff)
    scale = np.abs(vals).max()
    dv = float(np.abs(vals - c2["gpu_vals"]).max() / scale)
    free = np.abs(vals) < 1e20  # the penalty diagonal is set, not summed
    dvf = float(np.abs(vals[free] - c2["gpu_vals"][free]).max() / np.abs(vals[free]).max())
    drhs = float(np.abs(rhs - c2["gpu_rhs"]).max() / np.abs(rhs).max())
    c2["orc_vals"], c2["orc_rhs"] = vals, rhs
    quota = cgroup_cpu_limit()
    return {"value": round(n_own / tm / 1e6, 2), "unit": "MDoF/s", "cores": threads, "kind": "port",
            "nproc": nproc, "affinity_cores": aff, "cgroup_cpu_quota": quota,
            "value_lease_threads": round(n_own / t_lease / 1e6, 2), "lease_threads": lease,
            "value_all_cores": round(n_own / t_aff / 1e6, 2),
            "value_single_thread": round(n_own / t1 / 1e6, 2),
            "sample": f"C2 itself: Poisson-3D P1 Kuhn box ({n_own} DoF, {cells.shape[0]} tets, {cols.size} nnz), "
                      f"structure from the GPU run: median of {runs} assemblies (oracle/oracle.c cell loop, atomic adds, "
                      f"gcc -O3 -march=x86-64-v4; nproc {nproc}; cgroup CPU quota {quota}): {t_aff * 1e3:.0f} ms on "
                      f"{aff} OpenMP threads = every core of the affinity mask, {t_lease * 1e3:.0f} ms on the lease's "
                      f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')} ({lease} threads); value = the "
                      f"faster ({threads} threads); single thread "
                      f"{t1 * 1e3:.0f} ms = {n_own / t1 / 1e6:.2f} MDoF/s; oracle vs GPU values max rel diff "
                      f"{dvf:.1e} (free rows; {dv:.1e} overall), RHS {drhs:.1e}"}


def cpu_baseline_cg(c2, iters=50, runs=3):
    """the oracle's Jacobi-PCG with OpenMP on the C2 CSR
    the CPU baseline assembled, exactly `iters` iterations, median of `runs`
    after one warm-up."""
    from oracle import oracle as O

    rp, cols, vals, rhs = c2["rp"], c2["cols"], c2["orc_vals"], c2["orc_rhs"]
    lease, aff, _ = host_cores()

    def median_on(threads):
        O.omp_threads(threads)
        O.pcg_jacobi_omp(rp, cols, vals, rhs, max_iter=-iters)
        ts = []
        for _ in range(runs):
            t0 = time.perf_counter()
            O.pcg_jacobi_omp(rp, cols, vals, rhs, max_iter=-iters)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    runs_lease = runs
    t_lease = median_on(lease)
    # every core of the mask: one run when a cgroup quota caps the job below it
    # (the oversubscribed barrier-heavy loop took 27 s per run at 256 threads)
    quota = cgroup_cpu_limit()
    runs_aff = runs
    if aff != lease:
        runs_aff = runs = 1 if quota is not None and quota < aff else runs
        t_aff = median_on(aff)
    else:
        t_aff = t_lease
    t, threads = (t_lease, lease) if t_lease <= t_aff else (t_aff, aff)
    return {"value": round(iters / t, 2), "unit": "iter/s", "cores": threads, "kind": "port",
            "value_lease_threads": round(iters / t_lease, 2), "lease_threads": lease, "runs_lease_threads": runs_lease,
            "value_all_cores": round(iters / t_aff, 2), "affinity_cores": aff, "runs_all_cores": runs_aff,
            "cgroup_cpu_quota": quota,
            "sample": f"Jacobi-PCG (oracle/oracle.c orc_pcg_jacobi_omp) on the C2 system ({rp.size - 1} DoF, "
                      f"{int(rp[-1])} nnz): {iters} fixed iterations: {t_lease * 1e3:.1f} ms on the lease's {lease} "
                      f"OpenMP threads (median of {runs_lease}), {t_aff * 1e3:.1f} ms on {aff} (every core of the "
                      f"affinity mask; {'median of ' + str(runs_aff) if runs_aff > 1 else 'ONE run'}; cgroup CPU "
                      f"quota {quota}); value = the faster ({threads} threads)"}


def cpu_baseline_c1(runs=3):
    """config C1 end to end with the SequentialBasic
    semantics (femutils/DoFLinearSystem.cc:83-164): dense N x N `+=` assembly,
    penalty via matrixSetValue, dense -> CSR dropping zeros, PCG eps 1e-15.
    Single-threaded numpy/C; median of `runs`."""
    from oracle import oracle as O

    m = O.structured_mesh(2, 99)
    n = m["n_own"]
    cells, coords = m["cells"], m["coords"]
    ts, x = [], None
    for _ in range(runs):
        t0 = time.perf_counter()
        A = np.zeros((n, n))
        b = np.zeros(n)
        for c in cells:
            K, area = O.element_tri3(coords[c])
            A[np.ix_(c, c)] += K
            b[c] += 5.5 * area / 3
        for d in m["dirichlet"]:
            A[d, d] = 1e30
            b[d] = 1e30 * 0.5
        x = O.sequential_dense_solve(A, b)
        ts.append(time.perf_counter() - t0)
        del A
    t = float(np.median(ts))
    return {"value": round(t * 1e3, 1), "unit": "ms (assembly + solve)", "cores": 1, "kind": "port",
            "sample": f"C1: Poisson-2D P1 n=99 ({n} DoF, {cells.shape[0]} triangles), dense SequentialBasic "
                      f"semantics end to end, median of {runs}; max|u| = {np.abs(x).max():.6g}"}


def run_legs(ctx, af, args, legs):
    """The N = 1 side measurements named in `legs`, each with its own settle."""
    extras = {}
    sm = args.settle_ms
    if "c4" in legs and args.c4_n > 0:
        # the headline's CG iteration count (100): the solve's one-time setup (pattern flags, D^-1, x0, the
        # first SpMV: ~15 ms at C4) amortised as in the headline's CG
        extras["c4"] = poisson_c4(ctx, af, args.c4_n, cg_iters=args.cg_iters, settle_ms=sm)
    if "c3" in legs:
        extras["c3"] = elasticity_c3(ctx, af, args.c3_n, settle_ms=sm)
    if "c2_generic" in legs:
        extras["c2_generic"] = c2_generic_leg(ctx, af, 215, settle_ms=sm)
    if "c2_arrays" in legs:
        extras["c2_arrays"] = c2_arrays_leg(ctx, af, 215, settle_ms=sm)
    if "c2_arrays_natural" in legs:
        extras["c2_arrays_natural"] = c2_arrays_leg(ctx, af, 215, natural=True, settle_ms=sm)
    if ("unstructured" in legs or "unstructured_solve" in legs) and args.unstructured_levels > 0:
        extras["unstructured"] = unstructured_leg(ctx, af, "L-shape-3D.msh", args.unstructured_levels, settle_ms=sm,
                                                  solve="unstructured_solve" in legs)
    if "generic_unstructured" in legs and args.unstructured_levels > 0:
        extras["generic_unstructured"] = c2_generic_leg(ctx, af, 0, settle_ms=sm,
                                                        unstructured_levels=args.unstructured_levels)
    if "c5" in legs:
        extras["c5"] = elastodynamics_c5(ctx, af, args.c5_n, args.c5_steps)
    return extras


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)

    import arcanefem_amd as af

    ndev = af.device_count()
    if ndev < 1:
        raise SystemExit("bench.py needs a GPU (libafem.so has no CPU path)")
    if world > 1 and args.comm == "rccl" and ndev < world:
        # RCCL runs one rank per device; --comm host rehearses several ranks on one GPU
        raise SystemExit(f"bench.py: {world} ranks over RCCL need {world} GPUs, this host shows {ndev} "
                         f"(use --comm host to run them on one GPU over the host transport)")
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
    ctx = af.Context(local_rank % ndev)
    if args.no_headline:
        if world > 1:
            raise SystemExit("bench.py: --no-headline runs the N = 1 side legs only")
        print(json.dumps({"legs_only": True, "settle_ms": args.settle_ms,
                          **run_legs(ctx, af, args, set(args.legs.split(",")))}), flush=True)
        return
    n = args.n
    nz = n * world if args.scaling == "weak" else n
    t_setup = time.perf_counter()
    mesh, bsr, ls, bottom, dbottom, sparsity_ms = poisson_setup(ctx, af, n, nz, world, rank)
    nnz = bsr.view().nnz_blocks
    n_own, n_cells = mesh.n_own_nodes, mesh.n_cells
    comm = None
    if world > 1:
        if args.comm == "host":
            from arcanefem_amd.parallel import HostCommunicator

            comm = HostCommunicator(ctx)
        else:
            uid = [af.Communicator.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = af.Communicator(ctx, world, rank, uid[0])
        ls.set_halo_structured(comm, mesh)
    setup_s = time.perf_counter() - t_setup
    step = make_step(ctx, bsr, ls, bottom, dbottom)

    # unsettled: W warmup steps and K timed steps right after the setup, before
    # the clock-settle phase (the line reports both; the settled run
    # below is `value`)
    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    if dist:
        dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    uslots = min(args.steps, 27)
    for i in range(args.steps):
        step(200 + 2 * i if i < uslots else None)
    ctx.synchronize()
    if dist:
        dist.barrier()
    elapsed_unsettled = time.perf_counter() - t0
    kernel_ms_unsettled = [ctx.event_elapsed(200 + 2 * i, 201 + 2 * i) for i in range(uslots)]

    settle_steps = settle(ctx, step, args.settle_ms)
    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    if dist:
        dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    slots = min(args.steps, 100)
    for i in range(args.steps):
        step(2 * i if i < slots else None)
    ctx.synchronize()
    elapsed_own = time.perf_counter() - t0
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [ctx.event_elapsed(2 * i, 2 * i + 1) for i in range(slots)]
    if dist:
        import torch

        t = torch.tensor([elapsed, elapsed_unsettled], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, elapsed_unsettled = float(t[0]), float(t[1])
        tot = torch.tensor([float(n_own)], dtype=torch.float64)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        total_dof = float(tot[0])
    else:
        total_dof = float(n_own)
    ms_per_step = elapsed * 1e3 / args.steps
    value = total_dof * args.steps / elapsed / 1e6

    # ---- CG iter/s on the assembled system (fixed iteration count)
    ls.setSolverOptions(fixed_iterations=args.cg_iters)
    if dist:
        dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    st = ls.solve()
    ctx.synchronize()
    cg_s_own = time.perf_counter() - t0
    if dist:
        dist.barrier()
    cg_s = time.perf_counter() - t0
    if dist:
        import torch

        t = torch.tensor([cg_s], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        cg_s = float(t[0])
    cg_iter_per_s = args.cg_iters / cg_s
    per_rank = None
    if dist:
        # where each rank's time goes: its assembly kernel time,
        # and a separate short PCG run with the loop's halo waits and scalar
        # all-reduces timed by HIP events on the context stream (outside the
        # timed region above: the event records would perturb it)
        nit = min(20, args.cg_iters)
        ls.setSolverOptions(fixed_iterations=nit, profile_comm=True)
        ctx.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        sp = ls.solve()
        ctx.synchronize()
        prof_s = time.perf_counter() - t0
        ls.setSolverOptions(profile_comm=False)
        mine = {"rank": rank, "dof": int(n_own), "assembly_kernel_ms": round(float(np.median(kernel_ms)), 4),
                "step_ms_own": round(elapsed_own * 1e3 / args.steps, 4),
                "cg_ms_per_iter_own": round(cg_s_own * 1e3 / args.cg_iters, 4),
                "cg_device_ms_per_iter": round(st["solve_ms"] / max(st["iterations"], 1), 4),
                "profiled_cg_ms_per_iter": round(prof_s * 1e3 / nit, 4),
                "halo_wait_ms_per_iter": round(sp["halo_wait_ms"] / max(sp["n_halo"], 1), 5),
                "allreduce_ms_per_iter": round(sp["allreduce_ms"] / max(sp["iterations"], 1), 5),
                "allreduces_per_iter": round(sp["n_allreduce"] / max(sp["iterations"], 1), 2),
                "halo_bytes_per_exchange": int(sp["halo_bytes"])}
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        per_rank = gathered

    if rank == 0:
        kmed = float(np.median(kernel_ms))
        rf = roofline(bsr, mesh, kmed)
        rf["kernel_ms_mean"] = round(float(np.mean(kernel_ms)), 4)
        rf["kernel_ms_unsettled"] = round(float(np.median(kernel_ms_unsettled)), 4)
        rf["frac_unsettled"] = round(rf["algorithmic_bytes_per_launch"] / (rf["kernel_ms_unsettled"] * 1e-3) / 1e9
                                     / HBM_PEAK_GBS, 4)
        rf["traffic"] = None
        if world == 1:
            with_traffic(rf, "c2" if args.scaling == "weak" else "c4", n, kmed)
        extras = {}
        c2 = None
        if world == 1:
            if not args.no_cpu_baseline:
                c2 = download_c2(ctx, mesh, bsr, ls, bottom)
            # free the headline's buffers before the large side legs
            ctx.free(dbottom)
            ls.reset()
            bsr.close()
            mesh.close()
            dbottom = None
        legs = set() if args.no_extras or world > 1 else set(args.legs.split(","))
        if args.scaling == "strong" and n == args.c4_n:
            legs.discard("c4")
        extras = run_legs(ctx, af, args, legs)
        cpu = None
        if c2 is not None:
            cpu = cpu_baseline(c2)
            extras["cpu_baseline_cg"] = cpu_baseline_cg(c2)
            extras["cpu_baseline_c1"] = cpu_baseline_c1()
            del c2
        if args.scaling == "weak":
            workload = (f"C2 Poisson-3D P1, jittered Kuhn-tet box n={n} per GPU stacked in z "
                        f"({n_own} DoF, {n_cells} tets on rank 0), CSR assembly (matrix+RHS+penalty Dirichlet z=0) "
                        f"on fixed sparsity; CG = Jacobi-PCG on it")
        else:
            workload = (f"C4 Poisson-3D P1, ONE jittered Kuhn-tet box n={n} ({int(total_dof)} DoF) cut into "
                        f"{world} z-slab(s) ({n_own} DoF, {n_cells} tets on rank 0), CSR assembly "
                        f"(matrix+RHS+penalty Dirichlet z=0) on fixed sparsity; CG = Jacobi-PCG on it")
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "MDoF/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms,
            "settle_steps": settle_steps,
            "ms_per_step": round(ms_per_step, 4),
            "ms_per_step_unsettled": round(elapsed_unsettled * 1e3 / args.steps, 4),
            "value_unsettled": round(total_dof * args.steps / elapsed_unsettled / 1e6, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": workload,
                "n": n,
                "scaling": args.scaling,
                "dof_total": int(total_dof),
                "dof_rank0": int(n_own),
                "nnz_rank0": int(nnz),
                "parallelism": f"z-slab x{world}, {'RCCL' if args.comm == 'rccl' else 'host-transport'} halo + all-reduce in CG",
            },
            "roofline": rf,
            "cpu_baseline": cpu,
            "cg_iter_per_s": round(cg_iter_per_s, 2),
            "cg_ms_per_iter": round(cg_s * 1e3 / args.cg_iters, 4),
            "cg_roofline_frac": round(cg_bytes(nnz, n_own) * cg_iter_per_s / 1e9 / HBM_PEAK_GBS, 4),
            "cg_device_ms": round(st["solve_ms"], 3), "cg_spmv": SPMV_KERNELS.get(st["spmv_kernel"]),
            "sparsity_ms": round(sparsity_ms, 1),
            "setup_s": round(setup_s, 2),
            **({"per_rank": per_rank} if per_rank else {}),
            **extras,
        }
        if world == 1 and args.scaling == "weak":
            out.update(cg_traffic("c2_spmv", n, n_own, cg_iter_per_s))
        print(json.dumps({"bench_detail": out}), flush=True)
        print(json.dumps(compact_line(out)), flush=True)
    if dbottom is not None:
        ctx.free(dbottom)
    if comm:
        comm.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
