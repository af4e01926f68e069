"""3D elastodynamics time stepping on the assembly + CG path (BASELINE config C5).

Thin host mirror of the native time loop behind the C ABI
(``afem_elastodynamics_*``, arcanefem_amd/csrc/elastodynamics.cpp), which
restates the reference's time-stepping callers of the linear-system path:

* ``modules/elastodynamics/FemModule.cc`` (2D TRIA3): Newmark-beta with
  gamma = 1/2, beta = (gamma + 1/2)^2 / 4 (:256-270) or generalized-alpha
  (gamma = 1/2 + alpf - alpm, :275-290), Rayleigh damping etam / etak; LHS
  ``c1 div-div + c2 strain + c0 consistent mass`` (:1130-1340); RHS
  ``M (c0 U + c3 V + c4 A) - K(c5, c6) U + K(c7, c9) V + K(c8, c10) A`` + body
  force (:842-862); state update ``_updateVariables`` (:429-455); the matrix
  re-assembled every step (:149-153).
* ``modules/passmo/ElastodynamicModule.cc`` (3D): re-assembly every step on a
  fixed structure (:469-536).

Here the same scheme runs in 3D on P1 tetrahedra with block-3 BSR, on one
subdomain or on one ghosted z-slab per rank (``comm``: RCCL ``Communicator`` or
``parallel.HostCommunicator``): each step re-assembles ``c0 M + K`` and the
body-force RHS in one fused HIP kernel on the fixed sparsity, adds
``M (c0 U + c3 V + c4 A)`` (the mass operator shares the structure; its SpMV
exchanges the ghost values of the operand), clamps the fixed nodes by
penalty, solves with the PCG (3x3 node-block Jacobi by default, warm started
from the Newmark predictor; halo + all-reduces over the ranks) and
applies the Newmark update on the device.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _capi as C
from ._capi import call
from .core import Context, Mesh


SCHEMES = {"newmark-beta": 0, "generalized-alpha": 1}


def newmark_coefficients(rho: float, dt: float):
    """Newmark-beta constants of modules/elastodynamics/FemModule.cc:255-264
    (etam = etak = 0): returns gamma, beta, c0, c3, c4."""
    gamma = 0.5
    beta = 0.25 * (gamma + 0.5) ** 2
    c0 = rho / (beta * dt * dt)
    c3 = rho / beta / dt
    c4 = rho * ((1.0 - 2.0 * beta) / 2.0 / beta)
    return gamma, beta, c0, c3, c4


def young_from_lame(lam: float, mu: float):
    """(E, nu) of Lame parameters the way passmo converts its "lame" input
    (modules/passmo/ElastodynamicModule.cc:270-277): x = lambda/mu,
    nu = x/2/(1+x), E = 2 mu (1+nu)."""
    x = lam / mu
    nu = x / 2.0 / (1.0 + x)
    return 2.0 * mu * (1.0 + nu), nu


class Elastodynamics3D:
    def __init__(self, ctx: Context, mesh: Mesh, E: float, nu: float, rho: float, dt: float,
                 body_force=(0.0, 0.0, 0.0), fixed_nodes=None, penalty: float = 1.0e30, rtol: float = 1e-12,
                 comm=None, max_iter: int = 20000, preconditioner: str = "jacobi", etam: float = 0.0,
                 etak: float = 0.0, alpm: float = 0.0, alpf: float = 0.0, time_discretization: str = "newmark-beta"):
        """time_discretization, etam, etak, alpm, alpf: the module's
        timeDiscretization and damping options (Fem.axl of
        modules/elastodynamics; FemModule.cc:222-296)."""
        if mesh.dim != 3:
            raise ValueError("Elastodynamics3D needs a tetrahedral mesh")
        if time_discretization.lower() not in SCHEMES:
            raise ValueError("Only Newmark-beta | Generalized-alpha are supported for time-discretization")
        self.ctx, self.mesh, self.dt = ctx, mesh, dt
        self.n = 3 * mesh.n_own_nodes
        p = C.NewmarkParams(E, nu, rho, dt, (ctypes.c_double * 3)(*[float(x) for x in body_force]), penalty, 0.0, 0.0,
                            etam, etak, alpm, alpf, SCHEMES[time_discretization.lower()], 0)
        fixed = np.zeros(0, dtype=np.int32) if fixed_nodes is None else np.ascontiguousarray(fixed_nodes,
                                                                                            dtype=np.int32)
        h = ctypes.c_void_p()
        call("afem_elastodynamics_create", mesh.h, comm.h if comm is not None else None, ctypes.byref(p),
             ctypes.c_void_p(fixed.ctypes.data) if fixed.size else None, fixed.size, C.AFEM_MEM_HOST,
             ctypes.byref(h))
        self.h = h
        # "multigrid": the geometric multigrid V-cycle on structured boxes (one rank or z-slabs), built at
        # the first step and reused (the Newmark operator c0 M + K is the same every step)
        # "amg-reuse": the algebraic multigrid (any mesh; rebuilt when dt changes the operator)
        blk, mgm, amg = {"jacobi": (0, 0, 0), "block3": (3, 0, 0), "multigrid": (0, 2, 0),
                         "amg-reuse": (0, 0, 2)}[preconditioner]
        o = C.SolverOpts(C.AFEM_SOLVER_PCG, max_iter, rtol, 0.0, 8, 0, 0, blk, mgm)
        o.amg = amg
        call("afem_elastodynamics_set_solver_options", self.h, ctypes.byref(o))
        self.t = 0.0
        self.last_stats = None

    def step(self) -> dict:
        st = C.SolveStats()
        call("afem_elastodynamics_step", self.h, ctypes.byref(st))
        self.t += self.dt
        self.last_stats = dict(iterations=st.iterations, converged=bool(st.converged), rel_residual=st.rel_residual,
                               residual_norm=st.residual_norm, solve_ms=st.solve_ms, amg_levels=st.amg_levels,
                               amg_setup_ms=st.amg_setup_ms, precond_ms=st.precond_ms)
        return self.last_stats

    def setDirichlet(self, dofs, values):
        """Imposed displacements by penalty (passmo's dirichlet-surface /
        point conditions, modules/passmo/ElastodynamicModule.cc:1923-1939 and
        the re-application after the solve :2369-2371): local DoF ids
        (3 node + component) and their values; replaces the previous list."""
        d = np.ascontiguousarray(dofs, dtype=np.int32).ravel()
        v = np.ascontiguousarray(np.broadcast_to(np.asarray(values, dtype=np.float64), d.shape))
        call("afem_elastodynamics_set_dirichlet", self.h, ctypes.c_void_p(d.ctypes.data) if d.size else None,
             ctypes.c_void_p(v.ctypes.data) if v.size else None, d.size, C.AFEM_MEM_HOST)

    def setTimeStep(self, dt: float):
        """dt from the next step on (passmo's shortened final step, :525-530)."""
        call("afem_elastodynamics_set_time_step", self.h, float(dt))
        self.dt = float(dt)

    def profile(self, on: bool = True):
        """Per-phase HIP-event times of every following step (step_timing())."""
        call("afem_elastodynamics_profile", self.h, 1 if on else 0)

    def step_timing(self) -> dict:
        t = C.StepTiming()
        call("afem_elastodynamics_step_timing", self.h, ctypes.byref(t))
        return {f: getattr(t, f) for f, _ in C.StepTiming._fields_ if f != "reserved0"}

    def operators(self):
        """The last step's operators on the device: dict(lhs = CsrView of c0 M +
        K (block 3, CSR-row order), scalar_rows / scalar_cols = device pointers
        of the scalar CSR structure of those values, mass = device pointer of
        the mass values on it, c = the constants c0 .. c10)."""
        v = C.CsrView()
        sr, sc, mp = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        c = (ctypes.c_double * 11)()
        call("afem_elastodynamics_operators", self.h, ctypes.byref(v), ctypes.byref(sr), ctypes.byref(sc),
             ctypes.byref(mp), c)
        return dict(lhs=v, scalar_rows=sr.value, scalar_cols=sc.value, mass=mp.value, c=list(c))

    def state_dptrs(self):
        u, v, a = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        call("afem_elastodynamics_state", self.h, ctypes.byref(u), ctypes.byref(v), ctypes.byref(a))
        return u.value, v.value, a.value

    def state_host(self):
        return tuple(self.ctx.to_host(p, self.n, np.float64) for p in self.state_dptrs())

    def close(self):
        if self.h:
            call("afem_elastodynamics_destroy", self.h)
            self.h = None
