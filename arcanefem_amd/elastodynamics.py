"""3D elastodynamics time stepping on the assembly + CG path (BASELINE config C5).

Host-side mirror of the reference's time-stepping callers of the linear-system
path:

* ``modules/elastodynamics/FemModule.cc`` (2D TRIA3): Newmark-beta with
  gamma = 1/2, beta = (gamma + 1/2)^2 / 4 (:256-270); LHS
  ``c1 div-div + c2 strain + c0 consistent mass`` (:1130-1340, c1 = lambda and
  c2 = 2 mu without Rayleigh damping, etak = 0); RHS
  ``M (c0 U + c3 V + c4 A)`` + body force (:842-862); state update
  ``_updateVariables`` (:429-455); the linear system is re-created and the
  matrix re-assembled every step (:149-153).
* ``modules/passmo/ElastodynamicModule.cc`` (3D): re-assembly every step on a
  fixed structure (:469-536).

Here the same scheme runs in 3D on P1 tetrahedra with block-3 BSR: every step
re-assembles ``c0 M + K`` and the body-force RHS in one fused HIP kernel
(``afem_bsr_assemble_elasticity_p1_ex``) on the fixed sparsity, adds
``M (c0 U + c3 V + c4 A)`` (device lincomb + SpMV with the mass matrix
assembled once), imposes the clamped DoFs by penalty (the reference's
default Dirichlet treatment), solves with the Jacobi-PCG and applies the
Newmark update on the device.  Rayleigh damping (etam, etak) and the
generalized-alpha variant are not implemented (per-step
reassembly is the path; the damping terms only add more mass/stiffness
operands of the same shape).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._capi import call
from .core import BSRFormat, Context, DoFLinearSystem, Mesh


def newmark_coefficients(rho: float, dt: float):
    """Newmark-beta constants of modules/elastodynamics/FemModule.cc:255-264
    (etam = etak = 0): returns gamma, beta, c0, c3, c4."""
    gamma = 0.5
    beta = 0.25 * (gamma + 0.5) ** 2
    c0 = rho / (beta * dt * dt)
    c3 = rho / beta / dt
    c4 = rho * ((1.0 - 2.0 * beta) / 2.0 / beta)
    return gamma, beta, c0, c3, c4


class Elastodynamics3D:
    def __init__(self, ctx: Context, mesh: Mesh, E: float, nu: float, rho: float, dt: float,
                 body_force=(0.0, 0.0, 0.0), fixed_nodes=None, penalty: float = 1.0e30, rtol: float = 1e-12):
        if mesh.dim != 3:
            raise ValueError("Elastodynamics3D needs a tetrahedral mesh")
        if mesh.n_nodes != mesh.n_own_nodes:
            raise ValueError("Elastodynamics3D runs on one subdomain (no ghost nodes)")
        self.ctx, self.mesh, self.dt = ctx, mesh, dt
        self.lam = E * nu / ((1 + nu) * (1 - 2 * nu))
        self.mu2 = 2.0 * E / (2 * (1 + nu))
        self.gamma, self.beta, self.c0, self.c3, self.c4 = newmark_coefficients(rho, dt)
        self.f = tuple(float(x) for x in body_force)
        self.penalty = penalty
        n = 3 * mesh.n_own_nodes
        self.n = n
        # stiffness + c0 mass: per-scalar-row (CSR) values, used in place by the solver
        self.K = BSRFormat(mesh, 3).initialize(True)
        self.K.computeSparsity()
        self.ls = DoFLinearSystem().initialize(ctx, n, n)
        self.K.toLinearSystem(self.ls)
        self.ls.setSolverOptions(rtol=rtol)
        # consistent mass (assembled once) for the RHS operand
        self.M = BSRFormat(mesh, 3).initialize(True)
        self.M.computeSparsity()
        self.M.assembleElasticityP1Ex(0.0, 0.0, 1.0)
        self.ls_m = DoFLinearSystem().initialize(ctx, n, n)
        self.M.toLinearSystem(self.ls_m)
        self.U, self.V, self.A, self.W, self.MW = (ctx.malloc(8 * n) for _ in range(5))
        z = np.zeros(n)
        for p in (self.U, self.V, self.A):
            ctx.to_device(p, z)
        fixed = np.zeros(0, dtype=np.int32) if fixed_nodes is None else np.asarray(fixed_nodes, dtype=np.int64)
        self.fixed_dofs = (3 * fixed[:, None] + np.arange(3)[None, :]).ravel().astype(np.int32)
        self.d_fixed = ctx.malloc(max(4 * self.fixed_dofs.size, 4))
        if self.fixed_dofs.size:
            ctx.to_device(self.d_fixed, self.fixed_dofs)
        self.t = 0.0
        self.last_stats = None

    def step(self) -> dict:
        ctx, ls = self.ctx, self.ls
        rhs = ls.rhsVariable()
        # LHS c0 M + K and body-force RHS, re-assembled on the fixed structure
        self.K.assembleElasticityP1Ex(self.lam, self.mu2, self.c0, self.f, rhs, rhs_mode="set")
        # RHS += M (c0 U + c3 V + c4 A)
        call("afem_vec_lincomb", ctx.h, self.n, self.c0, ctypes.c_void_p(self.U), self.c3, ctypes.c_void_p(self.V),
             self.c4, ctypes.c_void_p(self.A), ctypes.c_void_p(self.W))
        self.ls_m.spmv(self.W, self.MW)
        call("afem_vec_lincomb", ctx.h, self.n, 1.0, ctypes.c_void_p(rhs), 1.0, ctypes.c_void_p(self.MW), 0.0, None,
             ctypes.c_void_p(rhs))
        if self.fixed_dofs.size:
            ls.applyDirichletViaPenaltyDevice(self.d_fixed, self.fixed_dofs.size, 0.0, self.penalty)
            ls.applyBoundaryConditions()
        st = ls.solve()
        call("afem_newmark_update", ctx.h, self.n, self.dt, self.beta, self.gamma,
             ctypes.c_void_p(ls.solutionVariable()), ctypes.c_void_p(self.U), ctypes.c_void_p(self.V),
             ctypes.c_void_p(self.A))
        self.t += self.dt
        self.last_stats = st
        return st

    def state_host(self):
        return tuple(self.ctx.to_host(p, self.n, np.float64) for p in (self.U, self.V, self.A))

    def close(self):
        for p in (self.U, self.V, self.A, self.W, self.MW, self.d_fixed):
            self.ctx.free(p)
        self.K.close()
        self.M.close()
        self.ls.reset()
        self.ls_m.reset()
