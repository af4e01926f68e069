// 3D elastodynamics time stepping on the assembly + CG path (BASELINE config
// C5), native behind the C ABI.  Mirrors the reference's time-stepping callers:
//   modules/elastodynamics/FemModule.cc  Newmark-beta constants (:255-270),
//     RHS M (c0 U + c3 V + c4 A) + body force (:842-862), state update
//     _updateVariables (:429-455), the matrix re-assembled every step (:149-153);
//   modules/passmo/ElastodynamicModule.cc  3D, re-assembly every step on a
//     fixed structure (:469-536).
// Per step: the fused block-3 kernel re-assembles c0 M + K and the body-force
// RHS (rhs_mode SET), the device lincomb + mass SpMV (the mass values share
// the stiffness structure, assembled once) add M (c0 U + c3 V + c4 A), the
// clamped DoFs are imposed by penalty, the Jacobi-PCG solves (halo exchange
// and dot-product sums over ranks when a communicator is attached; warm
// started from the Newmark predictor) and the Newmark update runs on the
// device.  Rayleigh damping (etam, etak) and the generalized-alpha scheme
// (alpm, alpf) follow the module's constants c0 .. c10 (:255-290): the LHS is
// c0 M + K(c1, c2) and the RHS adds K(lambda = 1) (-c5 U + c7 V + c8 A) +
// K(2 mu = 1) (-c6 U + c9 V + c10 A) (:842-862) -- two more operators on the
// same structure, assembled once.
#include <cmath>
#include <map>
#include <vector>

#include "afem_internal.hpp"

namespace afem {

namespace {

void halo_for(LinearSystem& ls, Comm* comm, Mesh& m)
{
  if (!comm || comm_nranks(comm) == 1) return;
  std::vector<int> nb;
  std::vector<int64_t> sc, rc;
  std::vector<int32_t> si, ri;
  if (m.part.valid) {  // partitioned general mesh (afem_mesh_create_subdomain)
    nb = m.part.nbr;
    sc = m.part.send_cnt;
    rc = m.part.recv_cnt;
    si = m.part.send_ids;
    ri = m.part.recv_ids;
  }
  else {
    AFEM_REQUIRE(m.st.valid, AFEM_ERR_NOT_IMPL,
                 "distributed elastodynamics: the mesh carries no halo plan (structured slab or "
                 "afem_mesh_create_subdomain)");
    structured_halo_lists(m.st.dim, m.st.n, m.st.nz, m.st.nranks, m.st.rank, nb, sc, rc, si, ri);
  }
  expand_dof_lists(3, sc, rc, si, ri);
  std::vector<int32_t> nb32(nb.begin(), nb.end());
  ls.halo.reset(new Halo());
  halo_setup(*ls.halo, *ls.ctx, comm, (int)nb.size(), nb32.data(), sc.data(), si.data(), rc.data(), ri.data());
}

void init_ls(LinearSystem& ls, Ctx* ctx, int64_t n, int64_t n_cols)
{
  ls.ctx = ctx;
  ls.n_rows = n;
  ls.n_cols = n_cols;
  ls.opts.method = AFEM_SOLVER_PCG;
  ls.opts.max_iter = 20000;
  ls.opts.rtol = 1e-8;
  ls.opts.atol = 0.0;
  ls.opts.check_every = 8;
  ls.opts.fixed_iterations = 0;
  ls.opts.initial_guess = 0;
  ls.opts.precond_block = 0;
  ls.rhs.alloc(n);
  ls.sol.alloc(n_cols);
  ls.forced_info.alloc(n);
  ls.elim_info.alloc(n);
  ls.forced_value.alloc(n);
  ls.elim_value.alloc(n);
  for (auto* b : { (void*)ls.rhs.p, (void*)ls.forced_value.p, (void*)ls.elim_value.p })
    AFEM_HIP(hipMemsetAsync(b, 0, n * sizeof(double), ctx->stream));
  AFEM_HIP(hipMemsetAsync(ls.sol.p, 0, n_cols * sizeof(double), ctx->stream));
  AFEM_HIP(hipMemsetAsync(ls.forced_info.p, 0, n, ctx->stream));
  AFEM_HIP(hipMemsetAsync(ls.elim_info.p, 0, n, ctx->stream));
}
}  // namespace

// modules/elastodynamics/FemModule.cc:255-290: the Newmark-beta and
// generalized-alpha constants with Rayleigh damping (etam, etak)
void dyn_coefficients(Elastodynamics* d)
{
  const afem_newmark_params& p = d->p;
  const double lambda = d->lambda, mu = 0.5 * d->mu2, rho = p.rho, dt = p.dt, etam = p.etam, etak = p.etak;
  double* c = d->c;
  if (p.scheme == 1) {
    const double alpm = p.alpm, alpf = p.alpf;
    const double gamma = 0.5 + alpf - alpm, beta = 0.25 * (gamma + 0.5) * (gamma + 0.5);
    d->gamma = gamma;
    d->beta = beta;
    c[0] = rho * (1. - alpm) / (beta * dt * dt) + etam * rho * gamma * (1 - alpf) / beta / dt;
    c[1] = lambda * (1. - alpf) + lambda * etak * gamma * (1. - alpf) / beta / dt;
    c[2] = 2. * mu * (1. - alpf) + 2. * mu * etak * gamma * (1. - alpf) / beta / dt;
    c[3] = rho * (1. - alpm) / beta / dt - etam * rho * (1 - gamma * (1 - alpf) / beta);
    c[4] = rho * ((1. - alpm) * (1. - 2. * beta) / 2. / beta - alpm - etam * dt * (1. - alpf) * (1. - gamma / 2 / beta));
    c[5] = lambda * alpf - lambda * etak * gamma * (1. - alpf) / beta / dt;
    c[6] = 2 * mu * alpf - 2. * mu * etak * gamma * (1. - alpf) / beta / dt;
    c[7] = etak * lambda * (gamma * (1. - alpf) / beta - 1);
    c[8] = etak * lambda * dt * (1. - alpf) * ((1. - 2 * beta) / 2. / beta - (1. - gamma));
    c[9] = etak * 2 * mu * (gamma * (1. - alpf) / beta - 1);
    c[10] = etak * 2 * mu * dt * (1. - alpf) * ((1. - 2 * beta) / 2. / beta - (1. - gamma));
  }
  else {
    const double gamma = p.gamma > 0 ? p.gamma : 0.5;
    const double beta = p.beta > 0 ? p.beta : 0.25 * (gamma + 0.5) * (gamma + 0.5);
    d->gamma = gamma;
    d->beta = beta;
    c[0] = rho / (beta * dt * dt) + etam * rho * gamma / beta / dt;
    c[1] = lambda + lambda * etak * gamma / beta / dt;
    c[2] = 2. * mu + 2. * mu * etak * gamma / beta / dt;
    c[3] = rho / beta / dt - etam * rho * (1 - gamma / beta);
    c[4] = rho * ((1. - 2. * beta) / 2. / beta - etam * dt * (1. - gamma / 2 / beta));
    c[5] = -lambda * etak * gamma / beta / dt;
    c[6] = -2. * mu * etak * gamma / beta / dt;
    c[7] = etak * lambda * (gamma / beta - 1);
    c[8] = etak * lambda * dt * ((1. - 2 * beta) / 2. / beta - (1. - gamma));
    c[9] = etak * 2 * mu * (gamma / beta - 1);
    c[10] = etak * 2 * mu * dt * ((1. - 2 * beta) / 2. / beta - (1. - gamma));
  }
}

Elastodynamics* dyn_create(Mesh* mesh, Comm* comm, const afem_newmark_params* prm, const int32_t* fixed_nodes,
                           int64_t n_fixed, int mem)
{
  {
    AFEM_REQUIRE(mesh->nv == 4 && mesh->dim == 3, AFEM_ERR_NOT_IMPL, "elastodynamics needs a tetrahedral mesh");
    AFEM_REQUIRE(prm->dt > 0 && prm->E > 0 && prm->nu > -1.0 && prm->nu < 0.5 && prm->rho >= 0, AFEM_ERR_ARG,
                 "elastodynamics: bad material or time step");
    AFEM_REQUIRE(n_fixed == 0 || fixed_nodes, AFEM_ERR_ARG, "fixed_nodes is NULL");
    AFEM_REQUIRE(prm->scheme == 0 || prm->scheme == 1, AFEM_ERR_ARG,
                 "elastodynamics: scheme 0 (Newmark-beta) or 1 (generalized-alpha)");
    if (comm)
      AFEM_REQUIRE(comm_nranks(comm) == 1 ||
                       (mesh->st.valid && mesh->st.nranks == comm_nranks(comm) && mesh->st.rank == comm_rank(comm)) ||
                       (mesh->part.valid && mesh->part.nranks == comm_nranks(comm) &&
                        mesh->part.rank == comm_rank(comm)),
                   AFEM_ERR_ARG, "the mesh's slab / subdomain rank and nranks differ from the communicator");
    mesh->ctx->set_device();
    auto* d = new Elastodynamics();
    try {
      Ctx& ctx = *mesh->ctx;
      d->mesh = mesh;
      d->ctx = &ctx;
      d->comm = comm;
      d->p = *prm;
      if (!(d->p.penalty > 0)) d->p.penalty = 1.0e30;  // modules/elasticity/Fem.axl:37-41
      // modules/elastodynamics/FemModule.cc:130-134 (Lame) and :255-290 (time scheme)
      d->mu2 = (prm->E / (2 * (1 + prm->nu))) * 2;
      d->lambda = prm->E * prm->nu / ((1 + prm->nu) * (1 - 2 * prm->nu));
      dyn_coefficients(d);
      d->damped = prm->etak != 0.0 || (prm->scheme == 1 && prm->alpf != 0.0);
      d->n = 3 * mesh->n_own;
      d->n_cols = 3 * mesh->n_nodes;
      // structure once; stiffness and mass share it
      d->K.mesh = mesh;
      d->K.nb_dof = 3;
      d->K.order_per_block = false;
      build_structure(*mesh, d->K.s);
      d->K.values.alloc((size_t)d->K.s.nnz * 9);
      d->K.has_sparsity = true;
      d->mvals.alloc((size_t)d->K.s.nnz * 9);
      std::swap(d->K.values, d->mvals);
      assemble_elasticity_tet(d->K, 0.0, 0.0, 1.0, nullptr, nullptr, 0);  // M (c0 = 1)
      std::swap(d->K.values, d->mvals);
      if (d->damped) {  // the RHS's stiffness operators K(lambda = 1) and K(2 mu = 1)
        d->klvals.alloc((size_t)d->K.s.nnz * 9);
        d->kmvals.alloc((size_t)d->K.s.nnz * 9);
        std::swap(d->K.values, d->klvals);
        assemble_elasticity_tet(d->K, 1.0, 0.0, 0.0, nullptr, nullptr, 0);
        std::swap(d->K.values, d->klvals);
        std::swap(d->K.values, d->kmvals);
        assemble_elasticity_tet(d->K, 0.0, 1.0, 0.0, nullptr, nullptr, 0);
        std::swap(d->K.values, d->kmvals);
      }
      bsr_expand_scalar(d->K, nullptr);  // scalar rows / columns of the block-3 CSR (shared)
      init_ls(d->ls, &ctx, d->n, d->n_cols);
      init_ls(d->lsm, &ctx, d->n, d->n_cols);
      if (d->damped) {
        init_ls(d->lsl, &ctx, d->n, d->n_cols);
        init_ls(d->lsu, &ctx, d->n, d->n_cols);
      }
      for (LinearSystem* l : { &d->ls, &d->lsm, &d->lsl, &d->lsu }) {
        if (!l->ctx) continue;  // lsl / lsu without damping
        l->has_csr = true;
        l->csr_n = d->n;
        l->csr_nnz = d->K.s.nnz * 9;
        l->csr_rows = d->K.csr_rows.p;
        l->csr_diag = nullptr;
        l->csr_cols = d->K.csr_cols.p;
        l->blk_k = 3;
        l->blk_n = d->K.s.n_rows;
        l->blk_rows = d->K.s.row_ptr.p;
        l->blk_cols = d->K.s.cols.p;
      }
      {  // structured box (or z-slab: block-Jacobi V-cycles over the ranks): the multigrid preconditioner
        const StructuredInfo& st = mesh->st;
        if (st.valid && st.dim == 3 && !mesh->part.valid) {
          d->ls.mg_k = 3;
          d->ls.mg_nx = st.n;
          d->ls.mg_nz = (st.k1 - st.k0) - 1;
          d->ls.mg_multi = st.nranks > 1;
          d->ls.mg_nzg = st.nz;
          d->ls.mg_k0 = st.k0;
          d->ls.mg_glo = st.ghost_lo >= 0;
        }
      }
      d->ls.csr_vals = d->K.values.p;
      d->lsm.csr_vals = d->mvals.p;
      halo_for(d->ls, d->comm, *mesh);
      halo_for(d->lsm, d->comm, *mesh);
      if (d->damped) {
        d->lsl.csr_vals = d->klvals.p;
        d->lsu.csr_vals = d->kmvals.p;
        halo_for(d->lsl, d->comm, *mesh);
        halo_for(d->lsu, d->comm, *mesh);
      }
      for (auto* b : { &d->U, &d->V, &d->A, &d->MW }) {
        b->alloc(d->n);
        AFEM_HIP(hipMemsetAsync(b->p, 0, b->bytes(), ctx.stream));
      }
      d->W.alloc(d->n_cols);  // ghost part filled by the mass SpMV's halo exchange
      AFEM_HIP(hipMemsetAsync(d->W.p, 0, d->W.bytes(), ctx.stream));
      std::vector<int32_t> hn(n_fixed);
      if (n_fixed) {
        AFEM_HIP(hipMemcpyAsync(hn.data(), fixed_nodes, n_fixed * 4,
                                mem == AFEM_MEM_HOST ? hipMemcpyHostToHost : hipMemcpyDeviceToHost, ctx.stream));
        ctx.sync();
      }
      std::vector<int32_t> dofs;
      for (int32_t nd : hn) {
        AFEM_REQUIRE(nd >= 0 && nd < mesh->n_nodes, AFEM_ERR_ARG, "fixed node id out of range");
        if (nd < mesh->n_own)
          for (int i = 0; i < 3; ++i) dofs.push_back(3 * nd + i);
      }
      d->fixed.alloc(dofs.size());
      if (!dofs.empty())
        AFEM_HIP(hipMemcpyAsync(d->fixed.p, dofs.data(), dofs.size() * 4, hipMemcpyHostToDevice, ctx.stream));
      ctx.sync();
    }
    catch (...) {
      delete d;
      throw;
    }
    return d;
  }
}

void dyn_step(Elastodynamics* d, afem_solve_stats* st)
{
  {
    Ctx& ctx = *d->ctx;
    ctx.set_device();
    const double f[3] = { d->p.body_force[0], d->p.body_force[1], d->p.body_force[2] };
    const double* c = d->c;
    const bool prof = d->profile;
    auto mark = [&](int i) {
      if (prof) AFEM_HIP(hipEventRecord(d->ev[i], ctx.stream));
    };
    const int32_t prof_opt = d->ls.opts.profile_comm;
    if (prof) d->ls.opts.profile_comm = 1;  // the PCG times its preconditioner applications
    mark(0);
    // LHS c0 M + K(c1, c2) and the body force (rhs = f |K|/4), re-assembled on the fixed structure
    assemble_elasticity_tet(d->K, c[1], c[2], c[0], f, d->ls.rhs.p, 0);
    mark(1);
    // rhs += M (c0 U + c3 V + c4 A)
    vec_lincomb(ctx, d->n, c[0], d->U.p, c[3], d->V.p, c[4], d->A.p, d->W.p);
    ls_spmv(d->lsm, d->W.p, d->MW.p);
    vec_lincomb(ctx, d->n, 1.0, d->ls.rhs.p, 1.0, d->MW.p, 0.0, nullptr, d->ls.rhs.p);
    if (d->damped) {  // rhs += K(lambda = 1) (-c5 U + c7 V + c8 A) + K(2 mu = 1) (-c6 U + c9 V + c10 A)
      vec_lincomb(ctx, d->n, -c[5], d->U.p, c[7], d->V.p, c[8], d->A.p, d->W.p);
      ls_spmv(d->lsl, d->W.p, d->MW.p);
      vec_lincomb(ctx, d->n, 1.0, d->ls.rhs.p, 1.0, d->MW.p, 0.0, nullptr, d->ls.rhs.p);
      vec_lincomb(ctx, d->n, -c[6], d->U.p, c[9], d->V.p, c[10], d->A.p, d->W.p);
      ls_spmv(d->lsu, d->W.p, d->MW.p);
      vec_lincomb(ctx, d->n, 1.0, d->ls.rhs.p, 1.0, d->MW.p, 0.0, nullptr, d->ls.rhs.p);
    }
    mark(2);
    // clamped DoFs by penalty (the reference's default Dirichlet treatment)
    if (d->fixed.n) ls_set_list(d->ls, d->fixed.p, (int64_t)d->fixed.n, AFEM_MEM_DEVICE, 0, 0.0, d->p.penalty);
    // imposed displacements: diagonal = penalty, rhs = u penalty
    // (modules/passmo/ElastodynamicModule.cc:1923-1939)
    if (d->imp_ids.n)
      ls_set_list(d->ls, d->imp_ids.p, (int64_t)d->imp_ids.n, AFEM_MEM_DEVICE, 0, 0.0, d->p.penalty, d->imp_vals.p);
    // warm start from the Newmark predictor U + dt V + dt^2 (1/2 - beta) A
    // (the PCG's stopping target is unchanged: the zero guess's residual)
    vec_lincomb(ctx, d->n, 1.0, d->U.p, d->p.dt, d->V.p, d->p.dt * d->p.dt * (0.5 - d->beta), d->A.p, d->ls.sol.p);
    d->ls.opts.initial_guess = 1;
    mark(3);
    ls_solve(d->ls, &d->last);
    d->ls.opts.profile_comm = prof_opt;
    mark(4);
    // the imposed values re-applied to the solution (_doSolve, :2369-2371)
    if (d->imp_ids.n) vec_scatter(ctx, (int64_t)d->imp_ids.n, d->imp_ids.p, d->imp_vals.p, d->ls.sol.p);
    newmark_update(ctx, d->n, d->p.dt, d->beta, d->gamma, d->ls.sol.p, d->U.p, d->V.p, d->A.p);
    mark(5);
    ctx.sync();
    if (prof) {
      float ms[5] = {};
      for (int i = 0; i < 5; ++i) AFEM_HIP(hipEventElapsedTime(&ms[i], d->ev[i], d->ev[i + 1]));
      float tot = 0.f;
      AFEM_HIP(hipEventElapsedTime(&tot, d->ev[0], d->ev[5]));
      afem_step_timing& t = d->timing;
      t.assemble_ms = ms[0];
      t.rhs_ms = ms[1];
      t.bc_ms = ms[2];
      t.solve_ms = ms[3];
      t.precond_ms = d->last.precond_ms;
      t.update_ms = ms[4];
      t.total_ms = tot;
      t.iterations = d->last.iterations;
    }
    if (st) *st = d->last;
  }
}

void dyn_set_dirichlet(Elastodynamics* d, const int32_t* dofs, const double* values, int64_t n, int mem)
{
  AFEM_REQUIRE(n == 0 || (dofs && values), AFEM_ERR_ARG, "afem_elastodynamics_set_dirichlet: dofs / values is NULL");
  AFEM_REQUIRE(n >= 0, AFEM_ERR_ARG, "afem_elastodynamics_set_dirichlet: negative count");
  Ctx& ctx = *d->ctx;
  ctx.set_device();
  std::vector<int32_t> hd(n);
  std::vector<double> hv(n);
  if (n) {
    const hipMemcpyKind k = mem == AFEM_MEM_HOST ? hipMemcpyHostToHost : hipMemcpyDeviceToHost;
    AFEM_HIP(hipMemcpyAsync(hd.data(), dofs, n * sizeof(int32_t), k, ctx.stream));
    AFEM_HIP(hipMemcpyAsync(hv.data(), values, n * sizeof(double), k, ctx.stream));
    ctx.sync();
  }
  // owned DoFs only (the reference loops over ownNodes(), :1923); the last
  // value of a DoF listed twice wins, as the module's successive conditions
  std::map<int32_t, double> m;
  for (int64_t i = 0; i < n; ++i) {
    AFEM_REQUIRE(hd[i] >= 0 && hd[i] < d->n_cols, AFEM_ERR_ARG, "imposed DoF id out of range");
    if (hd[i] < d->n) m[hd[i]] = hv[i];
  }
  std::vector<int32_t> ids;
  std::vector<double> vals;
  for (const auto& kv : m) {
    ids.push_back(kv.first);
    vals.push_back(kv.second);
  }
  d->imp_ids.alloc(ids.size());
  d->imp_vals.alloc(vals.size());
  if (!ids.empty()) {
    AFEM_HIP(hipMemcpyAsync(d->imp_ids.p, ids.data(), ids.size() * 4, hipMemcpyHostToDevice, ctx.stream));
    AFEM_HIP(hipMemcpyAsync(d->imp_vals.p, vals.data(), vals.size() * 8, hipMemcpyHostToDevice, ctx.stream));
  }
  ctx.sync();
}

void dyn_set_time_step(Elastodynamics* d, double dt)
{
  AFEM_REQUIRE(dt > 0, AFEM_ERR_ARG, "afem_elastodynamics_set_time_step: dt must be > 0");
  if (dt == d->p.dt) return;
  d->p.dt = dt;
  dyn_coefficients(d);
  // the operator c0 M + K(c1, c2) depends on dt: a reused multigrid hierarchy
  // is rebuilt at the next solve
  d->ls.mg.reset();
  d->ls.amg.reset();
}

void dyn_profile(Elastodynamics* d, bool on)
{
  d->ctx->set_device();
  if (on && !d->ev[0])
    for (auto& e : d->ev) AFEM_HIP(hipEventCreate(&e));
  d->profile = on;
  afem_step_timing& t = d->timing;
  t.nnz_blocks = d->K.s.nnz;
  t.n_incidences = d->K.s.n_incidences;
  t.n_nodes = d->mesh->n_nodes;
  t.n_own_nodes = d->mesh->n_own;
}

void dyn_destroy(Elastodynamics* d)
{
  if (!d) return;
  d->ctx->set_device();
  (void)hipStreamSynchronize(d->ctx->stream);
  for (auto& e : d->ev)
    if (e) (void)hipEventDestroy(e);
  if (d->ls.pinned) (void)hipHostFree(d->ls.pinned);
  for (LinearSystem* l : { &d->lsm, &d->lsl, &d->lsu })
    if (l->pinned) (void)hipHostFree(l->pinned);
  delete d;
}

}  // namespace afem
