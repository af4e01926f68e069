// -*- C++ -*-
/*
 * Arcane-side shim: ArcaneFEM's linear-system plugin surface on top of the
 * MI355X C ABI (include/arcanefem_amd.h, libafem.so).
 *
 *   DoFLinearSystemImpl        femutils/DoFLinearSystem.h:84-110
 *   IDoFLinearSystemFactory    femutils/IDoFLinearSystemFactory.h:34-44
 *   registration               as femutils/HypreDoFLinearSystem.cc:767-800
 *   options                    AfemDoFLinearSystemFactory.axl (as HypreDoFLinearSystemFactory.axl:4-11)
 *
 * Every virtual of DoFLinearSystemImpl is implemented, with the semantics of
 * the backend it replaces:
 *   - setCSRValues / hasSetCSRValues / getCSRValues and matrixAddValue /
 *     matrixSetValue on the view: HypreDoFLinearSystemImpl (:138-156, :199-204);
 *   - matrixAddValue / matrixSetValue without a view, eliminateRow /
 *     eliminateRowColumn: AlephDoFLinearSystemImpl (:192-246, _fillMatrix :501-583)
 *     -- libafem records them and applies them at solve;
 *   - rhsVariable / solutionVariable / getForced{Info,Value} /
 *     getElimination{Info,Value}: Arcane variables named solver_name + suffix
 *     (:106-115); the module's GPU boundary-condition kernels write them, the
 *     shim hands them to libafem at solve();
 *   - solve(): _applyRowElimination + _applyForcedValuesToLhs (:319-382) and
 *     the solve, on the device; the solution is synchronised over the
 *     subdomains (m_dof_variable.synchronize(), as after Hypre's solve);
 *   - clearValues(): :180-187.
 *
 * Numbering.  libafem wants the owned DoFs first ([0, n_own)) and the ghosts
 * after ([n_own, n_all)), which is also the row / column space of a
 * subdomain's CSR (owned rows, ghost columns).  Arcane numbers local DoFs in
 * node order with owned and ghost DoFs interleaved (femutils/FemDoFsOnNodes.cc:
 * 79-109), so the shim keeps the permutation lid -> afem index (owned DoFs in
 * own().index() order, then the ghosts): the global row numbering of the
 * Hypre backend (_computeMatrixNumerotation, :264-303) is the same
 * owned-first order.  When the permutation is the identity (one subdomain)
 * the CSR view is handed over without a copy; otherwise libafem keeps the
 * owned rows of a device view in its order on the device
 * (afem_ls_set_csr_values_mapped: the module's values stay the matrix, read
 * at solve) and a host view is copied permuted once per setCSRValues (ghost
 * rows are empty: the assembly filters isOwn(row), femutils/BSRFormat.h:815,870).
 *
 * Parallel: one process per GPU, one Arcane subdomain per rank.  The halo
 * lists are the DoF family's synchronisation lists built by
 * FemDoFsOnNodes::initialize -> computeSynchronizeInfos (femutils/
 * FemDoFsOnNodes.cc:125-126): per communicating rank, the shared (owned) DoFs
 * to send and the ghost DoFs to receive.  The transport is RCCL (rank 0's
 * ncclUniqueId broadcast with IParallelMng::broadcast) or, with
 * transport="host", IParallelMng itself through afem_comm_create_host.
 *
 * Built only where Arcane exists (shim/CMakeLists.txt, find_package(Arcane)).
 */

#include <arcane/core/IItemFamily.h>
#include <arcane/core/IParallelMng.h>
#include <arcane/core/IVariableSynchronizer.h>
#include <arcane/core/ItemGroup.h>
#include <arcane/core/ItemPrinter.h>
#include <arcane/core/VariableTypes.h>
#include <arcane/utils/FatalErrorException.h>
#include <arcane/utils/NotImplementedException.h>
#include <arcane/utils/PlatformUtils.h>
#include <arcane/accelerator/core/Runner.h>

#include <cstring>
#include <vector>

#include "DoFLinearSystem.h"
#include "IDoFLinearSystemFactory.h"
#include "arcanefem_amd.h"

#include "AfemDoFLinearSystemFactory_axl.h"

namespace Arcane::FemUtils
{

namespace
{
  //! ABI status -> exception, as hypreCheck does for Hypre (femutils/HypreDoFLinearSystem.cc:67-92).
  void afemCheck(int rc, const char* what)
  {
    if (rc != AFEM_OK)
      ARCANE_FATAL("libafem: {0} failed (code {1}): {2}", what, rc, afem_last_error());
  }

  //! IParallelMng as the host transport of afem_comm_create_host.
  struct ParallelMngTransport
  {
    IParallelMng* pm = nullptr;

    static int allreduce(void* user, double* buf, int64_t n)
    {
      auto* self = static_cast<ParallelMngTransport*>(user);
      try {
        self->pm->reduce(Parallel::ReduceSum, ArrayView<Real>(static_cast<Int32>(n), buf));
        return 0;
      }
      catch (...) {
        return 1;
      }
    }

    static int exchange(void* user, int n_nbr, const int32_t* nbr, const double* send, const int64_t* send_counts,
                        double* recv, const int64_t* recv_counts)
    {
      auto* self = static_cast<ParallelMngTransport*>(user);
      try {
        UniqueArray<Parallel::Request> requests;
        int64_t so = 0, ro = 0;
        for (int i = 0; i < n_nbr; ++i) {
          if (send_counts[i] > 0)
            requests.add(self->pm->send(ConstArrayView<Real>(static_cast<Int32>(send_counts[i]), send + so), nbr[i],
                                        false));
          if (recv_counts[i] > 0)
            requests.add(self->pm->recv(ArrayView<Real>(static_cast<Int32>(recv_counts[i]), recv + ro), nbr[i], false));
          so += send_counts[i];
          ro += recv_counts[i];
        }
        self->pm->waitAllRequests(requests);
        return 0;
      }
      catch (...) {
        return 1;
      }
    }
  };
} // namespace

/*---------------------------------------------------------------------------*/

class AfemDoFLinearSystemImpl
: public TraceAccessor
, public DoFLinearSystemImpl
{
 public:

  static constexpr Byte ELIMINATE_NONE = 0;

  AfemDoFLinearSystemImpl(IItemFamily* dof_family, const String& solver_name)
  : TraceAccessor(dof_family->traceMng())
  , m_dof_family(dof_family)
  , m_rhs_variable(VariableBuildInfo(dof_family, solver_name + "RHSVariable"))
  , m_dof_variable(VariableBuildInfo(dof_family, solver_name + "SolutionVariable"))
  , m_dof_forced_info(VariableBuildInfo(dof_family, solver_name + "DoFForcedInfo"))
  , m_dof_forced_value(VariableBuildInfo(dof_family, solver_name + "DoFForcedValue"))
  , m_dof_elimination_info(VariableBuildInfo(dof_family, solver_name + "DoFEliminationInfo"))
  , m_dof_elimination_value(VariableBuildInfo(dof_family, solver_name + "DoFEliminationValue"))
  {
    info() << "Creating AfemDoFLinearSystemImpl()";
  }

  ~AfemDoFLinearSystemImpl() override
  {
    if (m_ls)
      afem_ls_destroy(m_ls);
    if (m_comm)
      afem_comm_destroy(m_comm);
    if (m_ctx)
      afem_ctx_destroy(m_ctx);
  }

  void build(Int32 device, const String& transport)
  {
    IParallelMng* pm = m_dof_family->parallelMng();
    int nb_dev = 0;
    afemCheck(afem_device_count(&nb_dev), "afem_device_count");
    if (nb_dev < 1)
      ARCANE_FATAL("libafem: no GPU visible (the MI355X linear system has no CPU path)");
    if (device < 0)
      device = pm->commRank() % nb_dev;
    afemCheck(afem_ctx_create(device, nullptr, &m_ctx), "afem_ctx_create");
    _computeNumbering();
    afemCheck(afem_ls_create(m_ctx, m_nb_own, m_nb_all, &m_ls), "afem_ls_create");
    m_dof_forced_info.fill(false);
    m_dof_elimination_info.fill(ELIMINATE_NONE);
    m_dof_elimination_value.fill(0.0);
    if (pm->isParallel())
      _buildHalo(pm, transport);
  }

  void setSolverOptions(const afem_solver_opts& o) { afemCheck(afem_ls_set_solver_options(m_ls, &o), "solver options"); }

 public:

  // ------------------------------------------------ matrix entries
  void matrixAddValue(DoFLocalId row, DoFLocalId column, Real value) override
  {
    afemCheck(afem_ls_matrix_add_value(m_ls, m_index[row], m_index[column], value), "matrixAddValue");
  }

  void matrixSetValue(DoFLocalId row, DoFLocalId column, Real value) override
  {
    afemCheck(afem_ls_matrix_set_value(m_ls, m_index[row], m_index[column], value), "matrixSetValue");
  }

  void eliminateRow(DoFLocalId row, Real value) override
  {
    afemCheck(afem_ls_eliminate_row(m_ls, m_index[row], value), "eliminateRow");
  }

  void eliminateRowColumn(DoFLocalId row, Real value) override
  {
    afemCheck(afem_ls_eliminate_row_column(m_ls, m_index[row], value), "eliminateRowColumn");
  }

  // ------------------------------------------------ CSR view (Hypre semantics)
  void setCSRValues(const CSRFormatView& csr_view) override
  {
    m_csr_view = csr_view; // non-owning, valid until solve (femutils/DoFLinearSystem.h:251-258)
    CSRFormatView v = csr_view;
    const int mem = _isDeviceMemory() ? AFEM_MEM_DEVICE : AFEM_MEM_HOST;
    if (m_identity) {
      afemCheck(afem_ls_set_csr_values(m_ls, v.rows().data(), v.rowsNbColumn().data(), v.columns().data(),
                                       v.values().data(), m_nb_own, v.nbValue(), mem),
                "setCSRValues");
      return;
    }
    const Int32 nb_row = v.nbRow(), nnz = v.nbValue();
    if (mem == AFEM_MEM_DEVICE) {
      // device view (BSRFormat::toLinearSystem): libafem renumbers it on the
      // device, the module's values stay the matrix until solve()
      afemCheck(afem_ls_set_csr_values_mapped(m_ls, v.rows().data(), v.rowsNbColumn().data(), v.columns().data(),
                                              v.values().data(), nb_row, nnz, m_index.data(), m_index.size()),
                "setCSRValues");
      return;
    }
    // host view: owned rows in afem order, columns renumbered; a host copy
    // (once per view), kept in members: libafem reads a host view at solve()
    std::vector<Int32> rows(nb_row), cols(nnz);
    std::vector<Real> vals(nnz);
    afemCheck(afem_memcpy(m_ctx, rows.data(), v.rows().data(), sizeof(Int32) * nb_row, AFEM_MEM_HOST, mem), "copy");
    afemCheck(afem_memcpy(m_ctx, cols.data(), v.columns().data(), sizeof(Int32) * nnz, AFEM_MEM_HOST, mem), "copy");
    afemCheck(afem_memcpy(m_ctx, vals.data(), v.values().data(), sizeof(Real) * nnz, AFEM_MEM_HOST, mem), "copy");
    m_prow.assign(m_nb_own, 0);
    m_pcol.clear();
    m_pval.clear();
    m_pcol.reserve(nnz);
    m_pval.reserve(nnz);
    for (Int32 a = 0; a < m_nb_own; ++a) {
      const Int32 lid = m_lid_of[a];
      const Int32 b = rows[lid], e = lid == nb_row - 1 ? nnz : rows[lid + 1]; // end as HypreDoFLinearSystem.cc:140-141
      m_prow[a] = static_cast<Int32>(m_pcol.size());
      for (Int32 k = b; k < e; ++k) {
        m_pcol.push_back(m_index[cols[k]]);
        m_pval.push_back(vals[k]);
      }
    }
    afemCheck(afem_ls_set_csr_values(m_ls, m_prow.data(), nullptr, m_pcol.data(), m_pval.data(), m_nb_own,
                                     static_cast<Int32>(m_pcol.size()), AFEM_MEM_HOST),
              "setCSRValues");
  }

  CSRFormatView& getCSRValues() override { return m_csr_view; }
  bool hasSetCSRValues() const override { return true; }

  // ------------------------------------------------ variables
  VariableDoFReal& solutionVariable() override { return m_dof_variable; }
  VariableDoFReal& rhsVariable() override { return m_rhs_variable; }
  VariableDoFBool& getForcedInfo() override { return m_dof_forced_info; }
  VariableDoFReal& getForcedValue() override { return m_dof_forced_value; }
  VariableDoFByte& getEliminationInfo() override { return m_dof_elimination_info; }
  VariableDoFReal& getEliminationValue() override { return m_dof_elimination_value; }

  void setSolverCommandLineArguments(const CommandLineArguments&) override {}
  void setRunner(Runner* r) override { m_runner = r; }
  Runner* runner() const override { return m_runner; }

  void clearValues() override
  {
    info() << "[Afem-Info]: Clear values";
    m_csr_view = {};
    m_dof_forced_info.fill(false);
    m_dof_elimination_info.fill(ELIMINATE_NONE);
    m_dof_elimination_value.fill(0);
    afemCheck(afem_ls_clear_values(m_ls), "clearValues");
  }

  // ------------------------------------------------ solve
  void solve() override
  {
    Real t0 = platform::getRealTime();
    // the module wrote rhs / forced / elimination into the Arcane variables
    // (GPU BC kernels, femutils/ArcaneFemFunctionsGpu.h:434-482): hand the
    // owned part to libafem in its order
    std::vector<Real> rhs(m_nb_own), fval(m_nb_own), eval(m_nb_own);
    std::vector<uint8_t> finfo(m_nb_own), einfo(m_nb_own);
    for (Int32 a = 0; a < m_nb_own; ++a) {
      DoFLocalId lid(m_lid_of[a]);
      rhs[a] = m_rhs_variable[lid];
      finfo[a] = m_dof_forced_info[lid] ? 1 : 0;
      fval[a] = m_dof_forced_value[lid];
      einfo[a] = m_dof_elimination_info[lid];
      eval[a] = m_dof_elimination_value[lid];
    }
    double *d_rhs = nullptr, *d_fval = nullptr, *d_eval = nullptr, *d_sol = nullptr;
    uint8_t *d_finfo = nullptr, *d_einfo = nullptr;
    afemCheck(afem_ls_rhs(m_ls, &d_rhs), "rhs");
    afemCheck(afem_ls_forced_value(m_ls, &d_fval), "forced value");
    afemCheck(afem_ls_forced_info(m_ls, &d_finfo), "forced info");
    afemCheck(afem_ls_elimination_value(m_ls, &d_eval), "elimination value");
    afemCheck(afem_ls_elimination_info(m_ls, &d_einfo), "elimination info");
    const size_t n8 = sizeof(Real) * m_nb_own;
    afemCheck(afem_memcpy(m_ctx, d_rhs, rhs.data(), n8, AFEM_MEM_DEVICE, AFEM_MEM_HOST), "rhs upload");
    afemCheck(afem_memcpy(m_ctx, d_fval, fval.data(), n8, AFEM_MEM_DEVICE, AFEM_MEM_HOST), "forced upload");
    afemCheck(afem_memcpy(m_ctx, d_finfo, finfo.data(), m_nb_own, AFEM_MEM_DEVICE, AFEM_MEM_HOST), "forced upload");
    afemCheck(afem_memcpy(m_ctx, d_eval, eval.data(), n8, AFEM_MEM_DEVICE, AFEM_MEM_HOST), "elim upload");
    afemCheck(afem_memcpy(m_ctx, d_einfo, einfo.data(), m_nb_own, AFEM_MEM_DEVICE, AFEM_MEM_HOST), "elim upload");

    afem_solve_stats st{};
    afemCheck(afem_ls_solve(m_ls, &st), "solve");
    info() << "[Afem-Info] solve: iterations=" << st.iterations << " converged=" << st.converged
           << " rel_residual=" << st.rel_residual << " |r|=" << st.residual_norm << " device_ms=" << st.solve_ms;

    afemCheck(afem_ls_solution(m_ls, &d_sol), "solution");
    std::vector<Real> x(m_nb_own);
    afemCheck(afem_memcpy(m_ctx, x.data(), d_sol, n8, AFEM_MEM_HOST, AFEM_MEM_DEVICE), "solution download");
    for (Int32 a = 0; a < m_nb_own; ++a)
      m_dof_variable[DoFLocalId(m_lid_of[a])] = x[a];
    m_dof_variable.synchronize();
    info() << "[ArcaneFem-Timer] afem-solve = " << (platform::getRealTime() - t0);
  }

  afem_ls* handle() const { return m_ls; }

 private:

  IItemFamily* m_dof_family = nullptr;
  VariableDoFReal m_rhs_variable;
  VariableDoFReal m_dof_variable;
  VariableDoFBool m_dof_forced_info;
  VariableDoFReal m_dof_forced_value;
  VariableDoFByte m_dof_elimination_info;
  VariableDoFReal m_dof_elimination_value;
  CSRFormatView m_csr_view;
  Runner* m_runner = nullptr;

  afem_ctx* m_ctx = nullptr;
  afem_ls* m_ls = nullptr;
  afem_comm* m_comm = nullptr;
  ParallelMngTransport m_transport;

  Int32 m_nb_own = 0, m_nb_all = 0;
  bool m_identity = true;
  UniqueArray<Int32> m_index;  //!< DoF local id -> afem index (owned first)
  UniqueArray<Int32> m_lid_of; //!< afem index -> DoF local id
  //! the permuted copy of a view (several subdomains): libafem reads it at solve()
  std::vector<Int32> m_prow, m_pcol;
  std::vector<Real> m_pval;

 private:

  bool _isDeviceMemory() const
  {
    // the BSRFormat CSR arrays live in the queue's memory resource: device
    // memory with the accelerator runtime, host memory otherwise
    return m_runner && Accelerator::isAcceleratorPolicy(m_runner->executionPolicy());
  }

  void _computeNumbering()
  {
    DoFGroup all_dofs = m_dof_family->allItems();
    m_nb_all = all_dofs.size();
    m_index.resize(m_dof_family->maxLocalId());
    m_index.fill(-1);
    m_lid_of.resize(m_nb_all);
    Int32 next = 0;
    ENUMERATE_DOF (idof, all_dofs.own()) {
      m_index[idof.itemLocalId()] = next;
      m_lid_of[next++] = idof.itemLocalId();
    }
    m_nb_own = next;
    ENUMERATE_DOF (idof, all_dofs) {
      if (!(*idof).isOwn()) {
        m_index[idof.itemLocalId()] = next;
        m_lid_of[next++] = idof.itemLocalId();
      }
    }
    m_identity = true;
    for (Int32 a = 0; a < m_nb_all && m_identity; ++a)
      m_identity = m_lid_of[a] == a;
    info() << "[Afem-Info] DoFs own=" << m_nb_own << " all=" << m_nb_all << " identity numbering=" << m_identity;
  }

  void _buildHalo(IParallelMng* pm, const String& transport)
  {
    const Int32 nranks = pm->commSize(), rank = pm->commRank();
    if (transport == "host") {
      m_transport.pm = pm;
      afem_host_transport t{ &m_transport, &ParallelMngTransport::allreduce, &ParallelMngTransport::exchange };
      afemCheck(afem_comm_create_host(m_ctx, nranks, rank, &t, &m_comm), "afem_comm_create_host");
    }
    else {
      UniqueArray<Byte> id(AFEM_UNIQUE_ID_BYTES, 0);
      if (rank == 0)
        afemCheck(afem_comm_unique_id(reinterpret_cast<uint8_t*>(id.data())), "afem_comm_unique_id");
      pm->broadcast(id.view(), 0);
      afemCheck(afem_comm_create(m_ctx, reinterpret_cast<const uint8_t*>(id.data()), nranks, rank, &m_comm),
                "afem_comm_create");
    }
    // FemDoFsOnNodes::initialize -> computeSynchronizeInfos (femutils/FemDoFsOnNodes.cc:125-126)
    IVariableSynchronizer* sync = m_dof_family->allItemsSynchronizer();
    Int32ConstArrayView ranks = sync->communicatingRanks();
    std::vector<int32_t> nbr, send_ids, recv_ids;
    std::vector<int64_t> send_counts, recv_counts;
    for (Integer i = 0; i < ranks.size(); ++i) {
      Int32ConstArrayView shared = sync->sharedItems(i);
      Int32ConstArrayView ghosts = sync->ghostItems(i);
      nbr.push_back(ranks[i]);
      send_counts.push_back(shared.size());
      recv_counts.push_back(ghosts.size());
      for (Int32 lid : shared)
        send_ids.push_back(m_index[lid]);
      for (Int32 lid : ghosts)
        recv_ids.push_back(m_index[lid]);
    }
    afemCheck(afem_ls_set_halo(m_ls, m_comm, static_cast<int>(nbr.size()), nbr.data(), send_counts.data(),
                               send_ids.data(), recv_counts.data(), recv_ids.data()),
              "afem_ls_set_halo");
  }
};

/*---------------------------------------------------------------------------*/

class AfemDoFLinearSystemFactoryService
: public ArcaneAfemDoFLinearSystemFactoryObject
{
 public:

  explicit AfemDoFLinearSystemFactoryService(const ServiceBuildInfo& sbi)
  : ArcaneAfemDoFLinearSystemFactoryObject(sbi)
  {
    info() << "Create AfemDoF (MI355X linear system)";
  }

  DoFLinearSystemImpl*
  createInstance(ISubDomain* sd, IItemFamily* dof_family, const String& solver_name) override
  {
    auto* x = new AfemDoFLinearSystemImpl(dof_family, solver_name);
    x->build(options()->device(), options()->transport());
    afem_solver_opts o{};
    const String s = options()->solver();
    o.method = s == "pcg" ? AFEM_SOLVER_PCG : (s == "direct" ? AFEM_SOLVER_DIRECT : AFEM_SOLVER_AUTO);
    o.max_iter = options()->maxIter();
    o.rtol = options()->rtol();
    o.atol = options()->atol();
    o.check_every = options()->checkEvery();
    o.fixed_iterations = 0;
    const String pc = options()->preconditioner();
    o.precond_block = pc == "block3" ? 3 : 0;
    o.multigrid = pc == "multigrid" ? 1 : (pc == "multigrid-reuse" ? 2 : 0);
    x->setSolverOptions(o);
    return x;
  }
};

/*---------------------------------------------------------------------------*/

ARCANE_REGISTER_SERVICE_AFEMDOFLINEARSYSTEMFACTORY(AfemLinearSystem, AfemDoFLinearSystemFactoryService);
#if defined(AFEM_REGISTER_AS_HYPRE)
// The poisson / elasticity modules take their GPU BSR + device-BC branch only
// for serviceName() == "HypreLinearSystem" (modules/poisson/FemModule.cc:34,109,
// modules/elasticity/FemModule.cc:79,275): with FemUtils built without Hypre,
// the MI355X service answers to that name too, and the modules run unchanged.
ARCANE_REGISTER_SERVICE_AFEMDOFLINEARSYSTEMFACTORY(HypreLinearSystem, AfemDoFLinearSystemFactoryService);
#endif

} // namespace Arcane::FemUtils
