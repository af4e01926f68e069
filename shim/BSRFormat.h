// -*- C++ -*-
/*
 * Arcane-side BSRFormat<NB_DOF> backed by libafem (include/arcanefem_amd.h +
 * include/arcanefem_amd_generic.hpp): a drop-in for femutils/BSRFormat.h
 * with the methods the modules call --
 *
 *   BSRFormat(ITraceMng*, RunQueue&, const FemDoFsOnNodes&)   femutils/BSRFormat.h:356-362
 *   initialize(IMesh*, bool use_csr, bool atomic_free)        :389-409
 *   computeSparsity()                                         :775-781
 *   assembleBilinear(compute_element_matrix)                  :1105-1111
 *   toLinearSystem(DoFLinearSystem&)                          :414-430
 *   resetMatrixValues()                                       :1120-1123
 *
 * so modules/poisson/FemModule.cc:33-36, 76-77, 106-107, 261-272 and
 * modules/elasticity/FemModule.cc (BSRFormat<2>) compile unchanged when this
 * directory precedes femutils/ on the include path (shim/CMakeLists.txt,
 * AFEM_BSR_SHIM).  The module's element lambda
 *   [=] ARCCORE_HOST_DEVICE (CellLocalId c) { return _computeElementMatrixTetra4Gpu(c, cn_cv, in_node_coord); }
 * runs inside libafem's generic cell kernel (one lane per cell, binary search
 * of the sorted row, f64 atomics: the reference's assembleBilinearAtomic
 * semantics); it still reads the geometry through the Arcane views it
 * captured.  The module's own BC kernels then write the linear system's
 * variables, as with the reference.
 *
 * Numbering.  libafem numbers the owned nodes first, then the ghosts; cells
 * keep Arcane's local ids (so CellLocalId(c) in the lambda is the cell the
 * kernel scatters) and their nodes are renumbered.  With one subdomain and an
 * identity numbering (own nodes are lids 0..n_own-1) the CSR handed to the
 * linear system aliases libafem's device values (NB_DOF = 1, per-row layout:
 * no copy per assembly; rows / columns converted to the reference's int32
 * layout once per structure).  Otherwise toLinearSystem goes through
 * matrixAddValue per entry, as BSRMatrix::toLinearSystem does (:261-280).
 *
 * Status: written against the reference's interfaces; Arcane is not
 * installed here, so it is compiled against the single-subdomain Arcane mock
 * of tests/arcane_mock/ (test infrastructure) and run on the GPU by
 * tests/test_gpu_shim.py: initialize / computeSparsity / assembleBilinear(a
 * device element lambda) / toLinearSystem / solve on the reference's
 * sphere_3D case, equal to the oracle and the golden.
 */
#ifndef AFEM_SHIM_BSRFORMAT_H
#define AFEM_SHIM_BSRFORMAT_H

#include <arcane/accelerator/core/RunQueue.h>
#include <arcane/accelerator/NumArrayViews.h>
#include <arcane/core/IMesh.h>
#include <arcane/core/IParallelMng.h>
#include <arcane/core/ItemGroup.h>
#include <arcane/core/VariableTypes.h>
#include <arcane/utils/FatalErrorException.h>
#include <arcane/utils/NotImplementedException.h>
#include <arcane/utils/NumArray.h>
#include <arcane/utils/TraceAccessor.h>

#include <vector>

#include "DoFLinearSystem.h"
#include "FemDoFsOnNodes.h"
#include "arcanefem_amd.h"
#include "arcanefem_amd_generic.hpp"

namespace Arcane::FemUtils
{

template <int NB_DOF>
class BSRFormat : public TraceAccessor
{
 public:

  BSRFormat(ITraceMng* tm, RunQueue& queue, const FemDoFsOnNodes& dofs_on_nodes)
  : TraceAccessor(tm)
  , m_queue(queue)
  , m_dofs_on_nodes(dofs_on_nodes)
  {}

  ~BSRFormat()
  {
    if (m_bsr)
      afem_bsr_destroy(m_bsr);
    if (m_afem_mesh)
      afem_mesh_destroy(m_afem_mesh);
    if (m_ctx)
      afem_ctx_destroy(m_ctx);
  }

  void initialize(IMesh* mesh, bool does_linear_system_use_csr, bool use_atomic_free = false)
  {
    ARCANE_CHECK_POINTER(mesh);
    if (mesh->dimension() != 2 && mesh->dimension() != 3)
      ARCANE_THROW(NotImplementedException, "BSRFormat(initialize): Only supports 2D and 3D");
    m_mesh = mesh;
    m_use_csr = does_linear_system_use_csr;
    (void)use_atomic_free;  // libafem's fixed-physics paths are atomic-free; the generic one uses atomics
    int nb_dev = 0;
    _check(afem_device_count(&nb_dev), "afem_device_count");
    if (nb_dev < 1)
      ARCANE_FATAL("libafem: no GPU visible (the MI355X BSRFormat has no CPU path)");
    _check(afem_ctx_create(mesh->parallelMng()->commRank() % nb_dev, nullptr, &m_ctx), "afem_ctx_create");
    _buildMesh();
    _check(afem_bsr_create(m_afem_mesh, NB_DOF, m_use_csr ? 1 : 0, &m_bsr), "afem_bsr_create");
  }

  void computeSparsity()
  {
    _check(afem_bsr_compute_sparsity(m_bsr), "afem_bsr_compute_sparsity");
    m_csr_ready = false;
  }

  template <class Function>
  void assembleBilinear(Function compute_element_matrix)
  {
    m_queue.barrier();  // the module's previous device work (views it captured) is done
    auto f = [=] __device__(int32_t c) { return compute_element_matrix(CellLocalId(c)); };
    const int rc = m_mesh->dimension() == 2 ? afem::generic::assemble_bilinear<3, NB_DOF>(m_bsr, f)
                                            : afem::generic::assemble_bilinear<4, NB_DOF>(m_bsr, f);
    _check(rc, "BSRFormat::assembleBilinear");
  }

  void resetMatrixValues() { _check(afem_bsr_reset_values(m_bsr), "afem_bsr_reset_values"); }

  void toLinearSystem(DoFLinearSystem& linear_system)
  {
    if (m_use_csr && m_identity && NB_DOF == 1) {
      if (!linear_system.hasSetCSRValues())
        ARCANE_THROW(ArgumentException, "BSRFormat(toLinearSystem): Linear system was set to use CSR but is incompatible");
      _exportStructure();
      afem_csr_view v;
      _check(afem_bsr_view(m_bsr, &v), "afem_bsr_view");
      // values alias libafem's device array (per-row layout = CSR order for NB_DOF = 1)
      Span<Real> values(v.values, static_cast<Int64>(v.nnz_blocks));
      CSRFormatView view(m_rows.to1DSpan(), m_rows_nb_column.to1DSpan(), m_columns.to1DSpan(), values);
      linear_system.setCSRValues(view);
      return;
    }
    // BSRMatrix::toLinearSystem (femutils/BSRFormat.h:261-280): per-entry adds
    int64_t n_rows = 0, nnz = 0;
    _check(afem_bsr_get_sizes(m_bsr, &n_rows, &nnz), "afem_bsr_get_sizes");
    std::vector<int32_t> rows(n_rows), rnc(n_rows), cols(nnz);
    std::vector<double> vals(nnz);
    _check(afem_bsr_export_csr32(m_bsr, rows.data(), rnc.data(), cols.data(), vals.data()), "afem_bsr_export_csr32");
    auto node_dof(m_dofs_on_nodes.nodeDoFConnectivityView());
    for (int64_t r = 0; r < n_rows; ++r) {
      const NodeLocalId rn(m_node_of[r / NB_DOF]);
      const DoFLocalId rd = node_dof.dofId(rn, static_cast<Int32>(r % NB_DOF));
      for (int32_t t = rows[r]; t < rows[r] + rnc[r]; ++t) {
        const NodeLocalId cn(m_node_of[cols[t] / NB_DOF]);
        linear_system.matrixAddValue(rd, node_dof.dofId(cn, cols[t] % NB_DOF), vals[t]);
      }
    }
  }

  afem_bsr* handle() const { return m_bsr; }

 private:

  RunQueue& m_queue;
  const FemDoFsOnNodes& m_dofs_on_nodes;
  IMesh* m_mesh = nullptr;
  bool m_use_csr = false;
  bool m_identity = true;
  bool m_csr_ready = false;
  afem_ctx* m_ctx = nullptr;
  afem_mesh* m_afem_mesh = nullptr;
  afem_bsr* m_bsr = nullptr;
  std::vector<Int32> m_node_of; //!< libafem node -> Arcane node local id
  NumArray<Int32, MDDim1> m_rows, m_rows_nb_column, m_columns;

  static void _check(int rc, const char* what)
  {
    if (rc != AFEM_OK)
      ARCANE_FATAL("libafem: {0} failed (code {1}): {2}", what, rc, afem_last_error());
  }

  //! owned nodes first (own() order), then the ghosts; cells in local-id order
  void _buildMesh()
  {
    const Int32 max_lid = m_mesh->nodeFamily()->maxLocalId();
    std::vector<Int32> afem_of(max_lid, -1);
    m_node_of.clear();
    ENUMERATE_NODE (inode, m_mesh->ownNodes()) {
      afem_of[inode.itemLocalId()] = static_cast<Int32>(m_node_of.size());
      m_node_of.push_back(inode.itemLocalId());
    }
    const Int64 n_own = static_cast<Int64>(m_node_of.size());
    ENUMERATE_NODE (inode, m_mesh->allNodes()) {
      if (!(*inode).isOwn()) {
        afem_of[inode.itemLocalId()] = static_cast<Int32>(m_node_of.size());
        m_node_of.push_back(inode.itemLocalId());
      }
    }
    m_identity = true;
    for (size_t a = 0; a < m_node_of.size() && m_identity; ++a)
      m_identity = m_node_of[a] == static_cast<Int32>(a);
    const int nv = m_mesh->dimension() + 1;
    const Int32 max_cell = m_mesh->cellFamily()->maxLocalId();
    std::vector<int32_t> cell_node(static_cast<size_t>(max_cell) * nv, 0);
    ENUMERATE_CELL (icell, m_mesh->allCells()) {
      Cell cell = *icell;
      if (cell.nbNode() != nv)
        ARCANE_THROW(NotImplementedException, "BSRFormat: P1 simplices only (TRIA3 / TETRA4)");
      for (int i = 0; i < nv; ++i)
        cell_node[static_cast<size_t>(icell.itemLocalId()) * nv + i] = afem_of[cell.node(i).localId()];
    }
    VariableNodeReal3& node_coord = m_mesh->nodesCoordinates();
    std::vector<double> coords(3 * m_node_of.size());
    for (size_t a = 0; a < m_node_of.size(); ++a) {
      const Real3 x = node_coord[NodeLocalId(m_node_of[a])];
      coords[3 * a] = x.x;
      coords[3 * a + 1] = x.y;
      coords[3 * a + 2] = x.z;
    }
    _check(afem_mesh_create(m_ctx, m_mesh->dimension(), nv, static_cast<int64_t>(m_node_of.size()), n_own, max_cell,
                            cell_node.data(), coords.data(), AFEM_MEM_HOST, &m_afem_mesh),
           "afem_mesh_create");
  }

  //! rows / rows_nb_column / columns in the reference's int32 layout (once per structure)
  void _exportStructure()
  {
    if (m_csr_ready)
      return;
    int64_t n_rows = 0, nnz = 0;
    _check(afem_bsr_get_sizes(m_bsr, &n_rows, &nnz), "afem_bsr_get_sizes");
    std::vector<int32_t> rows(n_rows), rnc(n_rows), cols(nnz);
    _check(afem_bsr_export_csr32(m_bsr, rows.data(), rnc.data(), cols.data(), nullptr), "afem_bsr_export_csr32");
    m_rows.resize(n_rows);
    m_rows_nb_column.resize(n_rows);
    m_columns.resize(nnz);
    auto mem = m_queue.memoryRessource();
    m_rows = NumArray<Int32, MDDim1>(n_rows, mem);
    m_rows_nb_column = NumArray<Int32, MDDim1>(n_rows, mem);
    m_columns = NumArray<Int32, MDDim1>(nnz, mem);
    m_rows.copy(ConstArrayView<Int32>(static_cast<Int32>(n_rows), rows.data()));
    m_rows_nb_column.copy(ConstArrayView<Int32>(static_cast<Int32>(n_rows), rnc.data()));
    m_columns.copy(ConstArrayView<Int32>(static_cast<Int32>(nnz), cols.data()));
    m_csr_ready = true;
  }
};

} // namespace Arcane::FemUtils

#endif
