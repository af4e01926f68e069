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
 * runs inside libafem's cell-unit kernel (afem::generic::assemble_bilinear:
 * one wavefront per unit of rows, the element blocks added in LDS, every
 * value written once -- no global atomics, no column search; it still reads
 * the geometry through the Arcane views it captured).  Like the reference it
 * accumulates into the values; right after computeSparsity /
 * resetMatrixValues (values known to be zero) it writes them instead (same
 * result, no read of the old values).  The module's own BC kernels then
 * write the linear system's variables, as with the reference.
 *
 * Numbering.  libafem numbers the owned nodes first, then the ghosts, and
 * gets the mesh's cells in enumeration order (local ids may have holes): the
 * lambda is called with the Arcane CellLocalId of the cell the kernel
 * scatters (a device map), never with a hole.  toLinearSystem with
 * use_csr hands the linear system a DEVICE CSR view in the module's DoF
 * numbering (BSRMatrix::toCsr, femutils/BSRFormat.h:194-256: rows = DoF local
 * ids, columns = node DoF ids in block order) for every NB_DOF and any
 * numbering: libafem builds that CSR once from the DoF ids of
 * FemDoFsOnNodes and gathers the values into it at each hand-over (one
 * kernel; with the identity numbering and NB_DOF = 1 the values are the
 * matrix's own array, no copy).  Without use_csr, toLinearSystem goes
 * through matrixAddValue per entry, as BSRMatrix::toLinearSystem does
 * (:261-280).
 *
 * Status: written against the reference's interfaces; Arcane is not
 * installed here, so it is compiled against the Arcane mock of
 * tests/arcane_mock/ (test infrastructure) and run on the GPU by
 * tests/test_gpu_shim.py: BSRFormat<1> (Poisson) and BSRFormat<3>
 * (elasticity) on 1-3 subdomains with Arcane-style interleaved local ids,
 * against the oracle and the golden.
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
    if (m_d_cell_lid)
      afem_free(m_ctx, m_d_cell_lid);
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
    m_map_ready = false;
    m_values_zero = true;
  }

  template <class Function>
  void assembleBilinear(Function compute_element_matrix)
  {
    m_queue.barrier();  // the module's previous device work (views it captured) is done
    const int32_t* cell_lid = m_d_cell_lid;
    auto f = [=] __device__(int32_t c) { return compute_element_matrix(CellLocalId(cell_lid[c])); };
    const auto mode = m_values_zero ? afem::generic::Mode::Overwrite : afem::generic::Mode::Accumulate;
    const int rc = m_mesh->dimension() == 2 ? afem::generic::assemble_bilinear<3, NB_DOF>(m_bsr, f, mode)
                                            : afem::generic::assemble_bilinear<4, NB_DOF>(m_bsr, f, mode);
    _check(rc, "BSRFormat::assembleBilinear");
    m_values_zero = false;
  }

  void resetMatrixValues()
  {
    _check(afem_bsr_reset_values(m_bsr), "afem_bsr_reset_values");
    m_values_zero = true;
  }

  void toLinearSystem(DoFLinearSystem& linear_system)
  {
    if (m_use_csr) {
      if (!linear_system.hasSetCSRValues())
        ARCANE_THROW(ArgumentException, "BSRFormat(toLinearSystem): Linear system was set to use CSR but is incompatible");
      // BSRMatrix::toCsr in the module's DoF numbering, on the device
      afem_csr32_view v;
      if (!m_map_ready) {
        auto node_dof(m_dofs_on_nodes.nodeDoFConnectivityView());
        std::vector<int32_t> dof_of(m_node_of.size() * NB_DOF);
        Int32 n_dof_rows = 0;
        for (size_t a = 0; a < m_node_of.size(); ++a)
          for (Int32 i = 0; i < NB_DOF; ++i) {
            const Int32 d = node_dof.dofId(NodeLocalId(m_node_of[a]), i).localId();
            dof_of[a * NB_DOF + i] = d;
            n_dof_rows = d + 1 > n_dof_rows ? d + 1 : n_dof_rows;
          }
        _check(afem_bsr_to_csr32_mapped(m_bsr, dof_of.data(), n_dof_rows, &v), "BSRFormat::toLinearSystem");
        m_map_ready = true;
      }
      else
        _check(afem_bsr_to_csr32_mapped(m_bsr, nullptr, 0, &v), "BSRFormat::toLinearSystem");
      CSRFormatView view(Span<const Int32>(v.rows, v.n_rows), Span<const Int32>(v.rows_nb_column, v.n_rows),
                         Span<const Int32>(v.columns, v.nnz), Span<Real>(v.values, v.nnz));
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
  bool m_map_ready = false;   //!< libafem holds the DoF map of toLinearSystem
  bool m_values_zero = true;  //!< values known to be zero (computeSparsity / resetMatrixValues)
  afem_ctx* m_ctx = nullptr;
  afem_mesh* m_afem_mesh = nullptr;
  afem_bsr* m_bsr = nullptr;
  std::vector<Int32> m_node_of; //!< libafem node -> Arcane node local id
  int32_t* m_d_cell_lid = nullptr; //!< device: libafem cell -> Arcane cell local id

  static void _check(int rc, const char* what)
  {
    if (rc != AFEM_OK)
      ARCANE_FATAL("libafem: {0} failed (code {1}): {2}", what, rc, afem_last_error());
  }

  //! owned nodes first (own() order), then the ghosts; the cells in enumeration order
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
    // the mesh's cells only (local ids may have holes): libafem cell c is
    // Arcane cell m_cell_lid[c], which the element lambda is called with
    const int nv = m_mesh->dimension() + 1;
    std::vector<int32_t> cell_node, cell_lid;
    ENUMERATE_CELL (icell, m_mesh->allCells()) {
      Cell cell = *icell;
      if (cell.nbNode() != nv)
        ARCANE_THROW(NotImplementedException, "BSRFormat: P1 simplices only (TRIA3 / TETRA4)");
      cell_lid.push_back(icell.itemLocalId());
      for (int i = 0; i < nv; ++i)
        cell_node.push_back(afem_of[cell.node(i).localId()]);
    }
    const Int64 n_cells = static_cast<Int64>(cell_lid.size());
    if (m_d_cell_lid)
      _check(afem_free(m_ctx, m_d_cell_lid), "afem_free");
    m_d_cell_lid = nullptr;
    void* p = nullptr;
    _check(afem_malloc(m_ctx, sizeof(int32_t) * (n_cells > 0 ? n_cells : 1), &p), "afem_malloc");
    m_d_cell_lid = static_cast<int32_t*>(p);
    if (n_cells > 0)
      _check(afem_memcpy(m_ctx, m_d_cell_lid, cell_lid.data(), sizeof(int32_t) * n_cells, AFEM_MEM_DEVICE, AFEM_MEM_HOST),
             "afem_memcpy");
    VariableNodeReal3& node_coord = m_mesh->nodesCoordinates();
    std::vector<double> coords(3 * m_node_of.size());
    for (size_t a = 0; a < m_node_of.size(); ++a) {
      const Real3 x = node_coord[NodeLocalId(m_node_of[a])];
      coords[3 * a] = x.x;
      coords[3 * a + 1] = x.y;
      coords[3 * a + 2] = x.z;
    }
    _check(afem_mesh_create(m_ctx, m_mesh->dimension(), nv, static_cast<int64_t>(m_node_of.size()), n_own, n_cells,
                            cell_node.data(), coords.data(), AFEM_MEM_HOST, &m_afem_mesh),
           "afem_mesh_create");
  }
};

} // namespace Arcane::FemUtils

#endif
