/*
 * arcanefem_amd_generic.hpp -- generic element-functor assembly on libafem's
 * structure (HIP C++, header-only; compile the caller with hipcc
 * --offload-arch=gfx950).
 *
 * The reference's BSRFormat<NB_DOF>::assembleBilinear(compute_element_matrix)
 * (femutils/BSRFormat.h:786-837, 1105-1111) takes the module's element
 * functor -- e.g. modules/poisson/FemModule.cc:269-271:
 *     [=] ARCCORE_HOST_DEVICE (CellLocalId c) { return _computeElementMatrixTetra4Gpu(c, cn_cv, in_node_coord); }
 * -- and scatters the returned (NV*NB_DOF)^2 FixedMatrix into the BSR values
 * cell by cell (owned rows only, column found by a search of the row,
 * doAtomic<Add>).  afem::generic::assemble_bilinear<NV, NB_DOF>(bsr, f) is
 * that entry for ANY device functor f(int32_t cell) whose result has
 * operator()(int, int): one lane per cell evaluates f, finds each column by a
 * binary search of the sorted row (libafem's rows are sorted) and adds the
 * k x k block with f64 atomics into either value layout (ordered per block or
 * per row, the K9 indexing fixed for k >= 3).  Like the reference it
 * ACCUMULATES into the current values (afem_bsr_reset_values zeroes them) and
 * its summation order is not fixed.
 *
 * The fixed-physics entries (afem_bsr_assemble_poisson_p1 / _elasticity_p1)
 * stay the fast instances: atomic-free row-gather strip kernels whose element
 * arithmetic is compiled in.  This path is for element functors the library
 * does not know (other physics, the Arcane-side BSRFormat shim,
 * shim/AfemBSRFormat.h).
 *
 * The functor sees the cell id; for geometry it captures the device arrays of
 * afem_bsr_assembly_view (cell_node, coords: the mesh's own numbering) or its
 * own (an Arcane shim captures Arcane's views: cell ids are the caller's).
 */
#ifndef ARCANEFEM_AMD_GENERIC_HPP
#define ARCANEFEM_AMD_GENERIC_HPP

#include <hip/hip_runtime.h>

#include "arcanefem_amd.h"

namespace afem {
namespace generic {

/* FixedMatrix<N, M> of femutils/FemUtils.h:53-186 (row-major, host+device): a
 * result type a functor may return; any type with operator()(int, int) works. */
template <int N, int M>
struct FixedMatrix {
  double v[N * M];
  __host__ __device__ double& operator()(int i, int j) { return v[i * M + j]; }
  __host__ __device__ double operator()(int i, int j) const { return v[i * M + j]; }
};

/* The structure a generic kernel scatters into (device pointers). */
struct CellAccess {
  const int32_t* cell_node;
  const double* coords;
  __device__ int32_t node(int32_t cell, int i, int nv) const { return cell_node[(int64_t)cell * nv + i]; }
  __device__ double x(int32_t node, int c) const { return coords[3 * (int64_t)node + c]; }
};

template <int NV, int K, class F>
__global__ void __launch_bounds__(256) k_assemble_cells(afem_assembly_view v, F f)
{
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= v.n_cells) return;
  const auto ke = f((int32_t)c);
  int32_t nodes[NV];
#pragma unroll
  for (int a = 0; a < NV; ++a) nodes[a] = v.cell_node[c * NV + a];
#pragma unroll
  for (int a = 0; a < NV; ++a) {
    const int32_t r = nodes[a];
    if (r < 0 || r >= v.n_rows) continue;  // isOwn(row): owned rows only
    const int64_t rb = v.rows[r], re = v.rows[r + 1];
#pragma unroll
    for (int b = 0; b < NV; ++b) {
      const int32_t col = nodes[b];
      int64_t lo = rb, hi = re;  // sorted row: lower bound of col
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (v.columns[mid] < col)
          lo = mid + 1;
        else
          hi = mid;
      }
      if (lo >= re || v.columns[lo] != col) {  // not in the structure (BSRMatrix::findValueIndex throws)
        atomicOr(v.error_flag, 1);
        continue;
      }
#pragma unroll
      for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const int64_t idx = v.ordered_per_block ? lo * (K * K) + i * K + j
                                                  : rb * (K * K) + (int64_t)i * K * (re - rb) + K * (lo - rb) + j;
          atomicAdd(v.values + idx, (double)ke(K * a + i, K * b + j));
        }
    }
  }
}

/* BSRFormat<K>::assembleBilinear(f) for cells of NV nodes: returns AFEM_OK or
 * an AFEM_ERR_* code (afem_last_error() tells why for library errors;
 * AFEM_ERR_NOT_FOUND when an element coupled nodes outside the sparsity).
 * Enqueued on the structure's context stream; checks the error flag (one
 * synchronisation) unless check == false. */
template <int NV, int K, class F>
int assemble_bilinear(afem_bsr* bsr, F f, bool check = true)
{
  afem_assembly_view v;
  int rc = afem_bsr_assembly_view(bsr, &v);
  if (rc != AFEM_OK) return rc;
  if (v.nb_node_per_cell != NV || v.block_size != K) return AFEM_ERR_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(v.stream);
  if (hipMemsetAsync(v.error_flag, 0, sizeof(int32_t), st) != hipSuccess) return AFEM_ERR_HIP;
  if (v.n_cells > 0) {
    const unsigned blocks = (unsigned)((v.n_cells + 255) / 256);
    hipLaunchKernelGGL((k_assemble_cells<NV, K, F>), dim3(blocks), dim3(256), 0, st, v, f);
    if (hipGetLastError() != hipSuccess) return AFEM_ERR_HIP;
  }
  if (!check) return AFEM_OK;
  int32_t flag = 0;
  if (hipMemcpyAsync(&flag, v.error_flag, sizeof(flag), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return AFEM_ERR_HIP;
  return flag ? AFEM_ERR_NOT_FOUND : AFEM_OK;
}

}  // namespace generic
}  // namespace afem

#endif /* ARCANEFEM_AMD_GENERIC_HPP */
