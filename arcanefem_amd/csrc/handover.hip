// Device hand-over of an assembled matrix between numberings (one-time
// structure + one gather kernel per hand-over):
//
//  * BSRFormat::toLinearSystem with use_csr (femutils/BSRFormat.h:414-430)
//    goes through BSRMatrix::toCsr (:194-256): the scalar CSR of the block
//    matrix in the MODULE's DoF numbering -- rows = DoF local ids (empty for
//    DoFs that are not owned, the isOwn filter of :815, 870), columns =
//    node*NB_DOF + j in block order, values copied (:253).  libafem numbers
//    its nodes owned-first; bsr_csr32_mapped builds that CSR once from the
//    caller's DoF ids of libafem's scalar DoFs and gathers the values at each
//    hand-over (aliases them when the map is the identity: no copy);
//  * setCSRValues with a device view in a numbering that is not libafem's
//    (several subdomains: owned and ghost DoFs interleaved,
//    femutils/FemDoFsOnNodes.cc:79-109): ls_set_csr_mapped keeps the owned
//    rows in the linear system's order (columns renumbered) and a gather
//    index into the caller's values, which stay the matrix until solve()
//    (femutils/DoFLinearSystem.h:251-258): re-read at solve, point updates and
//    the boundary-condition pass written through to them (as Hypre edits the
//    view's values, femutils/HypreDoFLinearSystem.cc:148-156, 319-382).
#include "afem_internal.hpp"

#include <vector>

namespace afem {
namespace {

inline unsigned grid_for(int64_t n, int threads) { return (unsigned)((n + threads - 1) / threads); }

// scalar row lengths in the caller's numbering; flags duplicate / out-of-range DoF ids
__global__ void k_map_row_len(int64_t n_rows, int k, const int64_t* __restrict__ row_ptr,
                              const int32_t* __restrict__ dof_of, int64_t n_dof_rows, int32_t* __restrict__ rnc,
                              int32_t* __restrict__ err)
{
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_rows * k) return;
  const int64_t r = t / k;
  const int32_t R = dof_of[t];
  if (R < 0 || R >= n_dof_rows) {
    atomicOr(err, 1);
    return;
  }
  if (atomicAdd(&rnc[R], (int32_t)(k * (row_ptr[r + 1] - row_ptr[r]))) != 0) atomicOr(err, 2);
}

__global__ void k_map_fill(int64_t n_rows, int k, int per_block, const int64_t* __restrict__ row_ptr,
                           const int32_t* __restrict__ cols, const int32_t* __restrict__ dof_of, int64_t n_dof,
                           const int32_t* __restrict__ rows_out, int32_t* __restrict__ cols_out,
                           int64_t* __restrict__ src, int32_t* __restrict__ err)
{
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_rows * k) return;
  const int64_t r = t / k;
  const int i = (int)(t - r * k);
  const int64_t rb = row_ptr[r], len = row_ptr[r + 1] - rb;
  const int64_t kk = (int64_t)k * k;
  int64_t o = rows_out[dof_of[t]];
  for (int64_t s = 0; s < len; ++s) {
    const int64_t c = cols[rb + s];
    for (int j = 0; j < k; ++j, ++o) {
      const int64_t a = c * k + j;
      if (a >= n_dof) {
        atomicOr(err, 1);
        continue;
      }
      cols_out[o] = dof_of[a];
      src[o] = per_block ? (rb + s) * kk + i * k + j : rb * kk + (int64_t)i * k * len + k * s + j;
    }
  }
}

__global__ void k_not_identity(int64_t n, const int64_t* __restrict__ src, int32_t* __restrict__ flag)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n && src[p] != p) *flag = 1;
}

__global__ void k_gather(int64_t n, const int64_t* __restrict__ src, const double* __restrict__ in,
                         double* __restrict__ out)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) out[p] = in[src[p]];
}

__global__ void k_scatter_back(int64_t n, const int64_t* __restrict__ src, const double* __restrict__ in,
                               double* __restrict__ out)
{
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) out[src[p]] = in[p];
}

// the caller's view rows -> linear-system rows (owned ones); lengths, then fill.
// Every linear-system row must be claimed by exactly one caller row (claim
// counts, as k_map_row_len does for the other direction): a row claimed twice
// would make k_lsmap_fill write one row's entries past its own range
__global__ void k_lsmap_len(int32_t nb_row, int32_t nnz, const int32_t* __restrict__ rows,
                            const int32_t* __restrict__ index, int64_t n_index, int64_t n_ls_rows,
                            int64_t* __restrict__ len, int32_t* __restrict__ claim, int32_t* __restrict__ err)
{
  const int32_t R = (int32_t)((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (R >= nb_row || R >= n_index) return;
  const int32_t a = index[R];
  if (a < 0 || a >= n_ls_rows) return;
  if (atomicAdd(&claim[a], 1) != 0) {
    atomicOr(err, 2);
    return;
  }
  const int32_t e = R + 1 < nb_row ? rows[R + 1] : nnz;  // row end as femutils/HypreDoFLinearSystem.cc:140-141
  len[a] = e - rows[R];
}

// every owned linear-system row reached by one caller row, and not empty
__global__ void k_lsmap_check(int64_t n_ls_rows, const int64_t* __restrict__ len, const int32_t* __restrict__ claim,
                              int32_t* __restrict__ err)
{
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a < n_ls_rows && (claim[a] != 1 || len[a] <= 0)) atomicOr(err, 4);
}

__global__ void k_lsmap_fill(int32_t nb_row, int32_t nnz, const int32_t* __restrict__ rows,
                             const int32_t* __restrict__ cols, const int32_t* __restrict__ index, int64_t n_index,
                             int64_t n_ls_rows, int64_t n_ls_cols, const int64_t* __restrict__ ls_rows,
                             int32_t* __restrict__ ls_cols, int64_t* __restrict__ src, int32_t* __restrict__ err)
{
  const int32_t R = (int32_t)((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (R >= nb_row || R >= n_index) return;
  const int32_t a = index[R];
  if (a < 0 || a >= n_ls_rows) return;
  const int32_t b = rows[R], e = R + 1 < nb_row ? rows[R + 1] : nnz;
  int64_t o = ls_rows[a];
  for (int32_t q = b; q < e; ++q, ++o) {
    const int32_t c = cols[q];
    const int32_t lc = c >= 0 && c < n_index ? index[c] : -1;
    if (lc < 0 || lc >= n_ls_cols) atomicOr(err, 1);
    ls_cols[o] = lc < 0 ? 0 : lc;
    src[o] = q;
  }
}

__global__ void k_point_update_mapped(const int64_t* __restrict__ rows, const int32_t* __restrict__ cols,
                                      double* __restrict__ vals, const int64_t* __restrict__ src,
                                      double* __restrict__ caller_vals, int32_t row, int32_t col, double v, int set,
                                      int32_t* __restrict__ found)
{
  if (threadIdx.x != 0) return;
  for (int64_t k = rows[row]; k < rows[row + 1]; ++k)
    if (cols[k] == col) {
      const double x = set ? v : vals[k] + v;
      vals[k] = x;
      caller_vals[src[k]] = x;
      *found = 1;
      return;
    }
  *found = 0;
}

int32_t read_flag(Ctx& ctx, const int32_t* d)
{
  int32_t h = 0;
  AFEM_HIP(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  return h;
}

}  // namespace

void bsr_csr32_mapped_build(Bsr& b, const int32_t* dof_of_host, int64_t n_dof_rows)
{
  Ctx& ctx = *b.mesh->ctx;
  Structure& s = b.s;
  const int k = b.nb_dof;
  const int64_t n_dof = b.mesh->n_nodes * k;
  AFEM_REQUIRE(n_dof_rows >= s.n_rows * k && n_dof_rows < (int64_t)INT32_MAX, AFEM_ERR_ARG,
               "toLinearSystem: the DoF count must cover the owned DoFs and fit int32");
  const int64_t nnz = s.nnz * k * k;
  AFEM_REQUIRE(nnz < (int64_t)INT32_MAX, AFEM_ERR_LIMIT, "toLinearSystem: more than 2^31 scalar non-zeros (CSRFormatView is int32)");
  HandOver& H = b.hand;
  H = HandOver();
  DevBuf<int32_t> dof_of, err;
  dof_of.alloc(n_dof);
  err.alloc(1);
  AFEM_HIP(hipMemcpyAsync(dof_of.p, dof_of_host, dof_of.bytes(), hipMemcpyHostToDevice, ctx.stream));
  AFEM_HIP(hipMemsetAsync(err.p, 0, err.bytes(), ctx.stream));
  H.rnc.alloc(n_dof_rows);
  AFEM_HIP(hipMemsetAsync(H.rnc.p, 0, H.rnc.bytes(), ctx.stream));
  const int64_t nt = s.n_rows * k;
  if (nt > 0) {
    hipLaunchKernelGGL(k_map_row_len, dim3(grid_for(nt, 256)), dim3(256), 0, ctx.stream, s.n_rows, k, s.row_ptr.p,
                       dof_of.p, n_dof_rows, H.rnc.p, err.p);
    AFEM_LAUNCHED();
  }
  AFEM_REQUIRE(read_flag(ctx, err.p) == 0, AFEM_ERR_ARG,
               "toLinearSystem: the DoF numbering maps two owned DoFs to one id or out of range");
  DevBuf<int64_t> r64;
  r64.alloc(n_dof_rows + 1);
  exclusive_scan_i32_to_i64(ctx, H.rnc.p, r64.p, n_dof_rows);
  AFEM_REQUIRE(read_i64(ctx, r64.p + n_dof_rows) == nnz, AFEM_ERR_STATE, "toLinearSystem: row lengths do not add up");
  // int32 rows (CSRFormatView), no sentinel
  std::vector<int64_t> hr(n_dof_rows);
  AFEM_HIP(hipMemcpyAsync(hr.data(), r64.p, (size_t)n_dof_rows * 8, hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  std::vector<int32_t> hr32(hr.begin(), hr.end());
  H.rows.alloc(n_dof_rows);
  AFEM_HIP(hipMemcpyAsync(H.rows.p, hr32.data(), H.rows.bytes(), hipMemcpyHostToDevice, ctx.stream));
  H.cols.alloc(nnz > 0 ? nnz : 1);
  H.src.alloc(nnz > 0 ? nnz : 1);
  if (nt > 0) {
    hipLaunchKernelGGL(k_map_fill, dim3(grid_for(nt, 256)), dim3(256), 0, ctx.stream, s.n_rows, k,
                       b.order_per_block ? 1 : 0, s.row_ptr.p, s.cols.p, dof_of.p, n_dof, H.rows.p, H.cols.p, H.src.p,
                       err.p);
    AFEM_LAUNCHED();
  }
  AFEM_REQUIRE(read_flag(ctx, err.p) == 0, AFEM_ERR_ARG, "toLinearSystem: a column node has no DoF id");
  if (nnz > 0) {
    hipLaunchKernelGGL(k_not_identity, dim3(grid_for(nnz, 256)), dim3(256), 0, ctx.stream, nnz, H.src.p, err.p);
    AFEM_LAUNCHED();
  }
  H.identity = read_flag(ctx, err.p) == 0;
  if (H.identity)
    H.src.reset();
  else
    H.vals.alloc(nnz > 0 ? nnz : 1);
  H.n_rows = n_dof_rows;
  H.nnz = nnz;
  H.valid = true;
}

double* bsr_csr32_mapped_values(Bsr& b)
{
  HandOver& H = b.hand;
  AFEM_REQUIRE(H.valid, AFEM_ERR_STATE, "toLinearSystem: no DoF map (pass the numbering)");
  if (H.identity) return b.values.p;
  Ctx& ctx = *b.mesh->ctx;
  if (H.nnz > 0) {
    hipLaunchKernelGGL(k_gather, dim3(grid_for(H.nnz, 256)), dim3(256), 0, ctx.stream, H.nnz, H.src.p, b.values.p,
                       H.vals.p);
    AFEM_LAUNCHED();
  }
  return H.vals.p;
}

void ls_set_csr_mapped(LinearSystem& ls, const int32_t* rows, const int32_t* columns, double* values, int32_t nb_row,
                       int32_t nnz, const int32_t* index_host, int64_t n_index)
{
  Ctx& ctx = *ls.ctx;
  DevBuf<int32_t> index, err;
  index.alloc(n_index > 0 ? n_index : 1);
  err.alloc(1);
  if (n_index)
    AFEM_HIP(hipMemcpyAsync(index.p, index_host, (size_t)n_index * 4, hipMemcpyHostToDevice, ctx.stream));
  AFEM_HIP(hipMemsetAsync(err.p, 0, err.bytes(), ctx.stream));
  DevBuf<int64_t> len;
  len.alloc(ls.n_rows + 1);
  AFEM_HIP(hipMemsetAsync(len.p, 0, len.bytes(), ctx.stream));
  DevBuf<int32_t> claim;
  claim.alloc(ls.n_rows > 0 ? ls.n_rows : 1);
  AFEM_HIP(hipMemsetAsync(claim.p, 0, claim.bytes(), ctx.stream));
  if (nb_row > 0) {
    hipLaunchKernelGGL(k_lsmap_len, dim3(grid_for(nb_row, 256)), dim3(256), 0, ctx.stream, nb_row, nnz, rows, index.p,
                       n_index, ls.n_rows, len.p, claim.p, err.p);
    AFEM_LAUNCHED();
  }
  if (ls.n_rows > 0) {
    hipLaunchKernelGGL(k_lsmap_check, dim3(grid_for(ls.n_rows, 256)), dim3(256), 0, ctx.stream, ls.n_rows, len.p,
                       claim.p, err.p);
    AFEM_LAUNCHED();
  }
  const int32_t map_err = read_flag(ctx, err.p);
  AFEM_REQUIRE((map_err & 2) == 0, AFEM_ERR_ARG, "setCSRValues: two rows of the view map to one linear-system row");
  AFEM_REQUIRE((map_err & 4) == 0, AFEM_ERR_ARG,
               "setCSRValues: an owned linear-system row gets no row (or an empty one) from the view");
  ls.own_rows.alloc(ls.n_rows + 1);
  exclusive_scan_i64(ctx, len.p, ls.own_rows.p, ls.n_rows);
  const int64_t n_own_nz = read_i64(ctx, ls.own_rows.p + ls.n_rows);
  ls.own_cols.alloc(n_own_nz > 0 ? n_own_nz : 1);
  ls.own_vals.alloc(n_own_nz > 0 ? n_own_nz : 1);
  ls.mv_src.alloc(n_own_nz > 0 ? n_own_nz : 1);
  if (nb_row > 0) {
    hipLaunchKernelGGL(k_lsmap_fill, dim3(grid_for(nb_row, 256)), dim3(256), 0, ctx.stream, nb_row, nnz, rows,
                       columns, index.p, n_index, ls.n_rows, ls.n_cols, ls.own_rows.p, ls.own_cols.p, ls.mv_src.p,
                       err.p);
    AFEM_LAUNCHED();
  }
  AFEM_REQUIRE(read_flag(ctx, err.p) == 0, AFEM_ERR_ARG,
               "setCSRValues: a column of an owned row has no index in the linear system's column space");
  ls.mv_vals = values;
  ls.csr_rows = ls.own_rows.p;
  ls.csr_cols = ls.own_cols.p;
  ls.csr_vals = ls.own_vals.p;
  ls.csr_nnz = n_own_nz;
  ls.csr_n = ls.n_rows;
  ls_mapped_gather(ls);
}

void ls_mapped_gather(LinearSystem& ls)
{
  if (!ls.mv_vals || ls.csr_nnz == 0) return;
  Ctx& ctx = *ls.ctx;
  hipLaunchKernelGGL(k_gather, dim3(grid_for(ls.csr_nnz, 256)), dim3(256), 0, ctx.stream, ls.csr_nnz, ls.mv_src.p,
                     ls.mv_vals, ls.own_vals.p);
  AFEM_LAUNCHED();
}

void ls_mapped_scatter_back(LinearSystem& ls)
{
  if (!ls.mv_vals || ls.csr_nnz == 0) return;
  Ctx& ctx = *ls.ctx;
  hipLaunchKernelGGL(k_scatter_back, dim3(grid_for(ls.csr_nnz, 256)), dim3(256), 0, ctx.stream, ls.csr_nnz,
                     ls.mv_src.p, ls.own_vals.p, ls.mv_vals);
  AFEM_LAUNCHED();
}

void ls_mapped_point_update(LinearSystem& ls, int32_t row, int32_t col, double v, bool set)
{
  Ctx& ctx = *ls.ctx;
  AFEM_REQUIRE(row >= 0 && row < ls.csr_n, AFEM_ERR_ARG, "matrix{Add,Set}Value: row out of range");
  DevBuf<int32_t> found;
  found.alloc(1);
  hipLaunchKernelGGL(k_point_update_mapped, dim3(1), dim3(64), 0, ctx.stream, ls.csr_rows, ls.csr_cols, ls.own_vals.p,
                     ls.mv_src.p, ls.mv_vals, row, col, v, set ? 1 : 0, found.p);
  AFEM_LAUNCHED();
  AFEM_REQUIRE(read_flag(ctx, found.p) == 1, AFEM_ERR_NOT_FOUND,
               "matrix{Add,Set}Value: (row,col) is not in the CSR structure");
}

}  // namespace afem
