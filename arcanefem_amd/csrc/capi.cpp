// extern "C" boundary (include/arcanefem_amd.h).  Host-side C++ mirroring the
// reference's DoFLinearSystem / IDoFLinearSystemFactory / BSRFormat plugin
// surface; every entry point catches exceptions and returns a status code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "afem_internal.hpp"

using namespace afem;

namespace {
thread_local std::string g_last_error;

int fail(int code, const char* msg)
{
  g_last_error = msg ? msg : "unknown error";
  return code;
}
}  // namespace

#define API_BEGIN try {
#define API_END                                              \
  }                                                          \
  catch (const afem::Error& e) { return fail(e.code, e.what()); } \
  catch (const std::bad_alloc&) { return fail(AFEM_ERR_HIP, "host allocation failed"); } \
  catch (const std::exception& e) { return fail(AFEM_ERR_ARG, e.what()); } \
  catch (...) { return fail(AFEM_ERR_ARG, "unknown exception"); } \
  return AFEM_OK;

// roctx range over an entry point (the reference's Accelerator::ProfileRegion /
// [ArcaneFem-Timer] phases): visible in rocprofv3 --marker-trace
struct RoctxRange {
  explicit RoctxRange(const char* m) { roctxRangePushA(m); }
  ~RoctxRange() { roctxRangePop(); }
  RoctxRange(const RoctxRange&) = delete;
  RoctxRange& operator=(const RoctxRange&) = delete;
};
#define AFEM_RANGE(name) RoctxRange afem_range_(name)

#define NOT_NULL(p) AFEM_REQUIRE((p) != nullptr, AFEM_ERR_ARG, #p " must not be NULL")

static hipMemcpyKind kind_of(int dst_mem, int src_mem)
{
  if (dst_mem == AFEM_MEM_DEVICE)
    return src_mem == AFEM_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  return src_mem == AFEM_MEM_DEVICE ? hipMemcpyDeviceToHost : hipMemcpyHostToHost;
}

namespace afem {
// node halo lists -> DoF halo lists (DoF lid = node lid * k + i)
void expand_dof_lists(int k, std::vector<int64_t>& sc, std::vector<int64_t>& rc, std::vector<int32_t>& si,
                      std::vector<int32_t>& ri)
{
  auto expand = [k](std::vector<int32_t>& v) {
    std::vector<int32_t> o;
    o.reserve(v.size() * k);
    for (int32_t x : v)
      for (int i = 0; i < k; ++i) o.push_back(x * k + i);
    v.swap(o);
  };
  expand(si);
  expand(ri);
  for (auto& c : sc) c *= k;
  for (auto& c : rc) c *= k;
}

void structured_halo_lists(int dim, int n, int nz, int nranks, int rank, std::vector<int>& nbr,
                           std::vector<int64_t>& send_cnt, std::vector<int64_t>& recv_cnt,
                           std::vector<int32_t>& send_ids, std::vector<int32_t>& recv_ids)
{
  AFEM_REQUIRE(dim == 2 || dim == 3, AFEM_ERR_ARG, "dim must be 2 or 3");
  AFEM_REQUIRE(n >= 1 && nranks >= 1 && rank >= 0 && rank < nranks, AFEM_ERR_ARG, "bad n/rank/nranks");
  if (dim == 2 || nz <= 0) nz = n;
  const int64_t L = dim == 3 ? (int64_t)(n + 1) * (n + 1) : (int64_t)(n + 1);
  const int nl = nz + 1;
  AFEM_REQUIRE(nranks <= nl, AFEM_ERR_ARG, "more ranks than node layers");
  const int k0 = (int)((int64_t)rank * nl / nranks), k1 = (int)((int64_t)(rank + 1) * nl / nranks);
  const int64_t n_own = (int64_t)(k1 - k0) * L;
  nbr.clear();
  send_cnt.clear();
  recv_cnt.clear();
  send_ids.clear();
  recv_ids.clear();
  const bool lo = k0 > 0, hi = k1 < nl;
  if (lo) {  // neighbour rank-1 owns layer k0-1 (my first ghost layer), needs my layer k0
    nbr.push_back(rank - 1);
    send_cnt.push_back(L);
    recv_cnt.push_back(L);
    for (int64_t i = 0; i < L; ++i) send_ids.push_back((int32_t)i);
    for (int64_t i = 0; i < L; ++i) recv_ids.push_back((int32_t)(n_own + i));
  }
  if (hi) {  // neighbour rank+1 owns layer k1 (my last ghost layer), needs my layer k1-1
    nbr.push_back(rank + 1);
    send_cnt.push_back(L);
    recv_cnt.push_back(L);
    for (int64_t i = 0; i < L; ++i) send_ids.push_back((int32_t)(n_own - L + i));
    const int64_t base = n_own + (lo ? L : 0);
    for (int64_t i = 0; i < L; ++i) recv_ids.push_back((int32_t)(base + i));
  }
}
}  // namespace afem

extern "C" {

const char* afem_last_error(void) { return g_last_error.c_str(); }
int afem_version(void) { return 100; }

int afem_set_variant(const char* name, const char* value)
{
  API_BEGIN
  NOT_NULL(name);
  AFEM_REQUIRE(strncmp(name, "AFEM_", 5) == 0, AFEM_ERR_ARG, "afem_set_variant: knob names start with AFEM_");
  afem::set_variant(name, value);
  API_END
}

int afem_device_count(int* count)
{
  API_BEGIN
  NOT_NULL(count);
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  *count = (e == hipSuccess) ? c : 0;
  API_END
}

// ------------------------------------------------------------------ context
int afem_ctx_create(int device, void* hip_stream, afem_ctx** out)
{
  API_BEGIN
  NOT_NULL(out);
  *out = nullptr;
  auto* c = new afem_ctx();
  try {
    c->device = device;
    c->set_device();
    if (hip_stream) {
      c->stream = static_cast<hipStream_t>(hip_stream);
      c->own_stream = false;
    }
    else {
      AFEM_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      c->own_stream = true;
    }
    AFEM_HIP(hipEventCreate(&c->ev0));
    AFEM_HIP(hipEventCreate(&c->ev1));
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0)
      c->n_cu = cu;
  }
  catch (...) {
    delete c;
    throw;
  }
  *out = c;
  API_END
}

int afem_ctx_destroy(afem_ctx* ctx)
{
  API_BEGIN
  if (!ctx) return AFEM_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (hipEvent_t e : ctx->pool) (void)hipEventDestroy(e);
  if (ctx->aux) {
    (void)hipStreamSynchronize(ctx->aux);
    (void)hipStreamDestroy(ctx->aux);
    (void)hipEventDestroy(ctx->ev_fork);
    (void)hipEventDestroy(ctx->ev_join);
  }
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  API_END
}

int afem_ctx_synchronize(afem_ctx* ctx)
{
  API_BEGIN
  NOT_NULL(ctx);
  ctx->sync();
  API_END
}

int afem_ctx_stream(afem_ctx* ctx, void** s)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(s);
  *s = ctx->stream;
  API_END
}

int afem_ctx_timer_start(afem_ctx* ctx)
{
  API_BEGIN
  NOT_NULL(ctx);
  AFEM_HIP(hipEventRecord(ctx->ev0, ctx->stream));
  API_END
}

int afem_ctx_timer_stop(afem_ctx* ctx, float* ms)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(ms);
  AFEM_HIP(hipEventRecord(ctx->ev1, ctx->stream));
  AFEM_HIP(hipEventSynchronize(ctx->ev1));
  AFEM_HIP(hipEventElapsedTime(ms, ctx->ev0, ctx->ev1));
  API_END
}

int afem_ctx_event_record(afem_ctx* ctx, int slot)
{
  API_BEGIN
  NOT_NULL(ctx);
  AFEM_REQUIRE(slot >= 0 && slot < AFEM_EVENT_SLOTS, AFEM_ERR_ARG, "event slot out of range");
  if (ctx->pool.empty()) {
    ctx->set_device();
    ctx->pool.resize(AFEM_EVENT_SLOTS, nullptr);
    for (auto& e : ctx->pool) AFEM_HIP(hipEventCreate(&e));
  }
  AFEM_HIP(hipEventRecord(ctx->pool[slot], ctx->stream));
  API_END
}

int afem_ctx_event_elapsed(afem_ctx* ctx, int a, int b, float* ms)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(ms);
  AFEM_REQUIRE(!ctx->pool.empty() && a >= 0 && b >= 0 && a < AFEM_EVENT_SLOTS && b < AFEM_EVENT_SLOTS, AFEM_ERR_ARG,
               "event slot out of range or never recorded");
  AFEM_HIP(hipEventSynchronize(ctx->pool[b]));
  AFEM_HIP(hipEventElapsedTime(ms, ctx->pool[a], ctx->pool[b]));
  API_END
}

int afem_malloc(afem_ctx* ctx, size_t bytes, void** dptr)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(dptr);
  ctx->set_device();
  AFEM_HIP(hipMalloc(dptr, bytes));
  API_END
}

int afem_free(afem_ctx* ctx, void* dptr)
{
  API_BEGIN
  NOT_NULL(ctx);
  if (dptr) AFEM_HIP(hipFree(dptr));
  API_END
}

int afem_memcpy(afem_ctx* ctx, void* dst, const void* src, size_t bytes, int dst_mem, int src_mem)
{
  API_BEGIN
  NOT_NULL(ctx);
  if (!bytes) return AFEM_OK;
  NOT_NULL(dst);
  NOT_NULL(src);
  AFEM_HIP(hipMemcpyAsync(dst, src, bytes, kind_of(dst_mem, src_mem), ctx->stream));
  ctx->sync();
  API_END
}

// ------------------------------------------------------------------ mesh
int afem_mesh_create(afem_ctx* ctx, int dim, int nv, int64_t n_nodes, int64_t n_own, int64_t n_cells,
                     const int32_t* cell_node, const double* coords, int mem, afem_mesh** out)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(out);
  *out = nullptr;
  AFEM_REQUIRE(dim == 2 || dim == 3, AFEM_ERR_ARG, "mesh dimension must be 2 or 3");
  AFEM_REQUIRE(nv == dim + 1, AFEM_ERR_NOT_IMPL, "only P1 simplices (TRIA3 in 2D, TETRA4 in 3D) are supported");
  AFEM_REQUIRE(n_nodes >= 0 && n_own >= 0 && n_own <= n_nodes && n_cells >= 0, AFEM_ERR_ARG, "bad mesh sizes");
  AFEM_REQUIRE(n_nodes < (int64_t)INT32_MAX, AFEM_ERR_LIMIT, "more than 2^31-1 local nodes");
  if (n_cells) NOT_NULL(cell_node);
  if (n_nodes) NOT_NULL(coords);
  ctx->set_device();
  auto* m = new afem_mesh();
  try {
    m->ctx = ctx;
    m->dim = dim;
    m->nv = nv;
    m->n_nodes = n_nodes;
    m->n_own = n_own;
    m->n_cells = n_cells;
    m->cell_node.alloc((size_t)n_cells * nv);
    m->coords.alloc((size_t)n_nodes * 3);
    const hipMemcpyKind k = kind_of(AFEM_MEM_DEVICE, mem);
    if (n_cells) AFEM_HIP(hipMemcpyAsync(m->cell_node.p, cell_node, m->cell_node.bytes(), k, ctx->stream));
    if (n_nodes) AFEM_HIP(hipMemcpyAsync(m->coords.p, coords, m->coords.bytes(), k, ctx->stream));
    ctx->sync();
    if (mem == AFEM_MEM_HOST) {
      for (int64_t i = 0; i < n_cells * nv; ++i)
        AFEM_REQUIRE(cell_node[i] >= 0 && cell_node[i] < n_nodes, AFEM_ERR_ARG, "cell_node holds an out-of-range node id");
    }
  }
  catch (...) {
    delete m;
    throw;
  }
  *out = m;
  API_END
}

int afem_mesh_create_structured(afem_ctx* ctx, int dim, int n, int nz, double jitter, uint64_t seed, int nranks,
                                int rank, afem_mesh** out)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(out);
  *out = nullptr;
  auto* m = new afem_mesh();
  try {
    mesh_structured(*ctx, *m, dim, n, nz, jitter, seed, nranks, rank);
    ctx->sync();
  }
  catch (...) {
    delete m;
    throw;
  }
  *out = m;
  API_END
}

int afem_partition_rcb(int dim, int64_t n_nodes, const double* coords, int n_parts, int32_t* node_part)
{
  API_BEGIN
  AFEM_REQUIRE(n_nodes >= 0, AFEM_ERR_ARG, "bad node count");
  if (n_nodes) {
    NOT_NULL(coords);
    NOT_NULL(node_part);
  }
  partition_rcb(dim, n_nodes, coords, n_parts, node_part);
  API_END
}

int afem_subdomain_plan(int nv, int64_t n_nodes, int64_t n_cells, const int32_t* cell_node, const int32_t* node_part,
                        int nranks, int rank, afem_subdomain_info* info, int64_t* local_to_global, int64_t* cells,
                        int32_t* neighbor_ranks, int64_t* send_counts, int32_t* send_ids, int64_t* recv_counts,
                        int32_t* recv_ids)
{
  API_BEGIN
  NOT_NULL(info);
  AFEM_REQUIRE(nv >= 2 && n_nodes >= 0 && n_cells >= 0, AFEM_ERR_ARG, "bad mesh sizes");
  if (n_cells) NOT_NULL(cell_node);
  if (n_nodes) NOT_NULL(node_part);
  SubdomainPlan P;
  subdomain_plan(nv, n_nodes, n_cells, cell_node, node_part, nranks, rank, P);
  info->n_own_nodes = P.n_own;
  info->n_nodes = (int64_t)P.l2g.size();
  info->n_cells = (int64_t)P.cells.size();
  info->n_neighbors = (int)P.nbr.size();
  info->n_send = (int64_t)P.send_ids.size();
  info->n_recv = (int64_t)P.recv_ids.size();
  if (local_to_global) std::copy(P.l2g.begin(), P.l2g.end(), local_to_global);
  if (cells) std::copy(P.cells.begin(), P.cells.end(), cells);
  if (neighbor_ranks) std::copy(P.nbr.begin(), P.nbr.end(), neighbor_ranks);
  if (send_counts) std::copy(P.send_cnt.begin(), P.send_cnt.end(), send_counts);
  if (recv_counts) std::copy(P.recv_cnt.begin(), P.recv_cnt.end(), recv_counts);
  if (send_ids) std::copy(P.send_ids.begin(), P.send_ids.end(), send_ids);
  if (recv_ids) std::copy(P.recv_ids.begin(), P.recv_ids.end(), recv_ids);
  API_END
}

int afem_mesh_create_subdomain(afem_ctx* ctx, int dim, int nv, int64_t n_nodes, int64_t n_cells,
                               const int32_t* cell_node, const double* coords, const int32_t* node_part, int nranks,
                               int rank, afem_mesh** out)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(out);
  *out = nullptr;
  AFEM_REQUIRE(dim == 2 || dim == 3, AFEM_ERR_ARG, "mesh dimension must be 2 or 3");
  AFEM_REQUIRE(nv == dim + 1, AFEM_ERR_NOT_IMPL, "only P1 simplices (TRIA3 in 2D, TETRA4 in 3D) are supported");
  AFEM_REQUIRE(n_nodes >= 0 && n_cells >= 0, AFEM_ERR_ARG, "bad mesh sizes");
  if (n_cells) NOT_NULL(cell_node);
  if (n_nodes) {
    NOT_NULL(coords);
    NOT_NULL(node_part);
  }
  SubdomainPlan P;
  subdomain_plan(nv, n_nodes, n_cells, cell_node, node_part, nranks, rank, P);
  std::vector<double> xyz(P.l2g.size() * 3);
  for (size_t l = 0; l < P.l2g.size(); ++l)
    for (int d = 0; d < 3; ++d) xyz[3 * l + d] = coords[3 * P.l2g[l] + d];
  afem_mesh* m = nullptr;
  const int rc = afem_mesh_create(ctx, dim, nv, (int64_t)P.l2g.size(), P.n_own, (int64_t)P.cells.size(),
                                  P.cell_node.data(), xyz.data(), AFEM_MEM_HOST, &m);
  if (rc != AFEM_OK) return rc;
  P.cell_node.clear();
  P.cell_node.shrink_to_fit();
  m->part = std::move(P);
  *out = m;
  API_END
}

int afem_mesh_get_info(const afem_mesh* m, afem_mesh_info* info)
{
  API_BEGIN
  NOT_NULL(m);
  NOT_NULL(info);
  info->dim = m->dim;
  info->nb_node_per_cell = m->nv;
  info->n_nodes = m->n_nodes;
  info->n_own_nodes = m->n_own;
  info->n_cells = m->n_cells;
  API_END
}

int afem_mesh_download(afem_mesh* m, int32_t* cell_node, double* coords, int64_t* l2g)
{
  API_BEGIN
  NOT_NULL(m);
  Ctx& ctx = *m->ctx;
  ctx.set_device();
  if (cell_node && m->cell_node.n)
    AFEM_HIP(hipMemcpyAsync(cell_node, m->cell_node.p, m->cell_node.bytes(), hipMemcpyDeviceToHost, ctx.stream));
  if (coords && m->coords.n)
    AFEM_HIP(hipMemcpyAsync(coords, m->coords.p, m->coords.bytes(), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  if (l2g) mesh_local_to_global(*m, l2g);
  API_END
}

int afem_mesh_structured_bottom_nodes(afem_mesh* m, int32_t* ids, int64_t* count)
{
  API_BEGIN
  NOT_NULL(m);
  NOT_NULL(count);
  std::vector<int32_t> v;
  mesh_structured_bottom(*m, v);
  *count = (int64_t)v.size();
  if (ids) std::copy(v.begin(), v.end(), ids);
  API_END
}

int afem_mesh_destroy(afem_mesh* m)
{
  API_BEGIN
  if (m) {
    m->ctx->set_device();
    m->ctx->sync();
    delete m;
  }
  API_END
}

// ------------------------------------------------------------------ BSRFormat
int afem_bsr_create(afem_mesh* mesh, int nb_dof, int use_csr, afem_bsr** out)
{
  API_BEGIN
  NOT_NULL(mesh);
  NOT_NULL(out);
  *out = nullptr;
  AFEM_REQUIRE(nb_dof >= 1 && nb_dof <= 3, AFEM_ERR_ARG, "BSRFormat: NB_DOF must be 1, 2 or 3");
  auto* b = new afem_bsr();
  b->mesh = mesh;
  b->nb_dof = nb_dof;
  b->order_per_block = !use_csr;  // femutils/BSRFormat.h:402-403
  *out = b;
  API_END
}

int afem_bsr_compute_sparsity(afem_bsr* b)
{
  API_BEGIN
  AFEM_RANGE("afem: BSRFormat::computeSparsity");
  NOT_NULL(b);
  b->mesh->ctx->set_device();
  b->has_sparsity = false;
  b->fplan = FunctorPlan();
  b->hand = HandOver();
  build_structure(*b->mesh, b->s, b->nb_dof);
  b->values.alloc((size_t)b->s.nnz * b->nb_dof * b->nb_dof);
  AFEM_HIP(hipMemsetAsync(b->values.p, 0, b->values.bytes(), b->mesh->ctx->stream));
  b->mesh->ctx->sync();
  b->has_sparsity = true;
  API_END
}

int afem_bsr_assemble_poisson_p1(afem_bsr* b, double coef, double f, double* rhs)
{
  API_BEGIN
  NOT_NULL(b);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "assembleBilinear called before computeSparsity");
  b->mesh->ctx->set_device();
  assemble_scalar(*b, coef, f, rhs, 1);
  API_END
}

int afem_bsr_assemble_poisson_p1_ex(afem_bsr* b, double coef, double f, double* rhs, int rhs_mode)
{
  API_BEGIN
  AFEM_RANGE("afem: BSRFormat::assembleBilinear (Poisson P1)");
  NOT_NULL(b);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "assembleBilinear called before computeSparsity");
  AFEM_REQUIRE(rhs_mode == AFEM_RHS_ADD || rhs_mode == AFEM_RHS_SET, AFEM_ERR_ARG, "unknown rhs_mode");
  b->mesh->ctx->set_device();
  assemble_scalar(*b, coef, f, rhs, rhs_mode == AFEM_RHS_ADD ? 1 : 0);
  API_END
}

int afem_bsr_assemble_elasticity_p1(afem_bsr* b, double lambda, double mu2)
{
  API_BEGIN
  NOT_NULL(b);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "assembleBilinear called before computeSparsity");
  b->mesh->ctx->set_device();
  if (b->mesh->nv == 4)
    assemble_elasticity_tet(*b, lambda, mu2, 0.0, nullptr, nullptr, 1);
  else
    assemble_elasticity_tri(*b, lambda, mu2);
  API_END
}

int afem_bsr_assemble_elasticity_p1_ex(afem_bsr* b, double lambda, double mu2, double mass_coef, const double* body_force,
                                       double* rhs, int rhs_mode)
{
  API_BEGIN
  AFEM_RANGE("afem: BSRFormat::assembleBilinear (elasticity P1)");
  NOT_NULL(b);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "assembleBilinear called before computeSparsity");
  AFEM_REQUIRE(b->mesh->nv == 4 && b->nb_dof == 3, AFEM_ERR_NOT_IMPL,
               "the mass / body-force form is implemented for NB_DOF = 3 on tetrahedra");
  AFEM_REQUIRE(!body_force || rhs, AFEM_ERR_ARG, "body_force given without an rhs array");
  AFEM_REQUIRE(rhs_mode == AFEM_RHS_ADD || rhs_mode == AFEM_RHS_SET, AFEM_ERR_ARG, "unknown rhs_mode");
  b->mesh->ctx->set_device();
  assemble_elasticity_tet(*b, lambda, mu2, mass_coef, body_force, rhs, rhs_mode == AFEM_RHS_ADD ? 1 : 0);
  API_END
}

int afem_bsr_reset_values(afem_bsr* b)
{
  API_BEGIN
  NOT_NULL(b);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "no sparsity");
  AFEM_HIP(hipMemsetAsync(b->values.p, 0, b->values.bytes(), b->mesh->ctx->stream));
  API_END
}

int afem_bsr_set_value(afem_bsr* b, int32_t row, int32_t col, double v)
{
  API_BEGIN
  NOT_NULL(b);
  AFEM_REQUIRE(bsr_point(*b, row, col, 1, v, nullptr), AFEM_ERR_NOT_FOUND,
               "BSRMatrix(findValueIndex): Value not found");
  API_END
}

int afem_bsr_get_value(afem_bsr* b, int32_t row, int32_t col, double* v)
{
  API_BEGIN
  NOT_NULL(b);
  NOT_NULL(v);
  AFEM_REQUIRE(bsr_point(*b, row, col, 0, 0.0, v), AFEM_ERR_NOT_FOUND, "BSRMatrix(findValueIndex): Value not found");
  API_END
}

int afem_bsr_view(afem_bsr* b, afem_csr_view* v)
{
  API_BEGIN
  NOT_NULL(b);
  NOT_NULL(v);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "no sparsity");
  v->n_block_rows = b->s.n_rows;
  v->n_block_cols = b->s.n_cols;
  v->nnz_blocks = b->s.nnz;
  v->block_size = b->nb_dof;
  v->ordered_per_block = b->order_per_block ? 1 : 0;
  v->rows = b->s.row_ptr.p;
  v->columns = b->s.cols.p;
  v->values = b->values.p;
  API_END
}

int afem_bsr_assembly_view(afem_bsr* b, afem_assembly_view* v)
{
  API_BEGIN
  NOT_NULL(b);
  NOT_NULL(v);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "no sparsity (computeSparsity first)");
  if (!b->gen_flag.p) b->gen_flag.alloc(1);
  const Mesh& m = *b->mesh;
  v->n_rows = b->s.n_rows;
  v->n_nodes = m.n_nodes;
  v->n_cells = m.n_cells;
  v->nb_node_per_cell = m.nv;
  v->block_size = b->nb_dof;
  v->ordered_per_block = b->order_per_block ? 1 : 0;
  v->dim = m.dim;
  v->cell_node = m.cell_node.p;
  v->coords = m.coords.p;
  v->rows = b->s.row_ptr.p;
  v->columns = b->s.cols.p;
  v->values = b->values.p;
  v->error_flag = b->gen_flag.p;
  v->stream = (void*)m.ctx->stream;
  API_END
}

int afem_bsr_to_csr32_mapped(afem_bsr* b, const int32_t* dof_of, int64_t n_dof_rows, afem_csr32_view* v)
{
  API_BEGIN
  AFEM_RANGE("afem: BSRFormat::toLinearSystem (mapped CSR)");
  NOT_NULL(b);
  NOT_NULL(v);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "no sparsity (computeSparsity first)");
  b->mesh->ctx->set_device();
  if (dof_of) bsr_csr32_mapped_build(*b, dof_of, n_dof_rows);
  double* vals = bsr_csr32_mapped_values(*b);
  const HandOver& H = b->hand;
  v->n_rows = H.n_rows;
  v->nnz = H.nnz;
  v->rows = H.rows.p;
  v->rows_nb_column = H.rnc.p;
  v->columns = H.cols.p;
  v->values = vals;
  v->identity = H.identity ? 1 : 0;
  API_END
}

int afem_bsr_functor_plan(afem_bsr* b, afem_functor_plan* p)
{
  API_BEGIN
  AFEM_RANGE("afem: BSRFormat functor plan");
  NOT_NULL(b);
  NOT_NULL(p);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "no sparsity (computeSparsity first)");
  b->mesh->ctx->set_device();
  if (!b->fplan.valid) functor_plan_build(*b);
  const FunctorPlan& P = b->fplan;
  p->n_units = P.n_units;
  p->n_stages = P.n_stages;
  p->n_entries = P.n_entries;
  p->rows_per_layer = P.rl;
  p->width = P.w;
  p->nbuf = P.nbuf;
  p->wide = P.wide;
  p->block_size = b->nb_dof;
  p->nb_node_per_cell = b->mesh->nv;
  p->ordered_per_block = b->order_per_block ? 1 : 0;
  p->lattice = P.lattice;
  p->units = P.units.p;
  p->stage_ptr = P.stage_ptr.p;
  p->layer_rows = P.layer_rows.p;
  p->entries = P.ent.p;
  p->entries2 = P.wide ? P.ent2.p : nullptr;
  p->rows = b->s.row_ptr.p;
  p->values = b->values.p;
  p->stream = (void*)b->mesh->ctx->stream;
  p->patterns = P.packed ? P.patterns.p : nullptr;
  p->n_patterns = P.n_patterns;
  p->packed = P.packed;
  p->reserved0 = 0;
  API_END
}

int afem_bsr_get_stats(afem_bsr* b, afem_bsr_stats* st)
{
  API_BEGIN
  NOT_NULL(b);
  NOT_NULL(st);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "no sparsity");
  st->n_incidences = b->s.n_incidences;
  st->inc_table_entries = (int64_t)b->s.inc.n;
  st->max_row_len = b->s.max_row_len;
  st->rows_per_block = afem::assembly_uses_lds(*b) ? 64 : 0;
  st->max_seg = b->s.max_wave_seg;
  st->max_slice_nodes = b->s.max_slice_nodes;
  st->max_slice_width = b->s.max_slice_w;
  st->n_slices = b->s.n_slices;
  st->brick_order = b->s.lattice ? 2 : b->s.brick_order ? 1 : 0;
  st->cube_lattice = b->s.cube_natural ? 2 : (b->s.canon && b->s.cube_ok) ? 3
                     : (b->mesh->st.valid && b->mesh->st.dim == 3 && !b->s.canon) ? 1 : 0;
  st->uniform_slices = (int32_t)b->s.n_uni;
  st->stencil_slices = (int32_t)b->s.n_k;
  st->stencil_sig = b->s.sig_k;
  st->shared_strip_slices = b->s.n_strip_shared;
  st->uniform_instance_slices = b->s.n_ur;
  st->general_slices = b->s.n_ms + b->s.n_mb;
  st->cube_axes = b->s.cube_natural ? b->s.nat_axes[0] + 3 * b->s.nat_axes[1] + 9 * b->s.nat_axes[2] : 0;
  st->last_kernel = b->last_kernel;
  API_END
}

int afem_bsr_get_sizes(afem_bsr* b, int64_t* n_rows, int64_t* nnz)
{
  API_BEGIN
  NOT_NULL(b);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "no sparsity");
  if (n_rows) *n_rows = b->s.n_rows * b->nb_dof;
  if (nnz) *nnz = b->s.nnz * b->nb_dof * b->nb_dof;
  API_END
}

int afem_bsr_download(afem_bsr* b, int64_t* rows, int32_t* cols, double* vals)
{
  API_BEGIN
  NOT_NULL(b);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "no sparsity");
  Ctx& ctx = *b->mesh->ctx;
  ctx.set_device();
  if (rows) AFEM_HIP(hipMemcpyAsync(rows, b->s.row_ptr.p, b->s.row_ptr.bytes(), hipMemcpyDeviceToHost, ctx.stream));
  if (cols && b->s.nnz)
    AFEM_HIP(hipMemcpyAsync(cols, b->s.cols.p, (size_t)b->s.nnz * sizeof(int32_t), hipMemcpyDeviceToHost, ctx.stream));
  if (vals && b->values.n)
    AFEM_HIP(hipMemcpyAsync(vals, b->values.p, b->values.bytes(), hipMemcpyDeviceToHost, ctx.stream));
  ctx.sync();
  API_END
}

int afem_bsr_export_csr32(afem_bsr* b, int32_t* rows, int32_t* rows_nb_column, int32_t* columns, double* values)
{
  API_BEGIN
  NOT_NULL(b);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "no sparsity");
  const int k = b->nb_dof;
  const int64_t ns = b->s.n_rows * k, nnz = b->s.nnz * k * k;
  AFEM_REQUIRE(nnz < (int64_t)INT32_MAX, AFEM_ERR_LIMIT, "the Int32 CSRFormatView cannot hold more than 2^31-1 values");
  Ctx& ctx = *b->mesh->ctx;
  ctx.set_device();
  std::vector<int64_t> srows(ns + 1);
  if (k == 1) {
    AFEM_HIP(hipMemcpyAsync(srows.data(), b->s.row_ptr.p, srows.size() * 8, hipMemcpyDeviceToHost, ctx.stream));
    if (columns && nnz) AFEM_HIP(hipMemcpyAsync(columns, b->s.cols.p, nnz * 4, hipMemcpyDeviceToHost, ctx.stream));
    if (values && nnz) AFEM_HIP(hipMemcpyAsync(values, b->values.p, nnz * 8, hipMemcpyDeviceToHost, ctx.stream));
  }
  else {
    DevBuf<double> tmp;
    if (b->order_per_block) tmp.alloc(nnz);
    bsr_expand_scalar(*b, tmp.p);
    AFEM_HIP(hipMemcpyAsync(srows.data(), b->csr_rows.p, srows.size() * 8, hipMemcpyDeviceToHost, ctx.stream));
    if (columns && nnz) AFEM_HIP(hipMemcpyAsync(columns, b->csr_cols.p, nnz * 4, hipMemcpyDeviceToHost, ctx.stream));
    if (values && nnz)
      AFEM_HIP(hipMemcpyAsync(values, b->order_per_block ? tmp.p : b->values.p, nnz * 8, hipMemcpyDeviceToHost,
                              ctx.stream));
    ctx.sync();
  }
  ctx.sync();
  for (int64_t i = 0; i < ns; ++i) {
    if (rows) rows[i] = (int32_t)srows[i];
    if (rows_nb_column) rows_nb_column[i] = (int32_t)(srows[i + 1] - srows[i]);
  }
  API_END
}

int afem_bsr_to_linear_system(afem_bsr* b, afem_ls* ls)
{
  API_BEGIN
  NOT_NULL(b);
  NOT_NULL(ls);
  AFEM_REQUIRE(b->has_sparsity, AFEM_ERR_STATE, "toLinearSystem called before computeSparsity");
  const int k = b->nb_dof;
  AFEM_REQUIRE(ls->n_rows == b->s.n_rows * k, AFEM_ERR_ARG,
               "BSRFormat(toLinearSystem): linear system size differs from the matrix rows");
  AFEM_REQUIRE(ls->n_cols >= b->mesh->n_nodes * k, AFEM_ERR_ARG,
               "BSRFormat(toLinearSystem): the linear system's column space (n_cols_local) is smaller than the "
               "matrix columns (owned + ghost nodes x NB_DOF)");
  b->mesh->ctx->set_device();
  ls->blk_k = 0;
  if (k == 1) {
    ls->csr_rows = b->s.row_ptr.p;
    ls->csr_diag = b->s.diag_pos.n >= (size_t)b->s.n_rows ? b->s.diag_pos.p : nullptr;
    ls->csr_cols = b->s.cols.p;
    ls->csr_vals = b->values.p;
  }
  else {
    if (b->order_per_block) b->csr_vals.alloc(b->s.nnz * k * k);
    bsr_expand_scalar(*b, b->csr_vals.p);
    ls->csr_rows = b->csr_rows.p;
    ls->csr_diag = nullptr;
    ls->csr_cols = b->csr_cols.p;
    ls->csr_vals = b->order_per_block ? b->csr_vals.p : b->values.p;
    ls->blk_k = k;  // the SpMV reads the node-row structure instead of the scalar columns
    ls->blk_n = b->s.n_rows;
    ls->blk_rows = b->s.row_ptr.p;
    ls->blk_cols = b->s.cols.p;
  }
  // structured box on one rank: the multigrid preconditioner's fine grid
  const StructuredInfo& st = b->mesh->st;
  // (a z-slab of several ranks: its owned box, for the block-Jacobi V-cycle)
  const bool box = st.valid && st.dim == 3 && b->mesh->nv == 4 && !b->mesh->part.valid;
  ls->mg_k = box ? k : 0;
  ls->mg_nx = box ? st.n : 0;
  ls->mg_nz = box ? (st.k1 - st.k0) - 1 : 0;
  ls->mg_multi = box && st.nranks > 1;
  ls->mg_nzg = box ? st.nz : 0;
  ls->mg_k0 = box ? st.k0 : 0;
  ls->mg_glo = box && st.ghost_lo >= 0;
  ls->mg.reset();
  ls->amg.reset();
  ls->has_csr = true;
  ls->csr_from_coo = false;
  ls->hv_rows = nullptr;
  ls->hv_cols = nullptr;
  ls->hv_vals = nullptr;
  ls->mv_vals = nullptr;
  ls->csr_n = b->s.n_rows * k;
  ls->csr_nnz = b->s.nnz * k * k;
  API_END
}

int afem_bsr_destroy(afem_bsr* b)
{
  API_BEGIN
  if (b) {
    b->mesh->ctx->set_device();
    b->mesh->ctx->sync();
    delete b;
  }
  API_END
}

// ------------------------------------------------------------------ linear system
int afem_ls_create(afem_ctx* ctx, int64_t n_rows, int64_t n_cols_local, afem_ls** out)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(out);
  *out = nullptr;
  AFEM_REQUIRE(n_rows > 0 && n_cols_local >= n_rows, AFEM_ERR_ARG, "linear system: need 0 < n_rows <= n_cols_local");
  AFEM_REQUIRE(n_cols_local < (int64_t)INT32_MAX, AFEM_ERR_LIMIT, "more than 2^31-1 local DoFs");
  ctx->set_device();
  auto* ls = new afem_ls();
  try {
    ls->ctx = ctx;
    ls->n_rows = n_rows;
    ls->n_cols = n_cols_local;
    ls->opts.method = AFEM_SOLVER_AUTO;
    ls->opts.max_iter = 10000;
    ls->opts.rtol = 1.0e-15;  // SequentialBasic epsilon (femutils/DoFLinearSystem.cc:234)
    ls->opts.atol = 0.0;
    ls->opts.check_every = 8;
    ls->opts.fixed_iterations = 0;
    ls->opts.initial_guess = 0;
    ls->opts.precond_block = 0;
    ls->rhs.alloc(n_rows);
    ls->sol.alloc(n_cols_local);
    ls->forced_info.alloc(n_rows);
    ls->elim_info.alloc(n_rows);
    ls->forced_value.alloc(n_rows);
    ls->elim_value.alloc(n_rows);
    hipStream_t s = ctx->stream;
    AFEM_HIP(hipMemsetAsync(ls->rhs.p, 0, ls->rhs.bytes(), s));
    AFEM_HIP(hipMemsetAsync(ls->sol.p, 0, ls->sol.bytes(), s));
    AFEM_HIP(hipMemsetAsync(ls->forced_info.p, 0, ls->forced_info.bytes(), s));
    AFEM_HIP(hipMemsetAsync(ls->elim_info.p, 0, ls->elim_info.bytes(), s));
    AFEM_HIP(hipMemsetAsync(ls->forced_value.p, 0, ls->forced_value.bytes(), s));
    AFEM_HIP(hipMemsetAsync(ls->elim_value.p, 0, ls->elim_value.bytes(), s));
    ctx->sync();
  }
  catch (...) {
    delete ls;
    throw;
  }
  *out = ls;
  API_END
}

int afem_ls_set_solver_options(afem_ls* ls, const afem_solver_opts* o)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(o);
  AFEM_REQUIRE(o->method == AFEM_SOLVER_AUTO || o->method == AFEM_SOLVER_PCG || o->method == AFEM_SOLVER_DIRECT,
               AFEM_ERR_NOT_IMPL, "unknown solver method");
  AFEM_REQUIRE(o->max_iter >= 0 && o->rtol >= 0 && o->atol >= 0, AFEM_ERR_ARG, "bad solver options");
  AFEM_REQUIRE(o->initial_guess == 0 || o->initial_guess == 1, AFEM_ERR_ARG, "initial_guess must be 0 or 1");
  AFEM_REQUIRE(o->precond_block == 0 || o->precond_block == 1 || o->precond_block == 3, AFEM_ERR_ARG,
               "precond_block must be 0, 1 or 3");
  AFEM_REQUIRE(o->multigrid >= 0 && o->multigrid <= 2, AFEM_ERR_ARG, "multigrid must be 0, 1 or 2");
  AFEM_REQUIRE(o->amg >= 0 && o->amg <= 2, AFEM_ERR_ARG, "amg must be 0, 1 or 2");
  AFEM_REQUIRE(!(o->amg && o->precond_block == 3), AFEM_ERR_ARG,
               "amg and block Jacobi are alternative preconditioners");
  AFEM_REQUIRE(!(o->multigrid && o->precond_block == 3), AFEM_ERR_ARG,
               "multigrid and block Jacobi are alternative preconditioners");
  if (o->multigrid != ls->opts.multigrid) ls->mg.reset();
  if (o->amg != ls->opts.amg) ls->amg.reset();
  ls->opts = *o;
  API_END
}

int afem_ls_get_solver_options(afem_ls* ls, afem_solver_opts* o)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(o);
  *o = ls->opts;
  API_END
}

// With a CSR view (from the BSR, setCSRValues on host or device memory) the
// point updates go into it, as HypreDoFLinearSystemImpl::matrixAddValue does
// (femutils/HypreDoFLinearSystem.cc:148-156); a CSR rebuilt from the host COO
// maps is a derived copy, so further adds go to the maps.
static bool ls_uses_device_view(afem_ls* ls) { return ls->has_csr && !ls->csr_from_coo; }

// a point update of a host view also edits the caller's arrays (the solve
// re-reads them); the device copy is updated too (SpMV / getCSRValues before solve)
static void host_view_update(afem_ls* ls, int32_t row, int32_t col, double v, bool set)
{
  const int64_t b = ls->hv_rows[row], e = row + 1 < ls->csr_n ? ls->hv_rows[row + 1] : ls->csr_nnz;
  for (int64_t k = b; k < e; ++k)
    if (ls->hv_cols[k] == col) {
      ls->hv_vals[k] = set ? v : ls->hv_vals[k] + v;
      return;
    }
}

int afem_ls_matrix_add_value(afem_ls* ls, int32_t row, int32_t col, double v)
{
  API_BEGIN
  NOT_NULL(ls);
  AFEM_REQUIRE(row >= 0 && row < ls->n_rows && col >= 0 && col < ls->n_cols, AFEM_ERR_ARG,
               "matrixAddValue: row or column out of range");
  ls->ctx->set_device();
  if (ls_uses_device_view(ls)) {
    if (ls->mv_vals)
      ls_mapped_point_update(*ls, row, col, v, false);
    else
      ls_point_update(*ls, row, col, v, false);
    if (ls->hv_vals) host_view_update(ls, row, col, v, false);
  }
  else {
    if (v == 0.0) return AFEM_OK;  // femutils/AlephDoFLinearSystem.cc:198-199
    ls->has_csr = false;           // rebuilt from the maps at solve
    ls->csr_from_coo = false;
    ls->add_map[{ row, col }] += v;
  }
  API_END
}

int afem_ls_matrix_set_value(afem_ls* ls, int32_t row, int32_t col, double v)
{
  API_BEGIN
  NOT_NULL(ls);
  AFEM_REQUIRE(row >= 0 && row < ls->n_rows && col >= 0 && col < ls->n_cols, AFEM_ERR_ARG,
               "matrixSetValue: row or column out of range");
  ls->ctx->set_device();
  if (ls_uses_device_view(ls)) {
    if (ls->mv_vals)
      ls_mapped_point_update(*ls, row, col, v, true);
    else
      ls_point_update(*ls, row, col, v, true);
    if (ls->hv_vals) host_view_update(ls, row, col, v, true);
  }
  else {
    ls->has_csr = false;
    ls->csr_from_coo = false;
    ls->set_map[{ row, col }] = v;
  }
  API_END
}

static int eliminate(afem_ls* ls, int32_t row, double v, uint8_t info)
{
  AFEM_REQUIRE(row >= 0 && row < ls->n_rows, AFEM_ERR_ARG, "eliminateRow: row out of range");
  ls->ctx->set_device();
  ls->host_elim[row] = { info, v };
  AFEM_HIP(hipMemcpyAsync(ls->elim_info.p + row, &info, 1, hipMemcpyHostToDevice, ls->ctx->stream));
  AFEM_HIP(hipMemcpyAsync(ls->elim_value.p + row, &v, sizeof(double), hipMemcpyHostToDevice, ls->ctx->stream));
  ls->ctx->sync();
  return AFEM_OK;
}

int afem_ls_eliminate_row(afem_ls* ls, int32_t row, double v)
{
  API_BEGIN
  NOT_NULL(ls);
  eliminate(ls, row, v, 1);
  API_END
}

int afem_ls_eliminate_row_column(afem_ls* ls, int32_t row, double v)
{
  API_BEGIN
  NOT_NULL(ls);
  eliminate(ls, row, v, 2);
  API_END
}

int afem_ls_set_csr_values(afem_ls* ls, const int32_t* rows, const int32_t* rows_nb_column, const int32_t* columns,
                           double* values, int32_t nb_row, int32_t nb_nz, int mem)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(rows);
  NOT_NULL(columns);
  NOT_NULL(values);
  AFEM_REQUIRE(nb_row == ls->n_rows, AFEM_ERR_ARG, "setCSRValues: nb_row differs from the linear system size");
  AFEM_REQUIRE(nb_nz >= 0, AFEM_ERR_ARG, "setCSRValues: negative nb_nz");
  Ctx& ctx = *ls->ctx;
  ctx.set_device();
  std::vector<int32_t> hrows(nb_row);
  AFEM_HIP(hipMemcpyAsync(hrows.data(), rows, (size_t)nb_row * 4, kind_of(AFEM_MEM_HOST, mem), ctx.stream));
  ctx.sync();
  (void)rows_nb_column;  // derived from rows, as femutils/HypreDoFLinearSystem.cc:140-141 does
  std::vector<int64_t> r64(nb_row + 1);
  for (int32_t i = 0; i < nb_row; ++i) r64[i] = hrows[i];
  r64[nb_row] = nb_nz;
  for (int32_t i = 0; i < nb_row; ++i)
    AFEM_REQUIRE(r64[i] <= r64[i + 1], AFEM_ERR_ARG, "setCSRValues: rows are not non-decreasing");
  AFEM_REQUIRE(nb_row == 0 || r64[0] == 0, AFEM_ERR_ARG, "setCSRValues: rows[0] must be 0");
  if (mem == AFEM_MEM_HOST) {
    for (int32_t t = 0; t < nb_nz; ++t)
      AFEM_REQUIRE(columns[t] >= 0 && columns[t] < ls->n_cols, AFEM_ERR_ARG,
                   "setCSRValues: column index outside the linear system's column space");
  }
  else {
    int32_t lo = 0, hi = 0;
    device_minmax_i32(ctx, columns, nb_nz, &lo, &hi);
    AFEM_REQUIRE(nb_nz == 0 || (lo >= 0 && hi < ls->n_cols), AFEM_ERR_ARG,
                 "setCSRValues: column index outside the linear system's column space");
  }
  ls->own_rows.alloc(nb_row + 1);
  AFEM_HIP(hipMemcpyAsync(ls->own_rows.p, r64.data(), ls->own_rows.bytes(), hipMemcpyHostToDevice, ctx.stream));
  if (mem == AFEM_MEM_DEVICE) {
    ls->csr_cols = columns;
    ls->csr_vals = values;
    ls->own_vals.reset();
  }
  else {
    ls->own_cols.alloc(nb_nz);
    ls->own_vals.alloc(nb_nz);
    if (nb_nz) {
      AFEM_HIP(hipMemcpyAsync(ls->own_cols.p, columns, (size_t)nb_nz * 4, hipMemcpyHostToDevice, ctx.stream));
      AFEM_HIP(hipMemcpyAsync(ls->own_vals.p, values, (size_t)nb_nz * 8, hipMemcpyHostToDevice, ctx.stream));
    }
    ls->csr_cols = ls->own_cols.p;
    ls->csr_vals = ls->own_vals.p;
  }
  ctx.sync();
  ls->csr_rows = ls->own_rows.p;
  ls->csr_diag = nullptr;
  ls->mv_vals = nullptr;
  ls->blk_k = 0;
  ls->mg_k = 0;
  ls->mg.reset();
  ls->amg.reset();
  ls->csr_n = nb_row;
  ls->csr_nnz = nb_nz;
  ls->has_csr = true;
  ls->csr_from_coo = false;
  ls->hv_rows = nullptr;
  ls->hv_cols = nullptr;
  ls->hv_vals = nullptr;
  if (mem == AFEM_MEM_HOST) {
    // host view: the caller's arrays stay the matrix until solve (point
    // updates edit them, the solve re-reads the values); keep the COO maps empty
    ls->hv_rows = rows;
    ls->hv_cols = columns;
    ls->hv_vals = values;
    ls->add_map.clear();
    ls->set_map.clear();
  }
  API_END
}

int afem_ls_set_csr_values_mapped(afem_ls* ls, const int32_t* rows, const int32_t* rows_nb_column,
                                  const int32_t* columns, double* values, int32_t nb_row, int32_t nb_nz,
                                  const int32_t* index, int64_t n_index)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(rows);
  NOT_NULL(columns);
  NOT_NULL(values);
  NOT_NULL(index);
  AFEM_REQUIRE(nb_row >= 0 && nb_nz >= 0 && n_index >= 0, AFEM_ERR_ARG, "setCSRValues: negative size");
  (void)rows_nb_column;  // derived from rows, as femutils/HypreDoFLinearSystem.cc:140-141 does
  ls->ctx->set_device();
  ls->has_csr = false;
  ls_set_csr_mapped(*ls, rows, columns, values, nb_row, nb_nz, index, n_index);
  ls->csr_diag = nullptr;
  ls->blk_k = 0;
  ls->mg_k = 0;
  ls->mg.reset();
  ls->amg.reset();
  ls->has_csr = true;
  ls->csr_from_coo = false;
  ls->hv_rows = nullptr;
  ls->hv_cols = nullptr;
  ls->hv_vals = nullptr;
  ls->add_map.clear();
  ls->set_map.clear();
  API_END
}

int afem_ls_has_set_csr_values(afem_ls* ls, int* has)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(has);
  *has = 1;  // hasSetCSRValues() == true (femutils/HypreDoFLinearSystem.cc:204)
  API_END
}

int afem_ls_get_csr_values(afem_ls* ls, afem_csr_view* v)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(v);
  AFEM_REQUIRE(ls->has_csr, AFEM_ERR_STATE, "getCSRValues: no CSR view");
  v->n_block_rows = ls->csr_n;
  v->n_block_cols = ls->n_cols;
  v->nnz_blocks = ls->csr_nnz;
  v->block_size = 1;
  v->ordered_per_block = 1;
  v->rows = ls->csr_rows;
  v->columns = ls->csr_cols;
  v->values = ls->csr_vals;
  API_END
}

#define LS_PTR(name, field, T)            \
  int name(afem_ls* ls, T** p)            \
  {                                       \
    API_BEGIN                             \
    NOT_NULL(ls);                         \
    NOT_NULL(p);                          \
    *p = ls->field.p;                     \
    API_END                               \
  }
LS_PTR(afem_ls_rhs, rhs, double)
LS_PTR(afem_ls_solution, sol, double)
LS_PTR(afem_ls_forced_info, forced_info, uint8_t)
LS_PTR(afem_ls_forced_value, forced_value, double)
LS_PTR(afem_ls_elimination_info, elim_info, uint8_t)
LS_PTR(afem_ls_elimination_value, elim_value, double)

int afem_ls_dirichlet_penalty(afem_ls* ls, const int32_t* dofs, int64_t n, double value, double penalty, int mem)
{
  API_BEGIN
  NOT_NULL(ls);
  if (n > 0) NOT_NULL(dofs);
  ls->ctx->set_device();
  ls_set_list(*ls, dofs, n, mem, 0, value, penalty);
  API_END
}

int afem_ls_dirichlet_row_elimination(afem_ls* ls, const int32_t* dofs, int64_t n, double value, int mem)
{
  API_BEGIN
  NOT_NULL(ls);
  if (n > 0) NOT_NULL(dofs);
  ls->ctx->set_device();
  ls_set_list(*ls, dofs, n, mem, 1, value, 0.0);
  API_END
}

int afem_apply_neumann(afem_mesh* mesh, int nb_dof, int mode, const double value[3], int64_t n_faces,
                       const int32_t* face_nodes, const int32_t* face_cells, int mem, double* rhs)
{
  API_BEGIN
  NOT_NULL(mesh);
  NOT_NULL(value);
  AFEM_REQUIRE(mode == AFEM_NEUMANN_VALUE || mode == AFEM_NEUMANN_NORMAL || mode == AFEM_NEUMANN_TRACTION, AFEM_ERR_ARG,
               "applyNeumannToRhs: unknown mode");
  AFEM_REQUIRE(nb_dof >= 1 && nb_dof <= 3, AFEM_ERR_ARG, "applyNeumannToRhs: NB_DOF must be 1, 2 or 3");
  AFEM_REQUIRE(mode == AFEM_NEUMANN_TRACTION || nb_dof == 1, AFEM_ERR_ARG,
               "applyNeumannToRhs: the scalar modes need NB_DOF = 1 (vector data: AFEM_NEUMANN_TRACTION)");
  AFEM_REQUIRE(n_faces >= 0, AFEM_ERR_ARG, "negative face count");
  if (n_faces > 0) {
    NOT_NULL(face_nodes);
    NOT_NULL(rhs);
  }
  mesh->ctx->set_device();
  apply_neumann(*mesh, nb_dof, mode, value, n_faces, face_nodes, face_cells, mem, rhs);
  API_END
}

int afem_ls_apply_boundary_conditions(afem_ls* ls)
{
  API_BEGIN
  AFEM_RANGE("afem: applyBoundaryConditions");
  NOT_NULL(ls);
  Ctx& ctx = *ls->ctx;
  ctx.set_device();
  if (!ls->has_csr && (!ls->add_map.empty() || !ls->set_map.empty())) ls_build_from_host_coo(*ls);
  const bool host_view = ls->hv_vals && ls->has_csr && !ls->csr_from_coo && ls->csr_nnz > 0;
  if (host_view)  // the live host view (as afem_ls_solve reads it)
    AFEM_HIP(hipMemcpyAsync(ls->own_vals.p, ls->hv_vals, (size_t)ls->csr_nnz * 8, hipMemcpyHostToDevice, ctx.stream));
  const bool mapped = ls->mv_vals && ls->has_csr && !ls->csr_from_coo;
  if (mapped) ls_mapped_gather(*ls);
  ls_apply_bcs(*ls);
  if (mapped) ls_mapped_scatter_back(*ls);  // into the caller's view, as for a host view below
  if (host_view) {
    // Hypre applies the forced values to the view's own values
    // (femutils/HypreDoFLinearSystem.cc:319-382): write them back, so the
    // re-read at solve() sees the eliminated rows / columns and the second
    // pass there is a no-op (the right-hand side is not corrected twice)
    AFEM_HIP(hipMemcpyAsync(ls->hv_vals, ls->own_vals.p, (size_t)ls->csr_nnz * 8, hipMemcpyDeviceToHost, ctx.stream));
    ctx.sync();
  }
  API_END
}

int afem_ls_clear_values(afem_ls* ls)
{
  API_BEGIN
  NOT_NULL(ls);
  Ctx& ctx = *ls->ctx;
  ctx.set_device();
  ls->has_csr = false;
  ls->csr_from_coo = false;
  ls->csr_rows = nullptr;
  ls->csr_diag = nullptr;
  ls->blk_k = 0;
  ls->mg_k = 0;
  ls->mg.reset();
  ls->amg.reset();
  ls->csr_cols = nullptr;
  ls->csr_vals = nullptr;
  ls->hv_rows = nullptr;
  ls->hv_cols = nullptr;
  ls->hv_vals = nullptr;
  ls->mv_vals = nullptr;
  ls->add_map.clear();
  ls->set_map.clear();
  ls->host_elim.clear();
  AFEM_HIP(hipMemsetAsync(ls->forced_info.p, 0, ls->forced_info.bytes(), ctx.stream));
  AFEM_HIP(hipMemsetAsync(ls->elim_info.p, 0, ls->elim_info.bytes(), ctx.stream));
  AFEM_HIP(hipMemsetAsync(ls->elim_value.p, 0, ls->elim_value.bytes(), ctx.stream));
  ctx.sync();
  API_END
}

int afem_ls_solve(afem_ls* ls, afem_solve_stats* st)
{
  API_BEGIN
  AFEM_RANGE("afem: DoFLinearSystem::solve");
  NOT_NULL(ls);
  if (ls->hv_vals && ls->has_csr && !ls->csr_from_coo && ls->csr_nnz > 0) {
    // host view: the values as they are now (the module may have edited its
    // view since setCSRValues; Hypre reads the live view at solve,
    // femutils/HypreDoFLinearSystem.cc:148-156, 587-599)
    ls->ctx->set_device();
    AFEM_HIP(hipMemcpyAsync(ls->own_vals.p, ls->hv_vals, (size_t)ls->csr_nnz * 8, hipMemcpyHostToDevice,
                            ls->ctx->stream));
  }
  if (ls->mv_vals && ls->has_csr && !ls->csr_from_coo) {
    // a mapped device view: its values as they are now (same contract)
    ls->ctx->set_device();
    ls_mapped_gather(*ls);
  }
  ls_solve(*ls, st);
  API_END
}

int afem_ls_spmv(afem_ls* ls, const double* x, double* y)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(x);
  NOT_NULL(y);
  ls->ctx->set_device();
  ls_spmv(*ls, x, y);
  API_END
}

int afem_vec_lincomb(afem_ctx* ctx, int64_t n, double a, const double* x, double b, const double* y, double c,
                     const double* z, double* out)
{
  API_BEGIN
  NOT_NULL(ctx);
  AFEM_REQUIRE(n == 0 || (x && y && out), AFEM_ERR_ARG, "afem_vec_lincomb: x, y and out must not be NULL");
  ctx->set_device();
  vec_lincomb(*ctx, n, a, x, b, y, c, z, out);
  API_END
}

int afem_newmark_update(afem_ctx* ctx, int64_t n, double dt, double beta, double gamma, const double* u_new, double* u,
                        double* v, double* a)
{
  API_BEGIN
  NOT_NULL(ctx);
  AFEM_REQUIRE(n == 0 || (u_new && u && v && a), AFEM_ERR_ARG, "afem_newmark_update: NULL state array");
  AFEM_REQUIRE(dt > 0.0 && beta > 0.0, AFEM_ERR_ARG, "afem_newmark_update: dt and beta must be positive");
  ctx->set_device();
  newmark_update(*ctx, n, dt, beta, gamma, u_new, u, v, a);
  API_END
}

int afem_elastodynamics_create(afem_mesh* mesh, afem_comm* comm, const afem_newmark_params* p,
                               const int32_t* fixed_nodes, int64_t n_fixed, int mem, afem_elastodynamics** out)
{
  API_BEGIN
  NOT_NULL(mesh);
  NOT_NULL(p);
  NOT_NULL(out);
  *out = nullptr;
  auto* h = new afem_elastodynamics();
  try {
    h->d = dyn_create(mesh, comm ? comm->c : nullptr, p, fixed_nodes, n_fixed, mem);
  }
  catch (...) {
    delete h;
    throw;
  }
  *out = h;
  API_END
}

int afem_elastodynamics_set_solver_options(afem_elastodynamics* h, const afem_solver_opts* o)
{
  API_BEGIN
  NOT_NULL(h);
  NOT_NULL(o);
  AFEM_REQUIRE(o->method != AFEM_SOLVER_DIRECT, AFEM_ERR_NOT_IMPL, "elastodynamics solves with the Jacobi-PCG");
  AFEM_REQUIRE(o->max_iter >= 0 && o->rtol >= 0 && o->atol >= 0, AFEM_ERR_ARG, "bad solver options");
  AFEM_REQUIRE(o->precond_block == 0 || o->precond_block == 1 || o->precond_block == 3, AFEM_ERR_ARG,
               "precond_block must be 0, 1 or 3");
  AFEM_REQUIRE(o->multigrid >= 0 && o->multigrid <= 2, AFEM_ERR_ARG, "multigrid must be 0, 1 or 2");
  AFEM_REQUIRE(o->amg >= 0 && o->amg <= 2, AFEM_ERR_ARG, "amg must be 0, 1 or 2");
  AFEM_REQUIRE(!(o->amg && o->precond_block == 3), AFEM_ERR_ARG,
               "amg and block Jacobi are alternative preconditioners");
  AFEM_REQUIRE(!(o->multigrid && o->precond_block == 3), AFEM_ERR_ARG,
               "multigrid and block Jacobi are alternative preconditioners");
  h->d->ls.mg.reset();
  h->d->ls.amg.reset();
  h->d->ls.opts = *o;
  h->d->ls.opts.method = AFEM_SOLVER_PCG;
  API_END
}

int afem_elastodynamics_step(afem_elastodynamics* h, afem_solve_stats* st)
{
  API_BEGIN
  AFEM_RANGE("afem: elastodynamics step");
  NOT_NULL(h);
  dyn_step(h->d, st);
  API_END
}

int afem_elastodynamics_set_dirichlet(afem_elastodynamics* h, const int32_t* dofs, const double* values, int64_t n,
                                      int mem)
{
  API_BEGIN
  NOT_NULL(h);
  dyn_set_dirichlet(h->d, dofs, values, n, mem);
  API_END
}

int afem_elastodynamics_set_time_step(afem_elastodynamics* h, double dt)
{
  API_BEGIN
  NOT_NULL(h);
  dyn_set_time_step(h->d, dt);
  API_END
}

int afem_elastodynamics_state(afem_elastodynamics* h, double** u, double** v, double** a)
{
  API_BEGIN
  NOT_NULL(h);
  if (u) *u = h->d->U.p;
  if (v) *v = h->d->V.p;
  if (a) *a = h->d->A.p;
  API_END
}

int afem_elastodynamics_operators(afem_elastodynamics* h, afem_csr_view* lhs, const int64_t** scalar_rows,
                                  const int32_t** scalar_cols, const double** mass_values, double* c)
{
  API_BEGIN
  NOT_NULL(h);
  Elastodynamics* d = h->d;
  if (lhs) {
    lhs->n_block_rows = d->K.s.n_rows;
    lhs->n_block_cols = d->mesh->n_nodes;
    lhs->nnz_blocks = d->K.s.nnz;
    lhs->block_size = 3;
    lhs->ordered_per_block = d->K.order_per_block ? 1 : 0;
    lhs->rows = d->K.s.row_ptr.p;
    lhs->columns = d->K.s.cols.p;
    lhs->values = d->K.values.p;
  }
  if (scalar_rows) *scalar_rows = d->K.csr_rows.p;
  if (scalar_cols) *scalar_cols = d->K.csr_cols.p;
  if (mass_values) *mass_values = d->mvals.p;
  if (c)
    for (int i = 0; i < 11; ++i) c[i] = d->c[i];
  API_END
}

int afem_elastodynamics_profile(afem_elastodynamics* h, int on)
{
  API_BEGIN
  NOT_NULL(h);
  dyn_profile(h->d, on != 0);
  API_END
}

int afem_elastodynamics_step_timing(afem_elastodynamics* h, afem_step_timing* out)
{
  API_BEGIN
  NOT_NULL(h);
  NOT_NULL(out);
  *out = h->d->timing;
  API_END
}

int afem_elastodynamics_destroy(afem_elastodynamics* h)
{
  API_BEGIN
  if (h) {
    dyn_destroy(h->d);
    delete h;
  }
  API_END
}

int afem_ls_destroy(afem_ls* ls)
{
  API_BEGIN
  if (ls) {
    ls->ctx->set_device();
    ls->ctx->sync();
    if (ls->pinned) (void)hipHostFree(ls->pinned);
    for (hipEvent_t e : ls->prof_ev) (void)hipEventDestroy(e);
    delete ls;
  }
  API_END
}

// ------------------------------------------------------------------ communicator
int afem_comm_unique_id(uint8_t id[AFEM_UNIQUE_ID_BYTES])
{
  API_BEGIN
  NOT_NULL(id);
  comm_unique_id(id);
  API_END
}

int afem_comm_create(afem_ctx* ctx, const uint8_t id[AFEM_UNIQUE_ID_BYTES], int nranks, int rank, afem_comm** out)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(id);
  NOT_NULL(out);
  *out = nullptr;
  auto* c = new afem_comm();
  try {
    c->c = comm_create(*ctx, id, nranks, rank);
    c->ctx = ctx;
  }
  catch (...) {
    delete c;
    throw;
  }
  *out = c;
  API_END
}

int afem_comm_create_host(afem_ctx* ctx, int nranks, int rank, const afem_host_transport* t, afem_comm** out)
{
  API_BEGIN
  NOT_NULL(ctx);
  NOT_NULL(t);
  NOT_NULL(out);
  *out = nullptr;
  auto* c = new afem_comm();
  try {
    c->c = comm_create_host(nranks, rank, t);
    c->ctx = ctx;
  }
  catch (...) {
    delete c;
    throw;
  }
  *out = c;
  API_END
}

int afem_comm_destroy(afem_comm* c)
{
  API_BEGIN
  if (c) {
    comm_destroy(c->c);
    delete c;
  }
  API_END
}

int afem_comm_allreduce_sum(afem_comm* c, double* d, int64_t n)
{
  API_BEGIN
  NOT_NULL(c);
  NOT_NULL(d);
  AFEM_REQUIRE(n >= 0, AFEM_ERR_ARG, "negative count");
  c->ctx->set_device();
  comm_allreduce(c->c, *c->ctx, d, n);
  API_END
}

int afem_comm_host_async(afem_comm* comm, int enable)
{
  API_BEGIN
  NOT_NULL(comm);
  comm_set_host_async(comm->c, enable != 0);
  API_END
}

int afem_ls_set_halo(afem_ls* ls, afem_comm* comm, int n_nbr, const int32_t* nbr, const int64_t* send_counts,
                     const int32_t* send_ids, const int64_t* recv_counts, const int32_t* recv_ids)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(comm);
  AFEM_REQUIRE(n_nbr >= 0, AFEM_ERR_ARG, "negative neighbour count");
  int64_t ns = 0, nr = 0;
  for (int i = 0; i < n_nbr; ++i) {
    AFEM_REQUIRE(nbr[i] >= 0 && nbr[i] < comm_nranks(comm->c) && (nbr[i] != comm_rank(comm->c) || comm_self_loop()),
                 AFEM_ERR_ARG, "bad neighbour rank");
    ns += send_counts[i];
    nr += recv_counts[i];
  }
  for (int64_t i = 0; i < ns; ++i)
    AFEM_REQUIRE(send_ids[i] >= 0 && send_ids[i] < ls->n_rows, AFEM_ERR_ARG, "halo send ids must be owned DoFs");
  for (int64_t i = 0; i < nr; ++i)
    AFEM_REQUIRE(recv_ids[i] >= ls->n_rows && recv_ids[i] < ls->n_cols, AFEM_ERR_ARG, "halo recv ids must be ghost DoFs");
  ls->ctx->set_device();
  ls->halo.reset(new Halo());
  halo_setup(*ls->halo, *ls->ctx, comm->c, n_nbr, nbr, send_counts, send_ids, recv_counts, recv_ids);
  API_END
}

int afem_structured_halo_plan(int dim, int n, int nz, int nranks, int rank, int* n_neighbors, int32_t* neighbor_ranks,
                              int64_t* send_counts, int64_t* recv_counts, int32_t* send_ids, int32_t* recv_ids)
{
  API_BEGIN
  NOT_NULL(n_neighbors);
  std::vector<int> nb;
  std::vector<int64_t> sc, rc;
  std::vector<int32_t> si, ri;
  structured_halo_lists(dim, n, nz, nranks, rank, nb, sc, rc, si, ri);
  *n_neighbors = (int)nb.size();
  for (size_t i = 0; i < nb.size(); ++i) {
    if (neighbor_ranks) neighbor_ranks[i] = nb[i];
    if (send_counts) send_counts[i] = sc[i];
    if (recv_counts) recv_counts[i] = rc[i];
  }
  if (send_ids) std::copy(si.begin(), si.end(), send_ids);
  if (recv_ids) std::copy(ri.begin(), ri.end(), recv_ids);
  API_END
}

int afem_ls_set_halo_structured(afem_ls* ls, afem_comm* comm, afem_mesh* mesh)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(comm);
  NOT_NULL(mesh);
  std::vector<int> nb;
  std::vector<int64_t> sc, rc;
  std::vector<int32_t> si, ri;
  if (mesh->part.valid) {  // afem_mesh_create_subdomain
    const SubdomainPlan& P = mesh->part;
    AFEM_REQUIRE(P.nranks == comm_nranks(comm->c) && P.rank == comm_rank(comm->c), AFEM_ERR_ARG,
                 "subdomain rank/nranks differ from the communicator");
    nb = P.nbr;
    sc = P.send_cnt;
    rc = P.recv_cnt;
    si = P.send_ids;
    ri = P.recv_ids;
  }
  else {
    AFEM_REQUIRE(mesh->st.valid, AFEM_ERR_ARG, "mesh is neither a structured slab nor a partitioned subdomain");
    const StructuredInfo& st = mesh->st;
    AFEM_REQUIRE(st.nranks == comm_nranks(comm->c) && st.rank == comm_rank(comm->c), AFEM_ERR_ARG,
                 "mesh slab rank/nranks differ from the communicator");
    structured_halo_lists(st.dim, st.n, st.nz, st.nranks, st.rank, nb, sc, rc, si, ri);
  }
  std::vector<int32_t> nb32(nb.begin(), nb.end());
  AFEM_REQUIRE(mesh->n_own > 0 && ls->n_rows % mesh->n_own == 0, AFEM_ERR_ARG,
               "linear system rows are not a multiple of the mesh's owned nodes");
  const int k = (int)(ls->n_rows / mesh->n_own);
  AFEM_REQUIRE(k >= 1 && k <= 3 && ls->n_cols >= k * mesh->n_nodes, AFEM_ERR_ARG,
               "linear system does not span NB_DOF x (owned + ghost) nodes");
  if (k > 1) expand_dof_lists(k, sc, rc, si, ri);
  ls->ctx->set_device();
  ls->halo.reset(new Halo());
  halo_setup(*ls->halo, *ls->ctx, comm->c, (int)nb.size(), nb32.data(), sc.data(), si.data(), rc.data(), ri.data());
  API_END
}

int afem_ls_set_halo_mesh(afem_ls* ls, afem_comm* comm, afem_mesh* mesh)
{
  return afem_ls_set_halo_structured(ls, comm, mesh);
}

int afem_ls_synchronize(afem_ls* ls, double* x)
{
  API_BEGIN
  NOT_NULL(ls);
  NOT_NULL(x);
  ls->ctx->set_device();
  if (ls->halo) halo_exchange(*ls->halo, *ls->ctx, x);
  API_END
}

}  // extern "C"
