// BSRFormat<NB_DOF>::assembleBilinear(lambda) through libafem's generic
// element-functor entry (include/arcanefem_amd_generic.hpp), compiled with
// hipcc: the module's element functor is a device lambda, exactly as in
// modules/poisson/FemModule.cc:261-272 --
//   k = 1: _computeElementMatrixTetra4Gpu (modules/poisson/FemModule.h:177-186:
//          volume * (dx^dx + dy^dy + dz^dz), with the gradient formulas of
//          femutils/ArcaneFemFunctionsGpu.h:110-122, 280-392);
//   k = 3: the block-3 P1 elasticity element (the 3D form of
//          computeElementMatrixTRIA3Base, modules/elasticity/FemModule.h:112-140:
//          vol * [lambda g_r,i g_b,j + mu (g_r,j g_b,i + delta_ij g_r.g_b)]).
// The same structure is also assembled by the library's fixed-physics
// instance (afem_bsr_assemble_poisson_p1 / _elasticity_p1): both value arrays
// are written for the GPU test (tests/test_gpu_generic.py), which checks them
// against each other and against the oracle per entry.
// usage: generic_assembly <n> <k: 1|3> <layout: block|row> <out.bin>
//   out.bin: int64 n_rows, int64 nnz_blocks, int64 rows[n_rows+1],
//            int32 cols[nnz], float64 generic[nnz*k*k], float64 builtin[nnz*k*k]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "arcanefem_amd.h"
#include "arcanefem_amd_generic.hpp"

#define CHECK(call)                                                           \
  do {                                                                        \
    int rc_ = (call);                                                         \
    if (rc_ != AFEM_OK) {                                                     \
      fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, afem_last_error()); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

namespace {

struct Tet {
  double x[4][3];
};

// the cell's vertices (cn_cv.nodeId + in_node_coord of the reference)
__device__ Tet load_tet(const afem::generic::CellAccess& a, int32_t c)
{
  Tet t;
  for (int i = 0; i < 4; ++i) {
    const int32_t n = a.node(c, i, 4);
    for (int d = 0; d < 3; ++d) t.x[i][d] = a.x(n, d);
  }
  return t;
}

// Gpu::MeshOperation::computeVolumeTetra4 and FeOperation3D::computeGradient{X,Y,Z}Tetra4
__device__ void volume_gradients(const Tet& t, double& vol, double g[4][3])
{
  const double(*m)[3] = t.x;
  double v0[3], v1[3], v2[3];
  for (int d = 0; d < 3; ++d) {
    v0[d] = m[1][d] - m[0][d];
    v1[d] = m[2][d] - m[0][d];
    v2[d] = m[3][d] - m[0][d];
  }
  const double cx = v1[1] * v2[2] - v1[2] * v2[1], cy = v1[2] * v2[0] - v1[0] * v2[2], cz = v1[0] * v2[1] - v1[1] * v2[0];
  const double V6 = fabs(v0[0] * cx + v0[1] * cy + v0[2] * cz);
  vol = V6 / 6.0;
  // x: (y, z) cofactors; y: (z, x); z: (x, y) -- ArcaneFemFunctionsGpu.h:296-299, 341-344, 386-389
  for (int d = 0; d < 3; ++d) {
    const int p = (d + 1) % 3, q = (d + 2) % 3;
    g[0][d] = (m[1][p] * (m[3][q] - m[2][q]) + m[2][p] * (m[1][q] - m[3][q]) + m[3][p] * (m[2][q] - m[1][q])) / V6;
    g[1][d] = (m[0][p] * (m[2][q] - m[3][q]) + m[2][p] * (m[3][q] - m[0][q]) + m[3][p] * (m[0][q] - m[2][q])) / V6;
    g[2][d] = (m[0][p] * (m[3][q] - m[1][q]) + m[1][p] * (m[0][q] - m[3][q]) + m[3][p] * (m[1][q] - m[0][q])) / V6;
    g[3][d] = (m[0][p] * (m[1][q] - m[2][q]) + m[1][p] * (m[2][q] - m[0][q]) + m[2][p] * (m[0][q] - m[1][q])) / V6;
  }
}

int write_out(const char* path, afem_bsr* bsr, int k, const std::vector<double>& gen, const std::vector<double>& bi)
{
  afem_csr_view v;
  CHECK(afem_bsr_view(bsr, &v));
  std::vector<int64_t> rows(v.n_block_rows + 1);
  std::vector<int32_t> cols(v.nnz_blocks);
  std::vector<double> tmp(v.nnz_blocks * k * k);
  CHECK(afem_bsr_download(bsr, rows.data(), cols.data(), tmp.data()));
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  const int64_t hdr[2] = { v.n_block_rows, v.nnz_blocks };
  fwrite(hdr, sizeof(hdr), 1, f);
  fwrite(rows.data(), 8, rows.size(), f);
  fwrite(cols.data(), 4, cols.size(), f);
  fwrite(gen.data(), 8, gen.size(), f);
  fwrite(bi.data(), 8, bi.size(), f);
  fclose(f);
  return 0;
}

}  // namespace

int main(int argc, char** argv)
{
  if (argc < 5) {
    fprintf(stderr, "usage: %s <n> <k: 1|3> <layout: block|row> <out.bin>\n", argv[0]);
    return 2;
  }
  const int n = atoi(argv[1]), k = atoi(argv[2]);
  const int per_row = argv[3][0] == 'r';  // BSRFormat::initialize(use_csr_in_linear_system)
  if (k != 1 && k != 3) return 2;
  afem_ctx* ctx = nullptr;
  afem_mesh* mesh = nullptr;
  afem_bsr* bsr = nullptr;
  CHECK(afem_ctx_create(0, nullptr, &ctx));
  CHECK(afem_mesh_create_structured(ctx, 3, n, 0, 0.2, 20250220ull, 1, 0, &mesh));
  CHECK(afem_bsr_create(mesh, k, per_row, &bsr));
  CHECK(afem_bsr_compute_sparsity(bsr));
  afem_assembly_view av;
  CHECK(afem_bsr_assembly_view(bsr, &av));
  const afem::generic::CellAccess acc{ av.cell_node, av.coords };
  const double E = 21.0e5, nu = 0.28;
  const double lambda = E * nu / ((1 + nu) * (1 - 2 * nu)), mu = E / (2 * (1 + nu));
  // the module's lambdas (capturing the geometry views by value)
  CHECK(afem_bsr_reset_values(bsr));
  if (k == 1) {
    CHECK((afem::generic::assemble_bilinear<4, 1>(bsr, [=] __device__(int32_t c) {
      double vol, g[4][3];
      volume_gradients(load_tet(acc, c), vol, g);
      afem::generic::FixedMatrix<4, 4> K;
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) K(a, b) = vol * g[a][0] * g[b][0] + vol * g[a][1] * g[b][1] + vol * g[a][2] * g[b][2];
      return K;
    })));
  }
  else {
    CHECK((afem::generic::assemble_bilinear<4, 3>(bsr, [=] __device__(int32_t c) {
      double vol, g[4][3];
      volume_gradients(load_tet(acc, c), vol, g);
      afem::generic::FixedMatrix<12, 12> K;
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) {
          const double gg = g[a][0] * g[b][0] + g[a][1] * g[b][1] + g[a][2] * g[b][2];
          for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
              K(3 * a + i, 3 * b + j) = vol * (lambda * g[a][i] * g[b][j] + mu * (g[a][j] * g[b][i] + (i == j ? gg : 0.0)));
        }
      return K;
    })));
  }
  afem_csr_view v;
  CHECK(afem_bsr_view(bsr, &v));
  const size_t nv = (size_t)v.nnz_blocks * k * k;
  std::vector<double> gen(nv), bi(nv);
  CHECK(afem_memcpy(ctx, gen.data(), v.values, nv * 8, AFEM_MEM_HOST, AFEM_MEM_DEVICE));
  // the library's fixed-physics instance on the same structure
  if (k == 1)
    CHECK(afem_bsr_assemble_poisson_p1(bsr, 1.0, 0.0, nullptr));
  else
    CHECK(afem_bsr_assemble_elasticity_p1_ex(bsr, lambda, 2.0 * mu, 0.0, nullptr, nullptr, AFEM_RHS_ADD));
  CHECK(afem_memcpy(ctx, bi.data(), v.values, nv * 8, AFEM_MEM_HOST, AFEM_MEM_DEVICE));
  double mx = 0.0, d = 0.0;
  for (size_t i = 0; i < nv; ++i) {
    mx = fmax(mx, fabs(bi[i]));
    d = fmax(d, fabs(gen[i] - bi[i]));
  }
  if (write_out(argv[4], bsr, k, gen, bi)) return 1;
  printf("generic_assembly n=%d k=%d rows=%lld nnz_blocks=%lld max|generic-builtin|/max = %.3e\n", n, k,
         (long long)v.n_block_rows, (long long)v.nnz_blocks, d / mx);
  CHECK(afem_bsr_destroy(bsr));
  CHECK(afem_mesh_destroy(mesh));
  CHECK(afem_ctx_destroy(ctx));
  return 0;
}
