// Element functors of the reference's modules, as device callables for
// afem::generic::assemble_bilinear (include/arcanefem_amd_generic.hpp):
// the module's own arithmetic, evaluated per cell through the mesh views it
// captures (cn_cv.nodeId + in_node_coord of the reference: here the
// cell_node / coords arrays of afem_bsr_assembly_view).
//   PoissonTet4: _computeElementMatrixTetra4Gpu (modules/poisson/FemModule.h:177-186)
//                = volume (dx^dx + dy^dy + dz^dz), gradients of
//                femutils/ArcaneFemFunctionsGpu.h:280-392 (each divides by V6);
//   PoissonTri3: _computeElementMatrixTria3Gpu (modules/poisson/FemModule.h:139-147)
//                = area (dx^dx + dy^dy), the signed-A2 gradients of
//                femutils/ArcaneFemFunctionsGpu.h:218-252;
//   ElasticityTri3: computeElementMatrixTRIA3Gpu (modules/elasticity/FemModule.h:112-152),
//                [lambda d_a,i d_b,j + mu (d_a,j d_b,i + delta_ij d_a.d_b)] / (4 area);
//   ElasticityTet4: its 3D form, vol [lambda g_a,i g_b,j + mu (g_a,j g_b,i + delta_ij g_a.g_b)].
#pragma once
#include <cmath>

#include "arcanefem_amd_generic.hpp"

namespace elements {

using afem::generic::CellAccess;
using afem::generic::FixedMatrix;

struct Tet {
  double x[4][3];
};

__device__ inline Tet load_tet(const CellAccess& a, int32_t c)
{
  Tet t;
  for (int i = 0; i < 4; ++i) {
    const int32_t n = a.node(c, i, 4);
    for (int d = 0; d < 3; ++d) t.x[i][d] = a.x(n, d);
  }
  return t;
}

// Gpu::MeshOperation::computeVolumeTetra4 and FeOperation3D::computeGradient{X,Y,Z}Tetra4
__device__ inline void volume_gradients(const Tet& t, double& vol, double g[4][3])
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

struct PoissonTet4 {
  CellAccess acc;
  __device__ FixedMatrix<4, 4> operator()(int32_t c) const
  {
    double vol, g[4][3];
    volume_gradients(load_tet(acc, c), vol, g);
    FixedMatrix<4, 4> K;
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) K(a, b) = vol * g[a][0] * g[b][0] + vol * g[a][1] * g[b][1] + vol * g[a][2] * g[b][2];
    return K;
  }
};

// Poisson tet4 in the cofactor form (not a module's arithmetic: one
// reciprocal per cell instead of the module's 12 gradient divisions + 1): with
// e_k = x_k - x_0 and c_1 = e_2 x e_3, c_2 = e_3 x e_1, c_3 = e_1 x e_2,
// c_0 = -(c_1 + c_2 + c_3), K_ab = c_a . c_b / (6 |e_1 . c_1|) -- what the
// cell-unit kernel reaches with lean element physics
struct PoissonTet4Lean {
  CellAccess acc;
  __device__ FixedMatrix<4, 4> operator()(int32_t c) const
  {
    const Tet t = load_tet(acc, c);
    double e[3][3];
    for (int k = 0; k < 3; ++k)
      for (int d = 0; d < 3; ++d) e[k][d] = t.x[k + 1][d] - t.x[0][d];
    double cf[4][3];
    for (int k = 0; k < 3; ++k) {
      const double* a = e[(k + 1) % 3];
      const double* b = e[(k + 2) % 3];
      cf[k + 1][0] = a[1] * b[2] - a[2] * b[1];
      cf[k + 1][1] = a[2] * b[0] - a[0] * b[2];
      cf[k + 1][2] = a[0] * b[1] - a[1] * b[0];
    }
    for (int d = 0; d < 3; ++d) cf[0][d] = -(cf[1][d] + cf[2][d] + cf[3][d]);
    const double s = 1.0 / (6.0 * fabs(e[0][0] * cf[1][0] + e[0][1] * cf[1][1] + e[0][2] * cf[1][2]));
    FixedMatrix<4, 4> K;
    for (int a = 0; a < 4; ++a)
      for (int b = a; b < 4; ++b) {
        const double v = s * (cf[a][0] * cf[b][0] + cf[a][1] * cf[b][1] + cf[a][2] * cf[b][2]);
        K(a, b) = v;
        K(b, a) = v;
      }
    return K;
  }
};

struct ElasticityTet4 {
  CellAccess acc;
  double lambda, mu;
  __device__ FixedMatrix<12, 12> operator()(int32_t c) const
  {
    double vol, g[4][3];
    volume_gradients(load_tet(acc, c), vol, g);
    FixedMatrix<12, 12> K;
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) {
        const double gg = g[a][0] * g[b][0] + g[a][1] * g[b][1] + g[a][2] * g[b][2];
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j)
            K(3 * a + i, 3 * b + j) = vol * (lambda * g[a][i] * g[b][j] + mu * (g[a][j] * g[b][i] + (i == j ? gg : 0.0)));
      }
    return K;
  }
};

__device__ inline void tri_grad(const CellAccess& a, int32_t c, double m[3][2], double& A2)
{
  for (int i = 0; i < 3; ++i) {
    const int32_t n = a.node(c, i, 3);
    m[i][0] = a.x(n, 0);
    m[i][1] = a.x(n, 1);
  }
  A2 = (m[1][0] - m[0][0]) * (m[2][1] - m[0][1]) - (m[2][0] - m[0][0]) * (m[1][1] - m[0][1]);
}

struct PoissonTri3 {
  CellAccess acc;
  __device__ FixedMatrix<3, 3> operator()(int32_t c) const
  {
    double m[3][2], A2;
    tri_grad(acc, c, m, A2);
    const double area = fabs(A2) / 2.0;  // computeAreaTria3: |cross| / 2
    const double dx[3] = { (m[1][1] - m[2][1]) / A2, (m[2][1] - m[0][1]) / A2, (m[0][1] - m[1][1]) / A2 };
    const double dy[3] = { (m[2][0] - m[1][0]) / A2, (m[0][0] - m[2][0]) / A2, (m[1][0] - m[0][0]) / A2 };
    FixedMatrix<3, 3> K;
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) K(a, b) = area * dx[a] * dx[b] + area * dy[a] * dy[b];
    return K;
  }
};

struct ElasticityTri3 {
  CellAccess acc;
  double lambda, mu;
  __device__ FixedMatrix<6, 6> operator()(int32_t c) const
  {
    double m[3][2], A2;
    tri_grad(acc, c, m, A2);
    const double area = fabs(A2) / 2.0;
    const double d[3][2] = { { m[1][1] - m[2][1], m[2][0] - m[1][0] },
                             { m[2][1] - m[0][1], m[0][0] - m[2][0] },
                             { m[0][1] - m[1][1], m[1][0] - m[0][0] } };
    FixedMatrix<6, 6> K;
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        const double dd = d[a][0] * d[b][0] + d[a][1] * d[b][1];
        for (int i = 0; i < 2; ++i)
          for (int j = 0; j < 2; ++j)
            K(2 * a + i, 2 * b + j) = (lambda * d[a][i] * d[b][j] + mu * (d[a][j] * d[b][i] + (i == j ? dd : 0.0))) / (4.0 * area);
      }
    return K;
  }
};

}  // namespace elements
