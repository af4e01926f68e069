// Neumann / traction right-hand side on boundary faces (K15 of SURVEY.md §2.4):
// femutils/ArcaneFemFunctionsGpu.h:612-674 (BoundaryConditions2D::applyNeumannToRhs),
// :703-766 (BoundaryConditions3D::applyNeumannToRhs) and the vector traction of
// modules/elasticity/FemModule.cc:244-273.  One lane per face; the face's
// owned nodes receive their share with f64 atomics (a boundary group is
// O(N^(2/3)) faces: the launch is negligible next to the assembly).
#include "afem_internal.hpp"

namespace afem {
namespace {

__global__ void k_neumann(int dim, int64_t n_own, int k, int mode, double v0, double v1, double v2, int64_t n_faces,
                          const int32_t* __restrict__ face_nodes, const int32_t* __restrict__ face_cells, int nv,
                          const int32_t* __restrict__ cell_node, const double* __restrict__ coords,
                          double* __restrict__ rhs)
{
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n_faces) return;
  const int nf = dim;  // nodes per face: edge (2D) or triangle (3D)
  int32_t fn[3];
  for (int a = 0; a < nf; ++a) fn[a] = face_nodes[(int64_t)nf * f + a];
  const double* m0 = coords + 3 * (int64_t)fn[0];
  const double* m1 = coords + 3 * (int64_t)fn[1];
  double meas, nx, ny, nz = 0.0;
  if (dim == 2) {  // computeLengthFace / computeNormalFace (femutils/ArcaneFemFunctionsGpu.h:130-160)
    meas = sqrt((m1[0] - m0[0]) * (m1[0] - m0[0]) + (m1[1] - m0[1]) * (m1[1] - m0[1]));
    nx = (m1[1] - m0[1]) / meas;
    ny = (m0[0] - m1[0]) / meas;
  }
  else {  // computeAreaTria / computeNormalTriangle (:88-96, :172-196)
    const double* m2 = coords + 3 * (int64_t)fn[2];
    const double e1x = m1[0] - m0[0], e1y = m1[1] - m0[1], e1z = m1[2] - m0[2];
    const double e2x = m2[0] - m0[0], e2y = m2[1] - m0[1], e2z = m2[2] - m0[2];
    const double cx = e1y * e2z - e1z * e2y, cy = e1z * e2x - e1x * e2z, cz = e1x * e2y - e1y * e2x;
    const double nrm = sqrt(cx * cx + cy * cy + cz * cz);
    meas = nrm / 2.0;
    nx = cx / nrm;
    ny = cy / nrm;
    nz = cz / nrm;
  }
  if (mode == AFEM_NEUMANN_NORMAL && face_cells) {
    // the reference flips the normal of a face that is not
    // isSubDomainBoundaryOutside(): the outward normal, i.e. pointing away from
    // the centroid of the face's cell
    const int32_t* cn = cell_node + (int64_t)nv * face_cells[f];
    double s = 0.0;
    for (int d = 0; d < dim; ++d) {
      double fc = 0.0, cc = 0.0;
      for (int a = 0; a < nf; ++a) fc += coords[3 * (int64_t)fn[a] + d];
      for (int a = 0; a < nv; ++a) cc += coords[3 * (int64_t)cn[a] + d];
      s += (d == 0 ? nx : (d == 1 ? ny : nz)) * (fc / nf - cc / nv);
    }
    if (s < 0.0) {
      nx = -nx;
      ny = -ny;
      nz = -nz;
    }
  }
  for (int a = 0; a < nf; ++a) {
    const int32_t node = fn[a];
    if (node >= n_own) continue;  // nodes_infos.isOwn(node_lid)
    if (mode == AFEM_NEUMANN_VALUE) {
      atomicAdd(rhs + (int64_t)k * node, v0 * meas / nf);
    }
    else if (mode == AFEM_NEUMANN_NORMAL) {
      const double vn = dim == 2 ? nx * v0 + ny * v1 : nx * v0 + ny * v1 + nz * v2;
      atomicAdd(rhs + (int64_t)k * node, vn * meas / nf);
    }
    else {
      for (int i = 0; i < k; ++i) atomicAdd(rhs + (int64_t)k * node + i, (i == 0 ? v0 : (i == 1 ? v1 : v2)) * meas / nf);
    }
  }
}

}  // namespace

void apply_neumann(Mesh& m, int k, int mode, const double* v, int64_t n_faces, const int32_t* face_nodes,
                   const int32_t* face_cells, int mem, double* rhs)
{
  Ctx& ctx = *m.ctx;
  if (n_faces <= 0) return;
  const int nf = m.dim;
  const int32_t* dfn = face_nodes;
  const int32_t* dfc = face_cells;
  DevBuf<int32_t> tfn, tfc;
  if (mem == AFEM_MEM_HOST) {
    for (int64_t i = 0; i < n_faces * nf; ++i)
      AFEM_REQUIRE(face_nodes[i] >= 0 && face_nodes[i] < m.n_nodes, AFEM_ERR_ARG, "face_nodes holds an out-of-range node id");
    if (face_cells)
      for (int64_t i = 0; i < n_faces; ++i)
        AFEM_REQUIRE(face_cells[i] >= 0 && face_cells[i] < m.n_cells, AFEM_ERR_ARG, "face_cells holds an out-of-range cell id");
    tfn.alloc(n_faces * nf);
    AFEM_HIP(hipMemcpyAsync(tfn.p, face_nodes, tfn.bytes(), hipMemcpyHostToDevice, ctx.stream));
    dfn = tfn.p;
    if (face_cells) {
      tfc.alloc(n_faces);
      AFEM_HIP(hipMemcpyAsync(tfc.p, face_cells, tfc.bytes(), hipMemcpyHostToDevice, ctx.stream));
      dfc = tfc.p;
    }
  }
  hipLaunchKernelGGL(k_neumann, dim3((unsigned)((n_faces + 255) / 256)), dim3(256), 0, ctx.stream, m.dim, m.n_own, k,
                     mode, v[0], v[1], v[2], n_faces, dfn, dfc, m.nv, m.cell_node.p, m.coords.p, rhs);
  AFEM_LAUNCHED();
  if (tfn.p) ctx.sync();  // the staging copies die with this scope
}

}  // namespace afem
