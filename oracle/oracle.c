/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C, single-threaded restatement of the reference (toutane/arcanefem @
 * 2025-02-20) algorithms on the FEM assembly + solve hot path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product path
 * (arcanefem_amd/libafem.so) never links, loads or calls it.
 *
 * Pinning: the reference cannot be built here (Arcane 3.14.14, .NET, Hypre,
 * PETSc and MPI are absent), so this restatement is pinned by
 * the reference's own golden result files (tests/golden/<case>.txt replayed on the
 * reference's own meshes tests/golden/<mesh>.msh, see tests/test_oracle_golden.py).
 *
 * Every function names the reference lines it follows.  Compiled with
 * -ffp-contract=off so that no FMA contraction changes the rounding of the
 * restated expressions.
 */
#ifdef _OPENMP
#include <omp.h>
#endif
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Element matrices                                                          */
/* ------------------------------------------------------------------------ */

/* Tetrahedron volume: femutils/ArcaneFemFunctionsGpu.h:110-122
 * (computeVolumeTetra4): |dot(v1-v0, cross(v2-v0, v3-v0))| / 6. */
static double tet_volume(const double* c0, const double* c1, const double* c2, const double* c3)
{
  double v0x = c1[0] - c0[0], v0y = c1[1] - c0[1], v0z = c1[2] - c0[2];
  double v1x = c2[0] - c0[0], v1y = c2[1] - c0[1], v1z = c2[2] - c0[2];
  double v2x = c3[0] - c0[0], v2y = c3[1] - c0[1], v2z = c3[2] - c0[2];
  double cx = v1y * v2z - v1z * v2y;
  double cy = v1z * v2x - v1x * v2z;
  double cz = v1x * v2y - v1y * v2x;
  return fabs(v0x * cx + v0y * cy + v0z * cz) / 6.0;
}

/* P1 tetrahedron stiffness K = V (dx^dx + dy^dy + dz^dz):
 * modules/poisson/FemModule.h:177-186 (_computeElementMatrixTetra4Gpu) with the
 * gradients of femutils/ArcaneFemFunctionsGpu.h:280-392 (computeGradient{X,Y,Z}Tetra4)
 * and operator^ / FixedMatrix of femutils/FemUtils.h:191-226. */
void orc_element_tet4(const double* xyz /* [4][3] */, double* K /* [16] */, double* vol_out)
{
  const double *m0 = xyz, *m1 = xyz + 3, *m2 = xyz + 6, *m3 = xyz + 9;
  double V6; /* 6 x Volume, as computed in computeGradient{X,Y,Z}Tetra4 */
  {
    double v0x = m1[0] - m0[0], v0y = m1[1] - m0[1], v0z = m1[2] - m0[2];
    double v1x = m2[0] - m0[0], v1y = m2[1] - m0[1], v1z = m2[2] - m0[2];
    double v2x = m3[0] - m0[0], v2y = m3[1] - m0[1], v2z = m3[2] - m0[2];
    double cx = v1y * v2z - v1z * v2y, cy = v1z * v2x - v1x * v2z, cz = v1x * v2y - v1y * v2x;
    V6 = fabs(v0x * cx + v0y * cy + v0z * cz);
  }
  double vol = tet_volume(m0, m1, m2, m3);
  double dx[4], dy[4], dz[4];
  dx[0] = (m1[1] * (m3[2] - m2[2]) + m2[1] * (m1[2] - m3[2]) + m3[1] * (m2[2] - m1[2])) / V6;
  dx[1] = (m0[1] * (m2[2] - m3[2]) + m2[1] * (m3[2] - m0[2]) + m3[1] * (m0[2] - m2[2])) / V6;
  dx[2] = (m0[1] * (m3[2] - m1[2]) + m1[1] * (m0[2] - m3[2]) + m3[1] * (m1[2] - m0[2])) / V6;
  dx[3] = (m0[1] * (m1[2] - m2[2]) + m1[1] * (m2[2] - m0[2]) + m2[1] * (m0[2] - m1[2])) / V6;
  dy[0] = (m1[2] * (m3[0] - m2[0]) + m2[2] * (m1[0] - m3[0]) + m3[2] * (m2[0] - m1[0])) / V6;
  dy[1] = (m0[2] * (m2[0] - m3[0]) + m2[2] * (m3[0] - m0[0]) + m3[2] * (m0[0] - m2[0])) / V6;
  dy[2] = (m0[2] * (m3[0] - m1[0]) + m1[2] * (m0[0] - m3[0]) + m3[2] * (m1[0] - m0[0])) / V6;
  dy[3] = (m0[2] * (m1[0] - m2[0]) + m1[2] * (m2[0] - m0[0]) + m2[2] * (m0[0] - m1[0])) / V6;
  dz[0] = (m1[0] * (m3[1] - m2[1]) + m2[0] * (m1[1] - m3[1]) + m3[0] * (m2[1] - m1[1])) / V6;
  dz[1] = (m0[0] * (m2[1] - m3[1]) + m2[0] * (m3[1] - m0[1]) + m3[0] * (m0[1] - m2[1])) / V6;
  dz[2] = (m0[0] * (m3[1] - m1[1]) + m1[0] * (m0[1] - m3[1]) + m3[0] * (m1[1] - m0[1])) / V6;
  dz[3] = (m0[0] * (m1[1] - m2[1]) + m1[0] * (m2[1] - m0[1]) + m2[0] * (m0[1] - m1[1])) / V6;
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b)
      K[4 * a + b] = vol * (dx[a] * dx[b]) + vol * (dy[a] * dy[b]) + vol * (dz[a] * dz[b]);
  if (vol_out)
    *vol_out = vol;
}

/* P1 triangle stiffness K = A (dx^dx + dy^dy):
 * modules/poisson/FemModule.h:139-147 (_computeElementMatrixTria3Gpu),
 * area femutils/ArcaneFemFunctionsGpu.h:75-83 (|cross|/2), gradients
 * femutils/ArcaneFemFunctionsGpu.h:218-252 (signed A2). */
void orc_element_tri3(const double* xyz /* [3][3] */, double* K /* [9] */, double* area_out)
{
  const double *v0 = xyz, *v1 = xyz + 3, *v2 = xyz + 6;
  double ax = v1[0] - v0[0], ay = v1[1] - v0[1], az = v1[2] - v0[2];
  double bx = v2[0] - v0[0], by = v2[1] - v0[1], bz = v2[2] - v0[2];
  double cx = ay * bz - az * by, cy = az * bx - ax * bz, cz = ax * by - ay * bx;
  double area = sqrt(cx * cx + cy * cy + cz * cz) / 2.0;
  double A2 = (v1[0] - v0[0]) * (v2[1] - v0[1]) - (v2[0] - v0[0]) * (v1[1] - v0[1]);
  double dx[3] = { (v1[1] - v2[1]) / A2, (v2[1] - v0[1]) / A2, (v0[1] - v1[1]) / A2 };
  double dy[3] = { (v2[0] - v1[0]) / A2, (v0[0] - v2[0]) / A2, (v1[0] - v0[0]) / A2 };
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b)
      K[3 * a + b] = area * (dx[a] * dx[b]) + area * (dy[a] * dy[b]);
  if (area_out)
    *area_out = area;
}

/* ------------------------------------------------------------------------ */
/* Sparsity: femutils/BSRFormat.h:583-770 (computeSparsityAtomic)            */
/* ------------------------------------------------------------------------ */

static int cmp_u64(const void* a, const void* b)
{
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return (x > y) - (x < y);
}
static int cmp_i32(const void* a, const void* b)
{
  int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
  return (x > y) - (x < y);
}

/* pack/unpack: femutils/BSRFormat.h:583-597 */
static uint64_t pack_edge(int32_t n0, int32_t n1)
{
  int32_t mn = n0 > n1 ? n1 : n0, mx = n0 > n1 ? n0 : n1;
  return ((uint64_t)(uint32_t)mn << 32) | (uint64_t)(uint32_t)mx;
}

/* Builds the node-node (via edges) scalar structure of `n_rows` rows: row r
 * holds r itself plus every node sharing an edge with it
 * (computeSortedEdges :602-651, computeNeighbors :656-672, computeRowIndex
 * :677-688, computeColumns :703-744).  Rows are restricted to r < n_rows (the
 * owned nodes; ghost rows are not materialised).  Unlike the reference (whose
 * atomic column fill leaves the order run-dependent, doc/BSRFormat.md:86-89)
 * the columns of each row are emitted in ascending order: this is the
 * canonical form the GPU path is compared against.
 * Two calls: cols==NULL returns nnz and fills row_ptr[n_rows+1]; the second
 * call fills cols[nnz]. */
int64_t orc_sparsity(int64_t n_nodes, int64_t n_rows, int64_t n_cells, int nv, const int32_t* cell_node,
                     int64_t* row_ptr, int32_t* cols)
{
  int epc = (nv == 3) ? 3 : 6; /* edges per element (:757) */
  int64_t ne = n_cells * epc;
  uint64_t* edges = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(ne > 0 ? ne : 1));
  for (int64_t c = 0; c < n_cells; ++c) {
    const int32_t* n = cell_node + c * nv;
    uint64_t* e = edges + c * epc;
    if (nv == 3) {
      e[0] = pack_edge(n[0], n[1]);
      e[1] = pack_edge(n[0], n[2]);
      e[2] = pack_edge(n[1], n[2]);
    }
    else {
      e[0] = pack_edge(n[0], n[1]);
      e[1] = pack_edge(n[0], n[2]);
      e[2] = pack_edge(n[0], n[3]);
      e[3] = pack_edge(n[1], n[2]);
      e[4] = pack_edge(n[1], n[3]);
      e[5] = pack_edge(n[2], n[3]);
    }
  }
  qsort(edges, (size_t)ne, sizeof(uint64_t), cmp_u64);
  /* neighbors initialised to 1 (the diagonal, :679) */
  int64_t* cnt = (int64_t*)calloc((size_t)n_nodes + 1, sizeof(int64_t));
  for (int64_t r = 0; r < n_rows; ++r)
    cnt[r] = 1;
  for (int64_t t = 0; t < ne; ++t) {
    if (t == ne - 1 || edges[t] != edges[t + 1]) {
      int32_t n0 = (int32_t)(edges[t] >> 32), n1 = (int32_t)(edges[t] & 0xFFFFFFFFu);
      if (n0 < n_rows)
        cnt[n0]++;
      if (n1 < n_rows)
        cnt[n1]++;
    }
  }
  row_ptr[0] = 0;
  for (int64_t r = 0; r < n_rows; ++r)
    row_ptr[r + 1] = row_ptr[r] + cnt[r];
  int64_t nnz = row_ptr[n_rows];
  if (cols) {
    for (int64_t r = 0; r < n_rows; ++r) {
      cols[row_ptr[r]] = (int32_t)r; /* diagonal first, :712-717 */
      cnt[r] = 1;
    }
    for (int64_t t = 0; t < ne; ++t) {
      if (t == ne - 1 || edges[t] != edges[t + 1]) {
        int32_t n0 = (int32_t)(edges[t] >> 32), n1 = (int32_t)(edges[t] & 0xFFFFFFFFu);
        if (n0 < n_rows)
          cols[row_ptr[n0] + cnt[n0]++] = n1;
        if (n1 < n_rows)
          cols[row_ptr[n1] + cnt[n1]++] = n0;
      }
    }
    for (int64_t r = 0; r < n_rows; ++r)
      qsort(cols + row_ptr[r], (size_t)(row_ptr[r + 1] - row_ptr[r]), sizeof(int32_t), cmp_i32);
  }
  free(cnt);
  free(edges);
  return nnz;
}

/* ------------------------------------------------------------------------ */
/* Assembly: femutils/BSRFormat.h:786-837 (assembleBilinearOrderedPerBlock)   */
/* with NB_DOF = 1: cell loop, owned-row filter, linear column search, add.   */
/* The RHS source term of femutils/ArcaneFemFunctionsGpu.h:401-429            */
/* (applyConstantSourceToRhsBase: rhs[dof] += f*|K|/nbNode for own nodes) is  */
/* done in the same cell loop when rhs != NULL.                               */
/* Returns the number of (row,col) pairs not found in the structure.          */
/* ------------------------------------------------------------------------ */
int64_t orc_assemble_poisson(int64_t n_rows, int64_t n_cells, int nv, const int32_t* cell_node, const double* coords,
                             const int64_t* row_ptr, const int32_t* cols, double* vals, double f, double* rhs)
{
  int64_t missing = 0;
  double xyz[12], K[16], meas;
  for (int64_t c = 0; c < n_cells; ++c) {
    const int32_t* n = cell_node + c * nv;
    for (int a = 0; a < nv; ++a) {
      xyz[3 * a + 0] = coords[3 * (int64_t)n[a] + 0];
      xyz[3 * a + 1] = coords[3 * (int64_t)n[a] + 1];
      xyz[3 * a + 2] = coords[3 * (int64_t)n[a] + 2];
    }
    if (nv == 4)
      orc_element_tet4(xyz, K, &meas);
    else
      orc_element_tri3(xyz, K, &meas);
    for (int a = 0; a < nv; ++a) {
      int32_t row = n[a];
      if (row >= n_rows)
        continue; /* nodes_infos.isOwn(row_node_lid) (:815) */
      for (int b = 0; b < nv; ++b) {
        int32_t col = n[b];
        int64_t k = row_ptr[row], end = row_ptr[row + 1];
        while (k < end && cols[k] != col)
          ++k;
        if (k == end) {
          ++missing;
          continue;
        }
        vals[k] += K[nv * a + b];
      }
      if (rhs)
        rhs[row] += f * meas / nv;
    }
  }
  return missing;
}

/* The same cell loop run on all host threads, as the reference runs it on a
 * multi-core host (the RUNCOMMAND cell loop of BSRFormat::assembleBilinearAtomic,
 * femutils/BSRFormat.h:786-837, with Accelerator::doAtomic adds): cells split
 * over OpenMP threads, every add atomic.  Used only for bench.py's multi-core
 * CPU baseline (summation order is run-dependent, as in the reference). */
int orc_omp_threads(int n)
{
#ifdef _OPENMP
  if (n > 0)
    omp_set_num_threads(n);
  return omp_get_max_threads();
#else
  (void)n;
  return 1;
#endif
}

int64_t orc_assemble_poisson_omp(int64_t n_rows, int64_t n_cells, int nv, const int32_t* cell_node,
                                 const double* coords, const int64_t* row_ptr, const int32_t* cols, double* vals,
                                 double f, double* rhs)
{
  int64_t missing = 0;
#pragma omp parallel for schedule(static) reduction(+ : missing)
  for (int64_t c = 0; c < n_cells; ++c) {
    double xyz[12], K[16], meas;
    const int32_t* n = cell_node + c * nv;
    for (int a = 0; a < nv; ++a) {
      xyz[3 * a + 0] = coords[3 * (int64_t)n[a] + 0];
      xyz[3 * a + 1] = coords[3 * (int64_t)n[a] + 1];
      xyz[3 * a + 2] = coords[3 * (int64_t)n[a] + 2];
    }
    if (nv == 4)
      orc_element_tet4(xyz, K, &meas);
    else
      orc_element_tri3(xyz, K, &meas);
    for (int a = 0; a < nv; ++a) {
      int32_t row = n[a];
      if (row >= n_rows)
        continue;
      for (int b = 0; b < nv; ++b) {
        int32_t col = n[b];
        int64_t k = row_ptr[row], end = row_ptr[row + 1];
        while (k < end && cols[k] != col)
          ++k;
        if (k == end) {
          ++missing;
          continue;
        }
#pragma omp atomic
        vals[k] += K[nv * a + b];
      }
      if (rhs) {
#pragma omp atomic
        rhs[row] += f * meas / nv;
      }
    }
  }
  return missing;
}

/* Block (vector) P1 elasticity on triangles, NB_DOF = 2, "ordered per block"
 * BSR values (block_start*4 + i*2 + j, femutils/BSRFormat.h:820-829) with the
 * element matrix of modules/elasticity/FemModule.h:112-140
 * (computeElementMatrixTRIA3Base): K = (lambda*...)+(mu2*...) / (4A) on the
 * [u1,u2]-interleaved 6x6 matrix; mu2 = 2*mu as in modules/elasticity/FemModule.cc:133. */
void orc_element_elasticity_tri3(const double* xyz, double lambda, double mu2, double* K /* [36] */)
{
  const double *m0 = xyz, *m1 = xyz + 3, *m2 = xyz + 6;
  double ax = m1[0] - m0[0], ay = m1[1] - m0[1], az = m1[2] - m0[2];
  double bx = m2[0] - m0[0], by = m2[1] - m0[1], bz = m2[2] - m0[2];
  double cx = ay * bz - az * by, cy = az * bx - ax * bz, cz = ax * by - ay * bx;
  double area = sqrt(cx * cx + cy * cy + cz * cz) / 2.0;
  /* 2A * grad: dPhi0 = (y1-y2, x2-x1) etc. (FemModule.h:118-124) */
  double dPhi0x = m1[1] - m2[1], dPhi0y = m2[0] - m1[0];
  double dPhi1x = m2[1] - m0[1], dPhi1y = m0[0] - m2[0];
  double dPhi2x = m0[1] - m1[1], dPhi2y = m1[0] - m0[0];
  double b[3][6] = {
    { dPhi0x, 0., dPhi1x, 0., dPhi2x, 0. },
    { 0., dPhi0y, 0., dPhi1y, 0., dPhi2y },
    { dPhi0y, dPhi0x, dPhi1y, dPhi1x, dPhi2y, dPhi2x }
  };
  double s = 1.0 / (4.0 * area);
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) {
      double lam = (b[0][i] + b[1][i]) * (b[0][j] + b[1][j]);
      double shr = b[0][i] * b[0][j] + b[1][i] * b[1][j] + 0.5 * b[2][i] * b[2][j];
      K[6 * i + j] = (lambda * lam + mu2 * shr) * s;
    }
}

/* Global block-2 elasticity assembly on triangles, values "ordered per block"
 * (femutils/BSRFormat.h:786-850, assembleBilinearOrderedPerBlock: for every
 * cell, every owned row node a and every node b of the cell, the 2x2 block
 * K[2a+i][2b+j] is added at block_index*4 + i*2 + j).  Returns the number of
 * (row,col) blocks not found in the structure. */
int64_t orc_assemble_elasticity_tri(int64_t n_rows, int64_t n_cells, const int32_t* cell_node, const double* coords,
                                    const int64_t* row_ptr, const int32_t* cols, double lambda, double mu2,
                                    double* vals)
{
  int64_t missing = 0;
  double xyz[9], K[36];
  for (int64_t c = 0; c < n_cells; ++c) {
    const int32_t* n = cell_node + 3 * c;
    for (int a = 0; a < 3; ++a)
      for (int d = 0; d < 3; ++d)
        xyz[3 * a + d] = coords[3 * (int64_t)n[a] + d];
    orc_element_elasticity_tri3(xyz, lambda, mu2, K);
    for (int a = 0; a < 3; ++a) {
      int32_t row = n[a];
      if (row >= n_rows)
        continue;
      for (int b = 0; b < 3; ++b) {
        int64_t k = row_ptr[row], end = row_ptr[row + 1];
        while (k < end && cols[k] != n[b])
          ++k;
        if (k == end) {
          ++missing;
          continue;
        }
        for (int i = 0; i < 2; ++i)
          for (int j = 0; j < 2; ++j)
            vals[4 * k + 2 * i + j] += K[6 * (2 * a + i) + 2 * b + j];
      }
    }
  }
  return missing;
}

/* Block-3 P1 elasticity on tetrahedra (NB_DOF = 3).  No reference module has
 * it (the elasticity module is 2D TRIA3); this is the 3D
 * restatement of computeElementMatrixTRIA3Base (modules/elasticity/FemModule.h:112-140):
 * the same bilinear form lambda*div(u)div(v) + mu2*(eps(u):eps(v)) written with
 * the B matrix of the three normal strains and the three engineering shears
 * (the 2D code's dx/dy rows and its 0.5*shear term), integrated exactly on the
 * P1 tet: K = V * B^T D B with grad N_a = c_a / det, det = 6V signed.
 * Optional consistent mass term (modules/elastodynamics/FemModule.cc:1285-1340,
 * the TRIA3 u1v1/u2v2 blocks: area/12*(1+delta_ab); tetrahedron: V/20*(1+delta_ab))
 * scaled by c0 (rho/(beta dt^2) in the Newmark LHS, :259).  Interleaved dofs
 * [u1x,u1y,u1z,u2x,...], 12x12 row-major. */
void orc_element_elasticity_tet4(const double* xyz, double lambda, double mu2, double c0, double* K /* [144] */)
{
  const double *m0 = xyz, *m1 = xyz + 3, *m2 = xyz + 6, *m3 = xyz + 9;
  double e[3][3];
  for (int d = 0; d < 3; ++d) {
    e[0][d] = m1[d] - m0[d];
    e[1][d] = m2[d] - m0[d];
    e[2][d] = m3[d] - m0[d];
  }
  /* cofactors: c1 = e2 x e3, c2 = e3 x e1, c3 = e1 x e2, c0 = -(c1+c2+c3); det = e1.c1 */
  double c[4][3];
  const int A[3] = { 1, 2, 0 }, B[3] = { 2, 0, 1 };
  for (int d = 0; d < 3; ++d) {
    c[1][d] = e[1][A[d]] * e[2][B[d]] - e[1][B[d]] * e[2][A[d]];
    c[2][d] = e[2][A[d]] * e[0][B[d]] - e[2][B[d]] * e[0][A[d]];
    c[3][d] = e[0][A[d]] * e[1][B[d]] - e[0][B[d]] * e[1][A[d]];
    c[0][d] = -(c[1][d] + c[2][d] + c[3][d]);
  }
  const double det = e[0][0] * c[1][0] + e[0][1] * c[1][1] + e[0][2] * c[1][2];
  const double vol = fabs(det) / 6.0;
  double g[4][3];
  for (int a = 0; a < 4; ++a)
    for (int d = 0; d < 3; ++d)
      g[a][d] = c[a][d] / det;
  /* B: 6 strain rows (xx, yy, zz, xy, yz, zx engineering) x 12 dofs */
  double Bm[6][12];
  for (int a = 0; a < 4; ++a) {
    const double gx = g[a][0], gy = g[a][1], gz = g[a][2];
    const double col[3][6] = { { gx, 0., 0., gy, 0., gz }, { 0., gy, 0., gx, gz, 0. }, { 0., 0., gz, 0., gy, gx } };
    for (int i = 0; i < 3; ++i)
      for (int r = 0; r < 6; ++r)
        Bm[r][3 * a + i] = col[i][r];
  }
  for (int p = 0; p < 12; ++p)
    for (int q = 0; q < 12; ++q) {
      const double lam = (Bm[0][p] + Bm[1][p] + Bm[2][p]) * (Bm[0][q] + Bm[1][q] + Bm[2][q]);
      const double shr = Bm[0][p] * Bm[0][q] + Bm[1][p] * Bm[1][q] + Bm[2][p] * Bm[2][q] +
                         0.5 * (Bm[3][p] * Bm[3][q] + Bm[4][p] * Bm[4][q] + Bm[5][p] * Bm[5][q]);
      double v = vol * (lambda * lam + mu2 * shr);
      if (c0 != 0.0 && (p % 3) == (q % 3))
        v += c0 * vol / 20.0 * ((p / 3) == (q / 3) ? 2.0 : 1.0);
      K[12 * p + q] = v;
    }
}

/* Global block-3 assembly on tetrahedra (assembleBilinearOrderedPerBlock,
 * femutils/BSRFormat.h:786-837, with NB_DOF = 3: block_index*9 + i*3 + j) and
 * the vectorial constant source (femutils/ArcaneFemFunctionsGpu.h:514-586:
 * rhs[3n+i] += f_i * V / 4 on owned nodes; f may be NULL). */
int64_t orc_assemble_elasticity_tet(int64_t n_rows, int64_t n_cells, const int32_t* cell_node, const double* coords,
                                    const int64_t* row_ptr, const int32_t* cols, double lambda, double mu2, double c0,
                                    const double* f, double* vals, double* rhs)
{
  int64_t missing = 0;
  double xyz[12], K[144];
  for (int64_t cc = 0; cc < n_cells; ++cc) {
    const int32_t* n = cell_node + 4 * cc;
    for (int a = 0; a < 4; ++a)
      for (int d = 0; d < 3; ++d)
        xyz[3 * a + d] = coords[3 * (int64_t)n[a] + d];
    orc_element_elasticity_tet4(xyz, lambda, mu2, c0, K);
    const double vol = tet_volume(xyz, xyz + 3, xyz + 6, xyz + 9);
    for (int a = 0; a < 4; ++a) {
      const int32_t row = n[a];
      if (row >= n_rows)
        continue;
      if (f && rhs)
        for (int i = 0; i < 3; ++i)
          rhs[3 * (int64_t)row + i] += f[i] * vol / 4.0;
      for (int b = 0; b < 4; ++b) {
        int64_t k = row_ptr[row], end = row_ptr[row + 1];
        while (k < end && cols[k] != n[b])
          ++k;
        if (k == end) {
          ++missing;
          continue;
        }
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j)
            vals[9 * k + 3 * i + j] += K[12 * (3 * a + i) + 3 * b + j];
      }
    }
  }
  return missing;
}

/* ------------------------------------------------------------------------ */
/* Dirichlet via penalty: femutils/ArcaneFemFunctionsGpu.h:434-456 (forced    */
/* info/value, rhs = P*g) then femutils/HypreDoFLinearSystem.cc:356-382       */
/* (_applyForcedValuesToLhs: A[i,i] = P).                                     */
/* ------------------------------------------------------------------------ */
void orc_dirichlet_penalty(int64_t n_dofs, const int32_t* dofs, double value, double penalty, const int64_t* row_ptr,
                           const int32_t* cols, double* vals, double* rhs)
{
  for (int64_t t = 0; t < n_dofs; ++t) {
    int32_t d = dofs[t];
    for (int64_t k = row_ptr[d]; k < row_ptr[d + 1]; ++k)
      if (cols[k] == d)
        vals[k] = penalty;
    rhs[d] = penalty * value;
  }
}

/* Row elimination: femutils/HypreDoFLinearSystem.cc:319-351 */
void orc_row_elimination(int64_t n_dofs, const int32_t* dofs, double value, const int64_t* row_ptr, const int32_t* cols,
                         double* vals, double* rhs)
{
  for (int64_t t = 0; t < n_dofs; ++t) {
    int32_t d = dofs[t];
    for (int64_t k = row_ptr[d]; k < row_ptr[d + 1]; ++k)
      vals[k] = cols[k] == d ? 1.0 : 0.0;
    rhs[d] = value;
  }
}

/* ------------------------------------------------------------------------ */
/* CSR SpMV and Jacobi-preconditioned CG.  Restates the iterative branch of   */
/* SequentialDoFLinearSystemImpl::solve (femutils/DoFLinearSystem.cc:137-151: */
/* DiagonalPreconditioner + ConjugateGradientSolver; the reference starts at   */
/* x0 = 0, here constraint rows start at their Dirichlet value).  Arcane MatVec*/
/* is external and not vendored, so its stopping test is unpinned; this       */
/* oracle stops on sqrt(r.z) <= rtol*sqrt(r0.z0|free) or ||r||_2 <= atol,     */
/* where r0.z0|free sums the non-constraint rows only (see below).            */
/* ------------------------------------------------------------------------ */
void orc_spmv(int64_t n_rows, const int64_t* row_ptr, const int32_t* cols, const double* vals, const double* x, double* y)
{
  for (int64_t r = 0; r < n_rows; ++r) {
    double s = 0.0;
    for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k)
      s += vals[k] * x[cols[k]];
    y[r] = s;
  }
}

static double dot(int64_t n, const double* a, const double* b)
{
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i)
    s += a[i] * b[i];
  return s;
}

/* Returns iterations done; *res_out = final sqrt(r.z)/sqrt(r0.z0);
 * *rnorm_out = ||r||_2. max_iter < 0 means "exactly -max_iter iterations, no
 * stopping test" (fixed-work timing). */
int orc_pcg_jacobi(int64_t n, const int64_t* row_ptr, const int32_t* cols, const double* vals, const double* b,
                   double* x, double rtol, double atol, int max_iter, double* res_out, double* rnorm_out)
{
  int fixed = max_iter < 0;
  if (fixed)
    max_iter = -max_iter;
  double* r = (double*)malloc(sizeof(double) * (size_t)n);
  double* z = (double*)malloc(sizeof(double) * (size_t)n);
  double* p = (double*)malloc(sizeof(double) * (size_t)n);
  double* q = (double*)malloc(sizeof(double) * (size_t)n);
  double* dinv = (double*)malloc(sizeof(double) * (size_t)n);
  /* constraint rows (penalty or eliminated: the diagonal dominates the rest
   * of the row by > 1e10) are excluded from the reference value of the
   * stopping test, otherwise P = 1e30 makes any relative test meaningless */
  unsigned char* constraint = (unsigned char*)malloc((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    double d = 0.0, off = 0.0;
    for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k)
      if (cols[k] == i)
        d += vals[k]; /* duplicate (i,i) entries add up, as the SpMV applies them */
      else
        off += fabs(vals[k]);
    dinv[i] = d != 0.0 ? 1.0 / d : 0.0;
    constraint[i] = fabs(d) > 1e10 * off;
  }
  /* x0: constraint rows solved on their own (the Dirichlet values), 0
   * elsewhere -- lifts the Dirichlet data into x0 (see k_cg_x0). */
  for (int64_t i = 0; i < n; ++i)
    x[i] = constraint[i] ? b[i] * dinv[i] : 0.0;
  orc_spmv(n, row_ptr, cols, vals, x, q);
  double rz0 = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    r[i] = b[i] - q[i];
    z[i] = r[i] * dinv[i];
    p[i] = z[i];
    if (!constraint[i])
      rz0 += r[i] * z[i];
  }
  double rz = dot(n, r, z);
  if (rz0 == 0.0)
    rz0 = rz;
  free(constraint);
  int it = 0;
  double res = rz0 > 0 ? 1.0 : 0.0;
  while (it < max_iter) {
    if (!fixed) {
      if (rz0 == 0.0)
        break;
      res = sqrt(fabs(rz / rz0));
      if (res <= rtol)
        break;
      if (atol > 0 && sqrt(dot(n, r, r)) <= atol)
        break;
    }
    orc_spmv(n, row_ptr, cols, vals, p, q);
    double pq = dot(n, p, q);
    double alpha = rz / pq;
    for (int64_t i = 0; i < n; ++i) {
      x[i] += alpha * p[i];
      r[i] -= alpha * q[i];
      z[i] = r[i] * dinv[i];
    }
    double rz_new = dot(n, r, z);
    double beta = rz_new / rz;
    rz = rz_new;
    for (int64_t i = 0; i < n; ++i)
      p[i] = z[i] + beta * p[i];
    ++it;
  }
  if (res_out)
    *res_out = rz0 > 0 ? sqrt(fabs(rz / rz0)) : 0.0;
  if (rnorm_out)
    *rnorm_out = sqrt(dot(n, r, r));
  free(r);
  free(z);
  free(p);
  free(q);
  free(dinv);
  return it;
}

/* ------------------------------------------------------------------------ */
/* Neumann / traction right-hand side on boundary faces (K15).               */
/*   mode 0 (value):    rhs[k n]   += g |F| / nf                             */
/*                      femutils/ArcaneFemFunctionsGpu.h:636-650 (2D, length/2)*/
/*                      and :731-743 (3D, area/3)                            */
/*   mode 1 (normal):   rhs[k n]   += (v . N) |F| / nf, N outward unit normal */
/*                      :652-672 (2D computeNormalFace, :145-160) and        */
/*                      :745-766 (3D computeNormalTriangle, :172-196)        */
/*   mode 2 (traction): rhs[k n+i] += t_i |F| / nf, i < k                    */
/*                      modules/elasticity/FemModule.cc:244-273              */
/* |F|: 2D edge length in the xy plane (computeLengthFace, :130-137), 3D     */
/* triangle area |cross|/2 (computeAreaTria, :88-96).  Only owned nodes      */
/* (node < n_own) receive a contribution (nodes_infos.isOwn).                */
/* Orientation: the reference swaps the face's first two nodes when the face  */
/* is not isSubDomainBoundaryOutside(), i.e. it uses the outward normal of   */
/* the boundary face; here the outward side is the one away from the         */
/* centroid of the face's cell face_cells[f] (node order as given when       */
/* face_cells is NULL).                                                      */
/* ------------------------------------------------------------------------ */
void orc_neumann(int dim, int64_t n_own, int k, int mode, const double* v, int64_t n_faces, const int32_t* face_nodes,
                 const int32_t* face_cells, int nv, const int32_t* cell_node, const double* coords, double* rhs)
{
  const int nf = dim; /* nodes per face: 2 (edge) or 3 (triangle) */
  for (int64_t f = 0; f < n_faces; ++f) {
    const int32_t* fn = face_nodes + (int64_t)nf * f;
    const double* m0 = coords + 3 * (int64_t)fn[0];
    const double* m1 = coords + 3 * (int64_t)fn[1];
    double meas, N[3] = { 0.0, 0.0, 0.0 };
    if (dim == 2) {
      meas = sqrt((m1[0] - m0[0]) * (m1[0] - m0[0]) + (m1[1] - m0[1]) * (m1[1] - m0[1]));
      N[0] = (m1[1] - m0[1]) / meas;
      N[1] = (m0[0] - m1[0]) / meas;
    }
    else {
      const double* m2 = coords + 3 * (int64_t)fn[2];
      double e1[3] = { m1[0] - m0[0], m1[1] - m0[1], m1[2] - m0[2] };
      double e2[3] = { m2[0] - m0[0], m2[1] - m0[1], m2[2] - m0[2] };
      double c[3] = { e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0] };
      double nrm = sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
      meas = nrm / 2.0;
      N[0] = c[0] / nrm;
      N[1] = c[1] / nrm;
      N[2] = c[2] / nrm;
    }
    if (mode == 1 && face_cells) {
      /* outward: N . (face centroid - cell centroid) > 0 */
      const int32_t* cn = cell_node + (int64_t)nv * face_cells[f];
      double s = 0.0;
      for (int d = 0; d < dim; ++d) {
        double fc = 0.0, cc = 0.0;
        for (int a = 0; a < nf; ++a)
          fc += coords[3 * (int64_t)fn[a] + d];
        for (int a = 0; a < nv; ++a)
          cc += coords[3 * (int64_t)cn[a] + d];
        s += N[d] * (fc / nf - cc / nv);
      }
      if (s < 0.0) {
        N[0] = -N[0];
        N[1] = -N[1];
        N[2] = -N[2];
      }
    }
    for (int a = 0; a < nf; ++a) {
      const int32_t node = fn[a];
      if (node >= n_own)
        continue;
      if (mode == 0)
        rhs[(int64_t)k * node] += v[0] * meas / nf;
      else if (mode == 1) {
        double vn = dim == 2 ? N[0] * v[0] + N[1] * v[1] : N[0] * v[0] + N[1] * v[1] + N[2] * v[2];
        rhs[(int64_t)k * node] += vn * meas / nf;
      }
      else {
        for (int i = 0; i < k; ++i)
          rhs[(int64_t)k * node + i] += v[i] * meas / nf;
      }
    }
  }
}

/* ------------------------------------------------------------------------ */
/* Row / row+column elimination with Aleph semantics:                        */
/* femutils/AlephDoFLinearSystem.cc:501-583 (_fillMatrix).                   */
/*   info[d] = 1 (ELIMINATE_ROW) or 2 (ELIMINATE_ROW_COLUMN), value[d] = g.   */
/* Phase 1: for a row+column eliminated row r, every owned column c != r:     */
/*          rhs[c] -= A[r,c] * g_r; entries of row+column eliminated columns  */
/*          are dropped from the other rows.                                  */
/* Phase 2: eliminated rows become identity rows with rhs = g.               */
/* ------------------------------------------------------------------------ */
void orc_eliminate(int64_t n_rows, const uint8_t* info, const double* value, const int64_t* row_ptr,
                   const int32_t* cols, double* vals, double* rhs)
{
  for (int64_t r = 0; r < n_rows; ++r) {
    if (info[r] != 2)
      continue;
    for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
      int32_t c = cols[k];
      if (c == r || c >= n_rows)
        continue;
      rhs[c] = rhs[c] - vals[k] * value[r];
    }
  }
  for (int64_t j = 0; j < n_rows; ++j) {
    if (info[j] != 0)
      continue;
    for (int64_t k = row_ptr[j]; k < row_ptr[j + 1]; ++k)
      if (cols[k] != j && cols[k] < n_rows && info[cols[k]] == 2)
        vals[k] = 0.0;
  }
  for (int64_t d = 0; d < n_rows; ++d) {
    if (info[d] == 0)
      continue;
    for (int64_t k = row_ptr[d]; k < row_ptr[d + 1]; ++k)
      vals[k] = cols[k] == d ? 1.0 : 0.0;
    rhs[d] = value[d];
  }
}

/* ------------------------------------------------------------------------ */
/* OpenMP variant of orc_pcg_jacobi (same iteration, same stopping rule;     */
/* parallel loops with reductions, so the summation order of the dot          */
/* products differs from the serial one).  The BASELINE.md §4 CPU baseline   */
/* "Jacobi-PCG restatement with OpenMP, fixed 50 iterations" and the         */
/* solution-parity reference at >= 1e7 DoF.                                   */
/* ------------------------------------------------------------------------ */
static double dot_omp(int64_t n, const double* a, const double* b)
{
  double s = 0.0;
#pragma omp parallel for reduction(+ : s) schedule(static)
  for (int64_t i = 0; i < n; ++i)
    s += a[i] * b[i];
  return s;
}

static void spmv_omp(int64_t n_rows, const int64_t* row_ptr, const int32_t* cols, const double* vals, const double* x,
                     double* y)
{
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < n_rows; ++r) {
    double s = 0.0;
    for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k)
      s += vals[k] * x[cols[k]];
    y[r] = s;
  }
}

int orc_pcg_jacobi_omp(int64_t n, const int64_t* row_ptr, const int32_t* cols, const double* vals, const double* b,
                       double* x, double rtol, double atol, int max_iter, double* res_out, double* rnorm_out)
{
  int fixed = max_iter < 0;
  if (fixed)
    max_iter = -max_iter;
  double* r = (double*)malloc(sizeof(double) * (size_t)n);
  double* z = (double*)malloc(sizeof(double) * (size_t)n);
  double* p = (double*)malloc(sizeof(double) * (size_t)n);
  double* q = (double*)malloc(sizeof(double) * (size_t)n);
  double* dinv = (double*)malloc(sizeof(double) * (size_t)n);
  unsigned char* constraint = (unsigned char*)malloc((size_t)n);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double d = 0.0, off = 0.0;
    for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k)
      if (cols[k] == i)
        d += vals[k]; /* duplicate (i,i) entries add up, as the SpMV applies them */
      else
        off += fabs(vals[k]);
    dinv[i] = d != 0.0 ? 1.0 / d : 0.0;
    constraint[i] = fabs(d) > 1e10 * off;
    x[i] = constraint[i] ? b[i] * dinv[i] : 0.0;
  }
  spmv_omp(n, row_ptr, cols, vals, x, q);
  double rz0 = 0.0, rz = 0.0;
#pragma omp parallel for reduction(+ : rz0, rz) schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    r[i] = b[i] - q[i];
    z[i] = r[i] * dinv[i];
    p[i] = z[i];
    rz += r[i] * z[i];
    if (!constraint[i])
      rz0 += r[i] * z[i];
  }
  if (rz0 == 0.0)
    rz0 = rz;
  free(constraint);
  int it = 0;
  while (it < max_iter) {
    if (!fixed) {
      if (rz0 == 0.0 || sqrt(fabs(rz / rz0)) <= rtol)
        break;
      if (atol > 0 && sqrt(dot_omp(n, r, r)) <= atol)
        break;
    }
    spmv_omp(n, row_ptr, cols, vals, p, q);
    const double alpha = rz / dot_omp(n, p, q);
    double rz_new = 0.0;
#pragma omp parallel for reduction(+ : rz_new) schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      x[i] += alpha * p[i];
      r[i] -= alpha * q[i];
      z[i] = r[i] * dinv[i];
      rz_new += r[i] * z[i];
    }
    const double beta = rz_new / rz;
    rz = rz_new;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i)
      p[i] = z[i] + beta * p[i];
    ++it;
  }
  if (res_out)
    *res_out = rz0 > 0 ? sqrt(fabs(rz / rz0)) : 0.0;
  if (rnorm_out)
    *rnorm_out = sqrt(dot_omp(n, r, r));
  free(r);
  free(z);
  free(p);
  free(q);
  free(dinv);
  return it;
}
