// TEST DRIVER of the Arcane-side shim (shim/AfemDoFLinearSystem.cc, shim/BSRFormat.h)
// against the single-subdomain Arcane mock (tests/arcane_mock/arcane_mock.hpp): it does
// what an ArcaneFEM module does with the linear-system service, through the shim's
// classes only, and writes the solutions for tests/test_gpu_shim.py to compare with the
// oracle.
//
//   csr   : modules/poisson/FemModule.cc with the GPU BSR branch -- the module builds the
//           CSR, hands it over with setCSRValues (host memory), its BC code writes
//           rhs / forced info / forced value (penalty, femutils/ArcaneFemFunctionsGpu.h:
//           434-457), then solve() (HypreDoFLinearSystemImpl semantics);
//   add   : the sequential path -- matrixAddValue per entry, eliminateRow for the
//           Dirichlet DoFs (AlephDoFLinearSystemImpl semantics);
//   bsr   : BSRFormat<1> of the shim: initialize / computeSparsity / assembleBilinear(the
//           module's element lambda) / toLinearSystem (device CSR view), then the
//           penalty and solve() -- modules/poisson/FemModule.cc:261-272 unchanged.
//
// usage: shim_driver <case.bin> <out.bin>
//        shim_driver par <nranks> <case_prefix> <out_prefix>
//   par: the csr and bsr flows on nranks subdomains at once (threads sharing a MockWorld: the
//   transport is the shim's IParallelMng one, transport = "host"), with Arcane-style
//   local ids (owned and ghost DoFs interleaved), the halo from the DoF family's
//   IVariableSynchronizer (_buildHalo) and the solution synchronised by the shim.
//   <case_prefix><r>.bin: int64 n, n_cells; f64 coords[3 n]; i32 cells[4 nc];
//     u8 own[n]; int32 n_nbr; per neighbour: int32 rank, int64 ns, i32 shared[ns],
//     int64 ng, i32 ghosts[ng]; int64 n_dir; i32 dir[n_dir]; f64 dir_value;
//     int64 nnz; i32 rows[n+1]; i32 cols[nnz]; f64 vals[nnz]; f64 rhs[n];
//     f64 rhs3[3 n], lambda, mu (BSRFormat<3>: clamped nodes = dir, body-force right-hand side)
//   <out_prefix><r>.bin: f64 x_csr[n], x_bsr[n], x_bsr3[3 n] (every local DoF, ghosts synchronised)
//   case.bin: int32 dim, nv; int64 n_nodes, n_cells; f64 coords[3 n]; i32 cells[nv nc];
//             int64 n_dir; i32 dir[n_dir]; f64 dir_value; int64 nnz; i32 rows[n+1];
//             i32 cols[nnz]; f64 vals[nnz]; f64 rhs[n]; f64 coef
//   out.bin : f64 x_csr[n], x_add[n], x_bsr[n]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "BSRFormat.h"
#include "DoFLinearSystem.h"
#include "IDoFLinearSystemFactory.h"

using namespace Arcane::FemUtils;

namespace
{
template <class T>
bool rd(FILE* f, T* p, size_t n)
{
  return fread(p, sizeof(T), n, f) == n;
}

struct Case
{
  int32_t dim = 3, nv = 4;
  int64_t n = 0, nc = 0, nnz = 0;
  std::vector<double> coords, vals, rhs;
  std::vector<int32_t> cells, dir, rows, cols;
  double dir_value = 0, coef = 1;
};

bool load(const char* path, Case& c)
{
  FILE* f = fopen(path, "rb");
  if (!f)
    return false;
  int64_t nd = 0;
  bool ok = rd(f, &c.dim, 1) && rd(f, &c.nv, 1) && rd(f, &c.n, 1) && rd(f, &c.nc, 1);
  if (ok) {
    c.coords.resize(3 * c.n);
    c.cells.resize(c.nv * c.nc);
    ok = rd(f, c.coords.data(), c.coords.size()) && rd(f, c.cells.data(), c.cells.size()) && rd(f, &nd, 1);
  }
  if (ok) {
    c.dir.resize(nd);
    ok = rd(f, c.dir.data(), nd) && rd(f, &c.dir_value, 1) && rd(f, &c.nnz, 1);
  }
  if (ok) {
    c.rows.resize(c.n + 1);
    c.cols.resize(c.nnz);
    c.vals.resize(c.nnz);
    c.rhs.resize(c.n);
    ok = rd(f, c.rows.data(), c.n + 1) && rd(f, c.cols.data(), c.nnz) && rd(f, c.vals.data(), c.nnz) &&
         rd(f, c.rhs.data(), c.n) && rd(f, &c.coef, 1);
  }
  fclose(f);
  return ok;
}

// the service a case file names (AfemLinearSystem), made by its registered factory
DoFLinearSystemImpl* make_linear_system(IItemFamily* dofs)
{
  auto& reg = mockServiceRegistry<IDoFLinearSystemFactory>();
  auto it = reg.find("AfemLinearSystem");
  if (it == reg.end())
    throw FatalErrorException("service AfemLinearSystem is not registered");
  ServiceBuildInfo sbi;
  std::unique_ptr<IDoFLinearSystemFactory> factory(it->second(sbi));
  ISubDomain sd;
  return factory->createInstance(&sd, dofs, "Afem");
}

// the module's penalty BC kernel (ArcaneFemFunctionsGpu.h:434-457) on the variables
void penalty(DoFLinearSystem& ls, const Case& c, double p = 1.0e30)
{
  for (int32_t d : c.dir) {
    ls.getForcedInfo()[DoFLocalId(d)] = true;
    ls.getForcedValue()[DoFLocalId(d)] = p;
    ls.rhsVariable()[DoFLocalId(d)] = p * c.dir_value;
  }
}

std::vector<double> solution(DoFLinearSystem& ls, int64_t n)
{
  std::vector<double> x(n);
  for (int64_t i = 0; i < n; ++i)
    x[i] = ls.solutionVariable()[DoFLocalId((Int32)i)];
  return x;
}

std::vector<double> run_csr(IItemFamily* dofs, const Case& c)
{
  DoFLinearSystem ls(make_linear_system(dofs));
  std::vector<int32_t> rnc(c.n);
  for (int64_t i = 0; i < c.n; ++i)
    rnc[i] = c.rows[i + 1] - c.rows[i];
  std::vector<double> vals = c.vals;  // the module's CSR values (the view is not owning)
  CSRFormatView v(Span<const Int32>(c.rows.data(), c.n), Span<const Int32>(rnc.data(), c.n),
                  Span<const Int32>(c.cols.data(), c.nnz), Span<Real>(vals.data(), c.nnz));
  ls.setCSRValues(v);
  for (int64_t i = 0; i < c.n; ++i)
    ls.rhsVariable()[DoFLocalId((Int32)i)] = c.rhs[i];
  penalty(ls, c);
  ls.solve();
  return solution(ls, c.n);
}

std::vector<double> run_add(IItemFamily* dofs, const Case& c)
{
  DoFLinearSystem ls(make_linear_system(dofs));
  for (int64_t i = 0; i < c.n; ++i)
    for (int32_t k = c.rows[i]; k < c.rows[i + 1]; ++k)
      ls.matrixAddValue(DoFLocalId((Int32)i), DoFLocalId(c.cols[k]), c.vals[k]);
  for (int64_t i = 0; i < c.n; ++i)
    ls.rhsVariable()[DoFLocalId((Int32)i)] = c.rhs[i];
  for (int32_t d : c.dir)
    ls.eliminateRow(DoFLocalId(d), c.dir_value);
  ls.solve();
  return solution(ls, c.n);
}

// the element's geometry, read through the views the module's lambda captures:
// cofactors of the edge matrix det * grad(lambda_a) (grad(lambda_0) = -sum) and det
struct TetGeom
{
  double g[4][3], det;
};

__device__ TetGeom tet_geom(const double* d_coords, const int32_t* d_cells, Int32 cell)
{
  double x[4][3];
  for (int a = 0; a < 4; ++a)
    for (int d = 0; d < 3; ++d)
      x[a][d] = d_coords[3 * (int64_t)d_cells[4 * (int64_t)cell + a] + d];
  double e[3][3];
  for (int a = 0; a < 3; ++a)
    for (int d = 0; d < 3; ++d)
      e[a][d] = x[a + 1][d] - x[0][d];
  TetGeom t;
  for (int d = 0; d < 3; ++d) {
    const int p = (d + 1) % 3, q = (d + 2) % 3;
    t.g[1][d] = e[1][p] * e[2][q] - e[1][q] * e[2][p];
    t.g[2][d] = e[2][p] * e[0][q] - e[2][q] * e[0][p];
    t.g[3][d] = e[0][p] * e[1][q] - e[0][q] * e[1][p];
    t.g[0][d] = -(t.g[1][d] + t.g[2][d] + t.g[3][d]);
  }
  t.det = e[0][0] * t.g[1][0] + e[0][1] * t.g[1][1] + e[0][2] * t.g[1][2];
  return t;
}

// BSRFormat<NB_DOF> of the shim as the modules drive it: initialize /
// computeSparsity / assembleBilinear(element lambda) / toLinearSystem (device
// CSR view in the DoF numbering of FemDoFsOnNodes) / the module's BCs / solve
template <int NB_DOF, class Element>
std::vector<double> run_bsr_k(IMesh* mesh, IItemFamily* dofs, Element element, Int64 n_dofs,
                              const std::function<void(DoFLinearSystem&)>& rhs_and_bc)
{
  ITraceMng tm;
  RunQueue queue(eMemoryRessource::Device);
  FemDoFsOnNodes dofs_on_nodes(NB_DOF);
  Runner runner(eExecutionPolicy::HIP);
  std::vector<double> x;
  BSRFormat<NB_DOF> bsr(&tm, queue, dofs_on_nodes);
  bsr.initialize(mesh, true);
  bsr.computeSparsity();
  bsr.assembleBilinear(element);
  DoFLinearSystem ls(make_linear_system(dofs));
  ls.setRunner(&runner);  // the CSR arrays of toLinearSystem live in device memory
  bsr.toLinearSystem(ls);
  rhs_and_bc(ls);
  ls.solve();
  return solution(ls, n_dofs);
}

struct DeviceGeometry
{
  double* coords = nullptr;
  int32_t* cells = nullptr;
  DeviceGeometry(const std::vector<double>& c, const std::vector<int32_t>& cl)
  {
    if (hipMalloc(&coords, sizeof(double) * c.size()) != hipSuccess ||
        hipMalloc(&cells, sizeof(int32_t) * cl.size()) != hipSuccess)
      throw FatalErrorException("hipMalloc");
    (void)hipMemcpy(coords, c.data(), sizeof(double) * c.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(cells, cl.data(), sizeof(int32_t) * cl.size(), hipMemcpyHostToDevice);
  }
  ~DeviceGeometry()
  {
    (void)hipFree(coords);
    (void)hipFree(cells);
  }
};

std::vector<double> run_bsr(IMesh* mesh, IItemFamily* dofs, const Case& c,
                            const std::function<void(DoFLinearSystem&)>& rhs_and_bc = {})
{
  // the module's element lambda (modules/poisson/FemModule.cc:261-272 +
  // FemModule.h:177-186): vol * coef * grad_i . grad_j from the captured geometry
  DeviceGeometry geo(c.coords, c.cells);
  const double* d_coords = geo.coords;
  const int32_t* d_cells = geo.cells;
  const double coef = c.coef;
  auto element = [=] __device__(CellLocalId cell) {
    const TetGeom t = tet_geom(d_coords, d_cells, cell.localId());
    const double s = coef / (6.0 * fabs(t.det));
    afem::generic::FixedMatrix<4, 4> K;
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b)
        K(a, b) = s * (t.g[a][0] * t.g[b][0] + t.g[a][1] * t.g[b][1] + t.g[a][2] * t.g[b][2]);
    return K;
  };
  auto bc = [&](DoFLinearSystem& ls) {
    if (rhs_and_bc) {
      rhs_and_bc(ls);
      return;
    }
    for (int64_t i = 0; i < c.n; ++i)
      ls.rhsVariable()[DoFLocalId((Int32)i)] = c.rhs[i];
    penalty(ls, c);
  };
  return run_bsr_k<1>(mesh, dofs, element, c.n, bc);
}

// BSRFormat<3>: the block-3 P1 elasticity element (the 3D form of
// computeElementMatrixTRIA3Base, modules/elasticity/FemModule.h:112-140):
// vol [lambda g_a,i g_b,j + mu (g_a,j g_b,i + delta_ij g_a.g_b)]
std::vector<double> run_bsr3(IMesh* mesh, IItemFamily* dofs, const std::vector<double>& coords,
                             const std::vector<int32_t>& cells, double lambda, double mu, Int64 n_nodes,
                             const std::function<void(DoFLinearSystem&)>& rhs_and_bc)
{
  DeviceGeometry geo(coords, cells);
  const double* d_coords = geo.coords;
  const int32_t* d_cells = geo.cells;
  auto element = [=] __device__(CellLocalId cell) {
    const TetGeom t = tet_geom(d_coords, d_cells, cell.localId());
    const double s = 1.0 / (6.0 * fabs(t.det));  // vol * (1/det)^2
    afem::generic::FixedMatrix<12, 12> K;
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) {
        const double gg = t.g[a][0] * t.g[b][0] + t.g[a][1] * t.g[b][1] + t.g[a][2] * t.g[b][2];
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j)
            K(3 * a + i, 3 * b + j) =
            s * (lambda * t.g[a][i] * t.g[b][j] + mu * (t.g[a][j] * t.g[b][i] + (i == j ? gg : 0.0)));
      }
    return K;
  };
  return run_bsr_k<3>(mesh, dofs, element, 3 * n_nodes, rhs_and_bc);
}
struct RankCase
{
  int64_t n = 0, nc = 0, nnz = 0;
  std::vector<double> coords, vals, rhs, rhs3;
  std::vector<int32_t> cells, dir, rows, cols;
  std::vector<char> own;
  double lambda = 0, mu = 0;
  std::vector<Int32> nbr;
  std::vector<std::vector<Int32>> shared, ghosts;
  double dir_value = 0;
};

bool load_rank(const std::string& path, RankCase& c)
{
  FILE* f = fopen(path.c_str(), "rb");
  if (!f)
    return false;
  bool ok = rd(f, &c.n, 1) && rd(f, &c.nc, 1);
  int32_t nn = 0;
  int64_t nd = 0;
  if (ok) {
    c.coords.resize(3 * c.n);
    c.cells.resize(4 * c.nc);
    c.own.resize(c.n);
    ok = rd(f, c.coords.data(), c.coords.size()) && rd(f, c.cells.data(), c.cells.size()) && rd(f, c.own.data(), c.n) &&
         rd(f, &nn, 1);
  }
  for (int32_t i = 0; ok && i < nn; ++i) {
    int32_t r = 0;
    int64_t ns = 0, ng = 0;
    ok = rd(f, &r, 1) && rd(f, &ns, 1);
    c.nbr.push_back(r);
    c.shared.emplace_back(ns);
    ok = ok && rd(f, c.shared.back().data(), ns) && rd(f, &ng, 1);
    c.ghosts.emplace_back(ng);
    ok = ok && rd(f, c.ghosts.back().data(), ng);
  }
  if (ok) {
    ok = rd(f, &nd, 1);
    c.dir.resize(nd);
    ok = ok && rd(f, c.dir.data(), nd) && rd(f, &c.dir_value, 1) && rd(f, &c.nnz, 1);
  }
  if (ok) {
    c.rows.resize(c.n + 1);
    c.cols.resize(c.nnz);
    c.vals.resize(c.nnz);
    c.rhs.resize(c.n);
    ok = rd(f, c.rows.data(), c.n + 1) && rd(f, c.cols.data(), c.nnz) && rd(f, c.vals.data(), c.nnz) &&
         rd(f, c.rhs.data(), c.n);
  }
  if (ok) {
    c.rhs3.resize(3 * c.n);
    ok = rd(f, c.rhs3.data(), 3 * c.n) && rd(f, &c.lambda, 1) && rd(f, &c.mu, 1);
  }
  fclose(f);
  return ok;
}

// one rank of the par mode: the module's Hypre-path calls on its subdomain,
// then the shim's BSRFormat<1> on the same subdomain (element lambda over the
// rank's cells, toLinearSystem through matrixAddValue: the ids are not the
// identity), both solved over the shim's IParallelMng transport
void run_rank(MockWorld* world, Int32 rank, const RankCase& c, std::vector<double>& x, std::string& err)
{
  try {
    ITraceMng tm;
    IParallelMng pm(world, rank);
    IItemFamily dofs((Int32)c.n, 0, &pm, &tm);
    dofs.setOwnMask(c.own);
    IVariableSynchronizer* sync = dofs.allItemsSynchronizer();
    sync->ranks = c.nbr;
    sync->shared = c.shared;
    sync->ghosts = c.ghosts;
    auto bc = [&](DoFLinearSystem& ls) {
      for (int64_t i = 0; i < c.n; ++i)
        ls.rhsVariable()[DoFLocalId((Int32)i)] = c.rhs[i];
      for (int32_t d : c.dir) {
        ls.getForcedInfo()[DoFLocalId(d)] = true;
        ls.getForcedValue()[DoFLocalId(d)] = 1.0e30;
        ls.rhsVariable()[DoFLocalId(d)] = 1.0e30 * c.dir_value;
      }
    };
    {
      DoFLinearSystem ls(make_linear_system(&dofs));
      std::vector<int32_t> rnc(c.n);
      for (int64_t i = 0; i < c.n; ++i)
        rnc[i] = c.rows[i + 1] - c.rows[i];
      std::vector<double> vals = c.vals;
      // rows: the reference's layout without the sentinel (HypreDoFLinearSystem.cc:140-141)
      CSRFormatView v(Span<const Int32>(c.rows.data(), c.n), Span<const Int32>(rnc.data(), c.n),
                      Span<const Int32>(c.cols.data(), c.nnz), Span<Real>(vals.data(), c.nnz));
      ls.setCSRValues(v);
      bc(ls);
      ls.solve();
      x = solution(ls, c.n);
    }
    {
      IItemFamily nodes((Int32)c.n, 0, &pm, &tm);
      nodes.setOwnMask(c.own);
      IItemFamily cells((Int32)c.nc, (Int32)c.nc, &pm, &tm);
      cells.nv = 4;
      cells.cell_node = c.cells;
      IMesh mesh(3, &nodes, &cells, &pm);
      for (int64_t i = 0; i < c.n; ++i)
        mesh.nodesCoordinates()[NodeLocalId((Int32)i)] = Real3{ c.coords[3 * i], c.coords[3 * i + 1], c.coords[3 * i + 2] };
      Case one;
      one.n = c.n;
      one.nc = c.nc;
      one.coords = c.coords;
      one.cells = c.cells;
      std::vector<double> xb = run_bsr(&mesh, &dofs, one, [&](DoFLinearSystem& ls) { bc(ls); });
      x.insert(x.end(), xb.begin(), xb.end());
      // BSRFormat<3>: DoF lid = node lid * 3 + i (FemDoFsOnNodes), owners and
      // synchronisation lists of the nodes' DoFs
      IItemFamily dofs3((Int32)(3 * c.n), 0, &pm, &tm);
      std::vector<char> own3(3 * c.n);
      for (int64_t i = 0; i < 3 * c.n; ++i)
        own3[i] = c.own[i / 3];
      dofs3.setOwnMask(own3);
      IVariableSynchronizer* sync3 = dofs3.allItemsSynchronizer();
      sync3->ranks = c.nbr;
      for (size_t q = 0; q < c.nbr.size(); ++q) {
        std::vector<Int32> sh, gh;
        for (Int32 lid : c.shared[q])
          for (Int32 i = 0; i < 3; ++i)
            sh.push_back(3 * lid + i);
        for (Int32 lid : c.ghosts[q])
          for (Int32 i = 0; i < 3; ++i)
            gh.push_back(3 * lid + i);
        sync3->shared.push_back(sh);
        sync3->ghosts.push_back(gh);
      }
      auto bc3 = [&](DoFLinearSystem& ls) {
        for (int64_t i = 0; i < 3 * c.n; ++i)
          ls.rhsVariable()[DoFLocalId((Int32)i)] = c.rhs3[i];
        for (int32_t d : c.dir)
          for (Int32 i = 0; i < 3; ++i) {
            ls.getForcedInfo()[DoFLocalId(3 * d + i)] = true;
            ls.getForcedValue()[DoFLocalId(3 * d + i)] = 1.0e30;
            ls.rhsVariable()[DoFLocalId(3 * d + i)] = 0.0;  // clamped: u = 0
          }
      };
      std::vector<double> x3 = run_bsr3(&mesh, &dofs3, c.coords, c.cells, c.lambda, c.mu, c.n, bc3);
      x.insert(x.end(), x3.begin(), x3.end());
    }
  }
  catch (const std::exception& e) {
    err = e.what();
  }
}

int run_par(int nranks, const std::string& in, const std::string& out)
{
  std::vector<RankCase> cases(nranks);
  for (int r = 0; r < nranks; ++r)
    if (!load_rank(in + std::to_string(r) + ".bin", cases[r])) {
      fprintf(stderr, "bad case file %s%d.bin\n", in.c_str(), r);
      return 2;
    }
  MockWorld world(nranks);
  std::vector<std::vector<double>> xs(nranks);
  std::vector<std::string> errs(nranks);
  std::vector<std::thread> th;
  for (int r = 0; r < nranks; ++r)
    th.emplace_back(run_rank, &world, r, std::cref(cases[r]), std::ref(xs[r]), std::ref(errs[r]));
  for (auto& t : th)
    t.join();
  for (int r = 0; r < nranks; ++r) {
    if (!errs[r].empty()) {
      fprintf(stderr, "shim_driver rank %d: %s\n", r, errs[r].c_str());
      return 1;
    }
    FILE* f = fopen((out + std::to_string(r) + ".bin").c_str(), "wb");
    if (!f)
      return 1;
    fwrite(xs[r].data(), 8, xs[r].size(), f);
    fclose(f);
  }
  return 0;
}
} // namespace

int main(int argc, char** argv)
{
  if (argc >= 5 && std::string(argv[1]) == "par")
    return run_par(atoi(argv[2]), argv[3], argv[4]);
  if (argc < 3) {
    fprintf(stderr, "usage: %s <case.bin> <out.bin>\n", argv[0]);
    return 2;
  }
  Case c;
  if (!load(argv[1], c) || c.dim != 3 || c.nv != 4) {
    fprintf(stderr, "bad case file %s\n", argv[1]);
    return 2;
  }
  try {
    ITraceMng tm;
    IParallelMng pm;
    IItemFamily nodes((Int32)c.n, (Int32)c.n, &pm, &tm);
    IItemFamily cells((Int32)c.nc, (Int32)c.nc, &pm, &tm);
    cells.nv = c.nv;
    cells.cell_node = c.cells;
    IItemFamily dofs((Int32)c.n, (Int32)c.n, &pm, &tm);  // one DoF per node, lid = node lid
    IMesh mesh(3, &nodes, &cells, &pm);
    for (int64_t i = 0; i < c.n; ++i)
      mesh.nodesCoordinates()[NodeLocalId((Int32)i)] = Real3{ c.coords[3 * i], c.coords[3 * i + 1], c.coords[3 * i + 2] };
    const std::vector<double> a = run_csr(&dofs, c);
    const std::vector<double> b = run_add(&dofs, c);
    const std::vector<double> d = run_bsr(&mesh, &dofs, c);
    FILE* f = fopen(argv[2], "wb");
    if (!f)
      return 1;
    fwrite(a.data(), 8, a.size(), f);
    fwrite(b.data(), 8, b.size(), f);
    fwrite(d.data(), 8, d.size(), f);
    fclose(f);
  }
  catch (const std::exception& e) {
    fprintf(stderr, "shim_driver: %s\n", e.what());
    return 1;
  }
  return 0;
}
