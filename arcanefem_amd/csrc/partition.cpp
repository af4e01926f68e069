// Node partitioning and ghosted subdomains of a general (Gmsh) mesh: the part
// of a distributed run that Arcane does before the FEM module sees the mesh
// (partitioner + one ghost layer) and that femutils/FemDoFsOnNodes.cc:71-128
// does after it (DoF uid = node uid * NB_DOF + i, DoF owner = node owner,
// dof_family->computeSynchronizeInfos(): the send / receive lists).
//
// partition_rcb: recursive coordinate bisection of the nodes (cut the longest
//   axis of the current box at the weighted median; parts get node counts
//   proportional to their share of ranks) - balanced, compact, deterministic
//   (ties broken by node id).
// subdomain_plan: for rank r and a node partition, the subdomain the row-owned
//   assembly needs: owned nodes (part == r) first, then the ghost nodes (the
//   other nodes of every cell that has an owned node), both in global id
//   order; the local cells (every cell with an owned node, global order);
//   per neighbour rank s (ascending), the owned nodes that are ghosts on s
//   (send) and the ghosts owned by s (receive), both in global id order, so
//   rank r's send list to s is rank s's receive list from r entry by entry.
//   Every owned row is then complete locally (all its incident cells are
//   local), and the CG's SpMV needs exactly the ghost values of the receive
//   lists.
#include <algorithm>
#include <cmath>
#include <numeric>

#include "afem_internal.hpp"

namespace afem {

namespace {

void rcb(int dim, const double* xyz, int32_t* ids, int64_t n, int part0, int nparts, int32_t* part)
{
  if (nparts <= 1 || n == 0) {
    for (int64_t i = 0; i < n; ++i) part[ids[i]] = part0;
    return;
  }
  double lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
  for (int64_t i = 0; i < n; ++i)
    for (int d = 0; d < dim; ++d) {
      lo[d] = std::min(lo[d], xyz[3 * (int64_t)ids[i] + d]);
      hi[d] = std::max(hi[d], xyz[3 * (int64_t)ids[i] + d]);
    }
  int ax = 0;
  for (int d = 1; d < dim; ++d)
    if (hi[d] - lo[d] > hi[ax] - lo[ax]) ax = d;
  const int pl = nparts / 2;
  const int64_t nl = (int64_t)((double)n * pl / nparts + 0.5);
  auto less = [&](int32_t a, int32_t b) {
    const double xa = xyz[3 * (int64_t)a + ax], xb = xyz[3 * (int64_t)b + ax];
    return xa < xb || (xa == xb && a < b);
  };
  std::nth_element(ids, ids + nl, ids + n, less);
  rcb(dim, xyz, ids, nl, part0, pl, part);
  rcb(dim, xyz, ids + nl, n - nl, part0 + pl, nparts - pl, part);
}

}  // namespace

void partition_rcb(int dim, int64_t n, const double* xyz, int nparts, int32_t* part)
{
  AFEM_REQUIRE(dim == 2 || dim == 3, AFEM_ERR_ARG, "partition: dimension must be 2 or 3");
  AFEM_REQUIRE(nparts >= 1, AFEM_ERR_ARG, "partition: nparts must be >= 1");
  AFEM_REQUIRE(n < (int64_t)INT32_MAX, AFEM_ERR_LIMIT, "partition: more than 2^31-1 nodes");
  std::vector<int32_t> ids((size_t)n);
  std::iota(ids.begin(), ids.end(), 0);
  rcb(dim, xyz, ids.data(), n, 0, nparts, part);
}

void subdomain_plan(int nv, int64_t n_nodes, int64_t n_cells, const int32_t* cell_node, const int32_t* part,
                    int nranks, int rank, SubdomainPlan& P)
{
  AFEM_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, AFEM_ERR_ARG, "subdomain: bad rank / nranks");
  for (int64_t i = 0; i < n_nodes; ++i)
    AFEM_REQUIRE(part[i] >= 0 && part[i] < nranks, AFEM_ERR_ARG, "subdomain: node_part holds an out-of-range rank");
  for (int64_t i = 0; i < n_cells * nv; ++i)
    AFEM_REQUIRE(cell_node[i] >= 0 && cell_node[i] < n_nodes, AFEM_ERR_ARG,
                 "subdomain: cell_node holds an out-of-range node id");
  P = SubdomainPlan();
  P.nranks = nranks;
  P.rank = rank;
  // local cells: every cell with an owned node
  std::vector<uint8_t> is_ghost((size_t)n_nodes, 0);
  for (int64_t c = 0; c < n_cells; ++c) {
    const int32_t* cn = cell_node + c * nv;
    bool mine = false;
    for (int k = 0; k < nv; ++k) mine |= part[cn[k]] == rank;
    if (!mine) continue;
    P.cells.push_back(c);
    for (int k = 0; k < nv; ++k)
      if (part[cn[k]] != rank) is_ghost[cn[k]] = 1;
  }
  // local nodes: owned (global order), then ghosts (global order)
  for (int64_t i = 0; i < n_nodes; ++i)
    if (part[i] == rank) P.l2g.push_back(i);
  P.n_own = (int64_t)P.l2g.size();
  for (int64_t i = 0; i < n_nodes; ++i)
    if (is_ghost[i]) P.l2g.push_back(i);
  AFEM_REQUIRE((int64_t)P.l2g.size() < (int64_t)INT32_MAX, AFEM_ERR_LIMIT, "subdomain: more than 2^31-1 local nodes");
  std::vector<int32_t> g2l((size_t)n_nodes, -1);
  for (size_t l = 0; l < P.l2g.size(); ++l) g2l[P.l2g[l]] = (int32_t)l;
  P.cell_node.resize(P.cells.size() * nv);
  for (size_t c = 0; c < P.cells.size(); ++c)
    for (int k = 0; k < nv; ++k) P.cell_node[c * nv + k] = g2l[cell_node[P.cells[c] * nv + k]];
  // send (owned node u is a ghost on s: u shares a cell with a node owned by
  // s) and receive (ghost v owned by s) lists, per neighbour s, global order
  std::vector<std::vector<int64_t>> snd((size_t)nranks), rcv((size_t)nranks);
  for (int64_t c = 0; c < n_cells; ++c) {
    const int32_t* cn = cell_node + c * nv;
    bool mine = false;
    for (int k = 0; k < nv; ++k) mine |= part[cn[k]] == rank;
    if (!mine) continue;
    for (int k = 0; k < nv; ++k) {
      const int s = part[cn[k]];
      if (s == rank) continue;
      rcv[s].push_back(cn[k]);
      for (int j = 0; j < nv; ++j)
        if (part[cn[j]] == rank) snd[s].push_back(cn[j]);
    }
  }
  for (int s = 0; s < nranks; ++s) {
    auto& a = snd[s];
    auto& b = rcv[s];
    std::sort(a.begin(), a.end());
    a.erase(std::unique(a.begin(), a.end()), a.end());
    std::sort(b.begin(), b.end());
    b.erase(std::unique(b.begin(), b.end()), b.end());
    if (a.empty() && b.empty()) continue;
    P.nbr.push_back(s);
    P.send_cnt.push_back((int64_t)a.size());
    P.recv_cnt.push_back((int64_t)b.size());
    for (int64_t g : a) P.send_ids.push_back(g2l[g]);
    for (int64_t g : b) P.recv_ids.push_back(g2l[g]);
  }
  P.valid = true;
}

}  // namespace afem
