// libafem_generic_example.so: the reference modules' element functors
// (examples/elements.hpp) assembled through afem::generic::assemble_bilinear
// (include/arcanefem_amd_generic.hpp), callable from C / ctypes -- the
// benchmark's c2_generic leg and tests/test_gpu_generic.py drive it on any
// structure libafem built.
//   gx_assemble(bsr, kind, path, mode, lambda, mu):
//     kind 0: Poisson (tet4 / tri3 by the mesh), 1: elasticity (tet4 NB_DOF 3 / tri3 NB_DOF 2),
//          2: Poisson tet4 in the cofactor form (elements::PoissonTet4Lean);
//     path 0: cell-unit kernel (assemble_bilinear), 1: f64-atomic kernel (assemble_bilinear_atomic);
//     mode 0: accumulate into the values, 1: overwrite them.
//   gx_assemble_unrolled(bsr, kind, un, mode, pad): kinds 0 / 2 on tet4 through the cell-unit kernel
//     with un = 1..4, 6, 8 functor evaluations in flight per lane and LDS planes of rows + pad (the A/B of
//     the defaults, tools/generic_ab.py).
// Enqueued on the structure's context stream; no synchronisation (path 1 syncs for its error flag).
#include "arcanefem_amd.h"
#include "arcanefem_amd_generic.hpp"
#include "elements.hpp"

using afem::generic::Mode;

namespace {
template <int NV, int K, class F>
int run(afem_bsr* bsr, F f, int path, int mode)
{
  const Mode m = mode ? Mode::Overwrite : Mode::Accumulate;
  return path == 0 ? afem::generic::assemble_bilinear<NV, K>(bsr, f, m)
                   : afem::generic::assemble_bilinear_atomic<NV, K>(bsr, f, m);
}
}  // namespace

extern "C" int gx_assemble(afem_bsr* bsr, int kind, int path, int mode, double lambda, double mu)
{
  afem_assembly_view v;
  int rc = afem_bsr_assembly_view(bsr, &v);
  if (rc != AFEM_OK) return rc;
  const afem::generic::CellAccess acc{ v.cell_node, v.coords };
  if (kind == 0 && v.block_size == 1 && v.nb_node_per_cell == 4) return run<4, 1>(bsr, elements::PoissonTet4{ acc }, path, mode);
  if (kind == 0 && v.block_size == 1 && v.nb_node_per_cell == 3) return run<3, 1>(bsr, elements::PoissonTri3{ acc }, path, mode);
  if (kind == 2 && v.block_size == 1 && v.nb_node_per_cell == 4)
    return run<4, 1>(bsr, elements::PoissonTet4Lean{ acc }, path, mode);
  if (kind == 1 && v.block_size == 3 && v.nb_node_per_cell == 4)
    return run<4, 3>(bsr, elements::ElasticityTet4{ acc, lambda, mu }, path, mode);
  if (kind == 1 && v.block_size == 2 && v.nb_node_per_cell == 3)
    return run<3, 2>(bsr, elements::ElasticityTri3{ acc, lambda, mu }, path, mode);
  return AFEM_ERR_ARG;
}

namespace {
template <int UN>
int run_un(afem_bsr* bsr, const afem::generic::CellAccess& acc, int kind, int mode, int pad)
{
  const Mode m = mode ? Mode::Overwrite : Mode::Accumulate;
  if (kind == 2) return afem::generic::assemble_bilinear_unrolled<4, 1, UN>(bsr, elements::PoissonTet4Lean{ acc }, m, pad);
  return afem::generic::assemble_bilinear_unrolled<4, 1, UN>(bsr, elements::PoissonTet4{ acc }, m, pad);
}
}  // namespace

extern "C" int gx_assemble_unrolled(afem_bsr* bsr, int kind, int un, int mode, int pad)
{
  afem_assembly_view v;
  int rc = afem_bsr_assembly_view(bsr, &v);
  if (rc != AFEM_OK) return rc;
  if (v.block_size != 1 || v.nb_node_per_cell != 4 || (kind != 0 && kind != 2)) return AFEM_ERR_ARG;
  const afem::generic::CellAccess acc{ v.cell_node, v.coords };
  switch (un) {
    case 1: return run_un<1>(bsr, acc, kind, mode, pad);
    case 2: return run_un<2>(bsr, acc, kind, mode, pad);
    case 3: return run_un<3>(bsr, acc, kind, mode, pad);
    case 4: return run_un<4>(bsr, acc, kind, mode, pad);
    case 6: return run_un<6>(bsr, acc, kind, mode, pad);
    case 8: return run_un<8>(bsr, acc, kind, mode, pad);
    default: return AFEM_ERR_ARG;
  }
}
