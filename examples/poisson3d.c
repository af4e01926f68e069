/* The Poisson module's linear-system call sequence driven from C through the
 * C ABI alone (include/arcanefem_amd.h) -- what an Arcane-side shim does
 * (INTEGRATION.md), without Python:
 *   modules/poisson/FemModule.cc:24-117 -- BSRFormat initialize ->
 *   computeSparsity -> assembleBilinear(_computeElementMatrixTetra4Gpu) +
 *   applyConstantSourceToRhs(f) -> toLinearSystem -> Dirichlet via penalty
 *   -> solve.
 * usage: poisson3d <n> <out.bin>   (jittered Kuhn box n^3 cells, f = 5.5,
 * u = 0.5 on z = 0 by penalty 1e30); writes the owned solution (float64)
 * and prints one line of statistics. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "arcanefem_amd.h"

#define CHECK(call)                                                                 \
  do {                                                                              \
    int rc_ = (call);                                                               \
    if (rc_ != AFEM_OK) {                                                           \
      fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, afem_last_error());       \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

int main(int argc, char** argv)
{
  if (argc < 3) {
    fprintf(stderr, "usage: %s <n> <out.bin>\n", argv[0]);
    return 2;
  }
  const int n = atoi(argv[1]);
  afem_ctx* ctx = NULL;
  afem_mesh* mesh = NULL;
  afem_bsr* bsr = NULL;
  afem_ls* ls = NULL;
  CHECK(afem_ctx_create(0, NULL, &ctx));
  CHECK(afem_mesh_create_structured(ctx, 3, n, 0, 0.2, 20250220ull, 1, 0, &mesh));
  afem_mesh_info mi;
  CHECK(afem_mesh_get_info(mesh, &mi));
  CHECK(afem_bsr_create(mesh, 1, /*use_csr_in_linear_system*/ 1, &bsr));
  CHECK(afem_bsr_compute_sparsity(bsr));
  CHECK(afem_ls_create(ctx, mi.n_own_nodes, mi.n_nodes, &ls));
  double* rhs = NULL;
  CHECK(afem_ls_rhs(ls, &rhs));
  CHECK(afem_bsr_assemble_poisson_p1(bsr, 1.0, 5.5, rhs));
  CHECK(afem_bsr_to_linear_system(bsr, ls));
  int64_t nb = 0;
  CHECK(afem_mesh_structured_bottom_nodes(mesh, NULL, &nb));
  int32_t* bottom = (int32_t*)malloc((size_t)(nb > 0 ? nb : 1) * sizeof(int32_t));
  CHECK(afem_mesh_structured_bottom_nodes(mesh, bottom, &nb));
  CHECK(afem_ls_dirichlet_penalty(ls, bottom, nb, 0.5, 1.0e30, AFEM_MEM_HOST));
  afem_solver_opts o;
  CHECK(afem_ls_get_solver_options(ls, &o));
  o.rtol = 1e-13;
  CHECK(afem_ls_set_solver_options(ls, &o));
  afem_solve_stats st;
  CHECK(afem_ls_solve(ls, &st));
  double* dsol = NULL;
  CHECK(afem_ls_solution(ls, &dsol));
  double* sol = (double*)malloc((size_t)mi.n_own_nodes * sizeof(double));
  CHECK(afem_memcpy(ctx, sol, dsol, (size_t)mi.n_own_nodes * sizeof(double), AFEM_MEM_HOST, AFEM_MEM_DEVICE));
  FILE* f = fopen(argv[2], "wb");
  if (!f || fwrite(sol, sizeof(double), (size_t)mi.n_own_nodes, f) != (size_t)mi.n_own_nodes) {
    fprintf(stderr, "cannot write %s\n", argv[2]);
    return 1;
  }
  fclose(f);
  printf("poisson3d n=%d dofs=%lld iterations=%d converged=%d rel_residual=%.3e solve_ms=%.3f\n", n,
         (long long)mi.n_own_nodes, st.iterations, st.converged, st.rel_residual, st.solve_ms);
  free(sol);
  free(bottom);
  CHECK(afem_ls_destroy(ls));
  CHECK(afem_bsr_destroy(bsr));
  CHECK(afem_mesh_destroy(mesh));
  CHECK(afem_ctx_destroy(ctx));
  return 0;
}
