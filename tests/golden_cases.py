"""The reference's own Poisson regression cases (mesh, source, Dirichlet groups,
golden file), replayed by the oracle tests and by the GPU parity tests.

Sources (toutane/arcanefem @ 2025-02-20):
  circle_cut  modules/poisson/inputs/circle.2D.arc:22-34             check/poisson_test_ref_circle_2D.txt
  sphere_cut  modules/poisson/inputs/sphere.3D.arc (same BCs)         check/poisson_test_ref_sphere_3D.txt
              (used by modules/testlab/inputs/Test.sphere.3D.arc:21-33)
  L-shape     modules/testlab/inputs/Test.direct-solver.arc:22-30     tests/poisson_test_ref_L-shape_2D.txt
  L-shape-3D  modules/testlab/inputs/Test.L-shape.3D.arc:22-36        tests/poisson_test_ref_L-shape_3D.txt
  plancher    modules/poisson/inputs/perforatedSquare.pointDirichlet.2D.arc:22-42
                                                                      check/poisson_test_point_dirichlet_2D.txt
The reference checks each with checkNodeResultFile(..., 1.0e-4)
(modules/poisson/FemModule.cc:404, modules/testlab/FemModule.cc:1896-1898).
"""
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# name: (mesh file, f or None, [(group, value)], golden file, penalty)
CASES = {
    "circle_2D": ("circle_cut.msh", 5.5, [("horizontal", 0.5)], "poisson_test_ref_circle_2D.txt", 1.0e30),
    "sphere_3D": ("sphere_cut.msh", 5.5, [("horizontal", 0.5)], "poisson_test_ref_sphere_3D.txt", 1.0e30),
    "L-shape_2D": ("L-shape.msh", -5.5, [("boundary", 0.5)], "poisson_test_ref_L-shape_2D.txt", 1.0e30),
    "L-shape_3D": ("L-shape-3D.msh", 5.5, [("bot", 50.0), ("bc", 10.0)], "poisson_test_ref_L-shape_3D.txt", 1.0e30),
    "point_dirichlet_2D": ("plancher.msh", None,
                           [("topLeftCorner", 50.0), ("topRightCorner", 20.0), ("botLeftCorner", 20.0),
                            ("botRightCorner", 50.0)], "poisson_test_point_dirichlet_2D.txt", 1.0e30),
}

# max relative error of the restatement against each golden (measured; the
# golden files were themselves produced by iterative solvers, which bounds
# how tightly they pin the arithmetic)
GOLDEN_TOL = {"circle_2D": 1e-8, "sphere_3D": 1e-8, "L-shape_2D": 1e-12, "L-shape_3D": 1e-12,
              "point_dirichlet_2D": 1e-4}


def path(name):
    return os.path.join(GOLDEN, name)
