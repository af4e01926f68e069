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


# Neumann / traction cases (K15), same meshes:
#   circle_neumann_2D  modules/poisson/inputs/circle.neumann.2D.arc     check/poisson_test_ref_circle_neumann_2D.txt
#   sphere_neumann_3D  modules/poisson/inputs/sphere.neumann.3D.arc     check/poisson_test_ref_sphere_neumann_3D.txt
# name: (mesh, f, [(dirichlet group, value)], [(neumann face group, (vx, vy[, vz]))], golden, penalty)
NEUMANN_CASES = {
    "circle_neumann_2D": ("circle_cut.msh", 5.5, [("horizontal", 0.5)], [("curved", (-0.35, 1.65))],
                          "poisson_test_ref_circle_neumann_2D.txt", 1.0e30),
    "sphere_neumann_3D": ("sphere_cut.msh", 5.5, [("horizontal", 0.5)], [("curved", (0.35, 1.65, 3.75))],
                          "poisson_test_ref_sphere_neumann_3D.txt", 1.0e30),
}

# Block-2 elasticity with traction (modules/elasticity/inputs/bar.2D.traction.bsr.arc:22-35):
# E = 21e5, nu = 0.28, `left` clamped (u = 0, both components) by penalty 1e30
# (modules/elasticity/Fem.axl:32-41), traction (1, NULL) on `right`; golden
# modules/elasticity/check/elasticity_traction_bar_test_ref.txt, checked by the
# reference at epsilon 1e-3, min value 1e-16 (modules/elasticity/FemModule.cc:547-553).
ELASTICITY_BAR = dict(mesh="bar.msh", E=21.0e5, nu=0.28, clamp="left", traction_group="right",
                      traction=(1.0, 0.0), golden="elasticity_traction_bar_test_ref.txt", penalty=1.0e30)


def lame(E, nu):
    """modules/elasticity/FemModule.cc:132-133."""
    mu2 = (E / (2 * (1 + nu))) * 2
    lam = E * nu / ((1 + nu) * (1 - 2 * nu))
    return lam, mu2
