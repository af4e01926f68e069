"""The Arcane-side shim (shim/AfemDoFLinearSystem.cc, shim/BSRFormat.h) driven the
way an ArcaneFEM module drives its linear-system service, on the GPU, against
the single-subdomain Arcane mock (tests/arcane_mock/: test infrastructure, not
Arcane; tests/arcane_mock/shim_driver.cpp says what each flow does):

  csr  -- setCSRValues with a host CSR + the module's penalty BC variables +
          solve() (HypreDoFLinearSystemImpl semantics, femutils/HypreDoFLinearSystem.cc:138-156, 319-382);
  add  -- matrixAddValue per entry + eliminateRow (AlephDoFLinearSystemImpl, :192-246);
  bsr  -- the shim's BSRFormat<1>: initialize / computeSparsity /
          assembleBilinear(device element lambda) / toLinearSystem (device CSR
          view) / penalty / solve() (modules/poisson/FemModule.cc:261-272).

Case: the reference's sphere_3D Poisson regression (golden_cases.CASES), with
the oracle's system as the expected one; every flow must also meet the
reference golden at checkNodeResultFile's 1e-4 (modules/poisson/FemModule.cc:404).
"""
import os
import subprocess

import numpy as np
import pytest

from arcanefem_amd.gmsh import read_gmsh, read_node_result_file
from golden_cases import CASES, path
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "arcane_mock", "shim_driver")


def _write_case(fname, gm, f, dirichlet, value, coef=1.0):
    n = gm.n_nodes
    rp, cols = O.sparsity(n, n, gm.cells)
    vals, rhs = O.assemble_poisson(n, gm.cells, gm.coords, rp, cols, f)
    with open(fname, "wb") as fh:
        fh.write(np.array([3, 4], np.int32).tobytes())
        fh.write(np.array([n, gm.cells.shape[0]], np.int64).tobytes())
        fh.write(np.ascontiguousarray(gm.coords, np.float64).tobytes())
        fh.write(np.ascontiguousarray(gm.cells, np.int32).tobytes())
        fh.write(np.array([dirichlet.size], np.int64).tobytes())
        fh.write(np.ascontiguousarray(dirichlet, np.int32).tobytes())
        fh.write(np.array([value], np.float64).tobytes())
        fh.write(np.array([cols.size], np.int64).tobytes())
        fh.write(rp.astype(np.int32).tobytes())
        fh.write(cols.astype(np.int32).tobytes())
        fh.write(vals.astype(np.float64).tobytes())
        fh.write(rhs.astype(np.float64).tobytes())
        fh.write(np.array([coef], np.float64).tobytes())
    return rp, cols, vals, rhs


def test_shim_flows_match_oracle_and_golden(tmp_path):
    assert os.path.exists(EXE), "tests/arcane_mock/shim_driver not built (__graft_entry__.build())"
    mfile, f, bcs, gfile, P = CASES["sphere_3D"]
    gm = read_gmsh(path(mfile))
    (group, value), = bcs
    dirichlet = gm.group_nodes(group).astype(np.int32)
    case, out = tmp_path / "case.bin", tmp_path / "out.bin"
    rp, cols, vals, rhs = _write_case(str(case), gm, f, dirichlet, value)
    r = subprocess.run([EXE, str(case), str(out)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, AFEM_OPT_RTOL="1e-14", AFEM_OPT_SOLVER="pcg", AFEM_OPT_MAX_ITER="20000"))
    assert r.returncode == 0, r.stderr
    n = gm.n_nodes
    x = np.fromfile(str(out), np.float64)
    assert x.size == 3 * n
    x_csr, x_add, x_bsr = x[:n], x[n:2 * n], x[2 * n:]
    # expected: the oracle's systems, solved directly
    pv, pr = vals.copy(), rhs.copy()
    O.dirichlet_penalty(dirichlet, value, P, rp, cols, pv, pr)
    xp = np.linalg.solve(O.csr_to_dense(rp, cols, pv), pr)
    ev, er = vals.copy(), rhs.copy()
    O.row_elimination(dirichlet, value, rp, cols, ev, er)
    xe = np.linalg.solve(O.csr_to_dense(rp, cols, ev), er)
    scale = np.abs(xp).max()
    assert np.abs(x_csr - xp).max() / scale <= 1e-10
    assert np.abs(x_bsr - xp).max() / scale <= 1e-10
    assert np.abs(x_add - xe).max() / scale <= 1e-10
    gold = read_node_result_file(path(gfile))
    for x_ in (x_csr, x_add, x_bsr):
        nerr, _ = O.check_node_result({int(t): x_[i] for i, t in enumerate(gm.node_tags)}, gold, 1e-4)
        assert nerr == 0
