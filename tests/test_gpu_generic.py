"""GPU: BSRFormat::assembleBilinear(lambda) through the generic element-functor
entry (include/arcanefem_amd_generic.hpp) -- the module's own element functor
(a hipcc-compiled device lambda, examples/generic_assembly.hip) scattered cell
by cell with f64 atomics, as femutils/BSRFormat.h:786-837 does.

Gates per entry (summation order differs from the fixed-physics strip
kernels, as the reference's atomics differ run to run): against the library's
compiled-in instance on the same structure and against the oracle's cell loop
(orc_assemble_poisson / orc_assemble_elasticity_tet), |a - b| <= 1e-12 max|b|,
both value layouts (ordered per block, per row)."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "generic_assembly")


def _run(n, k, layout, tmp_path):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} is not built (make -C examples)")
    out = str(tmp_path / f"g{n}_{k}_{layout}.bin")
    r = subprocess.run([EXE, str(n), str(k), layout, out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(out, "rb").read()
    n_rows, nnz = np.frombuffer(raw[:16], dtype=np.int64)
    off = 16
    rows = np.frombuffer(raw[off:off + 8 * (n_rows + 1)], dtype=np.int64)
    off += 8 * (n_rows + 1)
    cols = np.frombuffer(raw[off:off + 4 * nnz], dtype=np.int32)
    off += 4 * nnz
    m = nnz * k * k
    gen = np.frombuffer(raw[off:off + 8 * m], dtype=np.float64)
    bi = np.frombuffer(raw[off + 8 * m:off + 16 * m], dtype=np.float64)
    return rows, cols, gen, bi


@pytest.mark.parametrize("layout", ["block", "row"])
@pytest.mark.parametrize("k", [1, 3])
def test_generic_lambda_matches_oracle(tmp_path, k, layout):
    n = 6
    rows, cols, gen, bi = _run(n, k, layout, tmp_path)
    ref = O.structured_mesh(3, n, jitter=0.2, seed=20250220)
    orp, ocols = O.sparsity(ref["n_local"], ref["n_own"], ref["cells"])
    assert np.array_equal(rows, orp) and np.array_equal(cols, ocols)
    if k == 1:
        ovals, _ = O.assemble_poisson(ref["n_own"], ref["cells"], ref["coords"], orp, ocols, 0.0)
    else:
        E, nu = 21.0e5, 0.28
        lam, mu = E * nu / ((1 + nu) * (1 - 2 * nu)), E / (2 * (1 + nu))
        ovals, _ = O.assemble_elasticity_tet(ref["n_own"], ref["cells"], ref["coords"], orp, ocols, lam, 2 * mu)
        if layout == "row":
            ovals = O.blocks_to_row_order_k(orp, ovals, 3)
    scale = np.abs(ovals).max()
    assert np.abs(gen - ovals).max() <= 1e-12 * scale, np.abs(gen - ovals).max() / scale
    assert np.abs(bi - ovals).max() <= 1e-12 * scale
    assert np.abs(gen - bi).max() <= 1e-12 * scale
