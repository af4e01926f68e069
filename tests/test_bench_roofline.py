"""bench.py's roofline bookkeeping (host logic, no GPU): the algorithmic bytes
of SURVEY §8(d), the cube kernel's own byte floor (generator boxes and the
staged canonical path), and the committed PMC summaries under profiles/ that
`roofline.traffic` / `frac_traffic` / `frac_profile` are recomputed from."""
import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

# C2: n = 215 Kuhn box
C2_N = 216 ** 3
C2_CELLS = 59_630_250
C2_NNZ = 150_048_286


def test_algorithmic_bytes_c2():
    """B_asm = 4 nv Ncell + 24 N + 8 (N + 1) + 4 nnz + 8 nnz + 8 N (SURVEY §8d with the int64 row
    offsets of DESIGN §2) ~ 3.16 GB at C2, the figure the headline's `frac` divides by the kernel time."""
    b = bench.algorithmic_bytes(4 * C2_CELLS, C2_N, C2_N, C2_NNZ)
    assert b == 4 * 4 * C2_CELLS + 24 * C2_N + 8 * (C2_N + 1) + 12 * C2_NNZ + 8 * C2_N
    assert 3.0e9 < b < 3.2e9


def test_cube_min_bytes():
    """The cube kernel's own floor: coordinates + row offsets + values + RHS
    (1.60 GB at C2); the staged canonical path adds the caller ids, the
    128-B lattice lines written and read back and the row maps."""
    box = bench.cube_min_bytes({"cube_lattice": 1}, C2_N, C2_N, C2_NNZ)
    assert box == 24 * C2_N + 8 * (C2_N + 1) + 8 * C2_NNZ + 8 * C2_N
    assert 1.55e9 < box < 1.65e9
    staged = bench.cube_min_bytes({"cube_lattice": 3}, C2_N, C2_N, C2_NNZ)
    assert staged - box == (4 + 256 + 12 + 8) * C2_N - 8 * (C2_N + 1)
    assert bench.cube_min_bytes({"cube_lattice": 1}, C2_N, C2_N, C2_NNZ, rhs_read=True) == box + 8 * C2_N


def test_cg_bytes():
    """Per Jacobi-PCG iteration: SpMV 12 nnz + 8 (N + 1) + 16 N, the two vector
    passes 80 N (SURVEY §8d's minimal fused 3-kernel form with int64 row offsets)."""
    assert bench.cg_bytes(C2_NNZ, C2_N) == 12 * C2_NNZ + 8 * (C2_N + 1) + 96 * C2_N


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))))
def test_committed_pmc_summaries(path):
    """Every profiles/pmc_<leg>.json carries the PMC bytes per launch as
    2 FETCH_SIZE + WRITE_SIZE (KiB), a one-GPU size, and -- for the round-5
    legs -- the kernel-trace mean that frac_profile is recomputed from."""
    with open(path) as f:
        pm = json.load(f)
    fetch, write = pm.get("fetch_kib"), pm.get("write_kib")
    assert fetch is not None and write is not None
    assert pm["hbm_bytes_per_launch"] == pytest.approx((2.0 * fetch + write) * 1024.0, rel=1e-6, abs=2)
    assert pm.get("world") in (None, 1)
    if "leg" in pm:
        assert pm["kernel_mean_ms"] > 0 and pm["kernels"]
        leg = os.path.basename(path)[len("pmc_"):-len(".json")]
        assert pm["leg"] == leg
        assert bench.leg_profile(leg, pm["size"]) == pm
        assert bench.leg_profile(leg, -1) is None  # another size: not attached


def test_with_traffic_recomputes_from_the_profile():
    """with_traffic attaches the committed profile's bytes and recomputes the
    fractions from this run's kernel time and from the profile's own mean."""
    pm = bench.leg_profile("c2", 215)
    assert pm is not None
    rf = {"algorithmic_bytes_per_launch": 3_157_771_280, "bytes_kernel_min": 1_603_494_136}
    out = bench.with_traffic(dict(rf), "c2", 215, 0.5)
    b = pm["hbm_bytes_per_launch"]
    assert out["traffic"] == int(b)
    assert out["frac_traffic"] == round(b / 0.5e-3 / 1e9 / bench.HBM_PEAK_GBS, 4)
    pk = pm["kernel_mean_ms"]
    assert out["frac_profile"] == round(rf["algorithmic_bytes_per_launch"] / (pk * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 4)
    assert out["traffic_over_min"] == round(b / rf["bytes_kernel_min"], 3)
    none = bench.with_traffic(dict(rf), "no_such_leg", 215, 0.5)
    assert none["traffic"] is None and none["frac_traffic"] is None
