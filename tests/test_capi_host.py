"""CPU: the C-ABI library loads, exports every symbol the header declares,
and its host-only logic (halo plans) is right.  No GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest

import arcanefem_amd as af
from arcanefem_amd import _capi
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "arcanefem_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(afem_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = af.load()
    names = declared_functions()
    assert len(names) > 50
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/arcanefem_amd.h but not exported"
    assert set(names) == set(_capi.exported_symbols())


def test_version_and_error_string():
    lib = af.load()
    assert lib.afem_version() >= 100
    with pytest.raises(af.AfemError) as e:
        _capi.call("afem_ctx_synchronize", None)
    assert e.value.code == 1 and "must not be NULL" in str(e.value)


@pytest.mark.parametrize("dim,n,nz,nranks", [(3, 4, 9, 3), (3, 3, 3, 4), (2, 7, None, 2), (3, 5, 5, 1)])
def test_structured_halo_plan_matches_mesh_spec(dim, n, nz, nranks):
    """Every ghost node of every slab is received from the rank that owns it,
    in the same order the owner sends it."""
    meshes = [O.structured_mesh(dim, n, nz=nz, nranks=nranks, rank=r) for r in range(nranks)]
    plans = [af.structured_halo_plan(dim, n, nz, nranks, r) for r in range(nranks)]
    for r in range(nranks):
        nbr, sc, rc, si, ri = plans[r]
        m = meshes[r]
        ghosts = set(range(m["n_own"], m["n_local"]))
        assert set(ri.tolist()) == ghosts
        off = np.concatenate([[0], np.cumsum(rc)])
        for k, q in enumerate(nbr):
            recv_g = m["local_to_global"][ri[off[k]:off[k + 1]]]
            qn, qsc, qrc, qsi, qri = plans[q]
            kk = list(qn).index(r)
            qoff = np.concatenate([[0], np.cumsum(qsc)])
            sent_g = meshes[q]["local_to_global"][qsi[qoff[kk]:qoff[kk + 1]]]
            assert np.array_equal(recv_g, sent_g)
            assert np.all(qsi[qoff[kk]:qoff[kk + 1]] < meshes[q]["n_own"])


def test_c_driver_builds_against_the_header():
    # examples/poisson3d.c uses only include/arcanefem_amd.h and links libafem.so
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "examples")], check=True)
    exe = os.path.join(root, "examples", "poisson3d")
    assert os.path.exists(exe)
    out = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "libafem.so" in out and "not found" not in out.split("libafem.so")[1].splitlines()[0]
