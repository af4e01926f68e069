"""CPU checks of the strip signatures compiled into the stencil kernels
(arcanefem_amd/csrc/stencil_sigs.inc): every signature is a well-formed
k_strip_classify slot stream whose window walk (shift / swap, the kernels'
compile-time tables: assembly.hip StencilWin) touches every off-diagonal slot
of a row of its length, never the diagonal, and emits one cell per step."""
import os
import re

import pytest

INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "arcanefem_amd", "csrc",
                   "stencil_sigs.inc")


def _sigs():
    text = open(INC).read()
    out = {}
    for m in re.finditer(r"inline constexpr StencilSig (\w+) = \{\s*(\d+),\s*(\d+),\s*(\d+),\s*(0x[0-9a-fA-F]+)ull,\s*"
                         r"\{([^}]*)\}", text):
        name, ns, w, d, pat, body = m.groups()
        slots = [int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", body)]
        out[name] = dict(nsteps=int(ns), w=int(w), dslot=int(d), pat=int(pat, 16), slot=slots)
    pack = re.search(r"#define AFEM_STENCIL_PACK\s*\\?\s*(.*?)\n\n", text + "\n\n", re.S).group(1)
    order = re.findall(r"kSig\w+", pack)
    return out, order


def test_signature_table_and_pack_agree():
    sigs, order = _sigs()
    assert order and set(order) == set(sigs), (order, list(sigs))
    assert order[0] == "kSigKuhn3D"  # index 0: the interior brick (the block-3 stencil instance's signature)
    xm = re.findall(r"X\((\d+), (kSig\w+)\)", open(INC).read())
    assert [n for _, n in sorted(xm, key=lambda t: int(t[0]))] == order


@pytest.mark.parametrize("name", sorted(_sigs()[0]))
def test_signature_window_walk(name):
    s = _sigs()[0][name]
    ns, w, d, pat, b = s["nsteps"], s["w"], s["dslot"], s["pat"], s["slot"]
    assert len(b) == 32 and 3 <= ns <= 32 and ns % 2 == 0 and 0 <= d < w <= 16
    assert b[0] >> 6 == 2 and b[1] >> 6 == 2  # two priming steps
    for j in range(2, ns):
        kind = b[j] >> 6
        assert kind in (0, 1) and kind == (pat >> j) & 1, (j, hex(b[j]))
    assert pat >> ns == 0 and pat & 3 == 0
    assert all(x == (0xC0 | d) for x in b[ns:])  # padding steps carry the diagonal slot
    # window walk: P, Q, R after each rotation; every cell's three nodes distinct,
    # never the diagonal, and every off-diagonal slot visited
    P, Q, R = d, b[0] & 63, b[1] & 63
    seen = {Q, R}
    for j in range(2, ns):
        if not (pat >> j) & 1:
            P = Q
        Q, R = R, b[j] & 63
        assert len({P, Q, R}) == 3 and d not in (P, Q, R), (j, P, Q, R)
        seen.add(R)
    assert seen == set(range(w)) - {d}
