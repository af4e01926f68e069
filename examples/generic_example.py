"""ctypes entry of examples/libafem_generic_example.so: the reference
modules' element functors (examples/elements.hpp) assembled through
afem::generic::assemble_bilinear (include/arcanefem_amd_generic.hpp), i.e.
what an unchanged module's BSRFormat::assembleBilinear(lambda) runs.  Used by
bench.py (leg c2_generic) and tests/test_gpu_generic.py.  No fallback: a
missing library raises."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("AFEM_GENERIC_LIB") or os.path.join(_HERE, "libafem_generic_example.so")  # env: A/B builds
POISSON, ELASTICITY, POISSON_LEAN = 0, 1, 2
UNITS, ATOMIC = 0, 1
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise OSError(f"{LIB} is missing: make -C examples")
        from arcanefem_amd import _capi
        _capi.load()  # libafem first (the example links it through its rpath)
        L = ctypes.CDLL(LIB)
        L.gx_assemble.restype = ctypes.c_int
        L.gx_assemble.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                  ctypes.c_double]
        L.gx_assemble_unrolled.restype = ctypes.c_int
        L.gx_assemble_unrolled.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


def assemble(bsr, kind=POISSON, path=UNITS, overwrite=False, lam=0.0, mu=0.0):
    """BSRFormat::assembleBilinear(<module element>) on bsr (core.BSRFormat);
    asynchronous on the structure's stream."""
    from arcanefem_amd import _capi
    rc = load().gx_assemble(bsr.h, kind, path, 1 if overwrite else 0, lam, mu)
    if rc != 0:
        L = _capi.load()
        raise _capi.AfemError(rc, "gx_assemble", L.afem_last_error().decode(errors="replace"))


def assemble_unrolled(bsr, kind, un, overwrite=False, pad=0):
    """The cell-unit kernel with un (1-4) functor evaluations in flight per
    lane and LDS planes padded by pad rows (tet4 Poisson kinds only): the A/B
    of assemble_bilinear's defaults."""
    from arcanefem_amd import _capi
    rc = load().gx_assemble_unrolled(bsr.h, kind, un, 1 if overwrite else 0, pad)
    if rc != 0:
        L = _capi.load()
        raise _capi.AfemError(rc, "gx_assemble_unrolled", L.afem_last_error().decode(errors="replace"))
