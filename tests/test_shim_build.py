"""CPU: the Arcane-side shim (shim/AfemDoFLinearSystem.cc with both service
names, shim/BSRFormat.h with a device element lambda) compiles against the
Arcane mock (tests/arcane_mock/, test infrastructure) and links with
libafem.so into the driver tests/test_gpu_shim.py runs on the GPU box; the
mock's service options come from the shim's own .axl (axl_mock.py)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOCK = os.path.join(ROOT, "tests", "arcane_mock")


def test_shim_compiles_and_links_against_the_mock():
    r = subprocess.run(["make", "-s", "-C", MOCK], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.path.exists(os.path.join(MOCK, "shim_driver"))
    # every option the shim reads exists in the generated service base (from the .axl)
    gen = open(os.path.join(MOCK, "build", "AfemDoFLinearSystemFactory_axl.h")).read()
    src = open(os.path.join(ROOT, "shim", "AfemDoFLinearSystem.cc")).read()
    for opt in ("device", "transport", "solver", "maxIter", "rtol", "atol", "checkEvery", "preconditioner"):
        assert f"options()->{opt}()" in src and f" {opt}() const" in gen
