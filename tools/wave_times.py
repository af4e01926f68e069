"""Per-workgroup timeline of the uniform strip assembly instance (diagnostic).

Needs the diagnostic build: make -C arcanefem_amd/csrc EXTRA=-DAFEM_WAVE_TIMES OBJDIR=build_wt OUT=../libafem_wt.so
usage: AFEM_LIB=arcanefem_amd/libafem_wt.so python tools/wave_times.py [n]
Prints, for the last of several assemblies, the start / end spread of the
persistent waves (s_memrealtime, 100 MHz) overall and per XCD."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import arcanefem_amd as af  # noqa: E402
from arcanefem_amd import _capi as C  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 215
ctx = af.Context(0)
mesh = af.Mesh.structured(ctx, 3, n, jitter=0.2, seed=20250220)
bsr = af.BSRFormat(mesh, 1).initialize(True)
bsr.computeSparsity()
ls = af.DoFLinearSystem().initialize(ctx, mesh.n_own_nodes)
for _ in range(5):
    bsr.assemblePoissonP1(1.0, 5.5, ls.rhsVariable(), rhs_mode="set")
ctx.synchronize()
N = 16384
buf = (ctypes.c_ulonglong * (3 * N))()
rc = C.load().afem_debug_wave_times(buf, N)
assert rc == 0, rc
a = np.frombuffer(buf, dtype=np.uint64).reshape(N, 3).astype(np.int64)
used = a[:, 0] > 0
g = np.nonzero(used)[0]
t0 = a[used, 0].min()
st = (a[used, 0] - t0) / 100.0  # us
en = (a[used, 1] - t0) / 100.0
cnt = a[used, 2]
print(f"workgroups {used.sum()}  span {en.max():.1f} us")
print(f"start: max {st.max():.1f} us  p50 {np.median(st):.1f}")
print(f"end:   min {en.min():.1f}  p10 {np.percentile(en, 10):.1f}  p50 {np.median(en):.1f}  p90 {np.percentile(en, 90):.1f}  max {en.max():.1f} us")
print(f"slices per wave: min {cnt.min()} p50 {np.median(cnt):.0f} max {cnt.max()}  total {cnt.sum()}")
for x in range(8):
    m = (g & 7) == x
    print(f"xcd {x}: waves {m.sum()} end p50 {np.median(en[m]):.1f} max {en[m].max():.1f} us  slices {cnt[m].sum()}  us/slice/wave {np.median(en[m] - st[m]) / np.median(cnt[m]):.2f}")
