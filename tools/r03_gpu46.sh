#!/bin/bash
# box edge / corner signatures compiled into the stencil kernel (168 VGPRs at 3 waves/SIMD forced):
# parity tests, A/B of the library against the previous build, bench
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "700:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_boundary.py tests/test_gpu_distributed.py tests/test_gpu_elasticity3d.py tests/test_gpu_shim.py -q --timeout 300 --timeout-method thread" \
  "400:ab215:python tools/ab_lib.py arcanefem_amd/libafem_base.so arcanefem_amd/libafem.so 215 30 3" \
  "500:ab400:python tools/ab_lib.py arcanefem_amd/libafem_base.so arcanefem_amd/libafem.so 400 10 3" \
  "300:bench:python bench.py --no-extras --no-cpu-baseline > gpurun_out/r03_v46_bench.json"
