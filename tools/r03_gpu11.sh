#!/bin/bash
# brick x-run write-back (scalar stencil + block-3 stencil instances): parity + C2/C3/C4 timing
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "500:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_elasticity3d.py tests/test_gpu_scale.py tests/test_gpu_multigrid.py tests/test_gpu_passmo.py -x -q --timeout 300 --timeout-method thread" \
  "400:bench:python bench.py --legs c4,c3 --no-cpu-baseline > gpurun_out/r03_v11_bench.json" \
  "400:bench2:python bench.py --legs c3 --no-cpu-baseline > gpurun_out/r03_v11_bench2.json"
