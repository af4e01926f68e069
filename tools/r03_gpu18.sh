#!/bin/bash
# block-3: 1/6 and c0/120 folded into kernel constants: every block-3 test + C3/C5 timing
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "600:pytest:python -u -m pytest tests/test_gpu_elasticity3d.py tests/test_gpu_passmo.py tests/test_gpu_multigrid.py tests/test_gpu_generic.py tests/test_gpu_distributed.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread" \
  "400:bench:python bench.py --legs c3,c5 --no-cpu-baseline > gpurun_out/r03_v18_bench.json"
