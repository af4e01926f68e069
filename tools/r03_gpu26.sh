#!/bin/bash
# boundary-aware order with box edges / corners in their own slices: pattern dump, parity, bench
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "200:patterns:AFEM_DEBUG_PATTERNS=1 python tools/pattern_probe.py 20 215" \
  "600:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_boundary.py tests/test_gpu_distributed.py tests/test_gpu_shim.py -q --timeout 300 --timeout-method thread" \
  "300:bench:python bench.py --no-extras --no-cpu-baseline > gpurun_out/r03_v26_bench.json"
