#!/bin/bash
# stencil kernel: non-run slices store per lane from registers (158 VGPRs: 3 waves/SIMD); parity + C2/C4 timing
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "500:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread" \
  "400:bench:python bench.py --legs c4 --no-cpu-baseline > gpurun_out/r03_v12_bench.json" \
  "400:bench2:python bench.py --legs c4 --no-cpu-baseline > gpurun_out/r03_v12_bench2.json"
