#!/bin/bash
# round-3 batch 3: stencil kernel with LDS-DMA coordinate staging (3 waves/SIMD) -- parity, A/B against
# the register-staged kernel, kernel stats
export TMPDIR=/tmp
B="bench.py --no-extras --no-cpu-baseline"
tools/gpu_steps.sh \
  "600:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread" \
  "200:dma:python $B > gpurun_out/r03_v4_dma.json" \
  "200:nodma:AFEM_STENCIL_DMA=0 python $B > gpurun_out/r03_v4_nodma.json" \
  "200:dma2:python $B > gpurun_out/r03_v4_dma2.json" \
  "200:c2trace:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r03_c2dma/trace -o run -- python3 $B --steps 10"
