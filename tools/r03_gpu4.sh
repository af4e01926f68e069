#!/bin/bash
# LDS-DMA probe + DMA stencil variants: parity on the small boxes, C2 timing
export TMPDIR=/tmp
B="bench.py --no-extras --no-cpu-baseline"
tools/gpu_steps.sh \
  "60:probe:tools/glds_probe" \
  "200:par2:AFEM_STENCIL_DMA=2 python -u -m pytest tests/test_gpu_parity.py -q -k 'structured_assembly_parity or stencil' --timeout 120 --timeout-method thread" \
  "200:par1:AFEM_STENCIL_DMA=1 python -u -m pytest tests/test_gpu_parity.py -q -k 'structured_assembly_parity or stencil' --timeout 120 --timeout-method thread" \
  "200:dma2:AFEM_STENCIL_DMA=2 python $B > gpurun_out/r03_v5_dma2.json" \
  "200:dma1:AFEM_STENCIL_DMA=1 python $B > gpurun_out/r03_v5_dma1.json" \
  "200:base:python $B > gpurun_out/r03_v5_base.json"
