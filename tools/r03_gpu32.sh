#!/bin/bash
# stencil kernel without the cross-slice coordinate prefetch (122 VGPRs, 4 waves/SIMD) vs with (158, 3): A/B
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:pf215:python tools/ab_asm_env.py AFEM_STENCIL_PREFETCH 1 0 215 40" \
  "300:pf300:python tools/ab_asm_env.py AFEM_STENCIL_PREFETCH 1 0 300 20"
