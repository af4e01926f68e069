#!/bin/bash
# A/B with afem_set_variant (the env is cached at first read): fused stencil accumulation,
# no coordinate prefetch (4 waves/SIMD), general list beside the stencil kernel
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:fu215:python tools/ab_asm_env.py AFEM_STENCIL_FUSE 0 1 215 40" \
  "300:pf215:python tools/ab_asm_env.py AFEM_STENCIL_PREFETCH 1 0 215 40" \
  "300:fu300:python tools/ab_asm_env.py AFEM_STENCIL_FUSE 0 1 300 20" \
  "300:pf300:python tools/ab_asm_env.py AFEM_STENCIL_PREFETCH 1 0 300 20" \
  "300:side215:python tools/ab_asm_env.py AFEM_ASSEMBLY_SIDE 0 2 215 40"
