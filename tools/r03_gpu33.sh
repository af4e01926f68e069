#!/bin/bash
# stencil entries' scale + accumulation fused into the dot products (41 instead of 44 FP64 ops per step): A/B
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:fu215:python tools/ab_asm_env.py AFEM_STENCIL_FUSE 0 1 215 40" \
  "300:fu300:python tools/ab_asm_env.py AFEM_STENCIL_FUSE 0 1 300 20"
