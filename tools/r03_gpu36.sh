#!/bin/bash
# AFEM_ASSEMBLY_SIDE=3 (stencil first, the small lists after it on the side stream) vs serial
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:s3_215:python tools/ab_asm_env.py AFEM_ASSEMBLY_SIDE 0 3 215 40" \
  "300:s3_300:python tools/ab_asm_env.py AFEM_ASSEMBLY_SIDE 0 3 300 20" \
  "300:s1_215:python tools/ab_asm_env.py AFEM_ASSEMBLY_SIDE 0 1 215 40"
