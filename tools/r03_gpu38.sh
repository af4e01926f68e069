#!/bin/bash
# stencil steps in one basic block with scheduling barriers (ALU may cross step boundaries, LDS reads not): A/B
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:sb215:python tools/ab_asm_env.py AFEM_STENCIL_SB 0 1 215 40" \
  "300:sb300:python tools/ab_asm_env.py AFEM_STENCIL_SB 0 1 300 20"
