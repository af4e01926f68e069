#!/bin/bash
# AFEM_STENCIL_STEAL A/B at n = 300 and at the C4 size (n = 463)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "400:st300:python tools/ab_asm_env.py AFEM_STENCIL_STEAL 0 1 300 20" \
  "600:st463:python tools/ab_asm_env.py AFEM_STENCIL_STEAL 0 1 463 12" \
  "300:st215b:python tools/ab_asm_env.py AFEM_STENCIL_STEAL 0 1 215 40"
