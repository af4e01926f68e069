#!/bin/bash
# stealing with a threshold on the victim's remaining slices per wave (AFEM_STENCIL_STEAL_MIN): A/B
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:a215:python tools/ab_asm_env.py AFEM_STENCIL_STEAL 0 1 215 40" \
  "300:b215:python tools/ab_asm_env.py AFEM_STENCIL_STEAL_MIN 1 3 215 40" \
  "600:a463:python tools/ab_asm_env.py AFEM_STENCIL_STEAL 0 1 463 12" \
  "600:b463:python tools/ab_asm_env.py AFEM_STENCIL_STEAL_MIN 0 1 463 12"
