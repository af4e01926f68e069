#!/bin/bash
# fold test + side-stream placement of the small general list, A/B on C2
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:pytest:python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k 'folded or stencil or uniform'" \
  "300:side2:python tools/ab_asm_env.py AFEM_ASSEMBLY_SIDE 0 2 215 40" \
  "300:side1:python tools/ab_asm_env.py AFEM_ASSEMBLY_SIDE 0 1 215 40"
