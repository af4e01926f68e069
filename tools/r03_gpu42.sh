#!/bin/bash
# stencil kernel: after its own eighth, a wave takes single slices from the other XCDs' eighths (AFEM_STENCIL_STEAL): A/B + parity
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:st215:python tools/ab_asm_env.py AFEM_STENCIL_STEAL 0 1 215 40" \
  "400:st400:python tools/ab_asm_env.py AFEM_STENCIL_STEAL 0 1 400 20" \
  "600:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_boundary.py tests/test_gpu_distributed.py -q --timeout 300 --timeout-method thread"
