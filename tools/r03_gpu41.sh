#!/bin/bash
# stencil tail pooled across XCDs (second launch beside the main one): A/B of AFEM_STENCIL_TAIL, parity tests
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:t215:python tools/ab_env.py AFEM_STENCIL_TAIL 0 8 215 40" \
  "400:t400:python tools/ab_env.py AFEM_STENCIL_TAIL 0 8 400 20" \
  "400:t400b:python tools/ab_env.py AFEM_STENCIL_TAIL 0 15 400 20" \
  "600:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_boundary.py tests/test_gpu_distributed.py -q --timeout 300 --timeout-method thread"
