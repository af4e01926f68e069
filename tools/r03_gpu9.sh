#!/bin/bash
# shared local-index streams of the stencil slices: parity + A/B (C2, C3, C4)
export TMPDIR=/tmp
B="bench.py --legs c4,c3 --no-cpu-baseline"
tools/gpu_steps.sh \
  "500:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_elasticity3d.py tests/test_gpu_scale.py tests/test_gpu_multigrid.py -x -q --timeout 300 --timeout-method thread" \
  "400:share:python $B > gpurun_out/r03_v9_share.json" \
  "400:noshare:AFEM_STRIP_SHARE=0 python $B > gpurun_out/r03_v9_noshare.json" \
  "400:share2:python $B > gpurun_out/r03_v9_share2.json"
