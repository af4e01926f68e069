#!/bin/bash
# ticket ring + 16-row k_apply_bcs: parity; A/B of the small general list serial vs beside the stencil kernel (AFEM_ASSEMBLY_SIDE=2)
export TMPDIR=/tmp
B="bench.py --no-extras --no-cpu-baseline --cg-iters 10 --steps 60"
tools/gpu_steps.sh \
  "500:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py tests/test_gpu_scale.py tests/test_gpu_elasticity3d.py -x -q --timeout 300 --timeout-method thread" \
  "200:a1:python $B > gpurun_out/r03_v15_s0a.json" \
  "200:b1:AFEM_ASSEMBLY_SIDE=2 python $B > gpurun_out/r03_v15_s2a.json" \
  "200:a2:python $B > gpurun_out/r03_v15_s0b.json" \
  "200:b2:AFEM_ASSEMBLY_SIDE=2 python $B > gpurun_out/r03_v15_s2b.json"
