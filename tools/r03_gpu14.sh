#!/bin/bash
# A/B: general-list slices before the stencil kernel (serial) vs beside it on the side stream
export TMPDIR=/tmp
B="bench.py --no-extras --no-cpu-baseline --cg-iters 10"
tools/gpu_steps.sh \
  "200:a1:python $B > gpurun_out/r03_v14_serial1.json" \
  "200:b1:AFEM_ASSEMBLY_SIDE=1 python $B > gpurun_out/r03_v14_side1.json" \
  "200:a2:python $B > gpurun_out/r03_v14_serial2.json" \
  "200:b2:AFEM_ASSEMBLY_SIDE=1 python $B > gpurun_out/r03_v14_side2.json"
