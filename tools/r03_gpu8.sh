#!/bin/bash
# slice balancing by strip length on the unstructured leg (A/B over the window size)
export TMPDIR=/tmp
B="bench.py --legs unstructured --no-cpu-baseline --steps 5 --warmup 2"
tools/gpu_steps.sh \
  "300:b0:python $B > gpurun_out/r03_sb0.json" \
  "300:b128:AFEM_SLICE_BALANCE=128 python $B > gpurun_out/r03_sb128.json" \
  "300:b256:AFEM_SLICE_BALANCE=256 python $B > gpurun_out/r03_sb256.json" \
  "300:b512:AFEM_SLICE_BALANCE=512 python $B > gpurun_out/r03_sb512.json" \
  "300:b1024:AFEM_SLICE_BALANCE=1024 python $B > gpurun_out/r03_sb1024.json"
