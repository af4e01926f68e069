#!/bin/bash
# round-3 final profiles: C4 (north-star size) and the unstructured leg with the final kernels
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "700:profc4:B='bench.py --legs c4 --no-cpu-baseline --steps 3 --warmup 1 --cg-iters 5 --c4-n 463' bash tools/profile_r1.sh gpurun_out/prof_r03_v39_c4" \
  "700:profu:B='tools/unstructured_probe.py 6' bash tools/profile_r1.sh gpurun_out/prof_r03_v39_u k_assemble_strip"
