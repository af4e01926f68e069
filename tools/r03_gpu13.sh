#!/bin/bash
# profiles of the current kernels: C2 (stencil, 3 waves/SIMD) and C3 (x-run write-back)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "700:prof:bash tools/profile_r1.sh gpurun_out/prof_r03_v13" \
  "700:profc3:bash tools/prof_c3.sh gpurun_out/prof_r03_v13_c3"
