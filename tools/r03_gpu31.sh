#!/bin/bash
# round 3 state after the edge/corner order: full GPU suite, default bench line, C2 + C3 rocprof stats + PMC
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "900:pytest:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "700:bench:python bench.py > gpurun_out/r03_v31_bench.json" \
  "700:prof:bash tools/profile_r1.sh gpurun_out/prof_r03_v31" \
  "700:profc3:bash tools/prof_c3.sh gpurun_out/prof_r03_v31_c3"
