#!/bin/bash
# round 3 re-entry: full GPU suite, the default bench line, C2 rocprof stats + PMC of the final kernel
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "900:pytest:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "600:bench:python bench.py > gpurun_out/r03_v10_bench.json" \
  "900:prof:bash tools/profile_r1.sh gpurun_out/prof_r03_v10"
