#!/bin/bash
# new boundary-aware order: all bench legs (no CPU baselines) + C3 kernel trace
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "700:bench:python bench.py --no-cpu-baseline > gpurun_out/r03_v29_bench.json" \
  "300:c3trace:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r03_v29_c3/trace -o run -- python3 tools/c3_probe.py 170 10"
