#!/bin/bash
# edge runs of 32: block-3 back on the workgroup kernel; tests + all bench legs + C3 trace
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "600:pytest:python -u -m pytest tests/test_gpu_elasticity3d.py tests/test_gpu_parity.py tests/test_gpu_passmo.py -q --timeout 300 --timeout-method thread" \
  "700:bench:python bench.py --no-cpu-baseline > gpurun_out/r03_v30_bench.json" \
  "300:c3trace:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r03_v30_c3/trace -o run -- python3 tools/c3_probe.py 170 10"
