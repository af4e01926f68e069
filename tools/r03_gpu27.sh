#!/bin/bash
# edge / corner slices folded into the compact general list: parity, bench, kernel trace
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "600:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_boundary.py tests/test_gpu_distributed.py tests/test_gpu_shim.py tests/test_gpu_elasticity3d.py -q --timeout 300 --timeout-method thread" \
  "300:bench:python bench.py --no-extras --no-cpu-baseline > gpurun_out/r03_v27_bench.json" \
  "300:trace:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r03_v27/trace -o run -- python3 bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2 --cg-iters 20"
