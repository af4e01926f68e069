#!/bin/bash
# k_apply_bcs 4 rows per thread: boundary/parity tests, C2 step timing + kernel trace, C4 profile of the final kernel
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "500:pytest:python -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_parity.py tests/test_gpu_shim.py -q --timeout 300 --timeout-method thread" \
  "300:bench:python bench.py --no-extras --no-cpu-baseline > gpurun_out/r03_v21_bench.json" \
  "300:trace:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r03_v21/trace -o run -- python3 bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2 --cg-iters 20" \
  "700:profc4:B='bench.py --legs c4 --no-cpu-baseline --steps 3 --warmup 1 --cg-iters 5 --c4-n 463' bash tools/profile_r1.sh gpurun_out/prof_r03_v21_c4"
