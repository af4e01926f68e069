#!/bin/bash
# final state after the vectorized CG kernels: smoke, whole GPU suite, default bench line, C2 kernel trace
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "900:pytest:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "700:bench:python bench.py > gpurun_out/r03_v55_bench.json" \
  "300:trace:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r03_v55/trace -o run -- python3 bench.py --no-extras --no-cpu-baseline --steps 10 --warmup 2 --cg-iters 20"
