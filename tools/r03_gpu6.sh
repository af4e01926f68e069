#!/bin/bash
# pattern SpMV full-block path: bitwise parity, distributed split, timing
export TMPDIR=/tmp
B="bench.py --no-extras --no-cpu-baseline"
tools/gpu_steps.sh \
  "400:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread" \
  "200:bench:python $B > gpurun_out/r03_v8_bench.json" \
  "200:bench2:python $B > gpurun_out/r03_v8_bench2.json" \
  "200:cgtrace:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r03_cg8/trace -o run -- python3 $B --steps 3"
