#!/bin/bash
# round-3 GPU batch: tests, bench, CG graph A/B, C4 kernel stats + HBM PMC with the final kernel
export TMPDIR=/tmp
B4="bench.py --n 463 --steps 5 --warmup 1 --cg-iters 20 --no-cpu-baseline --no-extras"
tools/gpu_steps.sh \
  "900:pytest:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "500:bench:python bench.py > gpurun_out/r03_v3_bench.json" \
  "200:cgnograph:AFEM_CG_GRAPH=0 python bench.py --no-extras --no-cpu-baseline > gpurun_out/r03_v3_nograph.json" \
  "200:c4trace:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r03_c4/trace -o run -- python3 $B4" \
  "200:c4fetch:rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_assemble -f csv -d gpurun_out/r03_c4/pmc_fetch -o run -- python3 $B4" \
  "200:c4write:rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_assemble -f csv -d gpurun_out/r03_c4/pmc_write -o run -- python3 $B4"
