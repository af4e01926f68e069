#!/bin/bash
# ELL pattern SpMV (one rank): full GPU suite + C2/C4 bench
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "900:pytest:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "500:bench:python bench.py --legs c4 --no-cpu-baseline > gpurun_out/r03_v19_bench.json" \
  "300:benchpat:AFEM_SPMV=pat python bench.py --no-extras --no-cpu-baseline > gpurun_out/r03_v19_pat.json"
