#!/bin/bash
# round-3 final state: smoke, the whole GPU suite, the default bench line
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "900:pytest:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "700:bench:python bench.py > gpurun_out/r03_v47_bench.json"
