#!/bin/bash
# global V-cycle over z-slabs: multigrid tests (one rank) + distributed solves
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "600:pytest:python -u -m pytest tests/test_gpu_multigrid.py tests/test_gpu_distributed.py -x -v -s --timeout 300 --timeout-method thread"
