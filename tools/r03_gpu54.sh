#!/bin/bash
# CG vector kernels with 16-B accesses (two rows per thread): A/B + CG tests
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:cgab:python tools/cg_probe.py AFEM_CG_VEC2 0 1 --iters 100 --reps 5" \
  "300:cgab2:python tools/cg_probe.py AFEM_CG_VEC2 1 0 --iters 100 --reps 5" \
  "600:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_multigrid.py tests/test_gpu_distributed.py tests/test_gpu_boundary.py -q --timeout 300 --timeout-method thread"
