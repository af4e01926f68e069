#!/bin/bash
# CG with the reductions fused into the SpMV / update kernels (last block sums the partials): A/B + CG tests + bench
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:cgab:python tools/cg_probe.py AFEM_CG_FUSED 0 1 --iters 100 --reps 5" \
  "600:pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_multigrid.py tests/test_gpu_distributed.py tests/test_gpu_boundary.py tests/test_gpu_shim.py -q --timeout 300 --timeout-method thread" \
  "300:bench:python bench.py --no-extras --no-cpu-baseline > gpurun_out/r03_v37_bench.json"
