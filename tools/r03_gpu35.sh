#!/bin/bash
# RCCL with 2 ranks on the one GPU of the box (diagnostic: does RCCL accept it?)
# (the bench.py override this run used was removed afterwards: RCCL refused)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "240:rccl2:AFEM_RCCL_SHARED_GPU=1 NCCL_DEBUG=WARN python bench.py --gpus 2 --comm rccl --no-extras --no-cpu-baseline --steps 3 --warmup 1 --cg-iters 10 --n 64 > gpurun_out/r03_v35_rccl2.json"
