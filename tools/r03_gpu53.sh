#!/bin/bash
# the N>1 bench flow rehearsed on one GPU (host transport): weak (C2 per rank) and strong (C4 in 2 slabs)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "400:weak2:python bench.py --gpus 2 --comm host --no-extras --no-cpu-baseline --steps 10 --warmup 3 --cg-iters 20 > gpurun_out/r03_v53_weak2.json" \
  "500:strong2:python bench.py --gpus 2 --comm host --scaling strong --no-extras --no-cpu-baseline --steps 5 --warmup 2 --cg-iters 10 > gpurun_out/r03_v53_strong2.json" \
  "200:rccl2:python bench.py --gpus 2 --comm rccl --no-extras --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r03_v53_rccl2.log 2>&1; echo rc=\$? >> gpurun_out/r03_v53_rccl2.log; true"
