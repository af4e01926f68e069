#!/bin/bash
# the box's edge / corner slices through the general list (fold, default) or the uniform instance: A/B
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:f215:python tools/ab_env.py AFEM_ASSEMBLY_FOLD 1 0 215 40" \
  "300:f215b:python tools/ab_env.py AFEM_ASSEMBLY_FOLD 0 1 215 40"
