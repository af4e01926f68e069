#!/bin/bash
# placement effect: two identical structures built one after the other, assemblies timed interleaved
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:d1:python tools/ab_env.py AFEM_NOTHING a b 215 40" \
  "300:d2:python tools/ab_env.py AFEM_NOTHING a b 215 40"
