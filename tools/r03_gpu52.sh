#!/bin/bash
# placement vs timing order: four identical structures, timed in reverse build order
export TMPDIR=/tmp
tools/gpu_steps.sh "400:d4r:AB_REVERSE=1 python tools/ab_env.py AFEM_NOTHING a b 215 40 c d" \
  "400:d4:python tools/ab_env.py AFEM_NOTHING a b 215 40 c d"
