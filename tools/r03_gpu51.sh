#!/bin/bash
# placement effect: four identical structures built one after the other, assemblies timed interleaved
export TMPDIR=/tmp
tools/gpu_steps.sh "400:d4:python tools/ab_env.py AFEM_NOTHING a b 215 40 c d"
