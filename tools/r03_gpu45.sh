#!/bin/bash
# strip patterns with the edge runs of 32 (AFEM_DEBUG_PATTERNS)
export TMPDIR=/tmp
tools/gpu_steps.sh "200:patterns:AFEM_DEBUG_PATTERNS=1 AFEM_DEBUG_SLICES=1 python tools/pattern_probe.py 40 215"
