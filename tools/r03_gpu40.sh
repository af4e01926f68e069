#!/bin/bash
# per-XCD end-time spread of the stencil kernel's persistent waves (diagnostic build libafem_wt.so)
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "200:wt215:AFEM_LIB=arcanefem_amd/libafem_wt.so python tools/wave_times.py 215" \
  "300:wt400:AFEM_LIB=arcanefem_amd/libafem_wt.so python tools/wave_times.py 400"
