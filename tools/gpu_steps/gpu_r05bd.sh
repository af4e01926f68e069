#!/bin/bash
# round-5 GPU step bd: C3 -- the small uniform list first with the stencil list beside it (AFEM_ELAST_SIDE=1)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/c3_ab.py 'serial: AFEM_ELAST_SIDE=0' 'side: AFEM_ELAST_SIDE=1' > gpurun_out/r05bd_ab.log 2>&1 || exit $?
