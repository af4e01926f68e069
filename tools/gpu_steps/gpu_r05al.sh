#!/bin/bash
# round-5 GPU step al: where the cube kernel's time goes now (diagnostic ablations on the default V = 880;
# values wrong by design): no full-flush value stores (+1), one LDS add per cube (+2), no tet arithmetic
# (+4), no complete-layer flush (+8)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_knobs.py --n 215 --rounds 4 'default:' 'nostore: AFEM_CUBES_V=881' 'oneadd: AFEM_CUBES_V=882' 'noarith: AFEM_CUBES_V=884' 'noflush: AFEM_CUBES_V=888' > gpurun_out/r05al_diag.log 2>&1 || exit $?
