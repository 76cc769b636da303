#!/bin/bash
# Round 6: every engine's time against the accumulation chunk (params.chunk, samples per work
# unit; each chunk is its own bit-exact Tier-B image): the megakernel f64 / f32 (mk_chunk_ab.py),
# the wavefront engine (wf_bench.py chunk=), the world kernel on the globe and the Cornell box
# (world_bench.run), configurations interleaved in one process per engine.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/chunk_sweep.txt
: > $O
timeout -k 10 300 python tools/mk_chunk_ab.py ${MKN:-8} ${MKCH:-32 16 20 24} >> $O 2>/dev/null || exit 1
PREC=f32 timeout -k 10 300 python tools/mk_chunk_ab.py ${MKN:-8} ${MKCH:-32 16 20 24} >> $O 2>/dev/null || exit 1
timeout -k 10 300 python tools/wf_bench.py ${WFN:-6} ${WFCH:-chunk=32 chunk=16 chunk=20 chunk=24} >> $O 2>/dev/null || exit 1
timeout -k 10 400 python -c "
import sys; sys.path.insert(0, 'tools')
from world_bench import run
for rnd in range(${WRN:-3}):
    for sc in (7, 6):
        for ch in (${WCH:-32, 16, 20, 24}):
            r = run(sc, 3, chunk=ch)
            print('world scene', sc, 'chunk', ch, 'round', rnd, r['ms'], flush=True)
" >> $O 2>/dev/null || exit 1
cat $O
