#!/bin/bash
# Per-rank sweep time of the 8-rank z-slab (SOLO transport) under fused-sweep tile /
# chunking variants, with the one-GPU sweep for reference.
set -e
run() { echo "== $*"; env "$@" timeout -k 10 150 python tools/bench_local_split.py --solo 1 8; }
run MAD_X=0
run MAD_FUSED_TILE=0
run MAD_FUSED_TILE=0 MAD_FUSED_BLOCKS=512
run MAD_BOUNDARY_PLANES=4
