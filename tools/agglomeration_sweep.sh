#!/bin/bash
# Per-rank sweep / V-cycle cost (SOLO transport, interior rank) against mad_desc.min_slab_planes
# (how deep the z-slab decomposition goes before the coarse levels are replicated).
#   tools/agglomeration_sweep.sh [values...]   -> one JSON line per (value, ranks)
set -e
for m in "${@:-0 8 16 32}"; do
  timeout -k 10 300 python tools/bench_local_split.py --msp "$m" --solo 1 2 4 8
done
