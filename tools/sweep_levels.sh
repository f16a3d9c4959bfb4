#!/bin/bash
# per-level smoother timing for the kernel variants (tools/bench_levels.py)
set -e
run() { timeout -k 10 120 python tools/bench_levels.py "$@"; }
run --gs-kernel 1
run --gs-kernel 2
MAD_FUSED_TILE=0 MAD_FUSED_BLOCKS=2048 run --gs-kernel 3
MAD_FUSED_TILE=1 MAD_FUSED_BLOCKS=1024 run --gs-kernel 3
MAD_FUSED_TILE=1 MAD_FUSED_BLOCKS=4096 run --gs-kernel 3
MAD_FUSED_TILE=0 MAD_FUSED_BLOCKS=8192 run --gs-kernel 3
run --smoother wj
