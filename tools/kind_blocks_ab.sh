# fused-sweep grid 256 (current default) vs 2048 (pre-change build) for the isotropic kind, fp32 / fp64
set -o pipefail
for r in 1 2; do
  for p in fp32 fp64; do
    timeout -k 10 150 python -u tools/kind_blocks_ab.py 1 $p && \
    MAD_HIP_LIB=tools/pglibs/libmad_b2048.so timeout -k 10 150 python -u tools/kind_blocks_ab.py 1 $p || exit 1
  done
done
