# FP64 fused-sweep grid size (MAD_FP64_FUSED_BLOCKS probe builds), alternated
set -o pipefail
for r in 1 2; do
  timeout -k 10 150 python -u tools/fp64_blocks_ab.py || exit 1
  for v in 256 512 1024; do MAD_HIP_LIB=tools/pglibs/libmad_f64b$v.so timeout -k 10 150 python -u tools/fp64_blocks_ab.py || exit 1; done
done
