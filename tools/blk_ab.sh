set -o pipefail
for lib in ${LIBS:-default blk128 blk512}; do
  if [ $lib = default ]; then unset MAD_HIP_LIB; else export MAD_HIP_LIB=tools/pglibs/libmad_$lib.so; fi
  for rep in 1 2; do
    echo "== $lib rep $rep 256^3 sweeps: $(timeout -k 10 60 python tools/vcycle_trace.py --size 256 --sweeps 400 | tail -1)"
    echo "== $lib rep $rep rank 4 of 8 slab sweeps: $(timeout -k 10 60 python tools/vcycle_trace.py --ranks 8 --sweeps 400 | tail -1)"
    echo "== $lib rep $rep rank 4 of 8 V-cycle (RCCL-SOLO): $(timeout -k 10 60 python tools/vcycle_trace.py --ranks 8 --rccl --cycles 40 2>&1 | grep ms_per | tail -1)"
  done
done
