# kernel traces of one 512^3 refined mad_run (tools/refine_fold_ab.py) with the zero-iterate sweep and
# with the -DMAD_NO_ZERO_SWEEP build: per-kernel totals (stats CSVs under gpurun_out/zu_prof_*)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/zu_prof_new -o zu -- python3 tools/refine_fold_ab.py /tmp/a.npy 512 && \
MAD_HIP_LIB=tools/pglibs/libmad_nozero.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/zu_prof_old -o zu -- python3 tools/refine_fold_ab.py /tmp/b.npy 512
