#!/bin/bash
# The round's closing GPU evidence on HEAD, as the driver runs it: build() from source on the
# box, the whole -m gpu suite, smoke(), the default bench line, then the rocprofv3 evidence for
# the bench kernel (kernel trace + stats of the bench command, FETCH_SIZE / WRITE_SIZE passes).
# Logs: gpurun_out/<tag>_*.log, profile CSVs: gpurun_out/<tag>_prof/   (tools/final_run.sh [tag])
T=${1:-final}
bash tools/gpu_steps.sh \
  "${T}_build|600|python -c 'import __graft_entry__ as g; g.build()'" \
  "${T}_gputests|1100|python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread" \
  "${T}_smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "${T}_bench|300|python bench.py" \
  "${T}_prof|900|bash tools/profile_round.sh ${T}_prof" \
  "${T}_vcycle_prof|700|bash tools/vcycle_profiles.sh"
# (not part of the driver's run) the bench's N = 2 torchrun launch and V-cycle forms with two RCCL
# ranks sharing the one GPU
bash tools/gpu_steps.sh "${T}_rehearse|500|bash tools/rehearse_vcycles.sh"
