#!/bin/bash
# kernel trace of one rank's pipelined frames (tools/rank_pipe_probe.py, 1080p, world 8, rank 3)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/rtl -o run --output-format csv -- python tools/rank_pipe_probe.py --world 8 --ranks 3 --frames 20 > gpurun_out/rtl.log 2>&1 || exit 1
python tools/trace_timeline.py $(find gpurun_out/rtl -name "*kernel_trace.csv" | head -1) 3 > gpurun_out/rtl_timeline.txt
tail -60 gpurun_out/rtl_timeline.txt
