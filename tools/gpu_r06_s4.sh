#!/bin/bash
# Round-6 session 4: the whole -m gpu suite, then the virtual-rank scaling probes (tools/gpu_scaling.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s4_pt.log 2>&1
rc=$?; tail -3 gpurun_out/s4_pt.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_scaling.sh
