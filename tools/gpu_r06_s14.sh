#!/bin/bash
# Round-6 session 14: the -m gpu suite on HEAD, then an A/B of VARIANTS (ab/<v>.so) at 1080p, 50M, 4K.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s14_pt.log 2>&1
rc=$?; tail -2 gpurun_out/s14_pt.log; [ $rc -eq 0 ] || exit $rc
NOTEST=1 bash tools/gpu_r06_s2.sh
