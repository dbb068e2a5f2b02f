#!/bin/bash
# Session: the new depth-cut table-size test, then the full GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_depth_split.py -x -v --timeout 300 --timeout-method thread -k cut_table_sizes > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "new test rc=$rc"; tail -5 gpurun_out/pytest_new.log; [ $rc -eq 0 ] || exit $rc
STEPS=tests bash tools/gpu_r05.sh
