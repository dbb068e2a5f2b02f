#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/pytest1.log 2>&1
rc=$?; tail -30 gpurun_out/pytest1.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 50 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?
cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err; echo "bench rc=$rc"
