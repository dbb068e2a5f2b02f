#!/bin/bash
# GPU: a subset of the -m gpu tests (PYTEST_K selects), verbose, bounded.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_subset.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_subset.log; echo "pytest rc=$rc"; exit $rc
