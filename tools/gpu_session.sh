#!/bin/bash
# Session: the duplicate counts the filtered first pass's digits (GS_DUP_FILTER_COUNT=1) now that
# the cut test there is an LDS lookup: A/B at configs 3, 5 and 4, then the depth-cut parity tests on fc.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=ab ROUNDS=2 VARIANTS="base fc" bash tools/gpu_r05.sh || exit 1
for cfg in 50m 4k; do
  STEPS=ab ROUNDS=1 VARIANTS="base fc" BENCH_ARGS="--config $cfg --steps 20 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit 1
done
GSPLAT_LIB=$PWD/ab/fc.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread \
  -k "depth or bands or oracle or parity" > gpurun_out/pytest_fc.log 2>&1; echo "fc tests rc=$?"; tail -3 gpurun_out/pytest_fc.log
