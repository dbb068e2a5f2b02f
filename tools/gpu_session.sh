#!/bin/bash
# Session: packed two-pixel composite body (GS_STRIP_PK) A/B at config 3 (+ 4K), then the
# GPU parity suite on the pk library (the packed body must keep every frame bit-exact).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=ab ROUNDS=2 VARIANTS="base pk" bash tools/gpu_r05.sh || exit 1
STEPS=ab ROUNDS=1 VARIANTS="base pk" BENCH_ARGS="--config 4k --steps 20 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit 1
GSPLAT_LIB=$PWD/ab/pk.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread \
  -k "composite or depth or oracle or parity or strip or mode or live" > gpurun_out/pytest_pk.log 2>&1; echo "pk tests rc=$?"; tail -3 gpurun_out/pytest_pk.log
