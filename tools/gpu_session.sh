#!/bin/bash
# Session: the longest-first composite in two launches (GS_STRIP_SPLIT = 20 / 40 % of the bins in the
# second launch, running into the next frame's chain) against one launch; 1080p 2 rounds, 4K 1 round;
# then the depth-cut GPU tests on split20.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=ab ROUNDS=2 VARIANTS="base split20 split40" BENCH_ARGS="--orbit-probe 0" bash tools/gpu_r05.sh || exit 1
STEPS=ab ROUNDS=1 VARIANTS="base split20 split40" BENCH_ARGS="--config 4k --steps 30 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit 1
GSPLAT_LIB=$PWD/ab/split20.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread \
  -k "depth or parity or oracle" > gpurun_out/pytest_split.log 2>&1; echo "split tests rc=$?"; tail -2 gpurun_out/pytest_split.log
