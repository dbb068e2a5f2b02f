#!/bin/bash
# Session: the ahead cut dilation on its own stream (base) against the dilation on the side stream before
# the projection (noahead); orbiting camera 1080p and 4K, 2 rounds; still camera 1 round; then the GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=ab ROUNDS=2 VARIANTS="base noahead" BENCH_ARGS="--camera orbit --steps 50 --settled-probe 0" bash tools/gpu_r05.sh || exit 1
STEPS=ab ROUNDS=2 VARIANTS="base noahead" BENCH_ARGS="--camera orbit --steps 50 --settled-probe 0 --config 4k" bash tools/gpu_r05.sh || exit 1
STEPS=ab ROUNDS=1 VARIANTS="base noahead" BENCH_ARGS="--orbit-probe 0" bash tools/gpu_r05.sh || exit 1
STEPS=tests bash tools/gpu_r05.sh
