#!/bin/bash
# Session: the host polls the pair count's sequence word in host-mapped memory (GS_HOST_POLL) instead of an
# event in the totals kernel's dispatch packet: GPU tests on poll first, then A/B 3 rounds at 1080p, 4K 1 round.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
GSPLAT_LIB=$PWD/ab/poll.so timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_poll.log 2>&1
rc=$?; echo "poll tests rc=$rc"; tail -2 gpurun_out/pytest_poll.log; [ $rc -eq 0 ] || exit 1
STEPS=ab ROUNDS=3 VARIANTS="base poll" bash tools/gpu_r05.sh || exit 1
STEPS=ab ROUNDS=1 VARIANTS="base poll" BENCH_ARGS="--config 4k --steps 30 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit 1
