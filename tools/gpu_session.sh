#!/bin/bash
# Session: the host waits for a buffer set's last reader instead of a wait packet on the side stream
# (GS_HOST_SET_WAIT) A/B, default bench (orbit probe on), 3 rounds; 4K 1 round.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=ab ROUNDS=3 VARIANTS="base hostwait" bash tools/gpu_r05.sh || exit 1
STEPS=ab ROUNDS=1 VARIANTS="base hostwait" BENCH_ARGS="--config 4k --steps 30 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit 1
