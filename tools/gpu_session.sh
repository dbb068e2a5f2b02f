#!/bin/bash
# Session: issue priority of the projection's waves in the co-run (GS_PRE_PRIO) A/B: base (0), pp1 (1), pp3 (3),
# pp3c2 (3, composite's first batches at 2 instead of 3); default bench (orbit probe off), 2 rounds; 4K 1 round.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
STEPS=ab ROUNDS=2 VARIANTS="base pp1 pp3 pp3c2" BENCH_ARGS="--orbit-probe 0" bash tools/gpu_r05.sh || exit 1
STEPS=ab ROUNDS=1 VARIANTS="base pp1 pp3 pp3c2" BENCH_ARGS="--config 4k --steps 30 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit 1
