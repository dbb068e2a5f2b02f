#!/bin/bash
# One-off GPU session of round 5 (overwritten per session; the committed copy
# is the last one run).  Every GPU step has its own time limit; the script
# stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS=tests bash tools/gpu_r05.sh || exit $?
STEPS=ab ROUNDS=2 VARIANTS="nofc8 fc8 noprio" bash tools/gpu_r05.sh || exit $?
for cfg in 50m 4k; do
  STEPS=ab ROUNDS=1 VARIANTS="nofc8 fc8" BENCH_ARGS="--config $cfg --steps 20 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit $?
done
STEPS=ab ROUNDS=1 VARIANTS="nofc8 fc8" BENCH_ARGS="--profile heavy --steps 20 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit $?
GSPLAT_LIB=$PWD/ab/trace.so timeout -k 10 240 python tools/composite_trace.py --out gpurun_out/trace_1080p_prio.json > gpurun_out/trace_prio.log 2>&1 || { tail -5 gpurun_out/trace_prio.log; exit 1; }
grep -E "span|mean_resident|drain|last_start" gpurun_out/trace_1080p_prio.json
