#!/bin/bash
# Round-6 session 3: kernel stats + PMC of the 50M frame (front-only emission), then the rows probes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS="prof pmc" VARIANTS=front1 BENCH_ARGS="--config 50m" PROF_ARGS="--config 50m" bash tools/gpu_r05.sh || exit 1
cp gpurun_out/prof_kernel_stats.csv gpurun_out/s3_50m_kernel_stats.csv
bash tools/gpu_r06_rows.sh
