#!/bin/bash
# Round artifacts: default bench line (CPU baseline + PMC traffic), kernel
# stats of an unpipelined run (standalone kernel durations, the roofline's
# timing) and of the default pipelined run, PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
TAG=fif1 bash tools/gpu_prof.sh --frames-in-flight 1 || exit $?
TAG=fif2 bash tools/gpu_prof.sh || exit $?
bash tools/pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 1; }
echo artifacts-done
