#!/bin/bash
# Session: the GPU suite and smoke() on HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS=tests bash tools/gpu_r05.sh || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_head.json 2> gpurun_out/bench_driver_head.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_driver_head.json'));print(d['ms_per_step'], d['value'], d['settled']['ms_per_step'], d['orbit']['ms_per_step'])"
