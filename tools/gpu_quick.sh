#!/bin/bash
# Quick GPU iteration: -m gpu tests, bench, composite phase timers (debug build ab/ct.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:---pmc 0 --cpu-baseline 0} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('ms/frame',d['ms_per_step'],'value',d['value']);print('standalone',d['standalone_kernel_ms']);print({k:v['ms'] for k,v in d['stages'].items()})"
if [ -f ab/ct.so ]; then GSPLAT_LIB=ab/ct.so timeout -k 10 300 python tools/composite_counters.py > gpurun_out/ct.txt 2>&1; echo "ct rc=$?"; cat gpurun_out/ct.txt; fi
