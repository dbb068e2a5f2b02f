#!/bin/bash
# A/B of the two-slab frame (GS_DEPTH_SPLIT=1) against one slab (=0) on the bench workload.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 0 1 0 1; do
  GS_DEPTH_SPLIT=$v timeout -k 10 300 python bench.py --pmc 0 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/ab_split_$v.json 2> gpurun_out/ab_split_$v.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/ab_split_$v.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/ab_split_$v.json'));print('split=$v','ms',d['ms_per_step'],'standalone',d['standalone_kernel_ms'],{k:v['ms'] for k,v in d['stages'].items()}, 'pairs', d['config']['pairs'], d['config'].get('pairs_sorted'), d['config'].get('open_tiles'))"
done
