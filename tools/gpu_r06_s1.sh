#!/bin/bash
# Round-6 session 1: depth-cut / parity / config GPU tests on the default library, then
# front-only emission A/B (ab/front0 = off, front1 = on, front1nc = on without the duplicate's digit counts).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_bench_ranks.py tests/test_gpu_depth_split.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/s1_pt.log 2>&1
rc=$?; tail -3 gpurun_out/s1_pt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s1_cfg.log 2>&1
rc=$?; tail -3 gpurun_out/s1_cfg.log; [ $rc -eq 0 ] || exit $rc
for cfg in 1080p 50m; do
 for r in 1 2; do for v in front0 front1 front1nc; do
  GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 300 python bench.py --config $cfg --cpu-baseline 0 --pmc 0 --steps 30 --settle 30 $([ $cfg = 50m ] && echo --orbit-probe 0 --settled-probe 0) > gpurun_out/s1_${cfg}_${v}_$r.json 2> gpurun_out/s1_${cfg}_${v}_$r.err
  rc=$?
  echo "$cfg $v r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/s1_${cfg}_${v}_$r.json'));print(d['ms_per_step'], 'orbit', (d.get('orbit') or {}).get('ms_per_step'), 'sa', d['standalone_kernel_ms'], {k:round(v['ms'],4) for k,v in d['stages'].items()})" 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/s1_${cfg}_${v}_$r.err; exit $rc; }
 done; done
done
