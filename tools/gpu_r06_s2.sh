#!/bin/bash
# Round-6 session 2: depth-cut / config tests on the default library, then the
# front-only emission A/B again (ab/front0 = off, front1 = on) at 1080p, 4K, 50M.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_depth_split.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s2_pt.log 2>&1
rc=$?; tail -3 gpurun_out/s2_pt.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-1080p 50m 4k}; do
 for r in 1 2; do for v in ${VARIANTS:-front0 front1}; do
  GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 300 python bench.py --config $cfg --cpu-baseline 0 --pmc 0 --steps 30 --settle 30 $([ $cfg = 50m ] && echo --orbit-probe 0 --settled-probe 0) > gpurun_out/s2_${cfg}_${v}_$r.json 2> gpurun_out/s2_${cfg}_${v}_$r.err
  rc=$?
  echo "$cfg $v r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/s2_${cfg}_${v}_$r.json'));print(d['ms_per_step'], 'orbit', (d.get('orbit') or {}).get('ms_per_step'), {k:round(v['ms'],4) for k,v in d['stages'].items()})" 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/s2_${cfg}_${v}_$r.err; exit $rc; }
 done; done
done
