#!/bin/bash
# Round-6: orbiting-camera A/B of library variants (VARIANTS, ab/<v>.so), 1080p and 4K, uniform and
# heavy scenes, interleaved; the depth-cut tests on the last variant first.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V="${VARIANTS:-fd0 fd1}"; last=${V##* }
GSPLAT_LIB=$PWD/ab/$last.so timeout -k 10 400 python -u -m pytest tests/test_gpu_depth_split.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/orb_pt.log 2>&1
rc=$?; tail -2 gpurun_out/orb_pt.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-1080p 4k}; do for p in uniform heavy; do for r in 1 2; do for v in $V; do
  GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 300 python bench.py --config $cfg --camera orbit --profile $p --steps 50 --cpu-baseline 0 --pmc 0 > gpurun_out/orb_${cfg}_${p}_${v}_$r.json 2> gpurun_out/orb_${cfg}_${p}_${v}_$r.err
  rc=$?
  echo "$cfg $p $v r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/orb_${cfg}_${p}_${v}_$r.json'));c=d['config'];print(d['ms_per_step'], 'pairs', c['pairs'], 'sorted', c['pairs_sorted'], 'open', c['open_tiles'], 'dil', c['cut_dilate'])" 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/orb_${cfg}_${p}_${v}_$r.err; exit $rc; }
done; done; done; done
