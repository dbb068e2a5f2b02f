#!/bin/bash
# band cull: the -m gpu suite on HEAD, then band_probe with (HEAD) and without (ab/bc0.so) it
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/bc_pt.log 2>&1
rc=$?; tail -2 gpurun_out/bc_pt.log; [ $rc -eq 0 ] || exit $rc
for cfg in "" "--width 3840 --height 2160" "--splats 50000000 --width 3840 --height 2160 --sh 0 --seed 4 --frames 8"; do
  for v in bc0 head; do
    L=""; [ $v = bc0 ] && L="GSPLAT_LIB=$PWD/ab/bc0.so"
    env $L timeout -k 10 400 python tools/band_probe.py --worlds 1,2,4,8 $cfg > gpurun_out/bc_$v.json 2> gpurun_out/bc_$v.err || exit 1
    echo "$v $cfg"; grep band_probe gpurun_out/bc_$v.err
  done
done
