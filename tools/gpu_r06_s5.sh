#!/bin/bash
# Round-6 session 5: the -m gpu suite; front-only A/B (1080p, 50M); the 4K rank render with the
# strip-composite threshold at 512 (default) and 1024 bins (8 virtual ranks).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/rows; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s5_pt.log 2>&1
rc=$?; tail -2 gpurun_out/s5_pt.log; [ $rc -eq 0 ] || exit $rc
NOTEST=1 CFGS="1080p 50m" bash tools/gpu_r06_s2.sh 2>&1 | grep -v "passed" || true
for v in front1 strip1024; do
  GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 300 python tools/rows_probe.py --frames 10 --worlds 8 --width 3840 --height 2160 \
    > gpurun_out/rows/4k_$v.json 2> gpurun_out/rows/4k_$v.err || { tail -3 gpurun_out/rows/4k_$v.err; exit 1; }
  echo "4k $v"; grep -h "world 8" gpurun_out/rows/4k_$v.err
done
