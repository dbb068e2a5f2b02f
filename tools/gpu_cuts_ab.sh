#!/bin/bash
# Depth cuts, A/B of library variants (ab/*.so) with the cuts on, plus the
# cuts-off baseline, and one kernel timeline per variant (rocprofv3 kernel trace).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" \
    > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head; exit $rc; }
fi
for r in $(seq ${ROUNDS:-2}); do
  for v in off $(ls ab/*.so | xargs -n1 basename | sed 's/\.so$//'); do
    if [ $v = off ]; then lib=$PWD/gaussian_splat_amd/libgsplat.so; ds=0; else lib=$PWD/ab/$v.so; ds=1; fi
    GSPLAT_LIB=$lib GS_DEPTH_SPLIT=$ds timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 ${BENCH_ARGS} \
      > gpurun_out/cab_${v}_$r.json 2> gpurun_out/cab_${v}_$r.err; rc=$?
    echo "$v r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/cab_${v}_$r.json'));c=d['config'];print(d['ms_per_step'], 'sorted', c['pairs_sorted'], 'open', c['open_tiles'], 'sa', d['standalone_kernel_ms'], {k:round(v['ms'],4) for k,v in d['stages'].items()})" 2>/dev/null)"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/cab_${v}_$r.err; exit $rc; }
  done
done
for v in ${TL:-}; do
  rm -rf gpurun_out/tl_$v
  GSPLAT_LIB=$PWD/ab/$v.so GS_DEPTH_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_$v -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --settle 20 --cpu-baseline 0 --pmc 0 --no-stage-timing ${BENCH_ARGS} > gpurun_out/tl_$v.log 2>&1; rc=$?
  echo "trace $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/tl_$v -name "*kernel_trace.csv" | head -1); python tools/trace_timeline.py $f 3 > gpurun_out/tl_$v.txt; tail -60 gpurun_out/tl_$v.txt
done
