#!/bin/bash
# Kernel timelines (rocprofv3 --kernel-trace) of the pipelined bench for each
# ab/<name>.so in VARIANTS: gpurun_out/tl_<name>.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${VARIANTS}; do
  rm -rf gpurun_out/tl_$v
  GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_$v -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --pmc 0 --no-stage-timing ${TL_ARGS} > gpurun_out/tl_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/tl_$v -name "*kernel_trace.csv" | head -1)
  python tools/trace_timeline.py $f 4 > gpurun_out/tl_$v.txt
  tail -14 gpurun_out/tl_$v.txt
done
