#!/bin/bash
# A/B on the GPU box: bench each ab/<name>.so in VARIANTS (default: all), ROUNDS times interleaved;
# optional PARITY variants run the parity tests first.  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${PARITY}; do
  GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -m gpu \
    -k "${AB_TESTS:-1080p or config1 or cap_parity or virtual_slabs or anisotropic or config2 or config3}" --timeout 200 --timeout-method thread \
    > gpurun_out/pt_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 gpurun_out/pt_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
VARIANTS="${VARIANTS:-$(ls ab/*.so | xargs -n1 basename | sed 's/\.so$//')}"
for r in $(seq ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 ${BENCH_ARGS} \
      > gpurun_out/ab_${v}_$r.json 2> gpurun_out/ab_${v}_$r.err
    rc=$?
    echo "$v r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab_${v}_$r.json'));print(d['ms_per_step'], 'sa', d['standalone_kernel_ms'], {k:round(v['ms'],4) for k,v in d['stages'].items()})" 2>/dev/null)"
    [ $rc -eq 0 ] || { tail -3 gpurun_out/ab_${v}_$r.err; exit $rc; }
  done
done
