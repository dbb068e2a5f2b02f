#!/bin/bash
# Depth cuts on the GPU box: the -m gpu suite, then the bench with the cuts
# off and on (GS_DEPTH_SPLIT), ROUNDS times interleaved; fixed and orbiting camera.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
fi
for r in $(seq ${ROUNDS:-2}); do
  for cam in ${CAMS:-fixed orbit}; do
    for ds in 0 1; do
      GS_DEPTH_SPLIT=$ds timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 --camera $cam ${BENCH_ARGS} \
        > gpurun_out/cuts_${cam}_${ds}_$r.json 2> gpurun_out/cuts_${cam}_${ds}_$r.err; rc=$?
      echo "cam=$cam cuts=$ds r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/cuts_${cam}_${ds}_$r.json'));c=d['config'];print(d['ms_per_step'], 'pairs', c['pairs'], 'sorted', c['pairs_sorted'], 'open', c['open_tiles'], 'sa', d['standalone_kernel_ms'], {k:round(v['ms'],4) for k,v in d['stages'].items()})" 2>/dev/null)"
      [ $rc -eq 0 ] || { tail -5 gpurun_out/cuts_${cam}_${ds}_$r.err; exit $rc; }
    done
  done
done
