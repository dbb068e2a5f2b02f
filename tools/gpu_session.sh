#!/bin/bash
# One-off GPU session of round 5 (overwritten per session; the committed copy
# is the last one run).  Every GPU step has its own time limit; the script
# stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS=tests bash tools/gpu_r05.sh || exit $?
STEPS=ab ROUNDS=2 VARIANTS="nofc fc prio" bash tools/gpu_r05.sh || exit $?
STEPS=ab ROUNDS=1 VARIANTS="nofc fc" BENCH_ARGS="--config 50m --steps 20 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit $?
# cut dilation on orbiting cameras: auto controller vs none (GS_CUT_DILATE=0)
for cfg in 1080p 4k; do for d in auto 0; do
  if [ $d = auto ]; then unset GS_CUT_DILATE; else export GS_CUT_DILATE=$d; fi
  timeout -k 10 300 python bench.py --config $cfg --camera orbit --steps 40 --cpu-baseline 0 --pmc 0 --settled-probe 0 \
    > gpurun_out/orbit_${cfg}_$d.json 2> gpurun_out/orbit_${cfg}_$d.err || { tail -3 gpurun_out/orbit_${cfg}_$d.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/orbit_${cfg}_$d.json'));c=d['config'];print('$cfg dilate=$d', d['ms_per_step'], c['pairs'], c['pairs_sorted'], c['open_tiles'], c['binning'], {k:round(v['ms'],4) for k,v in d['stages'].items()})"
done; done
unset GS_CUT_DILATE
