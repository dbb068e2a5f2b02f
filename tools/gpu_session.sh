#!/bin/bash
# Session: depth cuts on/off (GS_DEPTH_SPLIT) at the sparse configs: 1M @1080p SH0 and the heavy scene, 2 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do for cfg in "--config 1m" "--profile heavy"; do for ds in 1 0; do
  GS_DEPTH_SPLIT=$ds timeout -k 10 300 python bench.py $cfg --steps 50 --cpu-baseline 0 --pmc 0 --orbit-probe 0 > gpurun_out/ds.json 2> gpurun_out/ds.err || { tail -3 gpurun_out/ds.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ds.json'));c=d['config'];print('$cfg ds=$ds r$r', d['ms_per_step'], d['settled']['ms_per_step'], c['pairs'], c['pairs_sorted'], {k:round(v['ms'],4) for k,v in d['stages'].items()})"
done; done; done
