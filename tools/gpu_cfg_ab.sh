#!/bin/bash
# One config under several environments, interleaved: CFG (bench --config), ENVS ("name:ENV=VAL,ENV2=VAL ..."),
# ROUNDS.  Prints frame ms, binning, pairs, pairs sorted and the stage times of each run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-1}); do
for c in $ENVS; do
  name=${c%%:*}; envs=${c#*:}; [ "$envs" = "$c" ] && envs=""
  env ${envs//,/ } timeout -k 10 600 python bench.py --config ${CFG:-50m} --steps ${STEPS:-20} --cpu-baseline 0 --pmc 0 ${BENCH_ARGS} \
    > gpurun_out/cfg_${CFG:-50m}_$name.json 2> gpurun_out/cfg_${CFG:-50m}_$name.err; rc=$?
  echo "$name r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/cfg_${CFG:-50m}_$name.json'));c=d['config'];print(d['ms_per_step'], c['binning'], c['pairs'], c['pairs_sorted'], c['open_tiles'], {k:round(v['ms'],4) for k,v in d['stages'].items()})" 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/cfg_${CFG:-50m}_$name.err; exit $rc; }
done; done
