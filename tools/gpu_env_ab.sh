#!/bin/bash
# A/B of (library variant, environment) pairs: CASES="name:lib:ENV=VAL,ENV2=VAL ..." (lib = ab/<lib>.so or "base")
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-2}); do
for c in $CASES; do
  name=${c%%:*}; rest=${c#*:}; lib=${rest%%:*}; envs=${rest#*:}; [ "$envs" = "$rest" ] && envs=""
  if [ "$lib" = base ]; then libp=""; else libp="GSPLAT_LIB=$PWD/ab/$lib.so"; fi
  env $libp ${envs//,/ } timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 ${BENCH_ARGS} > gpurun_out/ea_$name.json 2> gpurun_out/ea_$name.err; rc=$?
  echo "$name r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ea_$name.json'));c=d['roofline']['kernels']['composite'];print(d['ms_per_step'], 'sa', d['standalone_kernel_ms'], 'bodies', c['records_fetched'])" 2>/dev/null)"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/ea_$name.err; exit $rc; }
done; done
