#!/bin/bash
# A/B timing of libgsplat variants on the GPU box: each ab/<name>.so (built
# here by copying gaussian_splat_amd/libgsplat.so after a variant build) runs
# the bench with GSPLAT_LIB pointing at it.  Usage (on the box):
#   bash tools/ab.sh [bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for so in ab/*.so; do
  name=$(basename "$so" .so)
  GSPLAT_LIB="$PWD/$so" timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 "$@" \
    > "gpurun_out/ab_$name.json" 2> "gpurun_out/ab_$name.err"
  rc=$?
  echo "$name rc=$rc $(python -c "import json,sys;d=json.load(open('gpurun_out/ab_$name.json'));print(d['ms_per_step'], {k:round(v['ms'],4) for k,v in d['stages'].items()})" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
