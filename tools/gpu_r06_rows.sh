#!/bin/bash
# Round-6: per-rank compute of the row scheme at 8 virtual ranks (tools/rows_probe.py),
# depth cuts on (default) and off (GS_DEPTH_SPLIT=0), with the rank-0 stage breakdown.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/rows; export TMPDIR=/tmp
for cfg in "1080p" "4k --width 3840 --height 2160" "50m --splats 50000000 --width 3840 --height 2160 --sh 0 --seed 4"; do
  set -- $cfg; n=$1; shift
  for ds in 1 0; do
    GS_DEPTH_SPLIT=$ds timeout -k 10 400 python tools/rows_probe.py --frames 10 --worlds 1,8 --stages 8 "$@" \
      > gpurun_out/rows/${n}_ds$ds.json 2> gpurun_out/rows/${n}_ds$ds.err || { tail -3 gpurun_out/rows/${n}_ds$ds.err; exit 1; }
    echo "$n ds=$ds"; grep -h "world 8: compute\|rank 0:" gpurun_out/rows/${n}_ds$ds.err
  done
done
