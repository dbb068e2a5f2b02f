#!/bin/bash
# Virtual-rank probes of both exact multi-GPU schemes at BASELINE configs 3, 4
# and 5 on one GPU, and the modelled 1/2/4/8 periods (tools/scaling_model.py).
# Each probe runs under its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/scaling
run() {  # name, time limit, probe and its arguments
  n=$1; t=$2; shift 2
  timeout -k 10 $t python "$@" > gpurun_out/scaling/$n.json 2> gpurun_out/scaling/$n.err || { tail -3 gpurun_out/scaling/$n.err; exit 1; }
  grep -h "world" gpurun_out/scaling/$n.err | tail -4
}
run rows_1080p 300 tools/rows_probe.py --frames 10
run bands_1080p 300 tools/band_probe.py --frames 10
run rows_4k 300 tools/rows_probe.py --frames 10 --width 3840 --height 2160
run bands_4k 300 tools/band_probe.py --frames 10 --width 3840 --height 2160
run rows_50m 500 tools/rows_probe.py --frames 8 --splats 50000000 --width 3840 --height 2160 --sh 0 --seed 4
run bands_50m 500 tools/band_probe.py --frames 8 --splats 50000000 --width 3840 --height 2160 --sh 0 --seed 4
python tools/scaling_model.py gpurun_out/scaling/rows_1080p.json gpurun_out/scaling/bands_1080p.json \
  gpurun_out/scaling/rows_4k.json gpurun_out/scaling/bands_4k.json \
  gpurun_out/scaling/rows_50m.json gpurun_out/scaling/bands_50m.json > gpurun_out/scaling/model.json
python -c "
import json; d=json.load(open('gpurun_out/scaling/model.json'))
for c in d['configs']:
    print(c['splats'], c['frame'], 'N=1', c['n1_frame_ms'], {k: (v['chosen'], v['chosen_ms']) for k, v in c['worlds'].items()}, 'monotone', c['monotone'])"
