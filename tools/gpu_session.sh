#!/bin/bash
# Session: GPU tests (band-local binning with depth cuts, behind-the-cut marks),
# then the band probes at configs 3, 4 and 5 (virtual ranks).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/scaling
STEPS=tests bash tools/gpu_r05.sh || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed" gpurun_out/pytest_gpu.log || exit 1
run() { n=$1; t=$2; shift 2
  timeout -k 10 $t python tools/band_probe.py "$@" > gpurun_out/scaling/$n.json 2> gpurun_out/scaling/$n.err || { tail -3 gpurun_out/scaling/$n.err; exit 1; }
  grep -h world gpurun_out/scaling/$n.err; }
run bands_1080p 300 --frames 10
run bands_4k 300 --frames 10 --width 3840 --height 2160
run bands_50m 500 --frames 8 --splats 50000000 --width 3840 --height 2160 --sh 0 --seed 4
# A/B: pw8 (every sort pass at 8 waves per SIMD), ipt4 (2048-pair sort tiles), nomask (timing
# ablation: no exclusion masks in the projection; changes the pairs) at configs 5 and 3
STEPS=ab ROUNDS=1 VARIANTS="base tag pw8 ipt4 nomask" BENCH_ARGS="--config 50m --steps 20 --settled-probe 0 --orbit-probe 0" bash tools/gpu_r05.sh || exit 1
STEPS=ab ROUNDS=2 VARIANTS="base notag tag" bash tools/gpu_r05.sh || exit 1
