set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS=tests bash tools/gpu_r05.sh || exit $?
GSPLAT_LIB=$PWD/ab/trace.so timeout -k 10 240 python tools/composite_trace.py --out gpurun_out/trace_1080p.json > gpurun_out/trace_1080p.log 2>&1 || { tail -5 gpurun_out/trace_1080p.log; exit 1; }
cat gpurun_out/trace_1080p.log | head -30
timeout -k 10 400 python tools/binning_probe.py --frames 40 --out gpurun_out/binning_heavy_orbit.json > gpurun_out/binning_probe.log 2>&1 || { tail -5 gpurun_out/binning_probe.log; exit 1; }
head -8 gpurun_out/binning_probe.log; grep -c '"bin"' gpurun_out/binning_probe.log
timeout -k 10 300 python bench.py --config 4k --cpu-baseline 0 --pmc 0 --steps 20 --settled-probe 0 > gpurun_out/bench_4k.json 2> gpurun_out/bench_4k.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_4k.json'));print('4k', d['ms_per_step'], d['standalone_kernel_ms'], d['orbit']['ms_per_step'])"
