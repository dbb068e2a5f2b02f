#!/bin/bash
# Round artifacts: GPU tests, driver-default bench, profiled unpipelined bench + rocprofv3 kernel
# stats of the same command, PMC summary, other BASELINE configs, heavy-tail scene, orbiting camera,
# 2-rank rehearsal, pipelined kernel timeline, virtual-rank row probes (config 4 and 5).
# Every GPU step has its own time limit; the script stops at the first failure.  STEPS selects.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
O=gpurun_out/art; mkdir -p $O
step() { name=$1; shift; echo "== $name"; "$@"; rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for s in ${STEPS:-tests driver bench prof pmc configs heavy orbit ranks timeline scaling}; do case $s in
driver) step driver bash -c "timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_command.json 2> $O/bench_driver_command.err"
       python -c "import json;d=json.load(open('$O/bench_driver_command.json'));print('driver', d['ms_per_step'], d['settled']['ms_per_step'], d['orbit']['ms_per_step'], d['roofline']['frac'], d['roofline']['kernels']['composite']['ms'])" ;;
tests) step tests bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1"
       tail -1 $O/pytest_gpu.log ;;
bench) step bench bash -c "timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err"; cat $O/bench_default.json ;;
prof)  step prof bash -c "timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
         python bench.py --frames-in-flight 1 --pmc 0 --cpu-baseline 0 > $O/bench_profiled.json 2> $O/bench_profiled.err"
       cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/bench_profiled_kernel_stats.csv; cat $O/bench_profiled.json ;;
pmc)   B="python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --pmc 0 --no-stage-timing --frames-in-flight 1"
       step sq1 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc/sq1 -o run --output-format csv -- $B > $O/pmc_sq1.log 2>&1
       step sq2 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $O/pmc/sq2 -o run --output-format csv -- $B > $O/pmc_sq2.log 2>&1
       step fetch timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc/fetch -o run --output-format csv -- $B > $O/pmc_fetch.log 2>&1
       step write timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc/write -o run --output-format csv -- $B > $O/pmc_write.log 2>&1
       python tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt; grep -A1 "composite_strip_kernel<0, 1>\|preprocess_kernel<3, 1>" $O/pmc_summary.txt ;;
pmc50m) B="python bench.py --config 50m --steps 3 --warmup 2 --cpu-baseline 0 --pmc 0 --no-stage-timing --frames-in-flight 1 --settled-probe 0 --orbit-probe 0"
       step p50sq1 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc50m/sq1 -o run --output-format csv -- $B > $O/pmc50m_sq1.log 2>&1
       step p50sq2 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $O/pmc50m/sq2 -o run --output-format csv -- $B > $O/pmc50m_sq2.log 2>&1
       step p50fetch timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc50m/fetch -o run --output-format csv -- $B > $O/pmc50m_fetch.log 2>&1
       step p50write timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc50m/write -o run --output-format csv -- $B > $O/pmc50m_write.log 2>&1
       python tools/pmc_summary.py $O/pmc50m > $O/pmc50m_summary.txt; grep -A1 "scan_duplicate\|rts_pass_kernel<1, 7, true" $O/pmc50m_summary.txt ;;
prof50m) for c in 4k 50m; do
         step prof_$c bash -c "timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- \
           python bench.py --config $c --steps 20 --frames-in-flight 1 --pmc 0 --cpu-baseline 0 --settled-probe 0 --orbit-probe 0 > $O/bench_${c}_profiled.json 2> $O/bench_${c}_profiled.err"
         cp $(find $O/prof_$c -name "*kernel_stats.csv" | head -1) $O/bench_${c}_profiled_kernel_stats.csv; done ;;
configs) for c in 1m 4k 50m; do
         step cfg_$c bash -c "timeout -k 10 600 python bench.py --config $c --steps 30 --cpu-baseline 0 > $O/bench_$c.json 2> $O/bench_$c.err"
         python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['ms_per_step'], d['value'], d['config']['binning'], d['roofline']['kernels']['composite']['ms'])"; done ;;
heavy) step heavy bash -c "timeout -k 10 600 python bench.py --profile heavy --steps 50 --cpu-baseline 0 > $O/bench_heavy.json 2> $O/bench_heavy.err"
       python -c "import json;d=json.load(open('$O/bench_heavy.json'));print('heavy', d['ms_per_step'], d['value'], d['config']['pairs'])" ;;
orbit) for p in uniform heavy; do
         step orbit_$p bash -c "timeout -k 10 600 python bench.py --camera orbit --profile $p --steps 50 --cpu-baseline 0 --pmc 0 > $O/bench_orbit_$p.json 2> $O/bench_orbit_$p.err"
         python -c "import json;d=json.load(open('$O/bench_orbit_$p.json'));c=d['config'];print('orbit $p', d['ms_per_step'], c['pairs'], c['pairs_sorted'], c['open_tiles'])"; done ;;
timeline) step timeline bash -c "timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pmc 0 --no-stage-timing --settled-probe 0 --orbit-probe 0 > $O/tl.log 2>&1"
       python tools/trace_timeline.py $(find $O/tl -name "*kernel_trace.csv" | head -1) 3 > $O/timeline_fif2.txt; head -30 $O/timeline_fif2.txt ;;
rows50m) step rows50m bash -c "timeout -k 10 900 python tools/rows_probe.py --splats 50000000 --width 3840 --height 2160 --sh 0 --frames 10 > $O/rows_probe_virtual_ranks_50m.json 2> $O/rows_probe_50m.err"
       tail -5 $O/rows_probe_50m.err ;;
rows4k) step rows4k bash -c "timeout -k 10 600 python tools/rows_probe.py --splats 6000000 --width 3840 --height 2160 --sh 3 > $O/rows_probe_virtual_ranks_4k.json 2> $O/rows_probe_4k.err"
       tail -5 $O/rows_probe_4k.err ;;
ranks) step ranks bash -c "GS_BENCH_BACKEND=gloo GS_BENCH_SAME_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --launcher ranks --steps 5 --warmup 2 --cpu-baseline 0 --pmc 0 > $O/rehearsal_2rank_gloo.log 2> $O/rehearsal_2rank_gloo.err"
       # (gloo's connection messages share stdout with the JSON line)
       grep '^{' $O/rehearsal_2rank_gloo.log > $O/rehearsal_2rank_gloo.json; cat $O/rehearsal_2rank_gloo.json
       # the one-process launcher (bench.py's default outside torchrun) through the group's RCCL
       # branches, on device 0 with the test stub of the RCCL entry points
       step group bash -c "GS_BENCH_SAME_DEVICE=1 GS_RCCL_LIB=$PWD/tests/cpp/librccl_stub.so timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 3 --cpu-baseline 0 --pmc 0 > $O/rehearsal_2rank_group_stub.json 2> $O/rehearsal_2rank_group_stub.err"
       cat $O/rehearsal_2rank_group_stub.json ;;
scaling) step scaling bash tools/gpu_scaling.sh
       mkdir -p $O/scaling && cp gpurun_out/scaling/* $O/scaling/ ;;
esac; done
