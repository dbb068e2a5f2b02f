#!/bin/bash
# Round-5 GPU session: the -m gpu suite on the default library, then
# interleaved A/B benches of ab/*.so (default bench + standalone kernel times),
# then a rocprofv3 kernel-stats pass of the default library's unpipelined frame.
# Every GPU step runs under its own time limit; a fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS="${STEPS:-tests ab prof}"
chk() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stop after $2"; exit "$rc"; fi; }
for s in $STEPS; do case $s in
  tests)
    timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread ${PYTEST_ARGS} \
      > gpurun_out/pytest_gpu.log 2>&1
    chk $? pytest; tail -4 gpurun_out/pytest_gpu.log ;;
  ab)
    VARIANTS="${VARIANTS:-$(ls ab/*.so | xargs -n1 basename | sed 's/\.so$//')}"
    for r in $(seq ${ROUNDS:-2}); do for v in $VARIANTS; do
      GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 ${BENCH_ARGS} \
        > gpurun_out/ab_${v}_$r.json 2> gpurun_out/ab_${v}_$r.err
      rc=$?
      echo "$v r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab_${v}_$r.json'));print(d['ms_per_step'], 'settled', d.get('settled'), 'sa', d['standalone_kernel_ms'], {k:round(v['ms'],4) for k,v in d['stages'].items()})" 2>/dev/null)"
      [ $rc -eq 0 ] || { tail -3 gpurun_out/ab_${v}_$r.err; exit $rc; }
    done; done ;;
  prof)
    rm -rf gpurun_out/prof
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --pmc 0 --frames-in-flight 1 ${PROF_ARGS} > gpurun_out/prof.json 2> gpurun_out/prof.err
    chk $? rocprof; find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_kernel_stats.csv \;
    head -30 gpurun_out/prof_kernel_stats.csv | cut -d, -f1-8 ;;
  pmc)
    # per-variant PMC of the unpipelined frame's kernels (one counter group per rocprofv3 run)
    VARIANTS="${VARIANTS:-$(ls ab/*.so | xargs -n1 basename | sed 's/\.so$//')}"
    for v in $VARIANTS; do
      for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
                 "SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_IFETCH SQ_IFETCH_LEVEL SQ_BUSY_CYCLES" \
                 ${PMC_TRAFFIC-"FETCH_SIZE" "WRITE_SIZE"}; do
        n=$(echo $grp | cut -d' ' -f1)
        rm -rf gpurun_out/pmc_$v/$n; mkdir -p gpurun_out/pmc_$v
        GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc_$v/$n -o run \
          --output-format csv -- python bench.py --steps 5 --warmup 2 --settled-probe 0 --orbit-probe 0 --cpu-baseline 0 \
          --pmc 0 --no-stage-timing --frames-in-flight 1 ${BENCH_ARGS} > gpurun_out/pmc_$v/$n.log 2>&1
        chk $? "pmc $v $n"
      done
      python tools/pmc_summary.py gpurun_out/pmc_$v > gpurun_out/pmc_$v/summary.txt
      grep -A1 "composite" gpurun_out/pmc_$v/summary.txt
    done ;;
esac; done
