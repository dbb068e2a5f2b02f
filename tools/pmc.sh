#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, --kernel-trace only,
# never combined with sys/runtime traces).  Output: gpurun_out/pmc/<pass>/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
ARGS="${PMC_BENCH_ARGS:---steps 3 --warmup 1 --cpu-baseline 0 --no-stage-timing}"
run() {
  name=$1; shift
  rm -rf gpurun_out/pmc/$name
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc/$name -o run --output-format csv -- \
    python bench.py $ARGS > gpurun_out/pmc/$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
mkdir -p gpurun_out/pmc
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run lds SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt && cat gpurun_out/pmc/summary.txt
