cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for sch in rows slabs; do
  GS_BENCH_BACKEND=gloo GS_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --scheme $sch > gpurun_out/rehearsal_$sch.json 2> gpurun_out/rehearsal_$sch.err
  rc=$?; echo "rehearsal $sch rc=$rc"; grep '^{' gpurun_out/rehearsal_$sch.json | tail -1; [ $rc -eq 0 ] || exit $rc
done
