cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in "" "--config 1m" "--config 4k"; do
  GS_LOOKBACK=2 timeout -k 10 200 python bench.py --steps 4 --warmup 2 --cpu-baseline 0 --pmc 0 $c > gpurun_out/lb_chk.json 2> gpurun_out/lb_chk.err || { tail -5 gpurun_out/lb_chk.err; exit 1; }
  echo "== check $c"; grep lookback gpurun_out/lb_chk.err | sort | uniq -c | head -5
done
CFGS="- GS_LOOKBACK=1" ROUNDS=3 TL="0 1" TL_LINES=14 bash tools/gpu_sched_ab.sh
