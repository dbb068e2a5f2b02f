#!/bin/bash
# Same-box A/B of HEAD against an earlier commit (e.g. the previous round's
# final tree), to catch regressions that per-change A/Bs miss.
#   here:    bash tools/round_ab.sh prepare <commit>   # worktree -> ./cmp_tree, built in place
#   GPU box: bash tools/round_ab.sh run [rounds]         # interleaved default benches
#   here:    bash tools/round_ab.sh clean
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
case "$1" in
prepare)
  rm -rf /tmp/cmp_wt cmp_tree && git worktree add -f /tmp/cmp_wt "$2" -q
  (cd /tmp/cmp_wt && python -c "import __graft_entry__ as g; g.build()")
  mkdir cmp_tree && (cd /tmp/cmp_wt && tar cf - --exclude=.git --exclude=gpurun_out --exclude=build --exclude=ab --exclude=profiles .) | (cd cmp_tree && tar xf -)
  grep -q "^cmp_tree/" .git/info/exclude || echo "cmp_tree/" >> .git/info/exclude ;;
run)
  set +e; mkdir -p gpurun_out; export TMPDIR=/tmp
  for r in $(seq "${2:-3}"); do
    timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 > gpurun_out/head_$r.json 2>/dev/null || exit 1
    (cd cmp_tree && timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 > ../gpurun_out/cmp_$r.json 2>/dev/null) || exit 1
    python -c "import json;a=json.load(open('gpurun_out/head_$r.json'));b=json.load(open('gpurun_out/cmp_$r.json'));print('round', $r, 'head', a['ms_per_step'], 'cmp', b['ms_per_step'])"
  done ;;
clean)
  rm -rf cmp_tree; git worktree remove --force /tmp/cmp_wt 2>/dev/null; git worktree prune ;;
esac
