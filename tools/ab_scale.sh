# A/B of ab/*.so at the default and the 50M @ 4K configs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/ab.sh --steps 30 && bash tools/ab.sh --steps 10 --warmup 2 --splats 50000000 --width 3840 --height 2160
