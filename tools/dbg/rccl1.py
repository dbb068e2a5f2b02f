#!/usr/bin/env python3
"""Debug: torch.distributed over RCCL with one rank on this box, step by step
(init, a plain all_to_all_single, then the rows scheme's exchange and render)."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
t0 = time.time()


def log(*a):
    print(f"[rccl1 {time.time() - t0:7.2f}s]", *a, flush=True)


import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
log("init")
from gaussian_splat_amd.distributed import init_ranks  # noqa: E402

init_ranks("nccl", 60, device=torch.device("cuda:0"), rank=0, world_size=1)
log("init done")
x = torch.arange(8, device="cuda", dtype=torch.int64)
y = torch.empty_like(x)
dist.all_to_all_single(y, x)
torch.cuda.synchronize()
log("all_to_all_single", y.tolist())
b = torch.arange(64, device="cuda", dtype=torch.uint8)
c = torch.empty_like(b)
dist.all_to_all_single(c, b, [64], [64])
torch.cuda.synchronize()
log("all_to_all_single splits uint8 ok", bool((c == b).all()))
from gaussian_splat_amd import Options, scene as S  # noqa: E402
from gaussian_splat_amd.api import default_camera  # noqa: E402
from gaussian_splat_amd.distributed import HipShardBackend, ShardedRenderer, exchange_start  # noqa: E402

W, H = 800, 600
sc = S.activate(S.synthetic_raw(60000, seed=51, aspect=W / H), 3)
be = HipShardBackend(sc, 0, 1, 0, Options(sh_degree=3, crop=False), 0)
cam = default_camera(W, H)
V, P = cam.getViewMatrix(), cam.getProjectionMatrix()
send, counts = be.project(V, P, W, H)
torch.cuda.synchronize()
log("projected", counts)
pend = exchange_start(send, counts, be.xregions, 1, None)
log("exchange started")
recv, n = pend.wait()
torch.cuda.synchronize()
log("exchange done", n)
band = be.render(recv, n, W, H)
torch.cuda.synchronize()
log("rendered")
f = ShardedRenderer(be, 0, 1).render(V, P, W, H)
torch.cuda.synchronize()
log("sharded frame", tuple(f.shape))
dist.destroy_process_group()
log("done")
