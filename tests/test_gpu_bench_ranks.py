"""The driver's multi-GPU bench path, rehearsed on one GPU: `bench.py --gpus 2`
starts two rank processes itself (torch.distributed.run, 127.0.0.1), both on
device 0 with gloo collectives (GS_BENCH_SAME_DEVICE / GS_BENCH_BACKEND are
rehearsal knobs the driver never sets).  Checks that every scheme runs and
rank 0 prints one well-formed JSON line whose value follows the headline rule
(rows, the splat-sharded scheme, whenever it is at least as fast as the
replicated bands; both timed and reported in `schemes`), named in
`scheme_choice` and `config.parallelism`.  The one-process launcher
(`--launcher group`, the default outside torchrun) runs the C-ABI group,
here over the test RCCL stub."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_bench_two_rank_rehearsal(built):
    env = dict(os.environ, GS_BENCH_BACKEND="gloo", GS_BENCH_SAME_DEVICE="1")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--launcher", "ranks", "--steps", "3", "--warmup",
           "1", "--splats", "300000", "--cpu-baseline", "0", "--pmc", "0", "--settle", "2", "--settled-probe", "4"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["config"]["global_splats"] == 300000
    assert set(d["schemes"]) == {"rows", "bands"}  # (slabs: opt-in, outside the 1e-4 tolerance)
    sc = d["schemes"]  # (rows, the splat-sharded scheme, whenever it is at least as fast as bands)
    head = "rows" if sc["rows"]["ms_per_step"] <= sc["bands"]["ms_per_step"] else "bands"
    assert abs(d["ms_per_step"] - d["schemes"][head]["ms_per_step"]) < 1e-3
    assert d["config"]["parallelism"].startswith(head + ":") and d["scheme_choice"].startswith(head + ":")
    assert "orbit" in d and d["orbit"] is None  # (the orbit probe is single-GPU)
    assert d["value"] > 0 and d["scaling"] == "strong"
    assert d["settle"]["frames"] == 2 * 2  # per timed scheme, the same count on every rank
    # the settled figure is reported beside the value, never as it
    assert d["settled"]["extra_frames"] == 4 and d["settled"]["ms_per_step"] > 0


def test_bench_group_launcher_rehearsal(built):
    """`bench.py --gpus 2` outside torchrun: one process drives both ranks
    through gs_create_sharded's group, rows pipelined (two frames in flight)
    and bands, collectives through the RCCL entry points (the test stub on
    this one-GPU box: GS_RCCL_LIB, every rank on device 0)."""
    from gaussian_splat_amd.build import RCCL_STUB
    env = dict(os.environ, GS_BENCH_SAME_DEVICE="1", GS_RCCL_LIB=str(RCCL_STUB))
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "2",
           "--splats", "300000", "--cpu-baseline", "0", "--pmc", "0", "--settled-probe", "4"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["launcher"].startswith("group")
    sc = d["schemes"]
    assert set(sc) == {"rows", "bands"} and all(v["transport"] == "rccl" for v in sc.values())
    head = "rows" if sc["rows"]["ms_per_step"] <= sc["bands"]["ms_per_step"] else "bands"
    assert abs(d["ms_per_step"] - sc[head]["ms_per_step"]) < 1e-3
    assert d["config"]["parallelism"].startswith(head + ":") and d["scheme_choice"].startswith(head + ":")
    assert "2 frames in flight" in d["config"]["parallelism"] or head == "bands"
    assert d["settled"]["ms_per_step"] > 0 and "rehearsal" in d
