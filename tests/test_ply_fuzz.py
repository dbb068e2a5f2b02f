"""PLY ingest under AddressSanitizer + UndefinedBehaviorSanitizer (host code
only): tests/host/fuzz_ply.cpp loads every golden PLY fixture and seeded
mutants of each (truncated headers and payloads, flipped header bytes,
absurd or malformed vertex counts, dropped / duplicated property lines)
through PLYLoader::load and the direct mmap path (planes_from_ply).  A loader
may reject a file; it must not touch memory it does not own, hit undefined
behaviour, or allocate for a vertex count the file cannot hold."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_ply_ingest_fuzz_asan_ubsan(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "fuzz_ply"
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           f"-I{ROOT / 'include'}", f"-I{ROOT / 'gaussian_splat_amd/csrc/host'}",
           str(ROOT / "tests/host/fuzz_ply.cpp"), str(ROOT / "gaussian_splat_amd/csrc/host/scene_io.cpp"),
           str(ROOT / "gaussian_splat_amd/csrc/host/ply_loader.cpp"), "-o", str(exe), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "sanitize" in r.stderr:
        pytest.skip("sanitizer runtime unavailable: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr[-2000:]
    files = sorted(str(p) for p in (ROOT / "tests/golden/ply").glob("*.ply"))
    assert files
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1", GS_LOAD_THREADS="4")
    work = tmp_path / "mut"
    work.mkdir()
    r = subprocess.run([str(exe), str(work), "120"] + files, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-1000:] + r.stderr[-3000:])
    assert "fuzz_ply:" in r.stdout
