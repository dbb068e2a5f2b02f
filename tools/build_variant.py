#!/usr/bin/env python3
"""Build a libgsplat.so variant into ab/<name>.so with extra compiler flags
(A/B timing with tools/ab.sh, or debug builds such as -DGS_COMPOSITE_COUNTERS).

  python tools/build_variant.py NAME [FLAG ...]
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gaussian_splat_amd.build import build_lib  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
print(build_lib(extra=flags, build_dir=ROOT / "build" / f"variant_{name}", lib=ROOT / "ab" / f"{name}.so"))
