"""The multi-GPU headline rule of bench.py (README): `value` is
the rows scheme's whenever rows is at least as fast as bands at that world
size; otherwise it is bands', named as the replicated scheme."""
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _bench():
    spec = importlib.util.spec_from_file_location("gs_bench", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)  # (defines the functions; main runs only as a script)
    return m


def test_rows_headline_when_at_least_as_fast():
    b = _bench()
    assert b.headline({"rows": {"ms": 0.30}, "bands": {"ms": 0.42}}, ["bands", "rows"]) == ("rows", ["rows", "bands"])
    assert b.headline({"rows": {"ms": 0.42}, "bands": {"ms": 0.42}}, ["bands", "rows"])[0] == "rows"  # (ties: rows)


def test_bands_headline_only_when_faster_and_named_replicated():
    b = _bench()
    head, exact = b.headline({"rows": {"ms": 1.4}, "bands": {"ms": 0.61}}, ["bands", "rows"])
    assert head == "bands" and exact == ["rows", "bands"]
    text = b.scheme_choice(head, exact, 2)
    assert text.startswith("bands:") and "replicated" in text and "world size 2" in text


def test_single_scheme_runs():
    b = _bench()
    assert b.headline({"rows": {"ms": 1.0}}, ["rows"]) == ("rows", ["rows"])
    assert b.headline({"bands": {"ms": 1.0}}, ["bands"]) == ("bands", ["bands"])
    assert b.headline({}, ["slabs"]) == ("slabs", [])
    assert b.scheme_choice("rows", ["rows"], 8) == "rows"
