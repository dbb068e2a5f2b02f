#!/usr/bin/env python3
"""Modelled 1->2->4->8 GPU frame period per BASELINE config, from the
virtual-rank probes of one GPU (tools/rows_probe.py, tools/band_probe.py):
the per-rank compute they measure, plus their xGMI link models.  NOT a
measured curve: the driver's 8-GPU run measures that.

For every world size it lists the two exact schemes as bench.py runs them:
  rows        splat-index shards with two frames in flight (bench.py's
              default, --pipeline-rows 1; gs_group_render_pipelined):
              max(project + render, busiest link) per rank
              (rows_probe pipelined_model_ms)
  rows_unpipelined  one frame at a time (--pipeline-rows 0): project +
              largest per-peer exchange over one link + render + its band to
              rank 0 (rows_probe link_model_ms)
  bands       the replicated scene, each rank its own bin rows:
              max(slowest rank, largest band over one link)
and `chosen` by bench.py's headline rule: rows (the splat-sharded scheme)
whenever its period is at most bands', else bands; `monotone` = every chosen
period at or below the previous world size's.

  python tools/scaling_model.py rows_1080p.json bands_1080p.json [more pairs ...] > model.json
"""
import json
import sys


def model(rows: dict, bands: dict) -> dict:
    rw, bw = rows["worlds"], bands["worlds"]
    one = rw.get("1") or rw.get(1)
    base = one["frame_ms_2_in_flight"]
    out = {"splats": rows["splats"], "frame": rows["frame"], "sh_degree": rows.get("sh_degree"),
           "n1_frame_ms": base, "worlds": {}}
    prev = base
    mono = True
    for g in sorted(int(k) for k in rw):
        if g == 1:
            continue
        r = rw.get(str(g)) or rw[g]
        b = bw.get(str(g)) or bw.get(g)
        e = {"rows": r["pipelined_model_ms"], "rows_unpipelined": r["link_model_ms"]}
        if b:
            e["bands"] = b["period_model_ms"]
        choice = "rows" if "bands" not in e or e["rows"] <= e["bands"] else "bands"
        e["chosen"] = choice
        e["chosen_ms"] = e[choice]
        e["speedup_vs_1"] = round(base / e[choice], 3)
        mono = mono and e[choice] <= prev
        prev = e[choice]
        out["worlds"][g] = e
    out["monotone"] = mono
    return out


def main():
    args = sys.argv[1:]
    if len(args) < 2 or len(args) % 2:
        sys.exit(__doc__)
    res = []
    for i in range(0, len(args), 2):
        rows = json.loads(open(args[i]).read().strip().splitlines()[-1])
        bands = json.loads(open(args[i + 1]).read().strip().splitlines()[-1])
        res.append(model(rows, bands))
    print(json.dumps({"note": "modelled from virtual-rank probes on one GPU (per-rank compute measured, links "
                              "priced at 76.8 GB/s per direction); not a measured multi-GPU curve",
                      "configs": res}, indent=1))


if __name__ == "__main__":
    main()
