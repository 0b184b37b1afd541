#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of tools/profile_round.sh into profiles/<tag>/.

Reads (under gpurun_out/<tag>/):
  trace/**/*kernel_stats.csv      --kernel-trace --stats of the default bench run
  pmc_<group>_<wl>/**/*counter_collection.csv   one --pmc pass per counter group
  bench.json, bench_<wl>.json     the bench lines of the same runs
Writes:
  profiles/<tag>/kernel_stats.csv (copy), profiles/<tag>/bench.json (copy),
  profiles/<tag>/pmc_<wl>.json    per-launch counters of the dominant kernel,
  profiles/latest_pmc.json        {workload: {...}} read by bench.py for roofline.traffic

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in kB and reports 1/2 of the
bytes of wide (16 B/lane) coalesced reads on gfx950, so bytes = FETCH_SIZE*1024*2;
WRITE_SIZE (kB) is exact for 16-B stores.  Infinity-Cache hits are counted by
FETCH_SIZE, so this is L2-miss (MALL + HBM) traffic.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOMINANT = {"expand": "stream_eval_kernel<3072", "big16m": "eval_net_kernel<3072", "small1m": "eval_net_kernel<128"}
# (round 1: expand_stream_kernel; pass --kernel expand=... to override)
N_SIMD = 256 * 4  # CUs x SIMDs


def find(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    return hits[-1] if hits else None


def counters(path, kname, names=None):
    """{counter: [value per dispatch]} of the dispatches whose name contains kname (their
    names added to `names`)."""
    per = defaultdict(lambda: defaultdict(float))
    with open(path) as f:
        for r in csv.DictReader(f):
            if kname in r["Kernel_Name"]:
                per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
                if names is not None:
                    names.add(r["Kernel_Name"])
    return {k: list(v.values()) for k, v in per.items()}


def main(tag):
    src, dst = os.path.join(ROOT, "gpurun_out", tag), os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    ks = find(os.path.join(src, "trace", "**", "*kernel_stats.csv"))
    if ks:
        shutil.copy(ks, os.path.join(dst, "kernel_stats.csv"))
    for b in glob.glob(os.path.join(src, "bench*.json")):
        shutil.copy(b, os.path.join(dst, os.path.basename(b)))
    latest_p = os.path.join(ROOT, "profiles", "latest_pmc.json")
    latest = json.load(open(latest_p)) if os.path.exists(latest_p) else {}
    for wl, kname in DOMINANT.items():
        vals, names = {}, set()
        for grp in ("fetch", "write", "mfma", "l2"):
            p = find(os.path.join(src, f"pmc_{grp}_{wl}", "**", "*counter_collection.csv"))
            if p:
                vals.update(counters(p, kname, names))
                shutil.copy(p, os.path.join(dst, f"pmc_{grp}_{wl}.csv"))
        if "FETCH_SIZE" not in vals:
            continue
        avg = {k: sum(v) / len(v) for k, v in vals.items()}
        bench_p = os.path.join(src, f"bench_{wl}.json")
        bl = json.load(open(bench_p)) if os.path.exists(bench_p) else None
        fetch = avg["FETCH_SIZE"] * 1024 * 2
        write = avg.get("WRITE_SIZE", 0.0) * 1024
        # the column-sliced stream (stream_eval_kernel<3072, 3>): three launches per step, the
        # counters per launch as the bench's roofline (per dispatch)
        sl = 3 if any("3072, 3>" in x for x in names) else 1
        s = {"kernel": kname, "launches": len(vals["FETCH_SIZE"]), "launches_per_step": sl, "abi": 4,
             "FETCH_SIZE_kB": avg["FETCH_SIZE"], "WRITE_SIZE_kB": avg.get("WRITE_SIZE"),
             "hbm_side_bytes_per_launch": fetch + write,
             "correction": "bytes = FETCH_SIZE kB x 1024 x 2 (gfx950 wide reads) + WRITE_SIZE kB x 1024; "
                           "Infinity-Cache hits included (L2-miss traffic)",
             "source": f"profiles/{tag}/pmc_fetch_{wl}.csv + pmc_write_{wl}.csv (rocprofv3 --pmc, one pass each)"}
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            s["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
            s["TCC_HIT_plus_MISS"] = avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]
        if "TCC_REQ_sum" in avg:
            s["TCC_REQ"] = avg["TCC_REQ_sum"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
            s["SQ_VALU_MFMA_BUSY_CYCLES"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"]
            s["GRBM_GUI_ACTIVE"] = avg["GRBM_GUI_ACTIVE"]
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs
            s["mfma_util"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8 * N_SIMD)
        if bl:
            cfg = bl["config"]
            s["positions"] = cfg.get("games_per_gpu", cfg.get("positions_per_gpu"))
            alg = bl["roofline"]["alg_bytes_per_launch"]
            s["alg_bytes_per_launch"] = alg
            s["traffic_over_alg"] = s["hbm_side_bytes_per_launch"] / alg
            # L2-side requests (128 B lines) against the algorithmic row bytes
            if "TCC_HIT_plus_MISS" in s:
                s["l2_request_bytes_over_alg"] = s["TCC_HIT_plus_MISS"] * 128 / alg
            s["kernel_ms_per_launch_bench"] = bl["roofline"]["kernel_ms_per_launch"]
        json.dump(s, open(os.path.join(dst, f"pmc_{wl}.json"), "w"), indent=1)
        latest[wl] = s
        print(wl, json.dumps(s))
    json.dump(latest, open(latest_p, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
