#!/usr/bin/env python3
"""Per-kernel sums of the SQ counter passes written by tools/sq_counters.sh.
Usage: python tools/sq_summary.py <tag> [kernel substring]"""
import collections
import csv
import glob
import os
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "sq"
kern = sys.argv[2] if len(sys.argv) > 2 else "expand"
root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", tag)
runs = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True)):
    name = os.path.relpath(f, root).split(os.sep)[0].rsplit("_", 1)[0]
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"] and "3072" in r["Kernel_Name"]:
            runs[name][r["Counter_Name"]] = runs[name].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for name, c in runs.items():
    print(name, " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))
    if "SQ_WAVE_CYCLES" in c:
        w = c["SQ_WAVE_CYCLES"]
        print("   wait %.2f  issue-stall %.2f  active %.2f  (fractions of wave cycles)" % (
            c["SQ_WAIT_ANY"] / w, c["SQ_WAIT_INST_ANY"] / w, c["SQ_ACTIVE_INST_ANY"] / w))
