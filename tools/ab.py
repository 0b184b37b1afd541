#!/usr/bin/env python3
"""A/B driver for the GPU box: runs bench.py once per variant and prints one line each.

A variant is a library build (fishnet_amd/lib/<name>.so, built beforehand on the CPU with
`python -m fishnet_amd.build -DNAME=VALUE --out=<name>.so`) and/or environment settings
(GN_ABLATE, GN_STREAM=old, GN_BLOCK_SORT=0, ...), plus bench.py arguments shared by all.

    python tools/ab.py --variants libgpu_nnue.so libgpu_nnue_gap7.so \
        --env "" "GN_BLOCK_SORT=0" -- --positions 16384 --steps 3

runs every (library x env) pair; each run gets its own time limit and the script stops at the
first failing run (no retries on the GPU).  Output: gpurun_out/ab/<tag>.json per run and a
summary line per run on stdout: kernel ms, plan ms, evals/s, stage times, oracle-check result.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="*", default=["libgpu_nnue.so"], help="library file names in fishnet_amd/lib")
    ap.add_argument("--env", nargs="*", default=[""], help="space-separated NAME=VALUE settings per env variant")
    ap.add_argument("--timeout", type=int, default=300, help="seconds per run")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ab"))
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    bargs = [x for x in a.bench_args if x != "--"] or ["--steps", "3"]
    bargs += [x for x in ("--no-cpu-baseline", "--no-secondary") if x not in bargs]
    os.makedirs(a.out, exist_ok=True)
    for lib in a.variants:
        for env in a.env:
            tag = lib.replace(".so", "") + ("." + env.replace(" ", ".").replace("=", "") if env else "")
            e = dict(os.environ, GPU_NNUE_LIB=os.path.join(ROOT, "fishnet_amd", "lib", lib))
            e.update(kv.split("=", 1) for kv in env.split())
            cmd = ["timeout", "-k", "10", str(a.timeout), sys.executable, "-u", os.path.join(ROOT, "bench.py")] + bargs
            with open(os.path.join(a.out, tag + ".json"), "w") as fo, open(os.path.join(a.out, tag + ".err"), "w") as fe:
                rc = subprocess.run(cmd, env=e, stdout=fo, stderr=fe).returncode
            if rc:
                print(f"{tag}: exit {rc} (see {a.out}/{tag}.err)", flush=True)
                sys.exit(rc)
            d = json.load(open(os.path.join(a.out, tag + ".json")))
            rf = d["roofline"]
            chk = d.get("oracle_check", {})
            ok = chk.get("vs_plain_path", {}).get("equal") if "vs_plain_path" in chk else chk.get("mismatches")
            print(f"{tag}: kernel {rf['kernel_ms_per_launch']:.2f} ms, plan {rf.get('plan_kernel_ms', 0):.2f} ms, "
                  f"{d['value']:.4g} evals/s, {d['ms_per_step']:.1f} ms/step, stages {rf.get('stage_ms')}, "
                  f"pads {d['config'].get('king_cache_gap_pads')}, check {ok}", flush=True)


if __name__ == "__main__":
    main()
