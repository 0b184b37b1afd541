#!/usr/bin/env python3
"""Per-kernel totals of the --pmc passes of tools/pmc_kernels.sh: python tools/pmc_kernels_summary.py <tag>
[kernel substrings...].  Prints, per kernel (dispatches summed), each counter and the derived
ratios (VALU / wave, wait share of wave cycles, L2 hit rate, TCP->L2 reads per access)."""
import csv
import glob
import sys
from collections import defaultdict


def main(tag, names):
    tot = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"gpurun_out/{tag}/pmc*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if names and not any(n in k for n in names):
                continue
            short = k.split("(")[0].replace("void ", "")
            tot[short][r["Counter_Name"]] += float(r["Counter_Value"])
            tot[short]["_vgpr"] = float(r["VGPR_Count"])
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        if not c.get("SQ_WAVE_CYCLES"):
            continue
        w = c.get("SQ_WAVES", 1) or 1
        print(f"== {k}  (VGPR {int(c['_vgpr'])})")
        for n in sorted(c):
            if not n.startswith("_"):
                print(f"   {n:32s} {c[n]:.4g}")
        wc = c["SQ_WAVE_CYCLES"]
        print(f"   -> per wave: cycles {wc / w:.0f}, VALU {c.get('SQ_INSTS_VALU', 0) / w:.0f}, SALU {c.get('SQ_INSTS_SALU', 0) / w:.0f}, "
              f"LDS {c.get('SQ_INSTS_LDS', 0) / w:.0f}, VMEM_RD {c.get('SQ_INSTS_VMEM_RD', 0) / w:.0f}, VMEM_WR {c.get('SQ_INSTS_VMEM_WR', 0) / w:.0f}, "
              f"SMEM {c.get('SQ_INSTS_SMEM', 0) / w:.0f}")
        print(f"   -> wait_inst_any / wave_cycles {c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}, wait_any {c.get('SQ_WAIT_ANY', 0) / wc:.3f}, "
              f"active_inst_any {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}; L2 hit "
              f"{c.get('TCC_HIT_sum', 0) / max(1, c.get('TCC_REQ_sum', 1)):.3f}; TCP->L2 reads / TCP accesses "
              f"{c.get('TCP_TCC_READ_REQ_sum', 0) / max(1, c.get('TCP_TOTAL_CACHE_ACCESSES_sum', 1)):.3f}; LDS bank conflict / LDS active "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, c.get('SQ_ACTIVE_INST_LDS', 1)):.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
