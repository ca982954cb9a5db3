#!/usr/bin/env python3
"""Summarise tools/mfma_pmc.sh's counter passes into profiles/TAG_mfma.json: per MFMA kernel and grid
size, the mean duration, the achieved clock, MFMA utilisation and MFMA flops.

    python tools/mfma_summary.py TAG [gpurun_out/mfma]

MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (rocprofv3's MfmaUtil
expression; the per-dispatch GRBM_GUI_ACTIVE value is the sum over the 8 XCDs, MI355X_MICROARCH.md
DVFS note); flops = (SQ_INSTS_VALU_MFMA_MOPS_F16 + _BF16) x 512.
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS, XCDS = 1024, 8


def load(path):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if "rtkv" not in r["Kernel_Name"] or not any(k in r["Kernel_Name"] for k in ("attn_lse", "qk_importance", "qk_head")):
            continue
        d = per[(r["Kernel_Name"], r["Grid_Size"], r["Dispatch_Id"])]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/mfma"
    out = {}
    for wl in ("lse", "qk"):
        merged = collections.defaultdict(lambda: collections.defaultdict(list))
        for path in glob.glob(os.path.join(src, wl, "*_counter_collection.csv")):
            for (name, grid, _), d in load(path).items():
                short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                for k, v in d.items():
                    merged[(short, grid)][k].append(v)
        for (name, grid), d in merged.items():
            m = {k: sum(v) / len(v) for k, v in d.items()}
            rec = {"dispatches": len(d["ns"]), "mean_us": round(m["ns"] / 1e3, 2)}
            if "GRBM_GUI_ACTIVE" in m:
                cyc = m["GRBM_GUI_ACTIVE"] / XCDS
                rec["clock_GHz"] = round(cyc / m["ns"], 3) if m["ns"] else None
                if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                    rec["mfma_util_pct"] = round(100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS), 2)
            mops = m.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0.0) + m.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0)
            if mops:
                rec["mfma_flops"] = mops * 512
            out[f"{wl}: {name} grid={grid}"] = rec
    doc = {"source": "rocprofv3 --pmc passes of tools/mfma_pmc.sh (tools/lse_bench.py: S = 4096 and 16384; "
                     "bench.py --importance qk --dtype float16, 4 cfg3 layers)",
           "definition": "mfma_util_pct = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs); "
                         "clock = GRBM_GUI_ACTIVE/8 / duration",
           "kernels": out}
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    with open(os.path.join(here, f"{tag}_mfma.json"), "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in out.items():
        print(k[:100], v)


if __name__ == "__main__":
    main()
