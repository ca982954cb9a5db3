#!/usr/bin/env python3
"""Summarise tools/mfma_pmc.sh's counter passes into profiles/TAG_mfma.json: per MFMA kernel and grid
size, the mean duration, the achieved clock, MFMA utilisation over the kernel's own duration, MFMA
flops and the LDS counters (instructions, bank-conflict cycles).

    python tools/mfma_summary.py TAG [gpurun_out/mfma]

Utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (duration x clock x 1024 SIMDs); the clock is GRBM_GUI_ACTIVE / 8
XCDs / duration (the per-dispatch value is the sum over the 8 XCDs, MI355X_MICROARCH.md DVFS note) unless
that exceeds 2.4 GHz — then the counter window was wider than the kernel (short kernels), the derived
clock is rejected and 2.4 GHz gives a lower bound.  flops = (SQ_INSTS_VALU_MFMA_MOPS_F16 + _BF16) x 512.
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS, XCDS, SES = 1024, 8, 32
PEAK_GHZ = 2.4  # MI355X peak engine clock (MI355X_MICROARCH.md chip parameters)
DENSE_BF16_TFLOPS = 2500.0  # dense f16/bf16 MFMA peak at PEAK_GHZ (MI355X_MICROARCH.md)


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
            if "GRBM_GUI_ACTIVE" in m and m["ns"]:
                # GRBM_GUI_ACTIVE counts the busy cycles of the counter window, which for a short kernel
                # extends past the kernel's own timestamps: a derived clock above the part's 2.4 GHz peak
                # means the window is wider than the kernel, and that clock is rejected.  Utilisation is
                # always taken over the kernel's OWN duration: busy / (duration x clock x 1024 SIMDs), with
                # the derived clock when it is plausible, else the 2.4 GHz peak (a lower bound).
                derived = m["GRBM_GUI_ACTIVE"] / XCDS / m["ns"]
                ok = derived <= PEAK_GHZ
                rec["clock_GHz_derived"] = round(derived, 3)
                rec["clock_window_ok"] = ok
                clk = derived if ok else PEAK_GHZ
                rec["clock_GHz_used"] = round(clk, 3)
                if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                    util = 100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["ns"] * clk * SIMDS)
                    rec["mfma_util_pct" if ok else "mfma_util_pct_lower_bound"] = round(util, 2)
            if m.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                # the same pass's SQ_BUSY_CYCLES (summed over the 32 shader engines) as the cycle base: a
                # busy-time window per engine instead of the counter window's wall clock, so it holds for
                # short dispatches too.  util = MFMA busy / (SQ busy x 1024 SIMDs / 32 engines)
                rec["sq_busy_clock_GHz"] = round(m["SQ_BUSY_CYCLES"] / SES / m["ns"], 3)
                rec["mfma_util_pct_sq_busy"] = round(100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] * SES /
                                                     (m["SQ_BUSY_CYCLES"] * SIMDS), 2)
            for k in ("SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAVES", "SQ_INSTS_MFMA",
                      "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
                if k in m:
                    rec[k] = m[k]
            if m.get("SQ_WAVE_CYCLES"):  # shares of wave time (all quad-cycle counters)
                for k, share in (("SQ_WAIT_ANY", "wait_any_pct"), ("SQ_WAIT_INST_ANY", "wait_inst_any_pct"),
                                 ("SQ_ACTIVE_INST_VALU", "valu_active_pct"), ("SQ_ACTIVE_INST_LDS", "lds_active_pct"),
                                 ("SQ_ACTIVE_INST_VMEM", "vmem_active_pct")):
                    if k in m:
                        rec[share] = round(100 * m[k] / m["SQ_WAVE_CYCLES"], 1)
            if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
                rec["lds_bank_conflict_pct"] = round(100 * m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 2)
            mops = m.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0.0) + m.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0)
            if mops:
                rec["mfma_flops"] = mops * 512
                # achieved rate against the dense f16/bf16 peak (2.5 PFLOP/s at 2.4 GHz, no sparsity)
                rate = mops * 512 / (m["ns"] * 1e-9) / 1e12
                rec["mfma_tflops"] = round(rate, 1)
                rec["frac_of_dense_bf16_peak"] = round(rate / DENSE_BF16_TFLOPS, 4)
            out[f"{wl}: {name} grid={grid}"] = rec
    doc = {"source": "rocprofv3 --pmc passes of tools/mfma_pmc.sh (tools/lse_bench.py: S = 4096 and 16384; "
                     "bench.py --importance qk --dtype float16, 4 cfg3 layers)",
           "definition": "mfma_util_pct = SQ_VALU_MFMA_BUSY_CYCLES / (kernel duration x clock x 1024 SIMDs), "
                         "clock = GRBM_GUI_ACTIVE/8 / duration when that is <= 2.4 GHz (the counter window is the "
                         "kernel's), else 2.4 GHz and the figure is reported as mfma_util_pct_lower_bound; "
                         "lds_bank_conflict_pct = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; "
                         "mfma_util_pct_sq_busy = SQ_VALU_MFMA_BUSY_CYCLES x 32 / (SQ_BUSY_CYCLES x 1024): the "
                         "same pass's per-engine busy cycles as the base (32 shader engines), valid for short "
                         "dispatches; on the long LSE dispatch it reads within 7 % of the clock-window figure; "
                         "mfma_tflops / frac_of_dense_bf16_peak = MOPS x 512 / duration against 2.5 PFLOP/s",
           "kernels": out}
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    with open(os.path.join(here, f"{tag}_mfma.json"), "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in out.items():
        print(k[:100], v)


if __name__ == "__main__":
    main()
