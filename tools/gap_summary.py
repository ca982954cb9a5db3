"""Summarise a rocprofv3 kernel trace of tools/dropin_profile.py: per kernel of the path (K1, K2, K4)
its mean duration and the idle gap before it (start minus the previous kernel's end), for the drop-in
region and the raw-driver region separately.

    python tools/gap_summary.py <trace dir> [--layers 32] [--warmup 2] [--reps 5]

dropin_profile.py runs the drop-in loop (warmup + reps runs of `layers` calls, a sync after each run),
then the raw driver (warmup + reps steps).  Gaps at run boundaries (the sync + reset between runs) are
reported apart from the per-layer gaps."""
import argparse
import csv
import glob
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--layers", type=int, default=32)
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()

path = glob.glob(f"{a.trace}/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(path)) if "rtkv" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def phase(name):
    if "aggregation" in name or "qk_head" in name:
        return "K1"
    if "quant_rows" in name:
        return "K4"
    if "prefetch" in name or "waiter" in name:
        return "PF"  # the drop-in's kept-row prefetch / the armed K4's waiter, between K2 and K4
    return "K2"


k1 = [i for i, r in enumerate(rows) if phase(r["Kernel_Name"]) == "K1"]
runs = a.warmup + a.reps


def region(label, first_layer, nlayers):
    if first_layer + nlayers >= len(k1):
        nlayers = len(k1) - first_layer - 1
    if nlayers <= 0:
        return
    dur = {"K1": [], "K2": [], "PF": [], "K4": []}
    gap = {"K1": [], "K2": [], "PF": [], "K4": []}
    boundary = []
    for li in range(first_layer, first_layer + nlayers):
        for i in range(k1[li], k1[li + 1]):
            r = rows[i]
            p = phase(r["Kernel_Name"])
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            dur[p].append((e - s) / 1e3)
            if i > 0:
                g = (s - int(rows[i - 1]["End_Timestamp"])) / 1e3
                if p == "K1" and (li - first_layer) % a.layers == 0:
                    boundary.append(g)  # first layer of a run: the sync + reset before it
                else:
                    gap[p].append(g)
    span = (int(rows[k1[first_layer + nlayers]]["Start_Timestamp"]) - int(rows[k1[first_layer]]["Start_Timestamp"])) / 1e3
    print(f"{label}: {nlayers} layers, {span / nlayers:.1f} us per layer start to start (run boundaries included)")
    for p in ("K1", "K2", "PF", "K4"):
        if not dur[p]:
            continue
        g = sorted(gap[p]) or [0.0]
        print(f"  {p}: dur {statistics.mean(dur[p]):7.2f} us   gap before: mean {statistics.mean(g):6.2f}  "
              f"p50 {g[len(g) // 2]:6.2f}  p90 {g[len(g) * 9 // 10]:6.2f}  max {g[-1]:7.2f} us")
    if boundary:
        print(f"  run boundaries: {len(boundary)}, mean {statistics.mean(boundary):.1f} us")


region("drop-in (timed runs)", a.warmup * a.layers, a.reps * a.layers)
region("raw driver (timed steps)", (runs + a.warmup) * a.layers, a.reps * a.layers)
