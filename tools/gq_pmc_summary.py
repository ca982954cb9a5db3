#!/usr/bin/env python3
"""HBM traffic of the rtkv-gq/1 kernels (the bench's gq leg) from separate rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes, against the leg's algorithmic bytes.

    python tools/gq_pmc_summary.py TAG [gpurun_out/r06g]   ->  profiles/TAG_gq_pmc.json

Bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): KiB counters; FETCH_SIZE doubled on gfx950 for wide
(16 B/lane) streaming reads, WRITE_SIZE as is.  The leg's algorithmic bytes per layer (bench.py gq_leg: kept
rows read by the pack, every vote_stride-th kept row by the vote, codes + scale/zero-points + outlier values
written) come from the profiled run's own bench line; the "workload" carries leg = gq, so bench.py never
takes these figures for the main line's roofline."""
import collections
import csv
import json
import os
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter and "gq_" in r["Kernel_Name"]:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def stats(path):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if "gq_" in r["Name"]:
                out[r["Name"]] = float(r["AverageNs"]) / 1e3
    return out


def bench_line(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/r06g"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) and --kernel-trace --stats of "
                     "`python3 bench.py --steps 1 --warmup 1 --dtype D --legs gq --leg-steps 2 --cpu-baseline-seconds 0`",
           "correction": "bytes = 2 * FETCH_SIZE KiB * 1024 + WRITE_SIZE KiB * 1024 (gfx950, MI355X_MICROARCH.md)",
           "dtypes": {}}
    for d in ("float32", "float16"):
        fetch = per_kernel(os.path.join(src, f"pmc_{d}", "fetch_counter_collection.csv"), "FETCH_SIZE")
        write = per_kernel(os.path.join(src, f"pmcw_{d}", "write_counter_collection.csv"), "WRITE_SIZE")
        us = stats(os.path.join(src, f"prof_{d}", "run_kernel_stats.csv"))
        line = bench_line(os.path.join(src, f"prof_{d}.log"))
        leg = line["legs"]["gq"] if line else {}
        ks, tot = {}, 0
        for k in sorted(fetch):
            fb, wb = 2 * fetch[k] * 1024, write.get(k, 0.0) * 1024
            if "unpack" not in k:  # (the leg's reconstruction check, not part of gq_compress)
                tot += fb + wb
            ks[k] = {"hbm_read_bytes": round(fb), "hbm_write_bytes": round(wb), "hbm_bytes": round(fb + wb),
                     "avg_us_rocprof": round(us.get(k, float("nan")), 2),
                     "GBs_of_traffic": round((fb + wb) / (us[k] * 1e3), 1) if k in us else None}
        alg = leg.get("algorithmic_bytes_per_layer")
        doc["dtypes"][d] = {"workload": {"dtype": d, "leg": "gq", "config": leg.get("config")},
                            "kernels": ks, "hbm_bytes_per_layer_vote_and_pack": round(tot),
                            "algorithmic_bytes_per_layer": alg,
                            "traffic_over_algorithmic": round(tot / alg, 3) if alg else None,
                            "leg_us_per_layer_events": leg.get("us_per_layer")}
    out = os.path.join(repo, "profiles", f"{tag}_gq_pmc.json")
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
