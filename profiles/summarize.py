#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of bench.py into the small files committed under profiles/.

    python profiles/summarize.py TAG [gpurun_out] [-- BENCH ARGS]

BENCH ARGS are the bench.py arguments of the profiled workload (default: bench.py's defaults); they
are recorded as the summary's "workload", which bench.py matches before using the traffic.

reads  gpurun_out/prof/run_kernel_stats.csv              (rocprofv3 --kernel-trace --stats)
       gpurun_out/pmc/fetch_counter_collection.csv       (rocprofv3 --pmc FETCH_SIZE, own pass)
       gpurun_out/pmcw/write_counter_collection.csv      (rocprofv3 --pmc WRITE_SIZE, own pass)
writes profiles/TAG_kernel_stats.csv                     (copy of the stats summary)
       profiles/TAG_pmc.json                             (per-kernel mean HBM bytes per dispatch)

HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): the counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores.
"""
import collections
import csv
import json
import os
import shutil
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    argv = sys.argv[1:]
    bench_args = argv[argv.index("--") + 1:] if "--" in argv else []
    argv = argv[:argv.index("--")] if "--" in argv else argv
    tag = argv[0]
    src = argv[1] if len(argv) > 1 else "gpurun_out"
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    import bench
    saved, sys.argv = sys.argv, ["bench.py"] + bench_args
    workload = bench.workload_key(bench.resolve_config(bench.parse(), 1))  # the config's shape filled in
    sys.argv = saved
    shutil.copy(os.path.join(src, "prof", "run_kernel_stats.csv"), os.path.join(here, f"{tag}_kernel_stats.csv"))
    fetch, n = per_kernel(os.path.join(src, "pmc", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write, _ = per_kernel(os.path.join(src, "pmcw", "write_counter_collection.csv"), "WRITE_SIZE")
    out = {}
    for k in fetch:
        if not k.startswith(("rtkv::", "void rtkv::")):
            continue
        fb = 2 * fetch[k] * 1024
        wb = write.get(k, 0.0) * 1024
        out[k] = {"dispatches": n[k], "fetch_kib_raw": round(fetch[k], 3), "write_kib_raw": round(write.get(k, 0.0), 3),
                  "hbm_read_bytes": round(fb), "hbm_write_bytes": round(wb), "hbm_bytes": round(fb + wb)}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                     "`python3 bench.py --steps 2 --warmup 1 --legs none --cpu-baseline-seconds 0 "
                     + " ".join(bench_args) + "`",
           "workload": workload,
           "correction": "bytes = 2 * FETCH_SIZE KiB * 1024 + WRITE_SIZE KiB * 1024 (gfx950, MI355X_MICROARCH.md)",
           "kernels": out}
    with open(os.path.join(here, f"{tag}_pmc.json"), "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in out.items():
        print(f"{v['hbm_bytes'] / 1e6:10.2f} MB/dispatch  {k[:90]}")


if __name__ == "__main__":
    main()
