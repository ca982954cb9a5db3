#!/usr/bin/env python3
"""Where the drop-in path's per-layer time goes (GPU tool): RealTimePrefillCompressor.
compress_layer_kv_cache over cfg3-shaped layers, cProfile of the host side and the raw driver's
per-layer time for comparison.

    python tools/dropin_profile.py [--dtype float32] [--layers 8]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "realtime-kv-cache-compression_amd"))

import bench  # noqa: E402
import rtkv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-cprofile", action="store_true", help="timings only (under a kernel trace)")
    a = ap.parse_args()
    sys.argv = ["bench.py", "--dtype", a.dtype, "--layers", str(a.layers)]
    args = bench.resolve_config(bench.parse(), 1)
    dev = torch.device("cuda", 0)
    job = bench.Job(args, dev, 0, 1)
    comp = rtkv.RealTimePrefillCompressor(job.cfg)
    ids = torch.zeros(1, job.S, dtype=torch.long, device=dev)

    def run():
        comp.reset_compression_state()
        for l in range(args.layers):
            K, V, W = job.inputs[l]
            comp.compress_layer_kv_cache(K, V, W, ids, l)
        torch.cuda.synchronize(dev)

    for _ in range(2):
        run()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        run()
    drop = (time.perf_counter() - t0) / (a.reps * args.layers) * 1e6
    raw_ms, kus = job.timed(a.reps, 2)
    print(f"drop-in {drop:.1f} us/layer; raw driver {raw_ms / args.layers * 1e3:.1f} us/layer "
          f"(K1 {kus[0]:.1f} K2 {kus[1]:.1f} K4 {kus[2]:.1f})", flush=True)
    if a.no_cprofile:
        return
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.reps):
        run()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
