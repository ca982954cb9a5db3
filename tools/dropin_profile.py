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


def device_stamps(comp, job, ids, layers, reps):
    """Without a profiler: each layer's device span (first K1 block start to last K4 row) and the idle
    time from one layer's last K4 row to the next layer's first K1 block, from rtkv_layer_times."""
    from rtkv import _lib as L
    comp = rtkv.RealTimePrefillCompressor(job.cfg, strict=False)  # keeps each layer's result in _unverified
    khz = L.wall_clock_khz(job.device)
    spans, gaps, walls = [], [], []
    for it in range(2 + reps):
        comp.reset_compression_state()
        torch.cuda.synchronize(job.device)
        t0 = time.perf_counter()
        res = []
        for l in range(layers):
            K, V, W = job.inputs[l]
            comp.compress_layer_kv_cache(K, V, W, ids, l)
            res.append(comp._unverified.get(job.device, (None,))[0])
        torch.cuda.synchronize(job.device)
        wall = time.perf_counter() - t0
        if it < 2 or any(r is None for r in res):
            continue
        walls.append(wall)
        be = []
        for r in res:
            t = r.bufs.stats[-L.TIMES_BYTES:].cpu().numpy().view("uint64")
            be.append((int(t[-1]), int(t[:-1:16].max())))
        spans += [(e - b) / khz * 1e3 for b, e in be]
        gaps += [(be[i + 1][0] - be[i][1]) / khz * 1e3 for i in range(len(be) - 1)]
    m = lambda v: sum(v) / len(v)
    print(f"stamps: wall {m(walls) * 1e3:.3f} ms per {layers} layers; device span per layer {m(spans):.1f} us; "
          f"idle between layers (last K4 row -> next K1 block) {m(gaps):.1f} us (p50 {sorted(gaps)[len(gaps) // 2]:.1f})",
          flush=True)


def host_timeline(comp, job, ids, layers, reps):
    """Per layer, host time from the return of the K4 launch (finish) to the next layer's K1 launch
    (begin), the begin call itself, the wait for the early statistics, and from the wait's return to
    the K4 launch — the host's share of the device gaps in the kernel trace."""
    from rtkv import _lib as L
    from rtkv import engine
    lib = L.lib()
    t = {"begin0": [], "begin1": [], "wait1": [], "fin0": [], "fin1": []}
    ob, of = lib.rtkv_compress_layer_begin, lib.rtkv_compress_layer_finish
    ow = engine.EarlyStatsBuffer.wait

    def begin(*x):
        t["begin0"].append(time.perf_counter())
        r = ob(*x)
        t["begin1"].append(time.perf_counter())
        return r

    def fin(*x):
        t["fin0"].append(time.perf_counter())
        r = of(*x)
        t["fin1"].append(time.perf_counter())
        return r

    def wait(self, *x, **k):
        r = ow(self, *x, **k)
        t["wait1"].append(time.perf_counter())
        return r
    lib.rtkv_compress_layer_begin, lib.rtkv_compress_layer_finish = begin, fin
    engine.EarlyStatsBuffer.wait = wait
    dev = job.device
    edges = []
    for it in range(2 + reps):
        for v in t.values():
            v.clear()
        comp.reset_compression_state()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for l in range(layers):
            K, V, W = job.inputs[l]
            comp.compress_layer_kv_cache(K, V, W, ids, l)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        if it >= 2:
            edges.append((t["begin0"][0] - t0, t1 - t["fin1"][-1], t2 - t1, t2 - t0))
    n = layers
    us = lambda v: 1e6 * sum(v) / len(v)
    post = [t["begin0"][i + 1] - t["fin1"][i] for i in range(n - 1)]
    print(f"host per layer (us): K4 launch return -> next begin call {us(post):.1f}; begin call (K1+K2 launch) "
          f"{us([t['begin1'][i] - t['begin0'][i] for i in range(n)]):.1f}; begin return -> wait return "
          f"{us([t['wait1'][i] - t['begin1'][i] for i in range(n)]):.1f}; wait return -> finish call "
          f"{us([t['fin0'][i] - t['wait1'][i] for i in range(n)]):.1f}; finish call (K4 launch) "
          f"{us([t['fin1'][i] - t['fin0'][i] for i in range(n)]):.1f}", flush=True)
    e = [sum(x[k] for x in edges) / len(edges) * 1e6 for k in range(4)]
    print(f"edges (us): loop start -> first begin call {e[0]:.1f}; last K4 launch -> last call returns {e[1]:.1f}; "
          f"final sync {e[2]:.1f}; wall {e[3]:.1f}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-cprofile", action="store_true", help="timings only (under a kernel trace)")
    ap.add_argument("--stamps", action="store_true",
                    help="per-layer device spans and inter-layer gaps from the kernels' own time stamps "
                         "(rtkv_layer_times; no profiler)")
    ap.add_argument("--host-timeline", action="store_true",
                    help="host timestamps around the begin / wait / finish calls (wrappers add ~1 us each)")
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

    if a.stamps:
        device_stamps(comp, job, ids, args.layers, a.reps)
        return
    if a.host_timeline:
        host_timeline(comp, job, ids, args.layers, a.reps)
        return
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
