#!/usr/bin/env python3
"""Interleaved A/B of environment-selected kernel variants on the GPU box (each variant is its own
bench.py process, since the library reads its knobs once per process).

    python tools/ab_env.py TAG --rounds 2 --variants 'A=' 'B=RTKV_K4_PK_WAVES=4' -- --dtype float16 --no-dequant

Every run: bench.py --legs none (unless --legs is among the arguments) --cpu-baseline-seconds 0 plus the
arguments after '--'.  Writes
gpurun_out/ab_TAG.json with, per variant, every run's ms_per_step and per-kernel event times, and the
means; prints one summary line per variant.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    argv = sys.argv[1:]
    bench_args = argv[argv.index("--") + 1:] if "--" in argv else []
    argv = argv[:argv.index("--")] if "--" in argv else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("--variants", nargs="+", required=True, help="NAME=VAR=VALUE,VAR=VALUE (empty: defaults)")
    a = ap.parse_args(argv)
    variants = []
    for v in a.variants:
        name, _, rest = v.partition("=")
        env = {}
        for kv in filter(None, rest.split(",")):
            k, _, val = kv.partition("=")
            env[k] = val
        variants.append((name, env))
    out = {"bench_args": bench_args, "variants": {n: {"env": e, "runs": []} for n, e in variants}}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    path = os.path.join(REPO, "gpurun_out", f"ab_{a.tag}.json")
    for r in range(a.rounds):
        for name, env in variants:
            e = dict(os.environ, **env)
            legs = [] if "--legs" in bench_args else ["--legs", "none"]
            cmd = [sys.executable, os.path.join(REPO, "bench.py"), *legs, "--cpu-baseline-seconds", "0", *bench_args]
            p = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=a.timeout)
            if p.returncode != 0:
                print(f"{name}: rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(p.returncode)
            line = json.loads(p.stdout.strip().splitlines()[-1])
            run = {"ms_per_step": line["ms_per_step"], "kernel_us_per_layer": line.get("kernel_us_per_layer")}
            if "legs" in line:  # extra legs asked for with --legs: their headline numbers
                run["legs"] = {k: {x: v[x] for x in ("ms_per_step", "ttft_ms", "ttft_device_span_ms",
                                                      "raw_driver_ms_per_prefill_same_state", "kernel_us_per_layer")
                                   if x in v} for k, v in line["legs"].items() if isinstance(v, dict)}
            out["variants"][name]["runs"].append(run)
            print(f"round {r} {name}: {run}", flush=True)
            with open(path, "w") as f:
                json.dump(out, f, indent=1)
    for name, v in out["variants"].items():
        runs = v["runs"]
        v["mean_ms_per_step"] = round(sum(x["ms_per_step"] for x in runs) / len(runs), 4)
        ks = [x["kernel_us_per_layer"] for x in runs if x["kernel_us_per_layer"]]
        if ks:
            v["mean_kernel_us"] = {k: round(sum(d[k] for d in ks) / len(ks), 2) for k in ks[0]}
        print(f"{name}: {v['mean_ms_per_step']} ms/step {v.get('mean_kernel_us')}", flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
