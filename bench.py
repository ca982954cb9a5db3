#!/usr/bin/env python3
"""Benchmark of the MI355X streaming prefill KV-cache compression path.

Metric (BASELINE.json): prefill KV-compress GB/s + TTFT, Llama-2-7B, S = 16k, 1 GPU.

One *step* = the compression of all 32 layers of one prefill (BASELINE config 3: B=1, S=16384,
32 heads × 128, K/V in the reference model's fp32 (modified_llama.py:368), prompt P=128, full
importance → quantization → selective propagation) through the C ABI's fused driver
(rtkv_compress_layer: 3 kernels per layer, no host sync inside the step).  Inputs are synthetic
(seeded, resident in HBM before timing).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg3|cfg4|cfg5]

Workloads (BASELINE.json configs): cfg3 (Llama-2-7B, 32 layers, S = 16384; the N = 1 default and
the headline), cfg4 (Llama-2-7B, S = 65536 in total; the N > 1 default) and cfg5 (Llama-2-13B,
40 layers, 40 heads, S = 32768 in total).  N > 1: sequence-chunk sharding of the SAME S_total
(strong scaling: rank j owns tokens [j·S_total/N, (j+1)·S_total/N); RCCL all-gather of the
per-token attention mass, global selection on every rank, local quantization, grouped RCCL
send/recv of the packed KV).  ``python bench.py --gpus N`` without WORLD_SIZE in the environment
starts ``python -m torch.distributed.run --nproc-per-node N ... bench.py ...`` as a child process
before anything touches a GPU, waits for it and exits with its code; it fails at once when fewer
than N GPUs are visible.  ``--launch-dry-run`` prints that command line and exits.

Rank 0 prints ONE JSON line.  ``value`` = algorithmic bytes of the whole job ÷ wall time (GB/s);
``ttft_ms`` = the step's wall time with every layer strictly after the previous one (the reference
caller's order: layer l+1's K/V come out of attention over layer l's compressed K'/V',
modified_llama.py:113-157), i.e. Σ per-layer compress time;
``roofline`` = the dominant kernel (K4: quantize+pack+compact) on its own algorithmic read+write
bytes over its average launch time (HIP events on the launch stream); ``roofline_path`` = the path's
HBM-read roofline as the north star defines it (R = 2·S·H·D·e + H·S·P·e bytes per layer
over the per-layer time of all the layer's kernels);
``cpu_baseline`` = the C oracle (OpenMP restatement of the reference) on a bounded sample of the
same workload.  Extra legs (``--legs``, single GPU): ``f16`` (the workload in fp16), ``packed_only``
(codes + scale/zp, no dequantized K'/V' — what the packed consumers read), ``drop_in`` (the reference
caller's path, RealTimePrefillCompressor.compress_layer_kv_cache per layer; ``ttft_ms`` = Σ
processing_time as longbench_eval.py:160 defines TTFT), ``s4096`` / ``s65536`` (the north star's other
sequence lengths), ``cfg2_s4096_quant`` (BASELINE config 2: S = 4096, quantization only) and
``independent_layers`` (layers on 4 streams: an upper bound for callers that own several layers'
inputs at once, not the reference caller's order).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "realtime-kv-cache-compression_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

# BASELINE.json configs 3-5 (SURVEY §8 shorthand): KV shapes of the named models, S_total = tokens of the
# whole prefill (split over the ranks at N > 1)
CONFIGS = {
    "cfg3": dict(model="Llama-2-7B", layers=32, heads=32, head_dim=128, seq_total=16384),
    "cfg4": dict(model="Llama-2-7B", layers=32, heads=32, head_dim=128, seq_total=65536),
    "cfg5": dict(model="Llama-2-13B", layers=40, heads=40, head_dim=128, seq_total=32768),
}


# Compression parameters of a workload.  "coverage": SURVEY §8d's coverage set (all three classes populated and
# tokens dropped in every layer group) at the reference tests' 8/4/2 bits — the main line and most legs;
# "pub16": the reference's second published run, alpha/beta/gamma .6/.2/.2, theta .6/.2, ratios .8/.6/.4 at the
# CompressionConfig default widths 16/8/4 (experiments/results/compression_exp_20251020_225951/config.json,
# configs/base_config.py:33-35).
PARAM_SETS = {
    "coverage": dict(alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25, high_precision_bits=8,
                     medium_precision_bits=4, low_precision_bits=2, early_layer_ratio=0.8, middle_layer_ratio=0.6,
                     later_layer_ratio=0.4),
    "pub16": dict(alpha=0.6, beta=0.2, gamma=0.2, theta_h=0.6, theta_m=0.2, high_precision_bits=16,
                  medium_precision_bits=8, low_precision_bits=4, early_layer_ratio=0.8, middle_layer_ratio=0.6,
                  later_layer_ratio=0.4),
}


def metric_label(args, world: int) -> str:
    """BASELINE.json's metric string for the headline (cfg3 on 1 GPU); other configs / N get their own."""
    if world == 1 and args.config == "cfg3":
        return "prefill KV-compress GB/s + TTFT, Llama-2-7B S=16k, 1 GPU"
    S_total = args.seq * world
    return (f"prefill KV-compress GB/s + TTFT, {args.model} S={S_total // 1024}k, "
            f"{world} GPU{'s' if world > 1 else ''}")


def scaling_fields(ms_per_step: float, single_ms: float, world: int, how: str) -> dict:
    """The N > 1 line's same-workload single-GPU reference: the SAME S_total prefill (same inputs) through
    the single-GPU driver on rank 0's GPU, so a 1 -> N curve never mixes workloads."""
    speedup = single_ms / ms_per_step
    return {"single_gpu_ms_same_workload": round(single_ms, 4), "speedup": round(speedup, 4),
            "strong_scaling_efficiency": round(speedup / world, 4), "how": how}


def resolve_config(args, world: int):
    """Fill --layers/--heads/--head-dim/--seq from --config (default: cfg3 at N = 1, cfg4 at N > 1)."""
    if args.config is None:
        args.config = "cfg3" if world == 1 else "cfg4"
    c = CONFIGS[args.config]
    args.model = c["model"]
    for k in ("layers", "heads", "head_dim"):
        if getattr(args, k) is None:
            setattr(args, k, c[k])
    if args.seq is None:
        if c["seq_total"] % world:
            raise SystemExit(f"bench.py: {args.config}'s S = {c['seq_total']} does not split over {world} ranks")
        args.seq = c["seq_total"] // world
    # a shape override makes it another workload: label it as the config it was derived from
    args.config_label = args.config if (args.layers, args.heads, args.head_dim, args.seq * world) == (
        c["layers"], c["heads"], c["head_dim"], c["seq_total"]) else f"{args.config}-derived"
    return args


def visible_gpu_count(dri: str = "/dev/dri", env=None) -> int:
    """GPUs this process could use, counted WITHOUT initialising HIP (the launcher runs before any GPU
    call, and a HIP-initialised parent must not spawn the ranks): the DRM render nodes this process can
    open (a container maps only its own GPUs' nodes, and the device cgroup refuses the others), limited
    by the visibility masks HIP honours (ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES).  Raises RuntimeError when the count cannot be determined (e.g. /dev/dri
    unreadable); no /dev/dri at all means no GPU."""
    env = os.environ if env is None else env
    if not os.path.exists(dri):
        n = 0
    else:
        try:
            nodes = sorted(x for x in os.listdir(dri) if x.startswith("renderD"))
        except OSError as e:
            raise RuntimeError(f"cannot list {dri}: {e}") from e
        n = 0
        for x in nodes:
            try:
                fd = os.open(os.path.join(dri, x), os.O_RDWR | os.O_CLOEXEC)
            except OSError:
                continue  # not this process's GPU (device cgroup / permissions)
            os.close(fd)
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is None:
            continue
        ids = [t for t in v.split(",") if t.strip() != ""]
        if any(not t.strip().lstrip("-").isdigit() for t in ids):
            raise RuntimeError(f"{var}={v!r}: cannot count the GPUs it selects (UUIDs are not supported here)")
        picked = []
        for t in ids:  # HIP stops at the first invalid ordinal
            i = int(t)
            if i < 0 or i >= n:
                break
            picked.append(i)
        n = len(picked)
    return n


def launch(args) -> int:
    """--gpus N > 1 without a torch.distributed environment: run this script under
    torch.distributed.run as a CHILD process (nothing here touches a GPU: visible_gpu_count() opens
    DRM render nodes only, no HIP call), relay its exit code.  Fails fast when fewer than N GPUs are
    visible or the count cannot be determined."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    rest = [a for a in sys.argv[1:] if a != "--launch-dry-run"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + rest
    try:
        visible = visible_gpu_count()
    except RuntimeError as e:
        print(f"bench.py: cannot determine the visible GPUs ({e}); not running", file=sys.stderr, flush=True)
        return 2
    if args.launch_dry_run:
        print(json.dumps({"launch": cmd, "visible_gpus": visible}), flush=True)
        return 0
    if visible < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, this process sees {visible}; "
              f"not running (a smaller run would be mislabelled)", file=sys.stderr, flush=True)
        return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # the box's drivers support dmabuf IPC only
    return subprocess.run(cmd, env=env).returncode


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="BASELINE workload: cfg3 (default at N = 1), cfg4 (default at N > 1) or cfg5")
    ap.add_argument("--layers", type=int, default=None, help="override the config's layer count")
    ap.add_argument("--seq", type=int, default=None, help="override: tokens per rank (default S_total / N)")
    ap.add_argument("--heads", type=int, default=None)
    ap.add_argument("--head-dim", type=int, default=None)
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="--gpus N > 1 without WORLD_SIZE: print the torch.distributed.run command line and exit")
    ap.add_argument("--dtype", default="float32", choices=["float16", "bfloat16", "float32"],
                    help="K/V/attention dtype (default: the reference model's fp32)")
    ap.add_argument("--params", default="coverage", choices=sorted(PARAM_SETS),
                    help="compression parameters: coverage (8/4/2 bits, the default workload) or pub16 (the "
                         "reference's published 16/8/4 run)")
    ap.add_argument("--quant-only", action="store_true",
                    help="every token kept (RTKV_NO_SELECTION): BASELINE config 2's quantization-only path")
    ap.add_argument("--no-same-workload", action="store_true",
                    help="N > 1: skip the same-workload single-GPU reference on rank 0")
    ap.add_argument("--no-packed", action="store_true", help="skip the packed-code output")
    ap.add_argument("--no-dequant", action="store_true", help="skip the dequantized K'/V' output (packed only)")
    ap.add_argument("--legs", default="f16,packed_only,f16_packed_only,bits16,drop_in,s4096,cfg2_s4096_quant,s65536,"
                                      "independent_layers,prefill_7b,prefill_7b_f32,gq",
                    help="extra single-GPU legs after the main line: comma list of f16, packed_only, f16_packed_only, "
                         "bits16, drop_in, s4096, cfg2_s4096_quant, s65536, independent_layers, prefill_7b, "
                         "prefill_7b_f32, gq (or 'none')")
    ap.add_argument("--prefill-dtype", default="float16", choices=["float16", "bfloat16", "float32"],
                    help="dtype of the prefill_7b leg's random-init model")
    ap.add_argument("--prefill-modes", default="none,fused,eager",
                    help="prefill_7b attention variants (tools/prefill_model.py): none, fused, eager")
    ap.add_argument("--streams", type=int, default=1,
                    help="single GPU: consecutive layers go to this many streams (layer l on stream l %% n, one "
                         "workspace each).  Default 1: strictly sequential, the reference caller's order "
                         "(layer l+1's K/V come out of attention over layer l's compressed K'/V')")
    ap.add_argument("--leg-steps", type=int, default=5)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0,
                    help="CPU work budget of the oracle sample (layers are added until it is spent; 0 = skip)")
    ap.add_argument("--cpu-baseline-layers", type=int, default=32, help="at most this many layers in the sample")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--importance", default="w", choices=["w", "qk"],
                    help="w: the reference's attention-weights input (prompt slice); qk: fused mode "
                         "(Q + prompt keys + row LSE, K1' on MFMA)")
    ap.add_argument("--sharded", action="store_true",
                    help="use the sequence-sharded driver even at world size 1 (plumbing check)")
    ap.add_argument("--collectives", default="torch", choices=["torch", "rtkv", "host"],
                    help="sharded driver: torch.distributed, or the C ABI's RCCL communicators "
                         "(rtkv_allgather_rows / rtkv_allgather_packed)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: nccl (RCCL over xGMI, one GPU per rank) or gloo (rehearsal of the multi-rank "
                         "control flow with every collective staged through host memory; ranks may share a GPU)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="sharded driver: exchange every layer's packed KV after the last layer instead of "
                         "overlapping each layer's exchange with the following layers")
    return ap.parse_args()


def synth_layer(l: int, S: int, H: int, D: int, P: int, dtype, device, gen, row0: int = 0):
    """K, V [1,S,H*D] ~ N(0,1); W prompt slice [1,H,S,P] = u^4 row-normalised × U(0,1), causal in
    the prompt.  row0: global index of the first token (sequence shards)."""
    F = H * D
    K = torch.randn(1, S, F, generator=gen, device=device, dtype=torch.float32).to(dtype)
    V = torch.randn(1, S, F, generator=gen, device=device, dtype=torch.float32).to(dtype)
    u = torch.rand(1, H, S, P, generator=gen, device=device, dtype=torch.float32)
    raw = (u * u) ** 2 + 1e-6
    causal = torch.arange(P, device=device)[None, :] <= row0 + torch.arange(S, device=device)[:, None]
    raw = raw * causal
    W = raw / raw.sum(-1, keepdim=True) * torch.rand(1, H, S, 1, generator=gen, device=device)
    return K, V, W.to(dtype)


def synth_qk(S: int, H: int, D: int, K, dtype, device, gen, causal=True):
    """Fused-mode inputs for one layer: Q [1,H,S,D] ~ N(0,1) and the exact fp32 row LSE of the causal
    softmax(Q·Kᵀ/√d) over all S keys (setup only; computed in row chunks)."""
    Q = torch.randn(1, H, S, D, generator=gen, device=device, dtype=torch.float32).to(dtype)
    Kh = K.view(1, S, H, D).permute(0, 2, 1, 3)
    lse = torch.empty(1, H, S, dtype=torch.float32, device=device)
    step = 2048
    for i0 in range(0, S, step):
        i1 = min(S, i0 + step)
        x = torch.matmul(Q[:, :, i0:i1].float(), Kh.float().transpose(2, 3)) * (1.0 / D ** 0.5)
        if causal:
            x.masked_fill_(torch.arange(S, device=device)[None, :] > torch.arange(i0, i1, device=device)[:, None],
                           float("-inf"))
        lse[:, :, i0:i1] = torch.logsumexp(x, dim=-1)
        del x
    return Q, lse


class Job:
    """Per-rank state: inputs and outputs of every layer, resident in HBM.

    dtype / emit_dequant / emit_packed override the command line (extra legs); ``inputs`` shares
    another job's resident inputs instead of generating new ones."""

    def __init__(self, args, device, rank, world, dtype=None, emit_dequant=None, emit_packed=None, inputs=None,
                 seq=None, slots=None, quant_only=None, param_set=None):
        """seq: tokens (default --seq); slots: distinct input/output sets, layer l uses slot l % slots
        (bounds the memory of long-sequence legs; default one per layer); ``inputs`` given: layer l reads
        inputs[l % len(inputs)] and only the outputs cycle over ``slots``; quant_only: every token kept
        (RTKV_NO_SELECTION: BASELINE config 2, quantization without propagation); param_set: PARAM_SETS key."""
        import rtkv
        from rtkv import _lib as L
        self.args, self.device, self.rank, self.world = args, device, rank, world
        self.dtype = getattr(torch, dtype or args.dtype)
        self.S, self.H, self.D = seq or args.seq, args.heads, args.head_dim
        self.F = self.H * self.D
        self.S_total = self.S * world
        self.P = rtkv.prompt_length(self.S_total)
        self.quant_only = quant_only = getattr(args, "quant_only", False) if quant_only is None else quant_only
        self.param_set = param_set = param_set or getattr(args, "params", "coverage")
        self.cfg = rtkv.CompressionConfig(**PARAM_SETS[param_set], num_hidden_layers=args.layers)
        self.bits = (self.cfg.low_precision_bits, self.cfg.medium_precision_bits, self.cfg.high_precision_bits)
        self.emit_packed = (not args.no_packed) if emit_packed is None else emit_packed
        self.emit_dequant = (not args.no_dequant) if emit_dequant is None else emit_dequant
        if not (self.emit_packed or self.emit_dequant):
            raise SystemExit("--no-packed and --no-dequant together leave nothing to compute")
        flags = (L.EMIT_DEQUANT if self.emit_dequant else 0) | (L.EMIT_PACKED if self.emit_packed else 0) | \
            (L.NO_SELECTION if quant_only else 0)
        prop = rtkv.SelectiveTokenPropagator(self.cfg)
        gen = torch.Generator(device=device)
        gen.manual_seed(1234 + 7919 * rank)
        self.slots = min(args.layers, slots or args.layers)
        self.inputs = list(inputs) if inputs is not None else []
        self.bufs, self.params = [], []
        for l in range(args.layers):
            if inputs is None and l < self.slots:
                K, V, W = synth_layer(l, self.S, self.H, self.D, self.P, self.dtype, device, gen)
                if args.importance == "qk":
                    Q, lse = synth_qk(self.S, self.H, self.D, K, self.dtype, device, gen)
                    self.inputs.append((K, V, Q, lse))
                    del W
                else:
                    self.inputs.append((K, V, W))
            if l < self.slots:
                self.bufs.append(rtkv.LayerBuffers(1, self.S, self.F, self.dtype, device, self.bits,
                                                   emit_dequant=self.emit_dequant, emit_packed=self.emit_packed))
            ratio = 1.0 if quant_only else prop.get_layer_propagation_ratio(l)
            self.params.append(rtkv.params_from_config(self.cfg, l, self.P, ratio, flags))
        self.in_slots = len(self.inputs)
        self._acct = None
        self.ws = rtkv.Workspace(device)
        self.ws.get(1, self.S)
        # layer pipelining (streams2 leg): layer l runs on stream l % n with that stream's workspace;
        # a layer's buffers always see the same stream, so steps stay ordered per layer
        self.streams, self.wss = [None], [self.ws]
        torch.cuda.synchronize(device)

    def set_streams(self, n):
        import rtkv
        self.streams = [None] + [torch.cuda.Stream(self.device) for _ in range(n - 1)]
        self.wss = [self.ws] + [rtkv.Workspace(self.device) for _ in range(n - 1)]
        for w in self.wss:
            w.get(1, self.S)
        torch.cuda.synchronize(self.device)

    def step(self, events=None):
        """Compress every layer (single GPU); events: list of 4-tuples of torch events or None."""
        import rtkv
        from rtkv import _lib as L
        import ctypes
        qk = self.args.importance == "qk"
        n = len(self.streams) if events is None else 1
        if n > 1:
            main = torch.cuda.current_stream(self.device)
            for st in self.streams[1:]:
                st.wait_stream(main)
        for l in range(self.args.layers):
            sl, si = l % self.slots, l % self.in_slots
            if n > 1:
                st = self.streams[l % n]
                with torch.cuda.stream(st if st is not None else torch.cuda.current_stream(self.device)):
                    if qk:
                        K, V, Q, lse = self.inputs[si]
                        rtkv.compress_layer_qk(K, V, Q, lse, self.params[l], self.bufs[sl], self.wss[l % n])
                    else:
                        K, V, W = self.inputs[si]
                        rtkv.compress_layer(K, V, W, self.params[l], self.bufs[sl], self.wss[l % n])
                continue
            if qk:
                K, V, Q, lse = self.inputs[si]
                if events is None:
                    rtkv.compress_layer_qk(K, V, Q, lse, self.params[l], self.bufs[sl], self.ws)
                    continue
                kd, wd = rtkv.engine.kv_desc(K, V), rtkv.engine.qk_desc(Q, K, lse)
                fn = L.lib().rtkv_compress_layer_qk_events
            else:
                K, V, W = self.inputs[si]
                if events is None:
                    rtkv.compress_layer(K, V, W, self.params[l], self.bufs[sl], self.ws)
                    continue
                kd, wd = rtkv.engine.kv_desc(K, V), rtkv.engine.attn_desc(W)
                fn = L.lib().rtkv_compress_layer_events
            out = self.bufs[sl].out_struct()
            out.o_stride_h = kd.D
            ev = (ctypes.c_void_p * 4)(*[e.cuda_event for e in events[l]])
            L.check(fn(ctypes.byref(kd), ctypes.byref(wd), ctypes.byref(self.params[l]), ctypes.byref(out),
                       self.ws.buf.data_ptr(), self.ws.buf.numel(), L.stream_ptr(self.device), ev),
                    "compress_layer_events")

    def join(self):
        """The main stream waits for the pipelining streams (end of a step)."""
        main = torch.cuda.current_stream(self.device)
        for st in self.streams[1:]:
            main.wait_stream(st)

    def elem(self):
        return torch.tensor([], dtype=self.dtype).element_size()

    def read_roofline_bytes(self):
        """R per layer (north star): every K/V element once + the prompt columns of W."""
        e = self.elem()
        return 2 * self.S * self.F * e + self.H * self.S * self.P * e

    def accounting(self):
        """(kept rows, packed bytes) of every layer: one untimed pass, each layer's statistics read right
        after it (slots are reused by later layers)."""
        if self._acct is None:
            from rtkv.engine import decode_stats
            torch.cuda.synchronize(self.device)
            acct = []
            for l in range(self.args.layers):
                self._step_one(l)
                st = decode_stats(self.bufs[l % self.slots].stats.cpu().numpy().tobytes(), 1)
                acct.append((st.max_kept, st.total_packed_bytes))
            self._acct = acct
        return self._acct

    def _step_one(self, l):
        import rtkv
        sl, si = l % self.slots, l % self.in_slots
        if self.args.importance == "qk":
            K, V, Q, lse = self.inputs[si]
            rtkv.compress_layer_qk(K, V, Q, lse, self.params[l], self.bufs[sl], self.ws)
        else:
            K, V, W = self.inputs[si]
            rtkv.compress_layer(K, V, W, self.params[l], self.bufs[sl], self.ws)

    def layer_bytes(self):
        """Algorithmic HBM bytes per layer: total and the K4 (quantize+pack+compact) part."""
        e = self.elem()
        tot, k4 = [], []
        for l, (Sp, pk) in enumerate(self.accounting()):
            if self.args.importance == "qk":                     # Q + row LSE + prompt keys
                w_read = self.H * self.S * self.D * e + 4 * self.H * self.S + self.P * self.F * e
            else:
                w_read = self.H * self.S * self.P * e               # prompt columns of W
            kv_read = 2 * Sp * self.F * e                        # kept rows of K and V, read once
            deq = 2 * Sp * self.F * e if self.emit_dequant else 0   # dequantized K', V'
            packed = (2 * pk + Sp * 16) if self.emit_packed else 0   # codes + scale/zp
            meta = self.S * (4 + 4 + 4 + 1 + 1) + Sp * (4 + 8 + 1)   # A, scores, labels, mask / index, offset
            k4.append(kv_read + deq + packed + Sp * (4 + 8 + 1))
            tot.append(w_read + kv_read + deq + packed + meta)
        return tot, k4

    def timed(self, steps, warmup):
        """(ms per step, per-layer event times [K1, K2, K4] in µs) of this job alone."""
        for _ in range(warmup):
            self.step()
            self.join()
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
            self.join()
        torch.cuda.synchronize(self.device)
        ms = (time.perf_counter() - t0) / steps * 1e3
        return ms, self.kernel_times()

    def kernel_times(self, reps=3):
        """Per-layer mean of K1, K2 and K4 (µs) from HIP events the C ABI records on the launch stream."""
        events = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(self.args.layers)]
        for evs in events:
            for e in evs:
                e.record()  # materialise the hipEvent_t
        torch.cuda.synchronize(self.device)
        k_ms = [0.0, 0.0, 0.0]
        for _ in range(reps):
            self.step(events=events)
            torch.cuda.synchronize(self.device)
            for evs in events:
                for k in range(3):
                    k_ms[k] += evs[k].elapsed_time(evs[k + 1])
        return [m / (reps * self.args.layers) * 1e3 for m in k_ms]


def drop_in_leg(args, job, steps, warmup):
    """The reference caller's path (modified_llama.py:113-117): RealTimePrefillCompressor.
    compress_layer_kv_cache per layer, with its host sync for the output shape.

    TTFTs: ``ttft_ms`` is what the caller sees — the wall time of the 32 calls plus the final sync;
    ``total_processing_time_ms`` is the reference's definition as the API reports it (Σ processing_time,
    longbench_eval.py:160, each processing_time the wall time of the call, unified_compressor.py:118,148;
    it misses only the last layer's K4 tail after the last return); ``ttft_device_span_ms`` is Σ
    device_processing_time (each layer's device span stamped by its kernels).  Measured for the default strict mode (each call waits for K4's start, so a late
    selection failure raises in its own layer) and for strict=False."""
    import rtkv
    ids = torch.zeros(1, job.S, dtype=torch.long, device=job.device)
    # the raw driver on the same inputs right before, in the same device state (legs that ran before
    # this one leave the device warmer: the drop-in's margin is measured against this, not the main line)
    raw_ms, _ = job.timed(steps, 1)
    # ... and timed like the drop-in: one prefill per timed region (sync, 32 layers, sync), so both pay the
    # same per-prefill start (the first launch after an idle device) and end (the final sync)
    raw_sample = []
    for it in range(warmup + steps):
        torch.cuda.synchronize(job.device)
        t0 = time.perf_counter()
        job.step()
        torch.cuda.synchronize(job.device)
        if it >= warmup:
            raw_sample.append((time.perf_counter() - t0) * 1e3)
    raw_sample_ms = sum(raw_sample) / len(raw_sample)
    out = {}
    for strict in (True, False):
        comp = rtkv.RealTimePrefillCompressor(job.cfg, emit_packed=job.emit_packed, strict=strict)
        span, wall, calls = [], [], []
        for it in range(warmup + steps):
            comp.reset_compression_state()
            torch.cuda.synchronize(job.device)
            t0 = time.perf_counter()
            for l in range(args.layers):
                K, V, W = job.inputs[l % job.in_slots]
                comp.compress_layer_kv_cache(K, V, W, ids, l)
            torch.cuda.synchronize(job.device)
            if it >= warmup:
                wall.append((time.perf_counter() - t0) * 1e3)
                span.append(sum(st["device_processing_time"] for st in comp.layer_states.values()) * 1e3)
                calls.append(comp.get_overall_compression_stats()["total_processing_time"] * 1e3)
        w, d, c = sum(wall) / len(wall), sum(span) / len(span), sum(calls) / len(calls)
        out["strict" if strict else "non_strict"] = {
            "ttft_ms": round(w, 4), "wall_ms_per_layer": round(w / args.layers, 4),
            "total_processing_time_ms": round(c, 4), "ttft_device_span_ms": round(d, 4), "over_raw_driver_ms": round(w - raw_ms, 4),
            "over_raw_driver_per_prefill_ms": round(w - raw_sample_ms, 4)}
        del comp
    s_ = out["strict"]
    return {"ttft_ms": s_["ttft_ms"], "ms_per_layer": s_["wall_ms_per_layer"],
            "total_processing_time_ms": s_["total_processing_time_ms"],
            "ttft_device_span_ms": s_["ttft_device_span_ms"], "wall_ms_per_step": s_["ttft_ms"],
            "raw_driver_ms_per_step_same_state": round(raw_ms, 4),
            "raw_driver_ms_per_prefill_same_state": round(raw_sample_ms, 4),
            "raw_driver_note": "ms_per_step: steps back to back (the main line's timing); per_prefill: each step "
                               "alone between two syncs, as the drop-in's wall time is taken",
            "modes": out, "steps": steps,
            "path": "rtkv.RealTimePrefillCompressor.compress_layer_kv_cache (dequant + packed, one host wait "
                    "per layer for the output shape; strict = the default)"}


def gq_leg(args, job, steps, warmup):
    """Extension rtkv-gq/1 (opt-in; per-channel outlier voting + per-head group-wise pack, csrc/outlier.hip) on
    the main line's layers: each layer is compressed as usual, then gq_compress (votes, outlier select, pack)
    runs on its kept rows, timed by events around the gq launches alone.  Algorithmic bytes per layer: the
    kept K/V rows read by the pack (plus every vote_stride-th row by the vote), the codes, per-head
    scale/zero-points and outlier values written.  Also the reconstruction MSE of K' and V' on the last
    layer: the reference's per-token scheme (the drop-in's K'/V') against gq, same kept rows and widths."""
    import rtkv
    if args.importance != "w" or job.F % 512 or not job.emit_packed or not job.emit_dequant:
        return {"skipped": "needs the W path with dequantized and packed outputs, F a multiple of 512"}
    cfg = rtkv.GroupQuantConfig()
    acct = job.accounting()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.layers)]
    tot, n, c = 0.0, 0, None
    for it in range(warmup + steps):
        for l in range(args.layers):
            job._step_one(l)
            K, V = job.inputs[l % job.in_slots][:2]
            b = job.bufs[l % job.slots]
            Sp, pk = acct[l]
            ev[l][0].record()
            c = rtkv.gq_compress(K, V, b.kept_index[0], b.labels[0], b.row_offset[0], b.stats, Sp, pk, job.bits, cfg)
            ev[l][1].record()
        torch.cuda.synchronize(job.device)
        if it >= warmup:
            tot += sum(a.elapsed_time(z) for a, z in ev)
            n += args.layers
    us = tot / n * 1e3
    # the same layers with the extension on a side stream (what the drop-in does): whole-step time against
    # the step without it, both between events on the main stream (the side stream joined at the end)
    side = torch.cuda.Stream(job.device)
    step_ms = {}
    for mode in ("without", "side_stream", "without", "side_stream"):
        for it in range(warmup + steps):
            a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a0.record()
            slot_ev = {}  # a buffer slot is not reused on the main stream before the side stream has read it
            for l in range(args.layers):
                if l % job.slots in slot_ev:
                    torch.cuda.current_stream(job.device).wait_event(slot_ev.pop(l % job.slots))
                job._step_one(l)
                if mode == "side_stream":
                    K, V = job.inputs[l % job.in_slots][:2]
                    b = job.bufs[l % job.slots]
                    Sp, pk = acct[l]
                    rtkv.gq_compress(K, V, b.kept_index[0], b.labels[0], b.row_offset[0], b.stats, Sp, pk, job.bits,
                                     cfg, stream=side)
                    slot_ev[l % job.slots] = torch.cuda.Event()
                    slot_ev[l % job.slots].record(side)
            torch.cuda.current_stream(job.device).wait_stream(side)
            a1.record()
            torch.cuda.synchronize(job.device)
            if it >= warmup:
                step_ms.setdefault(mode, []).append(a0.elapsed_time(a1))
    med = {m: sorted(v)[len(v) // 2] for m, v in step_ms.items()}
    e, H = job.elem(), job.F // 128
    nb = 0
    for Sp, pk in acct:
        nb += 2 * Sp * job.F * e + 2 * (Sp // cfg.vote_stride) * job.F * e  # pack reads + vote reads
        nb += 2 * pk + Sp * 2 * H * (2 + cfg.n_outlier) * e                   # codes + meta + outlier values
    nb /= len(acct)
    # reconstruction on the last layer (its buffers and K/V are still resident)
    l = args.layers - 1
    K, V = job.inputs[l % job.in_slots][:2]
    b = job.bufs[l % job.slots]
    Sp = acct[l][0]
    kept = b.kept_index[0, :Sp].long()
    kq, vq = c.dequantize()
    mse = {}
    for name, x, deq, gq in (("K", K, b.k_out, kq), ("V", V, b.v_out, vq)):
        src = x[0, kept].float()
        mse[name] = {"per_token": ((deq[: Sp * job.F].view(Sp, job.F).float() - src) ** 2).mean().item(),
                     "gq": ((gq[0].float() - src) ** 2).mean().item()}
    gbs = nb / (us / 1e6) / 1e9
    return {"us_per_layer": round(us, 2), "algorithmic_bytes_per_layer": int(nb), "GBs": round(gbs, 1),
            "hbm_frac": round(gbs / 8000.0, 4), "config": vars(cfg),
            "side_stream": {"step_ms_without": round(med["without"], 4), "step_ms_with": round(med["side_stream"], 4),
                            "overhead_us_per_layer": round((med["side_stream"] - med["without"]) * 1e3 / args.layers, 2),
                            "note": "the drop-in's mode: gq after each layer on a side stream, overlapping the next "
                                    "layers; medians of the steps, the side stream joined before the end event"},
            "reconstruction_mse_last_layer": mse,
            "note": "synthetic K/V ~ N(0,1) carry no outlier channels: the gq MSE gain here comes from the per-head "
                    "groups alone (tests/test_gpu_gq.py measures it with injected key outliers at the 13B shape)",
            "path": "rtkv.gq_compress after each layer's rtkv_compress_layer (events around the gq launches only)"}


def union_inputs(args, device, world, dtype):
    """The inputs of every layer of a sharded job's WHOLE prefill on one device: rank j's chunks drawn
    exactly as ShardedJob draws them (generator seed 1234 + 7919*j, row0 = j*S_local), concatenated in
    token order — the single-GPU reference of an N-rank line computes the same bytes."""
    import rtkv
    S_local, H, D = args.seq, args.heads, args.head_dim
    P = rtkv.prompt_length(S_local * world)
    gens = []
    for j in range(world):
        g = torch.Generator(device=device)
        g.manual_seed(1234 + 7919 * j)
        gens.append(g)
    inputs = []
    for l in range(args.layers):
        parts = [synth_layer(l, S_local, H, D, P, dtype, device, gens[j], row0=j * S_local) for j in range(world)]
        inputs.append(tuple(torch.cat([p[k] for p in parts], dim=2 if k == 2 else 1) for k in range(3)))
        del parts
    return inputs


class ShardedJob:
    """Sequence-sharded prefill: this rank owns tokens [rank*S, (rank+1)*S) of the config's
    S_total = N*S-token prefill (S = S_total / N: strong scaling over a fixed BASELINE workload).
    One step = every layer's shard stages (K1 on own rows, RCCL all-gather of A, global selection,
    K4 on own kept rows) + the exchange of the packed KV (overlapped with later layers by default)."""

    def __init__(self, args, device, rank, world):
        import rtkv
        from rtkv.sharded import ShardedPrefillCompressor
        self.args, self.device, self.rank, self.world = args, device, rank, world
        self.dtype = getattr(torch, args.dtype)
        self.S, self.H, self.D = args.seq, args.heads, args.head_dim
        self.F = self.H * self.D
        self.S_total = self.S * world
        self.P = rtkv.prompt_length(self.S_total)
        self.cfg = rtkv.CompressionConfig(**PARAM_SETS["coverage"], num_hidden_layers=args.layers)
        self.bits = (2, 4, 8)
        self.comp = ShardedPrefillCompressor(self.cfg, emit_packed=not args.no_packed, emit_dequant=True,
                                             device=device, overlap=not args.no_overlap,
                                             collectives=args.collectives)
        gen = torch.Generator(device=device)
        gen.manual_seed(1234 + 7919 * rank)
        self.inputs, self.params = [], []
        for l in range(args.layers):
            self.inputs.append(synth_layer(l, self.S, self.H, self.D, self.P, self.dtype, device, gen,
                                           row0=rank * self.S))
            self.params.append(self.comp.params(l, self.S_total))
        self.last = None
        torch.cuda.synchronize(device)

    def step(self, events=None):
        for l in range(self.args.layers):
            K, V, W = self.inputs[l]
            self.comp.enqueue_layer(K, V, W, l, params=self.params[l])
        self.last = self.comp.exchange()

    def layer_bytes(self):
        """Algorithmic HBM bytes per layer of the whole N*S-token job (same formula as Job)."""
        from rtkv.engine import decode_stats
        e = torch.tensor([], dtype=self.dtype).element_size()
        tot, k4 = [], []
        for sl in self.last:
            st = decode_stats(sl.bufs.g.stats.cpu().numpy().tobytes(), 1)
            Sp, pk = st.max_kept, st.total_packed_bytes
            w_read = self.H * self.S_total * self.P * e
            kv_read = 2 * Sp * self.F * e
            deq = 2 * Sp * self.F * e
            packed = (2 * pk + Sp * 16) if not self.args.no_packed else 0
            meta = self.S_total * (4 + 4 + 4 + 1 + 1) + Sp * (4 + 8 + 1)
            k4.append(kv_read + deq + packed + Sp * (4 + 8 + 1))
            tot.append(w_read + kv_read + deq + packed + meta)
        return tot, k4

    def split_times(self, barrier, reps=3):
        """This rank's milliseconds per step of the step's parts, each timed alone after the timed loop
        (end-of-prefill exchange mode, so the parts do not overlap): ``compute_ms`` = every layer's
        stages (K1, the all-gathers of A, the replicated selection, K4) with no packed KV moved;
        ``exchange_ms`` = the grouped send/recv of every layer's packed KV (after a barrier, so a
        slower peer's compute is not counted); ``allgather_A_ms`` = the layers' all-gathers of A alone
        (part of compute_ms)."""
        comp = self.comp
        overlap = comp.overlap
        comp.overlap = False
        try:
            def enqueue_all():
                for l in range(self.args.layers):
                    K, V, W = self.inputs[l]
                    comp.enqueue_layer(K, V, W, l, params=self.params[l])
            barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                enqueue_all()
                comp.exchange(transfer=False)
            torch.cuda.synchronize(self.device)
            compute = (time.perf_counter() - t0) / reps
            ex = 0.0
            for _ in range(reps):
                enqueue_all()
                torch.cuda.synchronize(self.device)
                barrier()
                t0 = time.perf_counter()
                self.last = comp.exchange()
                torch.cuda.synchronize(self.device)
                ex += time.perf_counter() - t0
            barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                for _l in range(self.args.layers):
                    comp.gather_A(1, self.S)
            torch.cuda.synchronize(self.device)
            ag = (time.perf_counter() - t0) / reps
        finally:
            comp.overlap = overlap
        return {"compute_ms": round(compute * 1e3, 4), "exchange_ms": round(ex / reps * 1e3, 4),
                "allgather_A_ms": round(ag * 1e3, 4)}

    def exchanged_bytes(self):
        """Bytes of packed KV (codes + scale/zero-point) this rank received in the exchange."""
        n = 0
        for sl in self.last:
            r = sl.ranges[0]
            mine = (int(r[self.rank + 1, 1] - r[self.rank, 1]) * 2 + int(r[self.rank + 1, 0] - r[self.rank, 0]) * 16)
            n += (int(r[-1, 1] - r[0, 1]) * 2 + int(r[-1, 0] - r[0, 0]) * 16) - mine
        return n


def workload_key(args):
    """Identifies the workload a committed PMC summary was collected on (profiles/*_pmc.json)."""
    key = {"seq": args.seq, "layers": args.layers, "heads": args.heads, "head_dim": args.head_dim,
           "dtype": args.dtype, "packed": not args.no_packed, "dequant": not args.no_dequant,
           "importance": args.importance}
    if getattr(args, "params", "coverage") != "coverage":  # summaries before round 5 are all "coverage"
        key["params"] = args.params
    if getattr(args, "quant_only", False):
        key["quant_only"] = True
    return key


def pmc_kernels(args):
    """Per-kernel HBM bytes per dispatch from the newest committed PMC summary of this exact workload
    (profiles/*_pmc.json, written by profiles/summarize.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of `bench.py --legs none`), or (None, None)."""
    import glob
    want = workload_key(args)
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc.json")), reverse=True):
        with open(path) as f:
            doc = json.load(f)
        if doc.get("workload") == want:  # round-1 summaries carry no workload key: never matched
            return doc["kernels"], os.path.relpath(path, REPO)
    return None, None


def cpu_baseline(args, job):
    """The C oracle (an OpenMP restatement of the reference: aggregation and per-row quantization
    over threads, selection serial) on a bounded sample: the first layers of the same workload, same
    inputs, added until --cpu-baseline-seconds of CPU time are spent."""
    if args.cpu_baseline_seconds <= 0 or args.importance != "w":
        return None
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import rtkv_oracle as orc
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = affinity
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():   # the host-core share of this job (16 on the GPU box)
        threads = max(1, min(threads, int(os.environ["OMP_NUM_THREADS"])))
    code = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}[job.dtype]
    nbytes, secs, n = 0.0, 0.0, 0
    tot, _ = job.layer_bytes()
    for l in range(min(args.cpu_baseline_layers, args.layers)):
        K, V, W = job.inputs[l]
        as_np = (lambda t: t.cpu().numpy()) if job.dtype == torch.float32 else \
            (lambda t: t.cpu().view(torch.int16).numpy().view(np.uint16))
        Kn, Vn, Wn = as_np(K), as_np(V), as_np(W)
        p = job.params[l]
        t0 = time.perf_counter()
        orc.compress_layer(Kn, Vn, code, Wn, code, job.P, p.alpha, p.beta, p.gamma, p.layer_weight, p.theta_h,
                           p.theta_m, job.bits, p.propagation_ratio, packed=job.emit_packed, threads=threads)
        secs += time.perf_counter() - t0
        nbytes += tot[l]
        n += 1
        if secs >= args.cpu_baseline_seconds:
            break
    return {"value": round(nbytes / secs / 1e9, 4), "unit": "GB/s", "cores": threads, "host_cpus": os.cpu_count(),
            "affinity_cpus": affinity,
            "threads_rule": "min(OMP_NUM_THREADS, CPUs in this process's affinity mask): the job's host-core share",
            "kind": "port", "ms_per_layer": round(secs / n * 1e3, 1),
            "sample": f"{n} of {args.layers} layers (S={job.S}, {job.H}x{job.D}, {args.dtype}), C oracle "
                      f"oracle/rtkv_oracle.c, OpenMP on {threads} host threads (aggregation and per-row "
                      f"quantization parallel, selection serial)"}


def roofline_objects(args, job, kus, k4_bytes):
    """(path read roofline, K4 roofline) from the per-layer event times kus = [K1, K2, K4] µs."""
    pmc, src = pmc_kernels(args)
    layer_us = sum(kus)
    R = job.read_roofline_bytes()
    achieved = R / (layer_us / 1e6) / 1e9
    traffic = None
    if pmc:
        traffic = round(sum(v["hbm_bytes"] for v in pmc.values()))
    path = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": src,
            "scope": "path: every kernel of a layer (K1 + K2 + K4), HIP events on the launch stream",
            "algorithmic_bytes_per_launch": R,
            "algorithmic_bytes_def": "R = 2*S*H*D*e + H*S*P*e (every K/V element once + W prompt columns; "
                                     "SURVEY §8d, the north star's HBM-read roofline)",
            "avg_launch_us": round(layer_us, 2)}
    k4_us = kus[2]
    k4_alg = sum(k4_bytes) / len(k4_bytes)
    k4_ach = k4_alg / (k4_us / 1e6) / 1e9
    k4_traffic = None
    name = "quant_rows_kernel"
    if pmc:  # the whole-row or the split-row K4 (quant_rows_split_kernel), whichever the workload ran
        hit = next(((k, v) for k, v in pmc.items() if "quant_rows_" in k), None)
        if hit:
            k4_traffic = round(hit[1]["hbm_bytes"])
            name = "quant_rows_split_kernel" if "quant_rows_split_kernel" in hit[0] else name
    k4 = {"bound": "hbm", "achieved": round(k4_ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
          "frac": round(k4_ach / HBM_PEAK_GBS, 4), "traffic": k4_traffic, "traffic_source": src,
          "algorithmic_bytes_per_launch": round(k4_alg),
          "kernel": f"{name} (K4), K4's read + write bytes",
          "avg_launch_us": round(k4_us, 2)}
    return path, k4


def job_args(args, job):
    """args as they would read for a bench run of exactly `job`'s workload (the PMC summary key)."""
    a = argparse.Namespace(**vars(args))
    a.seq, a.dtype, a.params, a.quant_only = job.S, str(job.dtype).split(".")[-1], job.param_set, job.quant_only
    a.no_dequant, a.no_packed = not job.emit_dequant, not job.emit_packed
    return a


def leg_summary(args, job, ms, kus):
    tot, k4 = job.layer_bytes()
    path, k4r = roofline_objects(job_args(args, job), job, kus, k4)
    return {"value": round(sum(tot) / (ms / 1e3) / 1e9, 2), "unit": "GB/s", "ms_per_step": round(ms, 4),
            "dtype": {"float16": "f16", "bfloat16": "bf16", "float32": "f32"}[str(job.dtype).split(".")[-1]],
            "outputs": "+".join(x for x, on in (("dequant", job.emit_dequant), ("packed", job.emit_packed)) if on),
            "bits": "/".join(map(str, job.bits[::-1])), "params": job.param_set,
            "kernel_us_per_layer": kernel_us(job, kus),
            "path_read_roofline_frac": path["frac"], "layer_us": round(sum(kus), 2), "roofline": k4r}


def kernel_us(job, kus):
    return {"K1_aggregation": round(kus[0], 2), "K2_select": round(kus[1], 2), "K4_quant_pack": round(kus[2], 2)}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))  # before any GPU call
    if args.launch_dry_run:
        raise SystemExit("--launch-dry-run: only with --gpus N > 1 outside torch.distributed.run")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: refusing a mislabelled run", file=sys.stderr)
        sys.exit(2)
    resolve_config(args, world)
    if args.dist_backend == "gloo":  # rehearsal: ranks may share the visible GPUs
        local = local % max(1, torch.cuda.device_count())
        args.collectives = "host"
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    sharded = world > 1 or args.sharded
    if sharded:
        import torch.distributed as dist
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29531")
            if args.dist_backend == "gloo":
                dist.init_process_group("gloo", rank=rank, world_size=world)
            else:
                dist.init_process_group("nccl", device_id=device, rank=rank, world_size=world)
        world = dist.get_world_size()
        job = ShardedJob(args, device, rank, world)
    else:
        dist = None
        # long sequences: 8 distinct layer inputs cycled over the layers (bounded HBM and setup time)
        job = Job(args, device, rank, world, slots=8 if args.seq > 16384 else None)
        job.set_streams(max(1, args.streams))

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(device)

    join = getattr(job, "join", lambda: None)
    for _ in range(args.warmup):
        job.step()
        join()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job.step()
        join()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3

    kus = None
    split = None
    if sharded:
        for _ in range(2):
            job.step()
        torch.cuda.synchronize(device)
        split = job.split_times(barrier)  # per-rank compute / all-gather / exchange, outside the timed loop
    else:
        kus = job.kernel_times()  # per-kernel timing (HIP events on the launch stream), outside the timed loop
    tot_bytes, k4_bytes = job.layer_bytes()
    step_bytes = sum(tot_bytes)  # whole-job algorithmic bytes (the sharded job counts all N*S tokens)
    value = step_bytes / (ms_per_step / 1e3) / 1e9

    ranks = None
    if sharded:
        props = torch.cuda.get_device_properties(device)
        me = dict(rank=rank, local_rank=local, device=torch.cuda.current_device(),
                  pci_bus_id=getattr(props, "pci_bus_id", None), received_bytes_per_step=job.exchanged_bytes(),
                  **split)
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
    single = None
    if sharded and world > 1 and rank == 0 and not args.no_same_workload:
        # the SAME S_total prefill through the single-GPU driver on this GPU (the other ranks wait in the
        # final barrier): the per-N lines of a 1 -> N curve then each carry their own same-workload time
        ref = Job(args, device, 0, 1, inputs=union_inputs(args, device, world, job.dtype), seq=args.seq * world,
                  slots=8)
        single_ms, _ = ref.timed(args.steps, args.warmup)
        single = scaling_fields(ms_per_step, single_ms, world,
                                f"the same {args.config_label} prefill (S={args.seq * world}, same inputs: every rank's "
                                f"chunks concatenated) through the single-GPU driver (rtkv_compress_layer; "
                                f"{'pipeline' if args.seq * world > 65536 else 'one-launch'} K2) on rank 0's GPU, "
                                f"{args.steps} timed steps, outputs cycled over 8 buffers")
        del ref
        torch.cuda.empty_cache()
    if rank == 0:
        outs = "+".join(x for x, on in (("dequant", not args.no_dequant), ("packed", not args.no_packed)) if on)
        line = {
            "metric": metric_label(args, world),
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "ttft_ms": round(ms_per_step, 4),
            "higher_is_better": True,
            # N > 1 splits the config's S_total over the ranks: total work fixed as N grows
            "scaling": "strong" if world > 1 else "weak",
            "vs_baseline": None,
            "dtype": {"float16": "f16", "bfloat16": "bf16", "float32": "f32"}[args.dtype],
            "data": "synthetic (seeded torch RNG; K,V ~ N(0,1), W = causal u^4-softmax-like prompt slice)",
            "config": {"workload": f"{args.config_label}: {args.model} prefill KV compression"
                                   f"{' (fused Q/LSE importance)' if args.importance == 'qk' else ''}, {args.layers} layers, "
                                   f"S={job.S * world} ({job.S}/rank), {args.heads}x{args.head_dim}, {args.dtype}, "
                                   f"P={job.P}, bits {'/'.join(map(str, job.bits[::-1]))}, {getattr(job, 'param_set', 'coverage')} "
                                   f"parameters, {'no selection (every token kept)' if getattr(job, 'quant_only', False) else 'ratios .8/.6/.4'}, "
                                   f"{outs} outputs"
                                   + (f", {job.in_slots} distinct layer inputs cycled" if getattr(job, "in_slots", args.layers) < args.layers else ""),
                       "model": f"{args.model} (KV shapes only)", "global_batch": 1, "seq_len": job.S * world,
                       "parallelism": f"sequence-shard x{world}" if world > 1 else "single GPU",
                       "layer_streams": 1 if sharded else max(1, args.streams)},
        }
        if sharded:
            line["world_size"] = world
            if single is not None:
                line.update(single)
            line["ranks"] = ranks
            line["exchange"] = {"received_bytes_per_rank_per_step": job.exchanged_bytes(),
                                "kind": ("grouped RCCL send/recv per layer of packed K/V codes + scale/zp (exact byte "
                                         "ranges, all peers at once), " +
                                         ("all after the last layer" if args.no_overlap else
                                          "each issued two layers later on its own communicator, overlapping "
                                          "the following layers' compute")),
                                "per_layer_collective": "RCCL all-gather of A (4 B/token)"}
        else:
            path, k4 = roofline_objects(args, job, kus, k4_bytes)
            line["roofline"] = k4  # the contract's object: the dominant kernel (K4) on its algorithmic bytes
            line["roofline_path"] = path  # the north star's: the whole layer path on its HBM-read bytes
            line["kernel_us_per_layer"] = kernel_us(job, kus)
            if args.importance == "qk":  # K1' on MFMA: the Q·K_P^T contraction against the dense peak
                flops = 2.0 * job.H * job.S * job.P * job.D
                tf = flops / (kus[0] / 1e6) / 1e12
                line["k1_mfma"] = {"bound": "mfma", "achieved": round(tf, 2), "peak": 2500.0, "unit": "TFLOP/s",
                                   "frac": round(tf / 2500.0, 4), "avg_launch_us": round(kus[0], 2),
                                   "hbm_GBs": round((job.H * job.S * job.D * 2 + 4 * job.H * job.S) / (kus[0] / 1e6) / 1e9, 1)}
            legs = {}
            wanted = [x for x in args.legs.split(",") if x and x != "none"] if args.importance == "w" else []
            wanted = sorted(wanted, key=lambda x: x not in ("f16", "f16_packed_only"))  # share the fp16 inputs
            f16_inputs = None
            for name in wanted:
                if name in ("f16", "f16_packed_only") and args.dtype != "float16":
                    # the workload in fp16, with dequantized + packed outputs or packed only (the north star's
                    # 60 % is defined on packed KV; SURVEY §8d's worked example is fp16)
                    packed_only = name == "f16_packed_only"
                    leg = Job(args, device, rank, world, dtype="float16", inputs=f16_inputs,
                              emit_dequant=not packed_only, emit_packed=True)
                    f16_inputs = leg.inputs
                    legs[name] = leg_summary(args, leg, *leg.timed(args.leg_steps, 2))
                    del leg
                elif name == "packed_only":
                    leg = Job(args, device, rank, world, emit_dequant=False, emit_packed=True, inputs=job.inputs)
                    legs["packed_only"] = leg_summary(args, leg, *leg.timed(args.leg_steps, 2))
                    del leg
                elif name == "bits16" and job.param_set != "pub16":
                    # the reference's default / second published widths 16/8/4 with the published run's
                    # parameters, on the main line's inputs
                    leg = Job(args, device, rank, world, inputs=job.inputs, param_set="pub16")
                    legs["bits16"] = leg_summary(args, leg, *leg.timed(args.leg_steps, 2))
                    del leg
                elif name == "independent_layers":
                    # NOT the reference caller's order: consecutive layers on 4 streams (layer l on stream
                    # l % 4), which only a caller holding several layers' K/V/W at once can do
                    job.set_streams(4)
                    ms4, _ = job.timed(args.leg_steps, 2)
                    job.set_streams(max(1, args.streams))
                    tot, _ = job.layer_bytes()
                    legs["independent_layers"] = {
                        "value": round(sum(tot) / (ms4 / 1e3) / 1e9, 2), "unit": "GB/s", "ms_per_step": round(ms4, 4),
                        "path": "layer l on stream l % 4 (cross-layer overlap of one layer's selection with its "
                                "neighbours' kernels; not reachable from the reference's sequential prefill)"}
                elif name in ("s4096", "cfg2_s4096_quant", "s65536"):
                    if f16_inputs is not None:
                        f16_inputs = None
                        torch.cuda.empty_cache()
                    # BASELINE configs: cfg2 (7B, S=4096, quantization only), the north star's S in {4k, 64k}
                    seq = 65536 if name == "s65536" else 4096
                    leg = Job(args, device, rank, world, seq=seq, slots=8 if seq > 16384 else None,
                              quant_only=name.startswith("cfg2"))
                    legs[name] = leg_summary(args, leg, *leg.timed(args.leg_steps, 2))
                    legs[name]["seq"] = seq
                    legs[name]["selection"] = "none (RTKV_NO_SELECTION, every token quantized)" \
                        if leg.quant_only else ("pipeline K2 (S > 65536)" if seq > 65536 else "one-launch K2")
                    if leg.slots < args.layers:
                        legs[name]["inputs"] = f"{leg.slots} distinct layer inputs cycled over {args.layers} layers"
                    del leg
                elif name == "prefill_7b":
                    # sync'd prefill wall time of a random-init 7B-shaped model at S (TTFT as
                    # benchmark runner.py:202-212 measures it), with / without compression
                    sys.path.insert(0, os.path.join(REPO, "tools"))
                    from prefill_model import prefill_leg
                    legs["prefill_7b"] = prefill_leg(device, S=job.S, dtype=getattr(torch, args.prefill_dtype),
                                                     modes=tuple(args.prefill_modes.split(",")))
                elif name == "prefill_7b_f32":
                    # the same at the reference model's own precision (modified_llama.py:368 builds the model
                    # with default fp32 parameters): fp32 states, fp32 LSE / K1' on the f32 MFMA
                    sys.path.insert(0, os.path.join(REPO, "tools"))
                    from prefill_model import prefill_leg
                    legs["prefill_7b_f32"] = prefill_leg(device, S=job.S, dtype=torch.float32,
                                                         modes=tuple(args.prefill_modes.split(",")))
                elif name == "gq":
                    legs["gq"] = gq_leg(args, job, args.leg_steps, 2)
                elif name == "drop_in":
                    legs["drop_in"] = drop_in_leg(args, job, args.leg_steps, 2)
                    legs["drop_in"]["raw_driver_ms_per_layer"] = round(ms_per_step / args.layers, 4)
                torch.cuda.empty_cache()
            if legs:
                line["legs"] = legs
            line["cpu_baseline"] = cpu_baseline(args, job)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
