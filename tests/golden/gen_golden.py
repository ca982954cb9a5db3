#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE implementation on synthetic inputs.

Run in the build container only (it imports the reference from /root/reference, which does not
exist on the GPU box):

    python tests/golden/gen_golden.py            # writes tests/golden/fixtures/

Numerics are pinned to PyTorch's CPU kernels with ATEN_CPU_CAPABILITY=avx2 and one thread (the
reduction order of torch's cascade sum depends on the vector width).  Inputs come from
tests/golden/synth.py (seeded, bit-reproducible), so fixtures store only expected outputs (full
arrays for small cases, sha256 for large ones) plus the input spec.

The script also runs the C oracle (oracle/rtkv_oracle.py) on the same inputs and reports every
mismatch: the oracle must agree with the reference bit-for-bit except where a selection depends on
the reference's unstable argsort tie order ("tie_ambiguous", recorded in the manifest).
"""
from __future__ import annotations

import os

os.environ.setdefault("ATEN_CPU_CAPABILITY", "avx2")
os.environ.setdefault("OMP_NUM_THREADS", "1")

import hashlib  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("RTKV_REFERENCE", "/root/reference")
OUT = os.path.join(HERE, "fixtures")
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REF)

import synth  # noqa: E402
import rtkv_oracle as orc  # noqa: E402
from configs.base_config import CompressionConfig  # noqa: E402
from src.compression.dynamic_quantization import DynamicPrecisionQuantizer  # noqa: E402
from src.compression.selective_propagation import SelectiveTokenPropagator  # noqa: E402
from src.compression.token_importance import PromptGuidedImportanceScorer  # noqa: E402
from src.compression.unified_compressor import RealTimePrefillCompressor  # noqa: E402

torch.set_num_threads(1)
TDT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}
SMALL = 1 << 16  # arrays up to this many bytes are stored whole; larger ones by sha256

PUBLISHED = dict(alpha=0.6, beta=0.2, gamma=0.2, theta_h=0.6, theta_m=0.2, high_precision_bits=8,
                 medium_precision_bits=4, low_precision_bits=2, early_layer_ratio=0.8,
                 middle_layer_ratio=0.6, later_layer_ratio=0.4)
COVERAGE = dict(PUBLISHED, alpha=0.8, beta=0.1, gamma=0.1, theta_h=0.4, theta_m=0.25)
# the second published run: same parameters at the CompressionConfig default widths 16/8/4
# (experiments/results/compression_exp_20251020_225951/config.json:50-52, configs/base_config.py:33-35)
PUB16 = dict(PUBLISHED, high_precision_bits=16, medium_precision_bits=8, low_precision_bits=4)
DEFAULT = {}  # CompressionConfig defaults: 16/8/4 bits, .4/.3/.3, θ .7/.3


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def t_of(stored: np.ndarray, dtype: str) -> torch.Tensor:
    return torch.from_numpy(synth.to_f32(stored, dtype).copy()).to(TDT[dtype])


def np_of(t: torch.Tensor) -> np.ndarray:
    """torch tensor → storage array (float32, or uint16 bits for half types)."""
    if t.dtype == torch.float32:
        return t.detach().numpy().copy()
    return t.detach().contiguous().view(torch.int16).numpy().view(np.uint16).copy()


def make_config(params: dict, L: int) -> CompressionConfig:
    kw = dict(params)
    kw["num_hidden_layers"] = L
    if L == 1:
        kw["layer_weights"] = [1.0]  # base_config.py:47-51 divides by L-1
    return CompressionConfig(**kw)


class Writer:
    def __init__(self):
        os.makedirs(OUT, exist_ok=True)
        self.manifest = []
        self.mismatches = []

    def put(self, name: str, kind: str, spec: dict, arrays: dict, scalars: dict):
        store, hashes = {}, {}
        for k, v in arrays.items():
            v = np.ascontiguousarray(v)
            hashes[k] = sha(v)
            if v.nbytes <= SMALL:
                store[k] = v
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **store)
        self.manifest.append(dict(name=name, kind=kind, spec=spec, sha256=hashes, scalars=scalars,
                                  shapes={k: list(np.shape(v)) for k, v in arrays.items()},
                                  dtypes={k: str(np.asarray(v).dtype) for k, v in arrays.items()}))

    def check(self, name: str, what: str, ok: bool, allowed: bool = False):
        if not ok:
            (print if allowed else print)(f"  [{'tie' if allowed else 'MISMATCH'}] {name}: {what}")
            if not allowed:
                self.mismatches.append(f"{name}: {what}")

    def finish(self, merge: bool = False):
        if merge:  # keep every other case, replace the regenerated ones in place
            with open(os.path.join(OUT, "manifest.json")) as f:
                old = json.load(f)["cases"]
            new = {c["name"]: c for c in self.manifest}
            merged = [new.pop(c["name"], c) for c in old]
            self.manifest = merged + list(new.values())
        with open(os.path.join(OUT, "manifest.json"), "w") as f:
            json.dump(dict(torch=torch.__version__, capability=torch.backends.cpu.get_cpu_capability(),
                           threads=torch.get_num_threads(), cases=self.manifest), f, indent=1)
        print(f"{len(self.manifest)} fixtures, {len(self.mismatches)} oracle mismatches")
        for m in self.mismatches:
            print("   ", m)


# ----------------------------------------------------------------------------- stage cases
def gen_position_bias(w: Writer):
    sc = PromptGuidedImportanceScorer(make_config(COVERAGE, 4))
    for S in [1, 2, 3, 10, 16, 17, 512, 4096, 16384, 73230, 110000]:
        ref = sc.compute_position_bias(S, torch.device("cpu")).numpy()
        mine = orc.position_bias(S)
        w.check(f"pos{S}", "position bias", np.array_equal(ref, mine))
        w.put(f"pos_{S}", "position_bias", dict(S=S), dict(pos=ref), {})


def gen_aggregation(w: Writer):
    cases = [  # (B, H, S, P, full?)  reference test shapes first
        (1, 8, 10, 3, True), (2, 8, 16, 4, True), (1, 8, 2, 1, True), (1, 4, 512, 102, False),
        (1, 32, 2048, 128, False), (1, 40, 256, 128, False), (2, 5, 37, 7, False), (1, 3, 1, 1, True),
    ]
    seed = 100
    for (B, H, S, P, full) in cases:
        for dt in ["float32", "float16", "bfloat16"]:
            seed += 1
            W = synth.attention_full(seed, B, H, S, dt) if full else synth.attention_slice(seed, B, H, S, P, dt)
            cfg = make_config(COVERAGE, 4)
            sc = PromptGuidedImportanceScorer(cfg)
            Wt = t_of(W, dt)
            idx = torch.arange(P)
            A = sc.compute_attention_aggregation(Wt, idx, 0)
            refA = A.float().numpy()
            mineA = orc.attention_aggregation(W, synth.DTYPES[dt], P)
            name = f"agg_B{B}H{H}S{S}P{P}{'full' if full else ''}_{dt}"
            w.check(name, "aggregation", np.array_equal(refA, mineA))
            out = {"A": refA}
            scal = {}
            for layer in [0, 3]:
                s = sc.compute_importance_scores(Wt, idx, layer).float().numpy()
                ms = orc.importance_scores(mineA, synth.DTYPES[dt], P, cfg.alpha, cfg.beta, cfg.gamma,
                                           cfg.layer_weights[layer])
                w.check(name, f"scores layer {layer}", np.array_equal(s, ms))
                out[f"scores_l{layer}"] = s
            N = sc.normalize_attention_scores(A, 0).float().numpy()
            w.check(name, "normalize", np.array_equal(N, orc.minmax_normalize(mineA, synth.DTYPES[dt])))
            out["N"] = N
            w.put(name, "aggregation", dict(seed=seed, B=B, H=H, S=S, P=P, full=full, dtype=dt,
                                            params="coverage", L=4, layers=[0, 3]), out, scal)


def gen_normalize_edge(w: Writer):
    sc = PromptGuidedImportanceScorer(make_config(COVERAGE, 4))
    for dt in ["float32", "float16", "bfloat16"]:
        A = np.stack([np.full(9, 0.37), synth.uniform(7, (9,)), np.linspace(0, 1e-9, 9)])
        stored = synth.cast(A, dt)
        N = sc.normalize_attention_scores(t_of(stored, dt), 0).float().numpy()
        mine = orc.minmax_normalize(synth.to_f32(stored, dt), synth.DTYPES[dt])
        w.check(f"norm_edge_{dt}", "normalize edge", np.array_equal(N, mine))
        w.put(f"norm_edge_{dt}", "normalize", dict(dtype=dt), dict(A=stored, N=N), {})


def gen_quant(w: Writer):
    seed = 300
    for dt in ["float32", "float16", "bfloat16"]:
        for params, bits in [(COVERAGE, (2, 4, 8)), (DEFAULT, (4, 8, 16))]:
            if dt == "float16" and bits[2] == 16:
                continue
            for (B, S, F) in [(2, 12, 64), (1, 33, 200), (1, 16, 4096)]:
                seed += 1
                cfg = make_config(params, 4)
                q = DynamicPrecisionQuantizer(cfg)
                K, V = synth.kv(seed, B, S, F, dt)
                # one constant row to exercise max == min (dynamic_quantization.py:83-86)
                Kf = synth.to_f32(K, dt)
                Kf[0, 1, :] = Kf[0, 1, 0]
                K = synth.cast(Kf.astype(np.float64), dt)
                scores = synth.scores_like(seed, B, S)
                labels_t, stats = q.assign_precision_levels(torch.from_numpy(scores))
                labels = labels_t.numpy().astype(np.uint8)
                ml, mc = orc.assign_precision(scores, cfg.theta_h, cfg.theta_m)
                name = f"quant_B{B}S{S}F{F}_b{''.join(map(str, bits))}_{dt}"
                w.check(name, "labels", np.array_equal(ml, labels))
                kq, vq, info = q.apply_mixed_precision_quantization(t_of(K, dt), t_of(V, dt), labels_t)
                kq, vq = np_of(kq), np_of(vq)
                w.check(name, "K fake-quant", np.array_equal(kq, orc.mixed_precision(K, synth.DTYPES[dt], labels, bits)))
                w.check(name, "V fake-quant", np.array_equal(vq, orc.mixed_precision(V, synth.DTYPES[dt], labels, bits)))
                w.put(name, "quant", dict(seed=seed, B=B, S=S, F=F, dtype=dt, bits=list(bits),
                                          theta=[cfg.theta_h, cfg.theta_m], const_row=[0, 1]),
                      dict(K=K, labels=labels, k_q=kq, v_q=vq),
                      dict(high=stats["high_count"], medium=stats["medium_count"], low=stats["low_count"]))
    # fp16 with 16-bit HIGH raises in the reference
    cfg = make_config(DEFAULT, 4)
    q = DynamicPrecisionQuantizer(cfg)
    K, V = synth.kv(999, 1, 4, 64, "float16")
    labels = torch.tensor([[2, 1, 0, 2]])
    try:
        q.apply_mixed_precision_quantization(t_of(K, "float16"), t_of(V, "float16"), labels)
        err = ""
    except RuntimeError as e:
        err = str(e)
    w.put("quant_f16_b16_error", "quant_error", dict(seed=999, B=1, S=4, F=64, dtype="float16",
                                                     bits=[4, 8, 16], labels=[[2, 1, 0, 2]]), {}, dict(error=err))


def gen_select(w: Writer):
    seed = 500
    cases = [(1, 10, 4, 0), (2, 64, 32, 5), (1, 4096, 32, 10), (1, 4096, 32, 25), (3, 333, 8, 1),
             (1, 16384, 32, 0), (1, 16384, 32, 31)]
    for (B, S, L, layer) in cases:
        for params, bits in [(COVERAGE, (2, 4, 8)), (DEFAULT, (4, 8, 16))]:
            seed += 1
            cfg = make_config(params, L)
            prop = SelectiveTokenPropagator(cfg)
            qz = DynamicPrecisionQuantizer(cfg)
            scores = synth.scores_like(seed, B, S)
            labels_t, _ = qz.assign_precision_levels(torch.from_numpy(scores))
            ratio = prop.get_layer_propagation_ratio(layer)
            mask_t, info = prop.select_tokens_with_budget(torch.from_numpy(scores), labels_t, ratio, layer)
            mask = mask_t.numpy().astype(np.uint8)
            labels = labels_t.numpy().astype(np.uint8)
            om, kept, units, fb = orc.select(scores, labels, bits, ratio)
            name = f"select_B{B}S{S}L{L}l{layer}_b{''.join(map(str, bits))}"
            tie = not np.array_equal(om, mask)
            w.check(name, "selection (tie order)", not tie, allowed=True)
            w.put(name, "select", dict(seed=seed, B=B, S=S, L=L, layer=layer, bits=list(bits),
                                       theta=[cfg.theta_h, cfg.theta_m], ratio=ratio, tie_ambiguous=tie),
                  dict(mask=mask, labels=labels), dict(selected_counts=info["selected_counts"]))
    # fallback: budget below the cheapest token → top-10% (selective_propagation.py:205-211)
    for (B, S) in [(1, 10), (2, 50)]:
        seed += 1
        cfg = make_config(dict(COVERAGE, early_layer_ratio=0.01, middle_layer_ratio=0.01,
                               later_layer_ratio=0.01), 4)
        prop = SelectiveTokenPropagator(cfg)
        qz = DynamicPrecisionQuantizer(cfg)
        scores = synth.scores_like(seed, B, S)
        labels_t, _ = qz.assign_precision_levels(torch.from_numpy(scores))
        K, V = synth.kv(seed, B, S, 16, "float32")
        ks, vs, ss, ls, pinfo = prop.apply_token_selection(t_of(K, "float32"), t_of(V, "float32"),
                                                           torch.from_numpy(scores), labels_t, 0)
        mask = pinfo["selection_mask"].numpy().astype(np.uint8)
        om, kept, units, fb = orc.select(scores, labels_t.numpy().astype(np.uint8), (2, 4, 8), 0.01)
        name = f"select_fallback_B{B}S{S}"
        w.check(name, "fallback mask", np.array_equal(om, mask), allowed=True)
        w.put(name, "select", dict(seed=seed, B=B, S=S, L=4, layer=0, bits=[2, 4, 8],
                                   theta=[cfg.theta_h, cfg.theta_m], ratio=0.01,
                                   tie_ambiguous=not np.array_equal(om, mask), fallback=True),
              dict(mask=mask, labels=labels_t.numpy().astype(np.uint8), k_sel=ks.numpy()),
              dict(max_selected=int(pinfo["max_selected_length"])))


# ----------------------------------------------------------------------------- full layer
LAYER_CASES = [
    # name, params, L, layer, B, H(attn), Hkv, D, S, kv dtype
    ("cfg1", COVERAGE, 1, 0, 1, 4, 4, 64, 512, "float32"),
    ("cfg1", COVERAGE, 1, 0, 1, 4, 4, 64, 512, "float16"),
    ("cfg1", COVERAGE, 1, 0, 1, 4, 4, 64, 512, "bfloat16"),
    ("pub_l0", PUBLISHED, 32, 0, 1, 8, 8, 32, 1024, "float32"),
    ("pub_l15", PUBLISHED, 32, 15, 1, 8, 8, 32, 1024, "float16"),
    ("pub_l31", PUBLISHED, 32, 31, 1, 8, 8, 32, 1024, "float32"),
    ("default", DEFAULT, 32, 5, 1, 4, 4, 64, 256, "float32"),
    ("gqa_b2", COVERAGE, 8, 6, 2, 8, 2, 64, 200, "float32"),
    ("small_s10", COVERAGE, 4, 0, 1, 8, 2, 32, 10, "float32"),
    ("small_s2", COVERAGE, 4, 3, 1, 8, 2, 32, 2, "float16"),
    ("cfg3_l0", COVERAGE, 32, 0, 1, 32, 32, 128, 16384, "float16"),
    ("cfg3_l20", PUBLISHED, 32, 20, 1, 32, 32, 128, 16384, "float16"),
    ("cfg2_quant", COVERAGE, 32, 0, 1, 32, 32, 128, 4096, "float16"),
    ("cfg5_13b_l39", COVERAGE, 40, 39, 1, 40, 40, 128, 8192, "bfloat16"),    # Llama-2-13B rows (F = 5120)
    ("cfg5_13b_l20", PUBLISHED, 40, 20, 1, 40, 40, 128, 4096, "float16"),
    # round 2: BASELINE cfg5 at its real size (Llama-2-13B, F = 5120, global selection over S = 32768)
    # and cfg3 in the reference model's own dtype (fp32, modified_llama.py:368)
    ("cfg5_13b_s32768_l39", COVERAGE, 40, 39, 1, 40, 40, 128, 32768, "float16"),
    ("cfg5_13b_s32768_l0", PUBLISHED, 40, 0, 1, 40, 40, 128, 32768, "bfloat16"),
    ("cfg5_13b_s32768_l20", COVERAGE, 40, 20, 1, 40, 40, 128, 32768, "float32"),
    ("cfg3_l0", COVERAGE, 32, 0, 1, 32, 32, 128, 16384, "float32"),
    ("cfg3_l25", PUBLISHED, 32, 25, 1, 32, 32, 128, 16384, "float32"),
    # round 4: BASELINE cfg4's whole sequence (Llama-2-7B, S = 65536: the single-GPU pipeline selection
    # and the 8-way shard union are compared with these), early (.8) and late (.4) ratio groups
    ("cfg4_s65536_l0", COVERAGE, 32, 0, 1, 32, 32, 128, 65536, "float32"),
    ("cfg4_s65536_l31", COVERAGE, 32, 31, 1, 32, 32, 128, 65536, "float32"),
    ("cfg4_s65536_l0", PUBLISHED, 32, 0, 1, 32, 32, 128, 65536, "float16"),
    ("cfg4_s65536_l31", PUBLISHED, 32, 31, 1, 32, 32, 128, 65536, "float16"),
    # round 5: the default / second published widths 16/8/4 at full size (16-bit packing at F = 4096, the
    # {0.5, 1, 2} cost units of selective_propagation.py:54-66, K2 quotas in 16-bit units); bf16 cannot
    # hold 2^16-1, so its HIGH rows take 17-bit fields (rtkv_field_width)
    ("cfg3_b16_l0", PUB16, 32, 0, 1, 32, 32, 128, 16384, "float32"),
    ("cfg3_b16_l25", PUB16, 32, 25, 1, 32, 32, 128, 16384, "float32"),
    ("cfg3_b16_l12", PUB16, 32, 12, 1, 32, 32, 128, 16384, "bfloat16"),
    ("cfg4_s65536_b16_l20", PUB16, 32, 20, 1, 32, 32, 128, 65536, "float32"),
    # round 6: BASELINE cfg2 (7B, S = 4096, quantization only) in the reference model's fp32, the launch the
    # bench's cfg2_s4096_quant leg times (rtkv_compress_layer with RTKV_NO_SELECTION)
    ("cfg2_quant", COVERAGE, 32, 0, 1, 32, 32, 128, 4096, "float32"),
]


def gen_layers(w: Writer):
    seed = 700
    for (tag, params, L, layer, B, H, Hkv, D, S, dt) in LAYER_CASES:
        seed += 1
        if not wanted(f"layer_{tag}_{dt}"):
            continue
        t0 = time.time()
        F = Hkv * D
        P = max(1, min(S // 5, 128))
        cfg = make_config(params, L)
        no_sel = tag.startswith("cfg2")
        if no_sel:  # quant-only (BASELINE config 2): the reference's quantizer alone
            cfg.early_layer_ratio = cfg.middle_layer_ratio = cfg.later_layer_ratio = 1.0
        comp = RealTimePrefillCompressor(cfg)
        K, V = synth.kv(seed, B, S, F, dt)
        W = synth.attention_slice(seed, B, H, S, P, dt)
        ids = torch.zeros((B, S), dtype=torch.long)
        Kt, Vt, Wt = t_of(K, dt), t_of(V, dt), t_of(W, dt)
        bits = (cfg.low_precision_bits, cfg.medium_precision_bits, cfg.high_precision_bits)
        if no_sel:
            scores_t = comp.importance_tracker.update_scores(layer, Wt, comp.identify_prompt_tokens(ids))
            labels_t, pstats = comp.quantizer.assign_precision_levels(scores_t)
            kq, vq, qinfo = comp.quantizer.apply_mixed_precision_quantization(Kt, Vt, labels_t)
            scores = scores_t.numpy()
            labels = labels_t.numpy().astype(np.uint8)
            mask = np.ones((B, S), np.uint8)
            k2, v2 = np_of(kq), np_of(vq)
            scal = dict(max_selected=S, high=pstats["high_count"], medium=pstats["medium_count"],
                        low=pstats["low_count"])
        else:
            kt2, vt2, info = comp.compress_layer_kv_cache(Kt, Vt, Wt, ids, layer)
            scores = comp.importance_tracker.layer_scores[layer].numpy()
            labels = info["quantization_info"]["bit_assignments"].astype(np.uint8)
            mask = info["propagation_info"]["selection_mask"].numpy().astype(np.uint8)
            k2, v2 = np_of(kt2), np_of(vt2)
            ps = info["precision_stats"]
            ist = info["importance_stats"]
            scal = dict(max_selected=int(info["propagation_info"]["max_selected_length"]),
                        high=ps["high_count"], medium=ps["medium_count"], low=ps["low_count"],
                        compression_ratio=info["compression_ratio"], mean_score=ist["mean_score"],
                        std_score=ist["std_score"], min_score=ist["min_score"], max_score=ist["max_score"],
                        ratio=info["propagation_info"]["propagation_ratio"])
        name = f"layer_{tag}_{dt}"
        o = orc.compress_layer(K, V, synth.DTYPES[dt], W, synth.DTYPES[dt], P, cfg.alpha, cfg.beta,
                               cfg.gamma, cfg.layer_weights[layer], cfg.theta_h, cfg.theta_m, bits,
                               comp.propagator.get_layer_propagation_ratio(layer), no_selection=no_sel)
        w.check(name, "scores", np.array_equal(o["scores"], scores))
        w.check(name, "labels", np.array_equal(o["labels"], labels))
        tie = not np.array_equal(o["mask"], mask)
        w.check(name, "mask (tie order)", not tie, allowed=True)
        if not tie:
            w.check(name, "K'", np.array_equal(o["k_out"], k2))
            w.check(name, "V'", np.array_equal(o["v_out"], v2))
        w.put(name, "layer", dict(seed=seed, tag=tag, params={k: v for k, v in cfg.__dict__.items()
                                                             if k in ("alpha", "beta", "gamma", "theta_h", "theta_m")},
                                  L=L, layer=layer, B=B, H=H, Hkv=Hkv, D=D, S=S, P=P, dtype=dt,
                                  bits=list(bits), layer_weight=cfg.layer_weights[layer],
                                  ratio=comp.propagator.get_layer_propagation_ratio(layer),
                                  no_selection=no_sel, tie_ambiguous=tie),
              dict(scores=scores, labels=labels, mask=mask, k_out=k2, v_out=v2), scal)
        print(f"  {name}: {time.time() - t0:.1f}s  S'={scal['max_selected']}  tie={tie}")


# ----------------------------------------------------------------------------- multi-layer state
# A sequence of layers through one compressor, then the aggregate API the reference's experiment
# scripts and LongBench "TTFT" read: get_overall_compression_stats (unified_compressor.py:174-230),
# get_cumulative_scores (token_importance.py:202-214) and reset_compression_state (:232-235).
STATS_CASES = [
    # name, params, L, processed layers (in call order), B, H, Hkv, D, S, dtype
    ("stats_seq8", PUBLISHED, 8, list(range(8)), 2, 8, 4, 32, 1024, "float32"),
    ("stats_sparse", COVERAGE, 12, [5, 0, 9, 2], 1, 4, 4, 64, 640, "float16"),
]
TIMING_KEYS = ("total_processing_time", "avg_processing_time_per_layer")


def gen_stats(w: Writer):
    seed = 900
    for (name, params, L, layers, B, H, Hkv, D, S, dt) in STATS_CASES:
        seed += 1
        if not wanted(name):
            continue
        cfg = make_config(params, L)
        comp = RealTimePrefillCompressor(cfg)
        F = Hkv * D
        P = max(1, min(S // 5, 128))
        ids = torch.zeros((B, S), dtype=torch.long)
        per_layer = []
        for k, layer in enumerate(layers):
            K, V = synth.kv(seed * 100 + k, B, S, F, dt)
            Wt = synth.attention_slice(seed * 100 + k, B, H, S, P, dt)
            _, _, info = comp.compress_layer_kv_cache(t_of(K, dt), t_of(V, dt), t_of(Wt, dt), ids, layer)
            per_layer.append(dict(layer=layer, compressed_len=int(info["compressed_shape"][1]),
                                  compression_ratio=info["compression_ratio"]))
        overall = comp.get_overall_compression_stats()
        for key in TIMING_KEYS:  # wall-clock sums: present, but not comparable across machines
            assert key in overall
            overall[key] = None
        arrays = {}
        queried = sorted(set(list(range(L)) + [L + 3]))
        cum_none = []
        for l in queried:
            try:
                c = comp.importance_tracker.get_cumulative_scores(l)
            except KeyError:  # zeros_like(layer_scores[0]) when layer 0 was never processed
                c = "KeyError"
            if c is None or isinstance(c, str):
                cum_none.append([l, c if isinstance(c, str) else None])
            else:
                arrays[f"cum_l{l}"] = c.numpy()
        comp.reset_compression_state()
        after = dict(overall=comp.get_overall_compression_stats(),
                     cumulative=comp.importance_tracker.get_cumulative_scores(0),
                     layer_states=len(comp.layer_states), layer_scores=len(comp.importance_tracker.layer_scores))
        after["cumulative"] = None if after["cumulative"] is None else "tensor"
        w.put(name, "stats", dict(seed=seed, params={k: v for k, v in cfg.__dict__.items()
                                                     if k in ("alpha", "beta", "gamma", "theta_h", "theta_m")},
                                  L=L, layers=layers, B=B, H=H, Hkv=Hkv, D=D, S=S, P=P, dtype=dt,
                                  bits=[cfg.low_precision_bits, cfg.medium_precision_bits, cfg.high_precision_bits],
                                  queried=queried),
              arrays, dict(overall=overall, per_layer=per_layer, cumulative_special=cum_none, after_reset=after))
        print(f"  {name}: {len(layers)} layers, overall {overall}")


ONLY = None  # fixture-name substrings (--only): regenerate just those and merge into the manifest


def wanted(name: str) -> bool:
    return ONLY is None or any(o in name for o in ONLY)


def main():
    global ONLY
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", help="regenerate only fixtures whose name contains one of these; "
                                               "other manifest entries are kept")
    args = ap.parse_args()
    ONLY = args.only
    print("torch", torch.__version__, torch.backends.cpu.get_cpu_capability(), "threads", torch.get_num_threads())
    assert torch.backends.cpu.get_cpu_capability() == "AVX2", "run with ATEN_CPU_CAPABILITY=avx2"
    orc.build()
    w = Writer()
    fns = [gen_position_bias, gen_aggregation, gen_normalize_edge, gen_quant, gen_select, gen_layers, gen_stats]
    if ONLY is not None:
        fns = [gen_layers, gen_stats]
    for fn in fns:
        t0 = time.time()
        fn(w)
        print(f"{fn.__name__}: {time.time() - t0:.1f}s")
    w.finish(merge=ONLY is not None)
    return 1 if w.mismatches else 0


if __name__ == "__main__":
    sys.exit(main())
