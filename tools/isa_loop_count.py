#!/usr/bin/env python3
"""Instruction mix of the loops of one kernel in a gfx950 assembly listing (hipcc --cuda-device-only -S).

    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \\
        -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -I include \\
        -I realtime-kv-cache-compression_amd/csrc -fno-slp-vectorize --cuda-device-only -S \\
        realtime-kv-cache-compression_amd/csrc/decode_f16.hip -o /tmp/decode_f16.s
    python tools/isa_loop_count.py /tmp/decode_f16.s decode_split_kernelILi1ELi2ELi1ELi16E

For every backward branch (a loop) of the first kernel whose symbol contains the pattern: the number of
VALU, vector-memory, DPP, v_exp, v_fma_mix, dot2, packed-math, readlane and SALU instructions between
the loop head and the branch (inner loops are counted inside their outer loops too).  Used for the
decode kernel's VALU-issue bound ("Decode details")."""
import re
import sys

src, pat = sys.argv[1], sys.argv[2]
text = open(src).read()
m = re.search(r"^(_Z\S*" + re.escape(pat) + r"\S*):", text, re.M)
if not m:
    sys.exit(f"no kernel matching {pat}")
start = m.start()
end = text.index(".Lfunc_end", start)
body = text[start:end].split("\n")
labels = {}
for n, line in enumerate(body):
    lm = re.match(r"^(\.LBB\d+_\d+):", line)
    if lm:
        labels[lm.group(1)] = n
print(m.group(1))
kinds = [("valu", r"^\s+v_"), ("vmem", r"^\s+(buffer_|global_)"), ("dpp", r"row_|quad_perm"), ("exp", r"v_exp"),
         ("fma_mix", r"fma_mix"), ("dot2", r"dot2"), ("pk", r"^\s+v_pk_"), ("readlane", r"readlane"),
         ("salu", r"^\s+s_")]
for n, line in enumerate(body):
    bm = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", line)
    if not bm:
        continue
    target = bm.group(1) or bm.group(2)
    if target in labels and labels[target] < n:
        seg = body[labels[target]:n + 1]
        counts = {k: sum(1 for x in seg if re.search(p, x)) for k, p in kinds}
        print(f"loop {target} (lines {labels[target]}-{n}): " + " ".join(f"{k} {v}" for k, v in counts.items()))
