#!/usr/bin/env python3
"""Instruction mix of selected kernels in a hipcc --cuda-device-only -S listing.
usage: isa_mix.py <file.s> <substring> [<substring> ...]"""
import collections
import re
import sys

txt = open(sys.argv[1]).read()
for key in sys.argv[2:]:
    m = re.search(r"\n(_Z\w*%s\w*):[^\n]*\n(.*?)\n\.Lfunc_end" % re.escape(key), txt, re.S)
    if not m:
        print("not found", key)
        continue
    name, body = m.group(1), m.group(2)
    ins = [l.split()[0] for l in body.split("\n")
           if l.startswith("\t") and l.strip() and not l.lstrip().startswith((".", ";"))]
    c = collections.Counter(ins)
    cat = collections.Counter()
    for k, v in c.items():
        if k.startswith("v_pk_"): cat["valu_pk"] += v
        elif k.startswith(("v_fma", "v_fmac", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32")): cat["valu_f32"] += v
        elif k.startswith("v_mov") or k.startswith("v_cndmask"): cat["valu_mov"] += v
        elif k.startswith("v_"): cat["valu_other"] += v
        elif k.startswith("ds_"): cat["lds"] += v
        elif k.startswith(("global_", "buffer_", "flat_", "scratch_")): cat["vmem"] += v
        elif k.startswith("s_"): cat["salu/ctl"] += v
    vg = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", txt)
    sp = re.search(re.escape(name) + r"\.private_seg_size, (\d+)", txt)
    print(name[:70], "instrs", len(ins), "vgpr", vg and vg.group(1), "scratch", sp and sp.group(1))
    print("  ", dict(cat))
    print("  ", sorted(c.items(), key=lambda x: -x[1])[:40])
