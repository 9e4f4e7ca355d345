#!/usr/bin/env python3
"""Per-kernel ISA statistics (loads, stores, VALU, scratch, VGPRs) of a hipcc -S device .s file."""
import re
import sys

s = open(sys.argv[1]).read()
pats = sys.argv[2:]
starts = [(m.start(), m.group(1)) for m in re.finditer(r"^(_Z\S+):", s, flags=re.M)]
vg = {m.group(1): m.group(2) for m in re.finditer(r"\.name:\s+(_ZN3mgp\S+)\n(?:.*\n){0,40}?\s+\.vgpr_count:\s+(\d+)", s)}
for idx, (pos, n) in enumerate(starts):
    end = starts[idx + 1][0] if idx + 1 < len(starts) else len(s)
    if pats and not any(p in n for p in pats):
        continue
    f = s[pos:end]
    c = lambda p: len(re.findall(p, f))
    cnt = [c(r"global_load_dword\s"), c(r"global_load_dwordx2"), c(r"global_load_dwordx4"), c(r"global_store"),
           c(r"\n\s+v_"), c(r"scratch_")]
    print("%-44s ld1 %3d ld2 %3d ld4 %3d st %3d valu %5d scratch %3d vgpr %s" % tuple([n[20:64]] + cnt + [vg.get(n, "?")]))
