#!/usr/bin/env python3
"""Instruction histogram and s_waitcnt list of one kernel in a hipcc -S device .s file.
usage: asm_hist.py file.s <substring of the mangled name> [out.s]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = [x for x in re.finditer(r"^(_Z\S+):", s, re.M) if sys.argv[2] in x.group(1)][0]
i = m.end()
j = s.index(".Lfunc_end", i)
body = s[i:j]
lines = [l.strip() for l in body.split("\n")]
c = collections.Counter()
for l in lines:
    if not l or l.startswith((".", ";")) or l.endswith(":"):
        continue
    c[l.split()[0]] += 1
for k, v in c.most_common(80):
    print(v, k)
print(sum(c.values()), "total")
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(body)
