"""Static VALU/SALU/LDS/VMEM instruction counts of one kernel attributed to source
lines (.loc directives of a -gline-tables-only hipcc -S output), weighted by an
issue-cost estimate (f64 / quarter-rate ops heavier).

    python tools/isa_lines.py file.s <kernel-symbol> [top]
"""
import collections
import re
import sys

s = open(sys.argv[1]).read().split("\n")
key = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
files = {}
start = next(i for i, l in enumerate(s) if l.startswith(key + ":"))
cur = None
cnt = collections.Counter()
wt = collections.Counter()
kinds = collections.defaultdict(collections.Counter)
HEAVY = {"v_mad_u64_u32": 8, "v_mul_lo_u32": 8, "v_mul_hi_u32": 8, "v_rcp_f64": 8}
for l in s:
    if l.startswith("\t.file"):
        m = re.match(r'\t\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
for l in s[start:]:
    if l.startswith(".Lfunc_end"):
        break
    if l.startswith("\t.loc"):
        p = l.split()
        cur = (files.get(p[1], p[1]), int(p[2]))
        continue
    if not l.startswith("\t") or l.strip().startswith((".", ";")) or not l.strip():
        continue
    op = l.strip().split()[0]
    if op.startswith("v_"):
        w = HEAVY.get(op, 4 if "f64" in op else 2)
        cnt[cur] += 1
        wt[cur] += w
        kinds[cur][op] += 1
tot = sum(wt.values())
print(f"VALU static instrs {sum(cnt.values())}, weighted cycles {tot}")
for k, v in wt.most_common(top):
    print(f"{v:6d} {100*v/tot:5.1f}%  n={cnt[k]:4d}  {k[0]}:{k[1]}  {dict(kinds[k].most_common(3))}")
