"""VALU instructions of one kernel attributed to the OUTERMOST line of the kernel source
(the inlined-at chain of each .loc), from a -gline-tables-only hipcc -S output.
    python tools/isa_src.py file.s <kernel-symbol> <kernel-source.hip> [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read().split("\n")
k = sys.argv[2]
src = open(sys.argv[3]).read().split("\n")
top = int(sys.argv[4]) if len(sys.argv) > 4 else 50
base = sys.argv[3].split("/")[-1]
st = next(i for i, l in enumerate(s) if l.startswith(k + ":"))
en = next(i for i in range(st, len(s)) if s[i].startswith(".Lfunc_end"))
cnt, kinds, seg, segc = collections.Counter(), collections.defaultdict(collections.Counter), 0, collections.Counter()
cur = None
for l in s[st:en]:
    if l.startswith("\t.loc"):
        m = re.findall(re.escape(base) + r":(\d+)", l)
        cur = int(m[-1]) if m else None
        continue
    t = l.strip()
    if not l.startswith("\t") or t.startswith((".", ";")) or not t:
        continue
    op = t.split()[0]
    if op == "s_barrier":
        seg += 1
    if op.startswith("v_"):
        cnt[cur] += 1
        kinds[cur][op] += 1
        segc[seg] += 1
print("VALU per barrier segment", dict(segc), "total", sum(segc.values()))
for ln, c in cnt.most_common(top):
    txt = src[ln - 1].strip()[:58] if ln else "(no line)"
    print(f"{c:4d} L{ln}: {txt:58s} {dict(kinds[ln].most_common(3))}")
