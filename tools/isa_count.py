"""VALU instruction counts of one kernel in a hipcc -S output (selected opcodes + total).
    python tools/isa_count.py file.s <kernel-symbol> [opcode ...]"""
import collections
import sys

s = open(sys.argv[1]).read().split("\n")
k = sys.argv[2]
st = next(i for i, l in enumerate(s) if l.startswith(k + ":"))
en = next(i for i in range(st, len(s)) if s[i].startswith(".Lfunc_end"))
c = collections.Counter(l.strip().split()[0] for l in s[st:en]
                        if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";")))
print("valu", sum(v for op, v in c.items() if op.startswith("v_")), " salu", sum(v for op, v in c.items() if op.startswith("s_")),
      " lds", sum(v for op, v in c.items() if op.startswith("ds_")))
for op in sys.argv[3:] or ("v_max_f64", "v_mov_b32_e32", "v_mov_b64_e32", "v_cndmask_b32_e32", "v_cndmask_b32_e64"):
    print(f"  {op} {c[op]}")
