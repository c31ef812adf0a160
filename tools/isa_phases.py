"""Weighted VALU / SALU / LDS / VMEM instruction counts of one kernel per barrier-delimited
segment (the step kernel's phases are separated by s_barrier), from a hipcc -S output.

    python tools/isa_phases.py file.s <kernel-symbol>
Weights: f64 and 64-bit-multiply VALU ops 4 (quarter... full-DP rate: a wave64 op on a 16-lane
SIMD), other VALU 2 (32-lane rate), transcendental / mad_u64 8."""
import collections
import sys

s = open(sys.argv[1]).read().split("\n")
key = sys.argv[2]
st = next(i for i, l in enumerate(s) if l.startswith(key + ":"))
en = next(i for i in range(st, len(s)) if s[i].startswith(".Lfunc_end"))
HEAVY = {"v_mad_u64_u32": 8, "v_mul_lo_u32": 8, "v_mul_hi_u32": 8, "v_rcp_f64": 8, "v_rcp_f32_e32": 4}
seg = [collections.Counter()]
for l in s[st:en]:
    t = l.strip()
    if not l.startswith("\t") or t.startswith((".", ";")) or not t:
        continue
    op = t.split()[0]
    c = seg[-1]
    if op == "s_barrier":
        seg.append(collections.Counter())
        continue
    if op.startswith("v_"):
        c["valu"] += 1
        c["valu_cyc"] += HEAVY.get(op, 4 if ("f64" in op or "b64" in op or "u64" in op or "i64" in op) else 2)
        if "f64" in op:
            c["f64"] += 1
    elif op.startswith("s_"):
        c["salu"] += 1
        if op.startswith("s_waitcnt"):
            c["waitcnt"] += 1
    elif op.startswith("ds_"):
        c["lds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        c["vmem"] += 1
tot = sum(c["valu_cyc"] for c in seg)
print(f"segments {len(seg)}  weighted VALU cycles {tot}")
for i, c in enumerate(seg):
    print(f"seg {i}: valu {c['valu']:5d} cyc {c['valu_cyc']:5d} ({100*c['valu_cyc']/max(tot,1):4.1f}%)  f64 {c['f64']:4d}"
          f"  salu {c['salu']:4d} (waitcnt {c['waitcnt']:3d})  lds {c['lds']:4d}  vmem {c['vmem']:3d}")
