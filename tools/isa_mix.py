"""Static instruction mix of one kernel in a hipcc -S output: python tools/isa_mix.py file.s <substr>"""
import collections
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2] if len(sys.argv) > 2 else "spgg_step_kernelILb0ELb0ELi2ELi4E"
i = s.index(key)
start = s.index(":\n", s.index("\n" + s[s.rfind("\n", 0, i) + 1:i].split()[0] if False else key + ":" if (key + ":") in s else key))
end = s.index(".Lfunc_end", i)
body = s[i:end].split("\n")
ins = [l.strip().split()[0] for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = collections.Counter(ins)
print("total", len(ins), " valu", sum(v for k, v in c.items() if k.startswith("v_")),
      " salu", sum(v for k, v in c.items() if k.startswith("s_")),
      " lds", sum(v for k, v in c.items() if k.startswith("ds_")),
      " vmem", sum(v for k, v in c.items() if k.startswith(("global_", "buffer_", "flat_"))))
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 25):
    print(f"{v:6d} {k}")
