import sys, numpy as np, torch
sys.path.insert(0, '.')
import bench
from spgg_amd.engine import BatchEngine
desc, L, M2, state, reps = bench.workload("cfg3", 0)
eng = BatchEngine(L, 220, reps, use_second_order=M2, state_representation=state, rng="philox")
eng.step(220); torch.cuda.synchronize()
st = eng.stop_iter.cpu().numpy()
print("stopped:", int((st > 0).sum()), "of", len(st))
for k, p in enumerate(reps):
    if st[k]: print(f"  rep {k} r={p.r} kappa={p.influence_factor} stop_iter={st[k]}")
