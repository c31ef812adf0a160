"""Compare the draw records of the single-wave generator (SPGG_GEN1=1) with the multi-wave one
(=0), iteration by iteration, for the chained Double-Q case of test_mt_chained_generator_vs_oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch
    from spgg_amd.engine import BatchEngine, ReplicaParams
    os.environ["SPGG_MT_CHAINS"] = "4"
    os.environ["SPGG_MT_PER_CHAIN"] = "4"
    alg = sys.argv[1] if len(sys.argv) > 1 else "double_qlearning"

    def P(**kw):
        base = dict(c=1, cost=1, alpha=0.8, gamma=0.9, epsilon=0.5, epsilon_decay=0.99, epsilon_min=0.01,
                    lambda_epsilon=0.01, delta_R_D=1, R_min=-10, R_max=10, rep_gain_C=1.0,
                    reward_weight_payoff=0.95, influence_factor=1.0, r=3.0)
        base.update(kw)
        return ReplicaParams(**base)
    reps = [P(r=0.5, epsilon=0.05, epsilon_decay=0.5, epsilon_min=0.0, seed=1),
            P(r=1.0, epsilon=0.1, epsilon_decay=0.5, epsilon_min=0.0, seed=1),
            P(r=3.0, influence_factor=0.0, seed=5), P(r=4.2, influence_factor=1.5, seed=6)]
    L, T = 40, 120
    recs = {}
    for mode in ("1", "0"):
        import importlib
        # the knob is read once per process in launch_gen: run each mode in a child
    mode = os.environ.get("SPGG_GEN1", "1")
    eng = BatchEngine(L, T, reps, use_second_order=False, rng="mt19937", algorithm=alg, streams=1)
    out = []
    for t in range(1, T + 1):
        eng.step(1)
        torch.cuda.synchronize()
        out.append(eng.draws[(t - 1) % eng.draw_slots].cpu().numpy().copy())
    eng.flush()
    torch.cuda.synchronize()
    keys = [eng.mt_state_host(k) for k in range(len(reps))]
    np.savez(f"/tmp/gen{mode}_{alg}.npz", recs=np.stack(out), keys=np.stack([k[0] for k in keys]),
             pos=np.array([k[1] for k in keys]), stop=eng.stop_iter.cpu().numpy())
    print("mode", mode, "stops", eng.stop_iter.cpu().numpy())


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "compare":
        import numpy as np
        a, b = np.load(f"/tmp/gen1_{sys.argv[1]}.npz"), np.load(f"/tmp/gen0_{sys.argv[1]}.npz")
        print("stops", a["stop"], b["stop"], "keys equal", np.array_equal(a["keys"], b["keys"]), a["pos"], b["pos"])
        ra, rb = a["recs"], b["recs"]
        for t in range(ra.shape[0]):
            d = np.argwhere(ra[t] != rb[t])
            if len(d):
                print("t", t + 1, "mismatching (rep, word):", d[:8].tolist(), "count", len(d))
                w = d[0]
                print("   gen1 %08x gen0 %08x" % (int(ra[t][tuple(w)]) & 0xffffffff, int(rb[t][tuple(w)]) & 0xffffffff))
                break
        else:
            print("records identical")
    else:
        main()
