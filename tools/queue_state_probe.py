"""Does work on ANOTHER hardware queue shortly before the bench's window slow it?  (round 6,
profiles/r06/mt_generator/occupier_queue_test.txt: one 1-us kernel on a torch side stream slowed
the next ~15 ms of step launches by up to 20 %).  cfg3, Philox, the bench's window (iterations
6-25 of a fresh engine), one process, variants interleaved over rounds:

  base        engine made, 5 warm-up iterations, the timed 20 (what bench.py does)
  idle50      ... a 50 ms host sleep (GPU idle) between the warm-up and the timed window
  idle50_tiny ... the sleep, then one tiny kernel on torch's current stream, then the window
  idle50_tinyside ... the sleep, then one tiny kernel on a new torch side stream
  pre50       a 50 ms sleep after the engine is made, then the warm-up on the group streams only
              (unordered: no event on torch's stream), the window right after
  pre50_ord   a 50 ms sleep after the engine is made, then bench.py's ordered warm-up

    python tools/queue_state_probe.py [rounds]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from spgg_amd import engine as E
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cfg = os.environ.get("PROBE_CONFIG", "cfg3")
    desc, L, M2, state, reps = bench.workload(cfg, 0)
    W, K = 5, 20
    res = {}
    x = torch.zeros(1, device="cuda")
    for rnd in range(rounds):
        for name in ("base", "idle50", "idle50_tiny", "idle50_tinyside", "pre50", "pre50_ord"):
            eng = E.BatchEngine(L, K + W, reps, use_second_order=M2, state_representation=state, rng="philox")
            if name.startswith("pre50"):
                torch.cuda.synchronize()
                time.sleep(0.05)
            eng.step(W, ordered=name != "pre50")
            torch.cuda.synchronize()
            if name.startswith("idle50"):
                time.sleep(0.05)
            if name == "idle50_tiny":
                x.add_(1.0)
                torch.cuda.synchronize()
            if name == "idle50_tinyside":
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    x.add_(1.0)
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.step(K, ordered=False)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / K * 1e6
            eng.close()
            res.setdefault(name, []).append(us)
            print(f"{rnd} {name:16s} {us:7.2f} us/step", flush=True)
    for name, v in res.items():
        print(f"{name:16s} median {statistics.median(v):7.2f}  min {min(v):7.2f}  max {max(v):7.2f}  n={len(v)}")


if __name__ == "__main__":
    main()
