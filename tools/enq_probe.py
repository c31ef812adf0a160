"""Window timing by host enqueue pattern: is a short window's step time the kernel's, or the
replica-group streams' start skew and drain?

    python tools/enq_probe.py [--config cfg3] [--rounds 3]

Each case makes a fresh engine, steps W untimed iterations, then times K iterations exactly as
bench.py does (HIP events on the current stream around eng.step(K), the group streams ordered
between them), with `enqueue_chunk` iterations enqueued per group and host call, or (interleave) every group
enqueued iteration by iteration by one spgg_step_groups call."""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--cases", default="5:20:8:0:0,5:20:1:0:0,5:20:8:0:1,400:20:8:0:0,400:20:8:0:1,400:200:8:0:1",
                    help="W:K:chunk[:streams (0 = the planner's)[:interleave (spgg_step_groups) 0/1]]")
    a = ap.parse_args()
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(a.config, 0)
    cases = [tuple(int(x) for x in c.split(":")) for c in a.cases.split(",")]
    res = {c: [] for c in cases}
    for r in range(a.rounds):
        for c in cases:
            W, K, chunk = c[:3]
            streams = (c[3] or None) if len(c) > 3 else None
            interleave = bool(c[4]) if len(c) > 4 else True
            eng = BatchEngine(L, W + K, reps, use_second_order=M2, state_representation=state, rng="philox",
                              streams=streams)
            eng.enqueue_chunk = chunk
            eng.interleave = interleave
            eng.step(W)
            torch.cuda.synchronize()
            cur = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(cur)
            eng.step(K)
            t_enq = time.perf_counter() - t0
            e1.record(cur)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            res[c].append(ms * 1e3 / K)
            print(f"round {r} W={W} K={K} chunk={chunk} streams={eng.resident} interleave={int(interleave)}: {ms * 1e3 / K:.2f} us/step "
                  f"(host enqueue {t_enq * 1e6:.0f} us)", flush=True)
            eng.close()
    print(desc)
    for c in cases:
        print(f"W={c[0]:4d} K={c[1]:4d} chunk={c[2]:3d} streams={c[3] if len(c) > 3 and c[3] else 'auto'} "
              f"interleave={c[4] if len(c) > 4 else 1}: median "
              f"{statistics.median(res[c]):.2f} us/step  all {[round(x, 2) for x in res[c]]}", flush=True)


if __name__ == "__main__":
    main()
