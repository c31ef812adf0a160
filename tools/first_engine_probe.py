"""Why is the FIRST engine of a process slower in the bench's window than later ones?
(tools/queue_state_probe.py, profiles/r06/first_engine/: the first engine's window 6-25 ran
57.3 us/step, every later engine's 54.5-55.5.)  One fresh process per call; before the timed
engine (cfg3, Philox, 5 warm-up + 20 timed iterations, as bench.py) it does MODE:

  none     nothing (bench.py today)
  busy     ~300 ms of unrelated GPU work on torch's stream (clocks / power state up)
  engine   a throwaway engine of the same batch: made, one iteration, closed (streams, allocator,
           code objects, the library's host caches all warm)
  engine0  the throwaway engine made and closed, no iteration
  engine_keep  the throwaway engine kept alive (the timed engine gets fresh memory and streams)
  engine_tiny  a 1-replica L=16 throwaway engine (kernel and launch paths, not the batch's memory)
  alloc    only torch allocations of the engine's size, written once and freed (allocator / pages)
  streams  only the library's pooled streams, made and handed back (its hardware queues)

    python tools/first_engine_probe.py MODE"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from spgg_amd import engine as E
    mode = sys.argv[1]
    desc, L, M2, state, reps = bench.workload(os.environ.get("PROBE_CONFIG", "cfg3"), 0)
    W, K = 5, 20
    torch.cuda.init()
    if mode == "busy":
        a = torch.randn(4096, 4096, device="cuda")
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            for _ in range(20):
                a = a @ a
                a = a / a.norm()
            torch.cuda.synchronize()
        del a
    elif mode in ("engine", "engine0", "engine_keep", "engine_tiny"):
        r0 = reps[:1] if mode == "engine_tiny" else reps
        e0 = E.BatchEngine(16 if mode == "engine_tiny" else L, 2, r0, use_second_order=M2, state_representation=state,
                           rng="philox")
        if mode != "engine0":
            e0.step(1)
        torch.cuda.synchronize()
        if mode != "engine_keep":
            e0.close()
            del e0
    elif mode == "alloc":
        n = len(reps) * L * L
        bufs = [torch.ones(n * 64, dtype=torch.uint8, device="cuda") for _ in range(2)]
        torch.cuda.synchronize()
        del bufs
    elif mode == "streams":
        lib = E.C.load()
        hs = [E._take_stream(lib, 0) for _ in range(2)]
        E._give_streams(hs)
    torch.cuda.synchronize()
    eng = E.BatchEngine(L, K + W, reps, use_second_order=M2, state_representation=state, rng="philox")
    eng.step(W)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step(K, ordered=False)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / K * 1e6
    eng.close()
    print(f"{mode} {us:.2f}", flush=True)


if __name__ == "__main__":
    main()
