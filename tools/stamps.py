"""Phase timeline of one step launch from a -DSPGG_STAMPS=1 build (one stream).

    python tools/stamps.py build_probe/stamps.so [--config cfg3]

Stamps (s_memrealtime, 10 ns) per workgroup: 0 start, 1 loads staged, 2 phase 1a
done, 3 phase 1b done, 4 ring barrier passed, 5 phase 2 done, 6 reductions'
barrier passed, 7 end."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--t", type=int, default=30)
    ap.add_argument("--rng", default="philox", choices=["philox", "mt19937"])
    ap.add_argument("--streams", type=int, default=1, help="replica groups (the bench's: 0 = the planner's)")
    args = ap.parse_args()
    import torch
    import bench
    from spgg_amd.engine import BatchEngine
    desc, L, M2, state, reps = bench.workload(args.config, 0)
    lib = os.path.abspath(args.lib)
    eng = BatchEngine(L, args.t + 5, reps, use_second_order=M2, state_representation=state, rng=args.rng,
                      lib_path=lib, streams=args.streams or None)
    eng.step(args.t + 2)
    torch.cuda.synchronize()
    h = ctypes.CDLL(lib)
    n = 8192 * 12   # (kStampSlots: 0-7 phases, 8 HW_ID, 9 XCC_ID, 10-11 persistent barrier)
    buf = np.zeros(n, dtype=np.uint64)
    rc = h.spgg_stamps_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
    assert rc == 0, rc
    eng.close()
    nwg = len(reps) * eng.tiles_per_rep if hasattr(eng, "tiles_per_rep") else 4200
    s = buf.reshape(-1, 12)[:nwg].astype(np.int64)
    s = s[s[:, 0] > 0]
    t0 = s[:, 0].min()
    st = (s[:, :8] - t0) * 10 / 1000.0  # us
    print(f"workgroups stamped {len(s)} (iteration {args.t}, {eng.resident} stream(s)); span {st[:, 7].max():.1f} us")
    names = ["loads+staging", "PC+1a", "barrier+1b", "1c+barrier", "phase2", "red barrier", "totals+atomics"]
    d = np.diff(st, axis=1)
    print("phase            mean   p10   p50   p90  (us per workgroup)")
    for k, nm in enumerate(names):
        print(f"{nm:15s} {d[:, k].mean():6.2f} {np.percentile(d[:, k], 10):5.2f} {np.percentile(d[:, k], 50):5.2f} "
              f"{np.percentile(d[:, k], 90):5.2f}")
    if (s[:, 11] > 0).any():   # persistent launch: the replica barrier after iteration t
        b = (s[:, 10:12] - t0) * 10 / 1000.0
        drain, wait = b[:, 0] - st[:, 7], b[:, 1] - b[:, 0]
        for nm, x in (("bar: drain", drain), ("bar: wait", wait)):
            print(f"{nm:15s} {x.mean():6.2f} {np.percentile(x, 10):5.2f} {np.percentile(x, 50):5.2f} "
                  f"{np.percentile(x, 90):5.2f}")
        print(f"barrier passed: first {b[:, 1].min():.2f} last {b[:, 1].max():.2f} us; last arrival "
              f"{b[:, 0].max():.2f} us")
    life = st[:, 7] - st[:, 0]
    print(f"lifetime        {life.mean():6.2f} {np.percentile(life, 10):5.2f} {np.percentile(life, 50):5.2f} "
          f"{np.percentile(life, 90):5.2f}")
    # start-time histogram (generations)
    hist, edges = np.histogram(st[:, 0], bins=20)
    print("start-time histogram (us):", " ".join(f"{e:.0f}:{c}" for e, c in zip(edges[:-1], hist)))
    hw = s[:, 8]
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    sh = (hw >> 12) & 1
    xcc = s[:, 9] & 0xF
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    u, c = np.unique(key, return_counts=True)
    print(f"distinct CUs {len(u)}; WGs per CU min/median/max {c.min()}/{int(np.median(c))}/{c.max()}")
    # concurrency on the busiest CU over time
    k0 = u[np.argmax(c)]
    m = key == k0
    ev = sorted([(a, 1) for a in st[m, 0]] + [(b, -1) for b in st[m, 7]])
    cur = mx = 0
    for _, e in ev:
        cur += e
        mx = max(mx, cur)
    print(f"busiest CU: {c.max()} WGs, max concurrent {mx}")
    for i in np.where(m)[0][:20]:
        print("   " + " ".join(f"{x:6.1f}" for x in st[i]))


if __name__ == "__main__":
    main()
