"""Cost of co-resident workgroups' RESOURCES vs their WORK on the cfg3 step kernels: occupier
workgroups (tools/occupier.hip: a chosen VGPR / LDS footprint, sleeping or spinning on VALU) run
on their own stream for the whole of a 100-iteration Philox window after 400 untimed iterations.

    python tools/occupier_probe.py        (needs build_probe/occupier.so)"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from spgg_amd import engine as E
    occ = ctypes.CDLL(os.path.join(ROOT, "build_probe", "occupier.so"))
    occ.occupier_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int]
    desc, L, M2, state, reps = bench.workload("cfg3", 0)
    K = 100
    base = [("wg420_slots", 420, 0, 0, 0), ("wg420_v56", 420, 0, 1, 0),
            ("wg420_lds18k", 420, 18436, 0, 0), ("wg420_v56_lds18k", 420, 18436, 1, 0),
            ("wg210_v56_lds18k", 210, 18436, 1, 0), ("wg420_valu", 420, 0, 0, 1), ("wg105_valu", 105, 0, 0, 1)]
    variants = []
    for v in base:  # "none" between every two variants: the drift of the chip's state
        variants += [("none", 0, 0, 0, 0), v]
    if os.environ.get("OCC_QUEUE_TEST"):  # windows with no occupier, before and after a 1-us occupier
        variants = [("none", 0, 0, 0, 0)] * 6 + [("tiny", 1, 0, 0, 0)] + [("none_after", 0, 0, 0, 0)] * 6
    eng = E.BatchEngine(L, 400 + K * (3 * len(variants) + 2), reps, use_second_order=M2, state_representation=state, rng="philox")
    eng.step(400)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    res = {}
    for rnd in range(1 if os.environ.get('OCC_QUEUE_TEST') else 3):
        for name, nwg, lds, v56, valu in variants:
            torch.cuda.synchronize()
            if nwg:
                rc = occ.occupier_launch(ctypes.c_void_p(side.cuda_stream), nwg, lds, v56, 1.0 if name == "tiny" else 12000.0, valu)
                assert rc == 0, rc
                time.sleep(0.0005)  # let its workgroups land first
            t0 = time.perf_counter()
            eng.step(K, ordered=False)
            s0 = time.perf_counter()
            # wait for the steps only (the occupier keeps running on its own stream)
            for s_ in eng.launch_streams():
                s_.synchronize()
            us = (time.perf_counter() - t0) / K * 1e6
            torch.cuda.synchronize()
            res.setdefault(name, []).append(us)
            print(f"{rnd} {name:20s} {us:7.2f} us/iter", flush=True)
    import statistics
    for name, v in res.items():
        print(f"{name:20s} median {statistics.median(v):7.2f}  min {min(v):7.2f} max {max(v):7.2f}  n={len(v)}")
    eng.close()


if __name__ == "__main__":
    main()
