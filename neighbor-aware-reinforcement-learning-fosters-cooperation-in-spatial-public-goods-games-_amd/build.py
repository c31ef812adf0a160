"""Build libspgg_hip.so in-tree for gfx950 (explicit hipcc, no JIT cache).

    python -m <pkg>.build      or     __graft_entry__.build()
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
SRC = [os.path.join(PKG_DIR, "csrc", "spgg_kernels.hip")]
INC = os.path.join(ROOT, "include")
OUT = os.path.join(PKG_DIR, "libspgg_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         # bit-exact f64: no FMA contraction of the reference's a*b+c
         "-ffp-contract=off",
         # f64 global atomics as hardware global_atomic_add_f64 (no CAS loop)
         "-munsafe-fp-atomics"]


def needs_build(out=OUT):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = SRC + [os.path.join(INC, "spgg_abi.h"), os.path.join(PKG_DIR, "csrc", "spgg_device.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC, *FLAGS, f"-I{INC}", "-o", OUT, *SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
