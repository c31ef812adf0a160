"""Build libspgg_hip.so in-tree for gfx950 (explicit hipcc, no JIT cache).

    python -m <pkg>.build      or     __graft_entry__.build()
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
SRC = [os.path.join(PKG_DIR, "csrc", "spgg_kernels.hip"),
       os.path.join(PKG_DIR, "csrc", "spgg_mt.hip")]   # MT19937 jump-ahead (its own object)
INC = os.path.join(ROOT, "include")
OUT = os.path.join(PKG_DIR, "libspgg_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# One translation unit per RL operator (its step kernels) + one for the C ABI,
# compiled in parallel and linked into one shared library (spgg_kernels.hip's
# SPGG_TU switch).
TUS = (0, 1, 2, 3, 9)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         # bit-exact f64: no FMA contraction of the reference's a*b+c
         "-ffp-contract=off",
         # f64 global atomics as hardware global_atomic_add_f64 (no CAS loop)
         "-munsafe-fp-atomics"]


DEPS = SRC + [os.path.join(INC, "spgg_abi.h"), os.path.join(INC, "spgg_test.h"), os.path.join(PKG_DIR, "csrc", "spgg_device.h"),
              os.path.join(PKG_DIR, "csrc", "spgg_mt.h")]


def build_id(defines=()):
    """16 hex digits of SHA-256 over the sources, compiler, flags and defines: embedded in
    the library (spgg_build_id(), and as the string "spgg-build:<id>") so that freshness is
    decided by content, not by file times."""
    h = hashlib.sha256()
    for d in DEPS:
        with open(d, "rb") as f:
            h.update(f.read())
    h.update(" ".join([HIPCC, *FLAGS, *sorted(defines)]).encode())
    return h.hexdigest()[:16]


def library_build_id(path):
    """The build id a built library carries, or None."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(b"spgg-build:")
    return data[i + 11:i + 27].decode("ascii", "replace") if i >= 0 else None


def needs_build(out=OUT, defines=()):
    return library_build_id(out) != build_id(defines)


def build(force=False, verbose=True, out=OUT, defines=()):
    if not force and not needs_build(out, defines):
        return out
    extra = [f"-D{d}" for d in defines] + [f'-DSPGG_BUILD_ID="{build_id(defines)}"']
    with tempfile.TemporaryDirectory() as tmp:
        objs = [os.path.join(tmp, f"tu{k}.o") for k in TUS] + [os.path.join(tmp, "mt.o")]
        cmds = [[HIPCC, *FLAGS, *extra, f"-DSPGG_TU={k}", f"-I{INC}", "-c", SRC[0], "-o", o]
                for k, o in zip(TUS, objs)]
        cmds.append([HIPCC, *FLAGS, *extra, f"-I{INC}", "-c", SRC[1], "-o", objs[-1]])
        if verbose:
            print(" ".join(cmds[0]).replace("-DSPGG_TU=0", "-DSPGG_TU={0,1,2,3,9}"), flush=True)
        jobs = max(1, min(len(cmds), os.cpu_count() or 1, int(os.environ.get("MAX_JOBS", "8"))))
        with ThreadPoolExecutor(jobs) as ex:
            for r in ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds):
                if r.returncode:
                    sys.stderr.write(r.stdout + r.stderr)
                    raise subprocess.CalledProcessError(r.returncode, r.args)
        link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs]
        subprocess.run(link, check=True)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
