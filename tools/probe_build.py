"""Probe builds for A/B timing: the step TUs (0-3) compiled once into a cache, TU 9 (C ABI +
generator) and the MT19937 jump object per variant, linked into build_probe/<name>.so.

    python tools/probe_build.py NAME [DEFINE ...]     (e.g. o1nb8 SPGG_GEN_OUT=1 SPGG_GEN_NB=8)
    python tools/probe_build.py --all-tus NAME DEFINE...   (every TU with the defines)"""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import spgg_amd.build as B  # noqa: E402

CACHE = "/tmp/spgg_probe_objs"


def obj(tu, defines, src=B.SRC[0]):
    key = hashlib.sha1(open(src, "rb").read() + repr((tu, sorted(defines))).encode()).hexdigest()[:12]
    for d in B.DEPS:
        key = hashlib.sha1((key + open(d, "rb").read().hex()[:0] + str(os.path.getmtime(d))).encode()).hexdigest()[:12]
    out = os.path.join(CACHE, f"tu{tu}_{key}.o")
    if not os.path.exists(out):
        cmd = [B.HIPCC, *B.FLAGS, *[f"-D{d}" for d in defines], '-DSPGG_BUILD_ID="probe000000000000"', f"-I{B.INC}", "-c", src, "-o", out]
        if tu is not None:
            cmd.insert(-4, f"-DSPGG_TU={tu}")
        subprocess.run(cmd, check=True, capture_output=True)
    return out


def main():
    args = sys.argv[1:]
    all_tus = args[0] == "--all-tus"
    if all_tus:
        args = args[1:]
    name, defines = args[0], args[1:]
    os.makedirs(CACHE, exist_ok=True)
    os.makedirs(os.path.join(ROOT, "build_probe"), exist_ok=True)
    jobs = [(tu, defines if (all_tus or tu == 9) else [], B.SRC[0]) for tu in B.TUS] + [(None, defines, B.SRC[1])]
    with ThreadPoolExecutor(6) as ex:
        objs = list(ex.map(lambda j: obj(*j), jobs))
    out = os.path.join(ROOT, "build_probe", f"{name}.so")
    subprocess.run([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs], check=True)
    print(out)


if __name__ == "__main__":
    main()
