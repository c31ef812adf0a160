"""Register / scratch budget of the built step kernels (CPU: reads the gfx950 code objects of
libspgg_hip.so, no GPU).

A step kernel that keeps a per-agent array in scratch memory runs ~2.6x slower (measured:
cfg3 178.6 vs 68.6 us/step when an InstCombine fold turned a select of two Q entries into a
load at a computed index, spgg_kernels.hip select_row), and one past 96 VGPRs loses the fifth
resident wave per SIMD.  Neither changes results, so the parity tests cannot see them."""
import os
import re
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "neighbor-aware-reinforcement-learning-fosters-cooperation-in-spatial-public-goods-games-_amd"
LIB = os.path.join(ROOT, PKG, "libspgg_hip.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# the bench's instance (cfg3: M=1, reputation, int8 R, Philox, 4 agents per thread, 40-wide
# tiles, Q-learning) and its VGPR ceiling for 5 waves per SIMD (512 / 5 -> 96, granule 8)
BENCH_KERNEL = "spgg_step_kernelILb0ELb0ELb1ELi2ELi4ELi40ELi0E"
BENCH_MAX_VGPR = 96


def _code_objects(path):
    """gfx950 code objects of every offload bundle in the library's fat binary."""
    data = open(path, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(MAGIC))[0]
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 1)
    return out


def _kernels(path):
    """{kernel symbol: metadata fields} from the code objects' AMDGPU notes."""
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        for i, co in enumerate(_code_objects(path)):
            f = os.path.join(tmp, f"co{i}.o")
            open(f, "wb").write(co)
            notes = subprocess.run([READELF, "--notes", f], capture_output=True, text=True, check=True).stdout
            for blk in notes.split("- .agpr_count:")[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk).group(1)
                res[name] = {k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))
                             for k in ("private_segment_fixed_size", "vgpr_count", "vgpr_spill_count",
                                       "sgpr_spill_count")}
    return res


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.skip("libspgg_hip.so not built")
    if not os.path.exists(READELF):
        pytest.skip("llvm-readelf not available")
    ks = _kernels(LIB)
    assert ks, "no gfx950 code object found in libspgg_hip.so"
    return ks


def test_step_kernels_use_no_scratch(kernels):
    steps = {k: v for k, v in kernels.items() if "spgg_step_kernel" in k}
    assert len(steps) >= 4 * 16, len(steps)  # every operator's instances
    bad = {k: v for k, v in steps.items() if v["private_segment_fixed_size"] or v["vgpr_spill_count"]}
    assert not bad, bad


def test_bench_kernel_register_budget(kernels):
    hit = [v for k, v in kernels.items() if BENCH_KERNEL in k]
    assert len(hit) == 1, [k for k in kernels if "spgg_step_kernel" in k][:8]
    assert hit[0]["vgpr_count"] <= BENCH_MAX_VGPR, hit[0]
