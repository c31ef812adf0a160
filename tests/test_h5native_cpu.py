"""The HDF5 sink without h5py (h5native: the HDF5 C library through ctypes).

The reference's own output files are the layout contract (spgg.py:339-633): every
golden fixture holds the complete dataset dictionary one reference run wrote.  Each
is written here through the sink the drop-in SPGG.run uses, then read back two
independent ways -- this package's reader and the HDF5 project's own h5dump -- and
must come back bit for bit: names, dtypes, shapes, values."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from spgg_amd import h5io, h5native
from _golden import Case, case_names

pytestmark = pytest.mark.skipif(not h5native.available(), reason="no HDF5 C library in this image")

H5DUMP = shutil.which("h5dump") or ("/opt/conda/bin/h5dump" if os.path.exists("/opt/conda/bin/h5dump") else None)


def _write(path, datasets):
    with h5native.Hdf5File(path, "w") as f:
        for k, v in datasets.items():
            f.create_dataset(k, data=v)


@pytest.mark.parametrize("name", case_names())
def test_reference_layout_round_trips_bit_exact(name, tmp_path):
    want = Case(name).datasets
    fn = str(tmp_path / "experiment_data.h5")
    _write(fn, want)
    assert h5io.is_hdf5(fn)
    got = h5native.read_all(fn)
    assert list(got) == sorted(want)                      # h5py's keys(): name order
    for k, w in want.items():
        g = got[k]
        assert g.dtype == w.dtype and g.shape == w.shape, (k, g.dtype, w.dtype, g.shape, w.shape)
        assert g.tobytes() == np.ascontiguousarray(w).tobytes(), k   # NaN payloads included
    assert h5native.read_one(fn, "coop_rate_history").tobytes() == want["coop_rate_history"].tobytes()
    assert h5native.read_one(fn, "no_such_dataset") is None


@pytest.mark.skipif(H5DUMP is None, reason="h5dump not installed")
@pytest.mark.parametrize("name", ["m1_rep_L50_cfg1", "m2_rep_L24_stopC", "dq_m1_rep_L16"])
def test_h5dump_reads_the_reference_layout(name, tmp_path):
    """The HDF5 project's own tool agrees: every dataset with the h5py type of its numpy
    dtype (IEEE F64LE / STD I64LE) and shape, and raw values identical (binary dump)."""
    want = Case(name).datasets
    fn = str(tmp_path / "experiment_data.h5")
    _write(fn, want)
    hdr = subprocess.run([H5DUMP, "-H", fn], capture_output=True, text=True, check=True).stdout
    for k, w in want.items():
        i = hdr.index(f'DATASET "{k}"')
        block = hdr[i:hdr.index("}", i)]
        assert ("H5T_IEEE_F64LE" if w.dtype.kind == "f" else "H5T_STD_I64LE") in block, (k, block)
        dims = "( " + ", ".join(str(d) for d in w.shape) + " )"
        assert f"SIMPLE {{ {dims} / {dims} " in block, (k, block)
    for k in ("coop_rate_history", "R_final", "Sn_final", "it_records_final"):
        out = str(tmp_path / f"{k}.bin")
        subprocess.run([H5DUMP, "-d", f"/{k}", "-b", "LE", "-o", out, fn], capture_output=True, check=True)
        assert open(out, "rb").read() == np.ascontiguousarray(want[k]).astype(want[k].dtype.newbyteorder("<")).tobytes(), k


def test_duplicate_name_refused_like_h5py(tmp_path):
    """h5py refuses a repeated dataset name with ValueError, and the file keeps what was
    written before (the reference's L <= 2 runs end this way, spgg.py:620-622)."""
    fn = str(tmp_path / "d.h5")
    with pytest.raises(ValueError, match="already exists"):
        with h5io.open_writer(fn) as f:
            f.create_dataset("q_c_pos_0_0_final", data=np.array([]))
            f.create_dataset("Sn_final", data=np.zeros((2, 2), dtype=np.int64))
            f.create_dataset("q_c_pos_0_0_final", data=np.array([]))
    got = h5io.read_datasets(fn)
    assert sorted(got) == ["Sn_final", "q_c_pos_0_0_final"]
    assert got["q_c_pos_0_0_final"].shape == (0,) and got["Sn_final"].dtype == np.int64


def test_sink_selection(tmp_path, monkeypatch):
    monkeypatch.setenv("SPGG_H5_SINK", "auto")
    assert h5io.sink() in ("h5py", "native")
    monkeypatch.setenv("SPGG_H5_SINK", "npz")
    fn = str(tmp_path / "x.h5")
    with h5io.open_writer(fn) as f:
        f.create_dataset("a", data=np.arange(3.0))
    assert not h5io.is_hdf5(fn) and h5io.read_dataset(fn, "a").tolist() == [0.0, 1.0, 2.0]
    monkeypatch.setenv("SPGG_H5_SINK", "hdf4")
    with pytest.raises(ValueError):
        h5io.sink()
