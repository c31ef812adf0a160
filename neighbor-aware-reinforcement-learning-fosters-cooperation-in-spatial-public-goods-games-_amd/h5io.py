"""Dataset sink for SPGG.run (the reference writes HDF5 via h5py, spgg.py:339-633).

Writers, first available wins ($SPGG_H5_SINK = auto | h5py | native | npz):
  * h5py, when importable (the reference's own writer);
  * the HDF5 C library through ctypes (`h5native`: this image has conda's libhdf5
    1.10 but no h5py) -- a real HDF5 file, same datasets as h5py would write;
  * a NumPy .npz archive at exactly the requested path (no HDF5 library at all).

A duplicate dataset name raises ValueError, as h5py does: the reference's run
fails that way when its three tracked positions coincide (L <= 2,
spgg.py:137, 620-622), after the state and the earlier datasets are written.
"""
from __future__ import annotations

import os

import numpy as np

from . import h5native

try:  # pragma: no cover - depends on the image
    import h5py  # type: ignore
except Exception:  # noqa: BLE001
    h5py = None

HDF5_MAGIC = b"\x89HDF\r\n\x1a\n"


class NpzFile:
    def __init__(self, filename, mode="w"):
        if mode != "w":
            raise ValueError("NpzFile only writes")
        self.filename = filename
        self.data = {}

    def create_dataset(self, name, data=None):
        if name in self.data:
            raise ValueError(f"dataset {name!r} already exists")
        self.data[name] = np.array(data)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, *a):
        # like closing an h5py.File: what was created so far is kept, and an error
        # raised inside the block (e.g. a duplicate dataset name) propagates
        with open(self.filename, "wb") as f:
            np.savez(f, **self.data)
        return False


def sink() -> str:
    """The writer open_writer uses: "h5py", "native" or "npz"."""
    want = os.environ.get("SPGG_H5_SINK", "auto")
    if want not in ("auto", "h5py", "native", "npz"):
        raise ValueError(f"SPGG_H5_SINK={want!r}: expected auto, h5py, native or npz")
    if want == "auto":
        return "h5py" if h5py is not None else ("native" if h5native.available() else "npz")
    if want == "h5py" and h5py is None:
        raise OSError("SPGG_H5_SINK=h5py but h5py is not importable")
    if want == "native" and not h5native.available():
        raise OSError("SPGG_H5_SINK=native but no HDF5 C library was found (SPGG_HDF5_LIB)")
    return want


def open_writer(filename):
    kind = sink()
    if kind == "h5py":
        return h5py.File(filename, "w")
    if kind == "native":
        return h5native.Hdf5File(filename, "w")
    return NpzFile(filename, "w")


def is_hdf5(filename) -> bool:
    with open(filename, "rb") as fh:
        return fh.read(8) == HDF5_MAGIC


def read_datasets(filename):
    """Every dataset of a file open_writer produced, {name: ndarray} (tests, plotting)."""
    if is_hdf5(filename):
        if h5py is not None:
            with h5py.File(filename, "r") as f:
                return {k: f[k][()] for k in f.keys()}
        return h5native.read_all(filename)
    with np.load(filename, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def read_dataset(filename, name):
    """One dataset, or None if the file has no dataset of that name."""
    if is_hdf5(filename):
        if h5py is not None:
            with h5py.File(filename, "r") as f:
                return f[name][()] if name in f else None
        return h5native.read_one(filename, name)
    with np.load(filename, allow_pickle=False) as z:
        return z[name] if name in z.files else None
