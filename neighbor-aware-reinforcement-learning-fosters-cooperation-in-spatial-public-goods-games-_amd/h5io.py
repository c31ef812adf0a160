"""Dataset sink for SPGG.run (the reference writes HDF5 via h5py, spgg.py:339-633).

h5py is used when importable.  This image has neither h5py nor an HDF5 library,
so the fallback writes the same dataset names/dtypes/shapes as a NumPy .npz
archive at exactly the requested path (readable with numpy.load).

A duplicate dataset name raises ValueError, as h5py does: the reference's run
fails that way when its three tracked positions coincide (L <= 2,
spgg.py:137, 620-622), after the state and the earlier datasets are written.
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - depends on the image
    import h5py  # type: ignore
except Exception:  # noqa: BLE001
    h5py = None


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


def open_writer(filename):
    if h5py is not None:
        return h5py.File(filename, "w")
    return NpzFile(filename, "w")


def read_datasets(filename):
    """Read back what open_writer produced (tests, plotting)."""
    if h5py is not None:
        try:
            with h5py.File(filename, "r") as f:
                return {k: f[k][()] for k in f.keys()}
        except OSError:
            pass
    with np.load(filename, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
