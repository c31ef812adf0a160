"""HDF5 files through the HDF5 C library itself (ctypes), for images without h5py.

The reference writes every result with `h5py.File(filename, "w")` and
`create_dataset(name, data=array)` into the root group (src/model/spgg.py:339-633),
and its plots read them back with h5py (src/visualization/plotting.py:36-63).  This
image has no h5py, but it does have the HDF5 C library (conda's libhdf5, 1.10.x).
Binding that library directly produces the same file h5py would: one contiguous,
uncompressed dataset per name in the root group, little-endian IEEE f64 / two's
complement integer types, default (earliest-format) file creation properties --
readable by h5py, h5dump and the reference's plotting code.

    with Hdf5File(path, "w") as f:           # h5py.File's writing subset
        f.create_dataset("coop_rate_history", data=np.arange(3.0))
    read_all(path)  -> {name: ndarray}       # every root-group dataset, name order
    read_one(path, name) -> ndarray | None

`available()` is False when no libhdf5 can be loaded ($SPGG_HDF5_LIB, the linker's
search path, or the conda prefix); callers then fall back (h5io).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os
import threading

import numpy as np

hid_t = ctypes.c_int64          # HDF5 >= 1.10: 64-bit identifiers
herr_t = ctypes.c_int
hsize_t = ctypes.c_ulonglong

H5F_ACC_RDONLY, H5F_ACC_TRUNC = 0x0000, 0x0002
H5P_DEFAULT = 0
H5S_ALL = 0
H5S_SCALAR = 0
H5E_DEFAULT = 0
H5T_INTEGER, H5T_FLOAT = 0, 1
H5T_SGN_NONE = 0
H5_INDEX_NAME, H5_ITER_INC = 0, 0

_CANDIDATES = ("libhdf5.so", "libhdf5.so.103", "libhdf5.so.200", "libhdf5.so.310")
_PREFIXES = (os.path.join(os.environ.get("CONDA_PREFIX", "/opt/conda"), "lib"), "/opt/conda/lib",
             "/usr/lib/x86_64-linux-gnu/hdf5/serial", "/usr/lib/x86_64-linux-gnu", "/usr/lib64", "/usr/lib")

_lock = threading.Lock()
_state = {"lib": None, "tried": False, "types": None}


def _find():
    env = os.environ.get("SPGG_HDF5_LIB")
    if env:
        return [env]
    found = ctypes.util.find_library("hdf5")
    paths = [found] if found else []
    paths += [os.path.join(p, c) for p in _PREFIXES for c in _CANDIDATES]
    return [p for p in paths if p and (os.path.isabs(p) is False or os.path.exists(p))]


def _bind(lib):
    P = ctypes.POINTER
    sig = {
        "H5open": (herr_t, []),
        "H5Eset_auto2": (herr_t, [hid_t, ctypes.c_void_p, ctypes.c_void_p]),
        "H5Fcreate": (hid_t, [ctypes.c_char_p, ctypes.c_uint, hid_t, hid_t]),
        "H5Fopen": (hid_t, [ctypes.c_char_p, ctypes.c_uint, hid_t]),
        "H5Fclose": (herr_t, [hid_t]),
        "H5Screate_simple": (hid_t, [ctypes.c_int, P(hsize_t), P(hsize_t)]),
        "H5Screate": (hid_t, [ctypes.c_int]),
        "H5Sclose": (herr_t, [hid_t]),
        "H5Sget_simple_extent_ndims": (ctypes.c_int, [hid_t]),
        "H5Sget_simple_extent_dims": (ctypes.c_int, [hid_t, P(hsize_t), P(hsize_t)]),
        "H5Dcreate2": (hid_t, [hid_t, ctypes.c_char_p, hid_t, hid_t, hid_t, hid_t, hid_t]),
        "H5Dopen2": (hid_t, [hid_t, ctypes.c_char_p, hid_t]),
        "H5Dwrite": (herr_t, [hid_t, hid_t, hid_t, hid_t, hid_t, ctypes.c_void_p]),
        "H5Dread": (herr_t, [hid_t, hid_t, hid_t, hid_t, hid_t, ctypes.c_void_p]),
        "H5Dget_type": (hid_t, [hid_t]),
        "H5Dget_space": (hid_t, [hid_t]),
        "H5Dclose": (herr_t, [hid_t]),
        "H5Tget_class": (ctypes.c_int, [hid_t]),
        "H5Tget_size": (ctypes.c_size_t, [hid_t]),
        "H5Tget_sign": (ctypes.c_int, [hid_t]),
        "H5Tclose": (herr_t, [hid_t]),
        "H5Lexists": (ctypes.c_int, [hid_t, ctypes.c_char_p, hid_t]),
        "H5Lget_name_by_idx": (ctypes.c_ssize_t, [hid_t, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, hsize_t,
                                                 ctypes.c_char_p, ctypes.c_size_t, hid_t]),
        "H5Gget_info": (herr_t, [hid_t, ctypes.c_void_p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.H5open() < 0:
        raise OSError("H5open failed")
    lib.H5Eset_auto2(H5E_DEFAULT, None, None)   # errors become return codes, not stderr dumps

    def g(sym):  # predefined type ids are globals, valid after H5open
        return hid_t.in_dll(lib, sym).value

    # numpy dtype -> (file type, memory type), as h5py maps them (little-endian file types)
    types = {}
    for kind, size, ftype, mtype in (
            ("f", 8, "H5T_IEEE_F64LE_g", "H5T_NATIVE_DOUBLE_g"), ("f", 4, "H5T_IEEE_F32LE_g", "H5T_NATIVE_FLOAT_g"),
            ("i", 8, "H5T_STD_I64LE_g", "H5T_NATIVE_LLONG_g"), ("i", 4, "H5T_STD_I32LE_g", "H5T_NATIVE_INT_g"),
            ("i", 2, "H5T_STD_I16LE_g", "H5T_NATIVE_SHORT_g"), ("i", 1, "H5T_STD_I8LE_g", "H5T_NATIVE_SCHAR_g"),
            ("u", 8, "H5T_STD_U64LE_g", "H5T_NATIVE_ULLONG_g"), ("u", 4, "H5T_STD_U32LE_g", "H5T_NATIVE_UINT_g"),
            ("u", 2, "H5T_STD_U16LE_g", "H5T_NATIVE_USHORT_g"), ("u", 1, "H5T_STD_U8LE_g", "H5T_NATIVE_UCHAR_g")):
        types[(kind, size)] = (g(ftype), g(mtype))
    return types


def library():
    """The bound libhdf5 (loaded once), or None."""
    with _lock:
        if not _state["tried"]:
            _state["tried"] = True
            for path in _find():
                try:
                    lib = ctypes.CDLL(path)
                    _state["types"] = _bind(lib)
                    _state["lib"] = lib
                    _state["path"] = path
                    break
                except (OSError, AttributeError):
                    continue
        return _state["lib"]


def available() -> bool:
    return library() is not None


def _check(rc, what):
    if rc < 0:
        raise OSError(f"HDF5: {what} failed")
    return rc


class Hdf5File:
    """h5py.File's writing subset the reference uses: create_dataset(name, data=...)
    into the root group; a repeated name raises ValueError (as h5py does) and what
    was written before stays in the file."""

    def __init__(self, filename, mode="w"):
        if mode != "w":
            raise ValueError("Hdf5File only writes (read_all / read_one read)")
        self.lib = library()
        if self.lib is None:
            raise OSError("no HDF5 C library found (set SPGG_HDF5_LIB)")
        self.filename = os.fspath(filename)
        self.fid = _check(self.lib.H5Fcreate(self.filename.encode(), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT),
                          f"create {self.filename}")

    def create_dataset(self, name, data=None):
        lib = self.lib
        bname = name.encode()
        if lib.H5Lexists(self.fid, bname, H5P_DEFAULT) > 0:
            raise ValueError(f"Unable to create dataset (name already exists): {name!r}")
        arr = np.ascontiguousarray(np.asarray(data))
        if arr.dtype == np.bool_:
            arr = arr.astype(np.int8)   # (not in the layout; h5py would write an enum)
        key = (arr.dtype.kind, arr.dtype.itemsize)
        if key not in _state["types"]:
            raise TypeError(f"dataset {name!r}: unsupported dtype {arr.dtype}")
        ftype, mtype = _state["types"][key]
        arr = arr.astype(arr.dtype.newbyteorder("="), copy=False)
        if arr.ndim == 0:
            sid = _check(lib.H5Screate(H5S_SCALAR), "H5Screate")
        else:
            dims = (hsize_t * arr.ndim)(*arr.shape)
            sid = _check(lib.H5Screate_simple(arr.ndim, dims, None), "H5Screate_simple")
        try:
            did = _check(lib.H5Dcreate2(self.fid, bname, ftype, sid, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT),
                         f"create dataset {name}")
            try:
                if arr.size:
                    _check(lib.H5Dwrite(did, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, arr.ctypes.data_as(ctypes.c_void_p)),
                           f"write dataset {name}")
            finally:
                lib.H5Dclose(did)
        finally:
            lib.H5Sclose(sid)

    def close(self):
        if self.fid is not None:
            self.lib.H5Fclose(self.fid)
            self.fid = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def _read(lib, fid, name):
    did = lib.H5Dopen2(fid, name.encode(), H5P_DEFAULT)
    if did < 0:
        return None
    try:
        tid = _check(lib.H5Dget_type(did), "H5Dget_type")
        try:
            cls, size = lib.H5Tget_class(tid), lib.H5Tget_size(tid)
            if cls == H5T_FLOAT:
                kind = "f"
            elif cls == H5T_INTEGER:
                kind = "u" if lib.H5Tget_sign(tid) == H5T_SGN_NONE else "i"
            else:
                raise TypeError(f"dataset {name!r}: HDF5 type class {cls} not supported")
        finally:
            lib.H5Tclose(tid)
        sid = _check(lib.H5Dget_space(did), "H5Dget_space")
        try:
            nd = _check(lib.H5Sget_simple_extent_ndims(sid), "ndims")
            dims = (hsize_t * max(nd, 1))()
            if nd:
                _check(lib.H5Sget_simple_extent_dims(sid, dims, None), "dims")
            shape = tuple(int(dims[i]) for i in range(nd))
        finally:
            lib.H5Sclose(sid)
        mtype = _state["types"][(kind, int(size))][1]
        out = np.empty(shape, dtype=np.dtype(f"={kind}{size}"))
        if out.size:
            _check(lib.H5Dread(did, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, out.ctypes.data_as(ctypes.c_void_p)),
                   f"read dataset {name}")
        return out
    finally:
        lib.H5Dclose(did)


def _names(lib, fid):
    info = (ctypes.c_char * 64)()
    _check(lib.H5Gget_info(fid, info), "H5Gget_info")
    nlinks = ctypes.c_ulonglong.from_buffer(info, 8).value   # H5G_info_t.nlinks (after the storage-type enum)
    names = []
    for i in range(nlinks):
        n = lib.H5Lget_name_by_idx(fid, b".", H5_INDEX_NAME, H5_ITER_INC, i, None, 0, H5P_DEFAULT)
        buf = ctypes.create_string_buffer(int(_check(n, "H5Lget_name_by_idx")) + 1)
        lib.H5Lget_name_by_idx(fid, b".", H5_INDEX_NAME, H5_ITER_INC, i, buf, len(buf), H5P_DEFAULT)
        names.append(buf.value.decode())
    return names


def _open(path):
    lib = library()
    if lib is None:
        raise OSError("no HDF5 C library found (set SPGG_HDF5_LIB)")
    fid = lib.H5Fopen(os.fspath(path).encode(), H5F_ACC_RDONLY, H5P_DEFAULT)
    if fid < 0:
        raise OSError(f"HDF5: cannot open {path}")
    return lib, fid


def read_all(path):
    """{name: ndarray} of every dataset in the root group, in name order (h5py's keys())."""
    lib, fid = _open(path)
    try:
        return {k: _read(lib, fid, k) for k in _names(lib, fid)}
    finally:
        lib.H5Fclose(fid)


def read_one(path, name):
    """One root-group dataset, or None if the file has no such dataset."""
    lib, fid = _open(path)
    try:
        if lib.H5Lexists(fid, name.encode(), H5P_DEFAULT) <= 0:
            return None
        return _read(lib, fid, name)
    finally:
        lib.H5Fclose(fid)
