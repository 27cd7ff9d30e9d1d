"""Reader / writer for the PAMGREC1 binary record files.

Written by the instrumented reference build (oracle/ref_hooks/pamg_ref_hooks.F90),
by the Fortran host driver (p-a_multigrids_amd/fortran/pamg_driver.F90) and by
tests/make_golden.py. Arrays are stored in Fortran (column-major) order; this
module returns numpy arrays with the Fortran shape (order='F').
"""
import struct

import numpy as np

MAGIC = b"PAMGREC1"


def read_records(path):
    out = {}
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos < len(data):
        if data[pos:pos + 8] != MAGIC:
            raise ValueError(f"{path}: bad magic at byte {pos}")
        pos += 8
        (nlen,) = struct.unpack_from("<i", data, pos); pos += 4
        name = data[pos:pos + nlen].decode(); pos += nlen
        dtype, ndim = struct.unpack_from("<ii", data, pos); pos += 8
        dims = struct.unpack_from("<%dq" % ndim, data, pos); pos += 8 * ndim
        dt = {1: np.float64, 2: np.int32}[dtype]
        count = int(np.prod(dims)) if ndim else 1
        arr = np.frombuffer(data, dtype=dt, count=count, offset=pos).copy()
        pos += count * np.dtype(dt).itemsize
        out[name] = arr.reshape(dims, order="F")
    return out


def write_records(path, records):
    with open(path, "wb") as f:
        for name, arr in records.items():
            arr = np.asarray(arr)
            if arr.dtype.kind == "f":
                arr, code = arr.astype(np.float64), 1
            else:
                arr, code = arr.astype(np.int32), 2
            nb = name.encode()
            f.write(MAGIC)
            f.write(struct.pack("<i", len(nb)))
            f.write(nb)
            f.write(struct.pack("<ii", code, arr.ndim))
            f.write(struct.pack("<%dq" % arr.ndim, *arr.shape))
            f.write(np.asfortranarray(arr).tobytes(order="F"))
