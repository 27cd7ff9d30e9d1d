"""Minimal reader of VTK XML UnstructuredGrid files (.vtu) with ascii or raw appended
data -- the reference's get_vtu output (get_vtk_files.F90:10-165, ascii) and
pamg_write_vtu's (raw appended, Float64). Test infrastructure only."""
import re
import xml.etree.ElementTree as ET

import numpy as np

_DT = {"Float32": np.float32, "Float64": np.float64, "Int32": np.int32, "Int64": np.int64, "UInt8": np.uint8,
       "UInt32": np.uint32, "UInt64": np.uint64}


def read_vtu(path):
    """Returns {"points": (n, 3), "cells": {...}, "point_data": {name: array}, "n_points", "n_cells"}."""
    raw = open(path, "rb").read()
    appended = b""
    m = re.search(rb"<AppendedData[^>]*>\s*_", raw)
    if m:
        end = raw.rfind(b"</AppendedData>")
        appended = raw[m.end():end]
        xml = raw[:m.start()] + b"<AppendedData/></VTKFile>"
    else:
        xml = raw
    root = ET.fromstring(xml.decode("latin-1"))
    header = _DT[root.get("header_type", "UInt32")]
    piece = root.find("./UnstructuredGrid/Piece")

    def data(da):
        dt = _DT[da.get("type")]
        if da.get("format", da.get("Format")) == "appended":
            off = int(da.get("offset"))
            nbytes = int(np.frombuffer(appended[off:off + np.dtype(header).itemsize], header)[0])
            start = off + np.dtype(header).itemsize
            return np.frombuffer(appended[start:start + nbytes], dt).copy()
        vals = np.array(da.text.split(), dtype=np.float64)   # ascii: keep every printed digit
        return vals if np.dtype(dt).kind == "f" else vals.astype(dt)

    out = {"n_points": int(piece.get("NumberOfPoints")), "n_cells": int(piece.get("NumberOfCells")),
           "point_data": {}, "cells": {}}
    for da in piece.find("PointData"):
        out["point_data"][da.get("Name")] = data(da)
    pts = data(piece.find("Points/DataArray"))
    out["points"] = pts.reshape(-1, int(piece.find("Points/DataArray").get("NumberOfComponents")))
    for da in piece.find("Cells"):
        out["cells"][da.get("Name")] = data(da)
    return out
