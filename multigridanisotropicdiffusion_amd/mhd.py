"""MetaImage (.mhd + raw / zlib .zraw) reader and writer.

The reference's VED test reads and writes its volumes through ITK's MetaImageIO
(test/itkVEDTest_GS.cxx:27-41 reads test_data/ved_test.mhd, :106-125 writes the
result with the input's direction); these are the header fields those files use:

    ObjectType NDims BinaryData BinaryDataByteOrderMSB CompressedData
    CompressedDataSize TransformMatrix Offset CenterOfRotation AnatomicalOrientation
    ElementSpacing DimSize ElementType ElementDataFile

`read_mhd` returns (array, info): array in numpy (z, y, x) order (ITK buffer order:
x fastest), info a dict with spacing / origin / direction (x first, as ITK) and the
raw header.  Only local data files are supported (ElementDataFile = LOCAL or a
file name next to the header), as in the reference's test data.
"""
import os
import zlib

import numpy as np

_TYPES = {
    "MET_UCHAR": np.uint8, "MET_CHAR": np.int8, "MET_USHORT": np.uint16,
    "MET_SHORT": np.int16, "MET_UINT": np.uint32, "MET_INT": np.int32,
    "MET_ULONG_LONG": np.uint64, "MET_LONG_LONG": np.int64,
    "MET_FLOAT": np.float32, "MET_DOUBLE": np.float64,
}
_NAMES = {np.dtype(v): k for k, v in _TYPES.items()}


def _parse_header(text):
    hdr = {}
    for line in text.splitlines():
        if "=" not in line:
            continue
        k, v = line.split("=", 1)
        hdr[k.strip()] = v.strip()
    return hdr


def read_mhd(path):
    with open(path, "rb") as f:
        head = f.read()
    # LOCAL data follows the ElementDataFile line in the same file
    marker = head.find(b"ElementDataFile")
    if marker < 0:
        raise ValueError(f"{path}: no ElementDataFile field")
    eol = head.find(b"\n", marker)
    eol = len(head) if eol < 0 else eol + 1
    hdr = _parse_header(head[:eol].decode("ascii", "replace"))
    ndims = int(hdr.get("NDims", "3"))
    dims = [int(v) for v in hdr["DimSize"].split()][:ndims]
    etype = hdr["ElementType"]
    if etype not in _TYPES:
        raise ValueError(f"{path}: unsupported ElementType {etype}")
    dt = np.dtype(_TYPES[etype])
    msb = hdr.get("BinaryDataByteOrderMSB", hdr.get("ElementByteOrderMSB", "False"))
    dt = dt.newbyteorder(">" if msb.lower() == "true" else "<")
    src = hdr["ElementDataFile"]
    if src == "LOCAL":
        data = head[eol:]
    else:
        with open(os.path.join(os.path.dirname(os.path.abspath(path)), src), "rb") as f:
            data = f.read()
    if hdr.get("CompressedData", "False").lower() == "true":
        data = zlib.decompress(data)
    n = int(np.prod(dims))
    arr = np.frombuffer(data, dtype=dt, count=n).astype(dt.newbyteorder("="))
    arr = arr.reshape(list(reversed(dims)))
    info = {
        "spacing": [float(v) for v in hdr.get("ElementSpacing", " ".join(["1"] * ndims)).split()][:ndims],
        "origin": [float(v) for v in hdr.get("Offset", hdr.get("Origin", " ".join(["0"] * ndims))).split()][:ndims],
        "direction": [float(v) for v in hdr.get("TransformMatrix", "").split()] or None,
        "header": hdr,
    }
    return arr, info


def write_mhd(path, arr, spacing=None, origin=None, direction=None, compress=True):
    """Write `arr` ((z, y, x) or (y, x)) as path (.mhd) + data file (.zraw / .raw)."""
    arr = np.ascontiguousarray(arr)
    if arr.dtype not in _NAMES:
        raise ValueError(f"unsupported dtype {arr.dtype}")
    nd = arr.ndim
    dims = list(reversed(arr.shape))
    spacing = list(spacing) if spacing is not None else [1.0] * nd
    origin = list(origin) if origin is not None else [0.0] * nd
    direction = list(direction) if direction is not None else list(np.eye(nd).ravel())
    base = os.path.splitext(path)[0]
    dfile = os.path.basename(base) + (".zraw" if compress else ".raw")
    raw = arr.astype(arr.dtype.newbyteorder("<")).tobytes()
    data = zlib.compress(raw) if compress else raw
    lines = [
        "ObjectType = Image",
        f"NDims = {nd}",
        "BinaryData = True",
        "BinaryDataByteOrderMSB = False",
        f"CompressedData = {'True' if compress else 'False'}",
    ]
    if compress:
        lines.append(f"CompressedDataSize = {len(data)}")
    lines += [
        "TransformMatrix = " + " ".join(f"{v:g}" for v in direction),
        "Offset = " + " ".join(f"{v:g}" for v in origin),
        "CenterOfRotation = " + " ".join(["0"] * nd),
        "ElementSpacing = " + " ".join(f"{v:g}" for v in spacing),
        "DimSize = " + " ".join(str(d) for d in dims),
        f"ElementType = {_NAMES[arr.dtype]}",
        f"ElementDataFile = {dfile}",
    ]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(os.path.dirname(os.path.abspath(path)), dfile), "wb") as f:
        f.write(data)
