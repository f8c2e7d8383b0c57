"""oracle/codec_ref.py — TEST INFRASTRUCTURE: pure-Python restatement of the reference wire
codec, used only to check libbloomstage's bs_codec_* byte for byte.

Follows utils::SerializeTensorVectorToBytes (utils.cpp:124-264): size_t count; per tensor
int32 ONNXTensorElementDataType (utils.cpp:144-146), size_t ndim (:153-155), int64 dims
(:158-161), raw data (:166-247); and DeserializeTensorVectorFromBytes (:266-368).
LP64 little endian (arm64 Android).
"""
import struct

import numpy as np

# ONNX enum -> numpy dtype, exactly the reference's switch cases (utils.cpp:166-247)
SUPPORTED = {1: np.float32, 3: np.int8, 2: np.uint8, 4: np.uint16, 5: np.int16, 6: np.int32,
             7: np.int64, 9: np.bool_, 11: np.float64, 12: np.uint32, 13: np.uint64}
TO_ENUM = {np.dtype(v): k for k, v in SUPPORTED.items()}


def serialize(arrays) -> bytes:
    out = [struct.pack("<Q", len(arrays))]
    for a in arrays:
        a = np.asarray(a)
        a = a if a.flags.c_contiguous else a.copy(order="C")
        out.append(struct.pack("<i", TO_ENUM[a.dtype]))
        out.append(struct.pack("<Q", a.ndim))
        out.extend(struct.pack("<q", d) for d in a.shape)
        out.append(a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes())
    return b"".join(out)


def deserialize(data: bytes):
    n, = struct.unpack_from("<Q", data, 0)
    off, res = 8, []
    for _ in range(n):
        dt, = struct.unpack_from("<i", data, off); off += 4
        nd, = struct.unpack_from("<Q", data, off); off += 8
        shape = struct.unpack_from("<" + "q" * nd, data, off); off += 8 * nd
        dtype = np.dtype(SUPPORTED[dt])
        cnt = int(np.prod(shape)) if nd else 1
        res.append(np.frombuffer(data, dtype=dtype, count=cnt, offset=off).reshape(shape).copy())
        off += cnt * dtype.itemsize
    return res
