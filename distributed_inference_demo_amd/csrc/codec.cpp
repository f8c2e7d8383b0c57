// codec.cpp — the reference's tensor-vector wire format, byte for byte.
//
// Format (utils.cpp:124-264 SerializeTensorVectorToBytes, :266-368 Deserialize...; LP64
// little-endian as on the arm64 phones):
//   size_t n_tensors (8 B)
//   per tensor: int32 ONNXTensorElementDataType, size_t ndim (8 B), int64 dims[ndim],
//               raw element data (no padding, no alignment)
// Supported element types are exactly the reference's switch cases (utils.cpp:166-247):
// FLOAT, INT8, UINT8, UINT16, INT16, INT32, INT64, BOOL, DOUBLE, UINT32, UINT64.
// Divergence by design: an unsupported type is an error (BS_ERR_UNSUPPORTED) instead of the
// reference's silent stream desynchronisation (utils.cpp:244-246, :359-361).
// A zero-tensor-count buffer is legal (8 bytes).  Deserialisation never copies: views point
// into the caller's byte buffer (the reference copies 4-6 times per hop).
#include <cstdint>
#include <cstring>

#include "../../include/bloomstage.h"

extern "C" int64_t bs_dtype_size(int32_t dt) {
  switch (dt) {
    case BS_DT_FLOAT: return 4;
    case BS_DT_UINT8: return 1;
    case BS_DT_INT8: return 1;
    case BS_DT_UINT16: return 2;
    case BS_DT_INT16: return 2;
    case BS_DT_INT32: return 4;
    case BS_DT_INT64: return 8;
    case BS_DT_BOOL: return 1;
    case BS_DT_DOUBLE: return 8;
    case BS_DT_UINT32: return 4;
    case BS_DT_UINT64: return 8;
    default: return -1;  // includes FLOAT16/BFLOAT16/STRING: not carried by the reference codec
  }
}

static bool elem_count(const bs_tensor_view& t, uint64_t* n) {
  if (t.ndim < 0 || t.ndim > BS_CODEC_MAX_DIMS) return false;
  uint64_t c = 1;
  for (int i = 0; i < t.ndim; i++) {
    if (t.dims[i] < 0) return false;
    const uint64_t d = (uint64_t)t.dims[i];
    if (d && c > UINT64_MAX / d) return false;  // a crafted wire shape must not wrap the count
    c *= d;
  }
  *n = c;
  return true;
}

extern "C" int64_t bs_codec_serialize(const bs_tensor_view* tensors, int32_t n, void* out, uint64_t cap) {
  if (n < 0 || (n > 0 && !tensors)) return BS_ERR_INVALID;
  uint64_t total = 8;
  for (int i = 0; i < n; i++) {
    const int64_t es = bs_dtype_size(tensors[i].dtype);
    if (es < 0) return BS_ERR_UNSUPPORTED;
    uint64_t cnt;
    if (!elem_count(tensors[i], &cnt)) return BS_ERR_INVALID;
    if (cnt && !tensors[i].data) return BS_ERR_INVALID;
    if (cnt > (UINT64_MAX / 2 - total) / (uint64_t)es) return BS_ERR_INVALID;
    total += 4 + 8 + 8ull * tensors[i].ndim + cnt * (uint64_t)es;
  }
  if (!out || cap < total) return (int64_t)total;
  char* p = (char*)out;
  const uint64_t nt = (uint64_t)n;
  std::memcpy(p, &nt, 8); p += 8;
  for (int i = 0; i < n; i++) {
    const bs_tensor_view& t = tensors[i];
    const int32_t dt = t.dtype;
    std::memcpy(p, &dt, 4); p += 4;
    const uint64_t nd = (uint64_t)t.ndim;
    std::memcpy(p, &nd, 8); p += 8;
    for (int k = 0; k < t.ndim; k++) { std::memcpy(p, &t.dims[k], 8); p += 8; }
    uint64_t cnt;
    elem_count(t, &cnt);
    const uint64_t bytes = cnt * (uint64_t)bs_dtype_size(dt);
    if (bytes) std::memcpy(p, t.data, bytes);
    p += bytes;
  }
  return (int64_t)total;
}

extern "C" int bs_codec_deserialize(const void* bytes, uint64_t len, bs_tensor_view* views, int32_t max_views,
                                    int32_t* n_out) {
  if (!bytes || !n_out) return BS_ERR_INVALID;
  const char* p = (const char*)bytes;
  const char* end = p + len;
  if (len < 8) return BS_ERR_INVALID;
  uint64_t n;
  std::memcpy(&n, p, 8); p += 8;
  if (n > (1u << 20)) return BS_ERR_INVALID;
  *n_out = (int32_t)n;
  for (uint64_t i = 0; i < n; i++) {
    if (end - p < 12) return BS_ERR_INVALID;
    int32_t dt;
    uint64_t nd;
    std::memcpy(&dt, p, 4); p += 4;
    std::memcpy(&nd, p, 8); p += 8;
    if (nd > BS_CODEC_MAX_DIMS) return BS_ERR_INVALID;
    if ((uint64_t)(end - p) < 8 * nd) return BS_ERR_INVALID;
    bs_tensor_view v;
    std::memset(&v, 0, sizeof(v));
    v.dtype = dt;
    v.ndim = (int32_t)nd;
    for (uint64_t k = 0; k < nd; k++) { std::memcpy(&v.dims[k], p, 8); p += 8; }
    const int64_t es = bs_dtype_size(dt);
    if (es < 0) return BS_ERR_UNSUPPORTED;
    uint64_t cnt;
    if (!elem_count(v, &cnt)) return BS_ERR_INVALID;
    if (cnt > (uint64_t)(end - p) / (uint64_t)es) return BS_ERR_INVALID;  // before cnt * es can wrap
    const uint64_t nb = cnt * (uint64_t)es;
    v.data = p;
    p += nb;
    if ((int64_t)i < max_views && views) views[i] = v;
  }
  return BS_OK;
}

extern "C" void bs_serialize_int(int32_t value, uint8_t out[4]) { std::memcpy(out, &value, 4); }

extern "C" int bs_deserialize_int(const uint8_t* bytes, uint64_t len, int32_t* value) {
  // utils.cpp:17-25 throws std::invalid_argument on a size mismatch; here: status code.
  if (!bytes || !value || len != 4) return BS_ERR_INVALID;
  std::memcpy(value, bytes, 4);
  return BS_OK;
}

extern "C" int bs_binary_classify(const void* bytes, uint64_t len, int32_t* cls) {
  // binaryClassify (native-lib.cpp:128-160): first tensor of the vector = logits; binary_classify
  // (inference.cpp:57-69) scans the first two floats with a strict >, so the first maximum wins.
  if (!cls) return BS_ERR_INVALID;
  bs_tensor_view v;
  int32_t n = 0;
  const int rc = bs_codec_deserialize(bytes, len, &v, 1, &n);
  if (rc != BS_OK) return rc;
  uint64_t cnt = 0;
  if (n < 1 || v.dtype != BS_DT_FLOAT || !elem_count(v, &cnt) || cnt < 2) return BS_ERR_INVALID;
  float l[2];
  std::memcpy(l, v.data, sizeof l);  // the view may be unaligned inside the wire buffer
  *cls = l[1] > l[0] ? 1 : 0;
  return BS_OK;
}
