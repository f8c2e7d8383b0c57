"""ctypes binding of libbloomstage.so + the host-side mirror of the reference's stage interface.

Reference interface (Java side `Communication.java:1153-1182`, C++ side `native-lib.cpp`):

    long   createSession(String modelPath)                                   native-lib.cpp:671-678
    void   releaseSession(long session)                                      native-lib.cpp:1290-1303
    Object[] runInferenceMasterResidual(long, int[] ids, int[] seq, int[][] res)   :942-1034
    Object[] runInferenceWorkerResidual(long, byte[] seq, ArrayList<byte[]> res, int[], int[][])  :1036-1194
    byte[] runInferenceWorkerResidualLastGeneration(long, byte[] seq, ArrayList<byte[]> res, int k, float temp)  :1368-1443
    byte[] runInferenceWorkerResidualLastClassification(long, byte[] seq, ArrayList<byte[]> res)  :1305-1366
    int    binaryClassify(byte[])                                            :128-160
    int    deserializeInt(byte[])                                            :1445-1471

`create_session`, `release_session`, `run_inference_master_residual`,
`run_inference_worker_residual`, `run_inference_worker_residual_last_generation`,
`run_inference_worker_residual_last_classification`, `binary_classify` and `deserialize_int` below keep those names, argument meanings and wire formats (activations as
the utils.cpp tensor-vector bytes, the tail's token as 4 little-endian bytes) so the
reference's driver loop ports over unchanged.  They run the stage with host I/O.  The fast
path is `Stage.forward()` on device buffers (what the RCCL pipeline uses).

Behavioural differences, all deliberate (DESIGN.md "Boundary"): errors raise `BloomStageError`
with the library's message instead of C++ exceptions crossing JNI; the header stage feeds the
whole new-token slice and keeps a KV cache (the reference feeds only the last token with no
cache, Communication.java:322-326, so it ignores context); the tail picks the greedy argmax
(k == 1) or a seeded top-k sample (k > 1) rather than an unseeded one (decoding.cpp:61-63).
"""
import ctypes
import os
import struct

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "lib", "libbloomstage.so")

BS_DT_FLOAT = 1
BS_DT_BFLOAT16 = 16
BS_WEIGHTS_SYNTHETIC = 0
BS_WEIGHTS_HOST = 1
BS_STEP_HOST_IO = 1
BS_STEP_LOGITS = 2
BS_FLAG_INT8_WEIGHTS = 1  # bs_stage_desc.flags: weight-only int8 block matrices
BS_FLAG_CLASSIFIER = 2    # bs_stage_desc.flags: sequence-classification tail (score head, class ids out)

DTYPES = {
    1: np.float32, 2: np.uint8, 3: np.int8, 4: np.uint16, 5: np.int16, 6: np.int32, 7: np.int64,
    9: np.bool_, 11: np.float64, 12: np.uint32, 13: np.uint64,
}
NP_TO_DT = {np.dtype(v): k for k, v in DTYPES.items()}


class BloomStageError(RuntimeError):
    pass


class StageDesc(ctypes.Structure):
    _fields_ = [
        ("hidden", ctypes.c_int32), ("n_head", ctypes.c_int32), ("n_layer", ctypes.c_int32),
        ("vocab", ctypes.c_int32), ("ln_eps", ctypes.c_float),
        ("layer_begin", ctypes.c_int32), ("layer_end", ctypes.c_int32),
        ("is_first", ctypes.c_int32), ("is_last", ctypes.c_int32),
        ("dtype", ctypes.c_int32), ("device", ctypes.c_int32),
        ("max_batch", ctypes.c_int32), ("max_ctx", ctypes.c_int32), ("max_tokens", ctypes.c_int32),
        ("weight_source", ctypes.c_int32), ("seed", ctypes.c_uint64),
        ("host_weights", ctypes.c_void_p), ("host_weight_count", ctypes.c_uint64),
        ("head_vocab_begin", ctypes.c_int32), ("head_vocab_end", ctypes.c_int32),
        ("flags", ctypes.c_int32), ("n_labels", ctypes.c_int32),
    ]


class Step(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("seq", ctypes.c_int32), ("slot", ctypes.c_int32),
                ("past_len", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("past_lens", ctypes.POINTER(ctypes.c_int32))]


class TensorView(ctypes.Structure):
    _fields_ = [("dtype", ctypes.c_int32), ("ndim", ctypes.c_int32), ("dims", ctypes.c_int64 * 8),
                ("data", ctypes.c_void_p)]


EXPORTS = [
    "bs_init_stage", "bs_forward", "bs_reset_kv", "bs_read_kv", "bs_release", "bs_last_error", "bs_stage_info",
    "bs_stage_weight_count", "bs_abi_version", "bs_profile_enable", "bs_profile_read",
    "bs_codec_serialize", "bs_codec_deserialize", "bs_dtype_size", "bs_serialize_int", "bs_deserialize_int",
    "bs_prompt_ids", "bs_read_weights", "bs_head_norm", "bs_head_slice", "bs_stream_delay", "bs_set_sampling",
    "bs_build_id", "bs_hbm_probe", "bs_mfma_probe", "bs_init_stage_file", "bs_weights_file_probe",
    "bs_set_graphs", "bs_binary_classify",
]

_LIB = None


def lib():
    """Load the HIP library.  There is no CPU fallback: a missing library is an error.

    A process that also uses PyTorch must import torch before the first call: torch ships its own
    libamdhip64.so.7, and the copy loaded first serves the whole process (torch fails to find the
    device on the system ROCm copy)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise BloomStageError(f"{LIB_PATH} not built: run `python -m distributed_inference_demo_amd.build`")
        L = ctypes.CDLL(LIB_PATH)
        vp, i32 = ctypes.c_void_p, ctypes.c_int32
        L.bs_build_id.restype = ctypes.c_char_p
        want, got = source_build_id(), L.bs_build_id().decode()
        if want is not None and got != want:
            raise BloomStageError(f"{LIB_PATH} was built from other sources (stamp {got[:12]}, sources {want[:12]}): "
                                  "rebuild with `python -m distributed_inference_demo_amd.build`")
        L.bs_init_stage.argtypes = [ctypes.POINTER(StageDesc), ctypes.POINTER(vp)]
        L.bs_init_stage_file.argtypes = [ctypes.POINTER(StageDesc), ctypes.c_char_p, ctypes.POINTER(vp)]
        L.bs_weights_file_probe.argtypes = [ctypes.c_char_p] + [ctypes.POINTER(i32)] * 3
        L.bs_forward.argtypes = [vp, ctypes.POINTER(Step), vp, vp, vp, vp]
        L.bs_reset_kv.argtypes = [vp, i32]
        L.bs_read_kv.argtypes = [vp, i32, i32, i32, i32, vp]
        L.bs_release.argtypes = [vp]
        L.bs_release.restype = None
        L.bs_last_error.restype = ctypes.c_char_p
        L.bs_stage_info.argtypes = [vp, ctypes.POINTER(StageDesc)] + [ctypes.POINTER(ctypes.c_uint64)] * 3
        L.bs_stage_weight_count.argtypes = [ctypes.POINTER(StageDesc)]
        L.bs_stage_weight_count.restype = ctypes.c_uint64
        L.bs_profile_enable.argtypes = [vp, i32]
        L.bs_profile_read.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_double)]
        L.bs_stream_delay.argtypes = [vp, i32]
        L.bs_codec_serialize.argtypes = [ctypes.POINTER(TensorView), i32, vp, ctypes.c_uint64]
        L.bs_codec_serialize.restype = ctypes.c_int64
        L.bs_codec_deserialize.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(TensorView), i32, ctypes.POINTER(i32)]
        L.bs_dtype_size.argtypes = [i32]
        L.bs_dtype_size.restype = ctypes.c_int64
        L.bs_serialize_int.argtypes = [i32, ctypes.c_char_p]
        L.bs_serialize_int.restype = None
        L.bs_deserialize_int.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(i32)]
        L.bs_binary_classify.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(i32)]
        L.bs_prompt_ids.argtypes = [ctypes.c_uint64, i32, i32, vp]
        L.bs_read_weights.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, vp]
        L.bs_head_norm.argtypes = [vp, vp, i32, i32, vp, vp]
        L.bs_head_slice.argtypes = [vp, vp, i32, vp, vp, vp, vp]
        L.bs_set_sampling.argtypes = [vp, i32, ctypes.c_float, ctypes.c_uint64]
        L.bs_set_graphs.argtypes = [vp, i32]
        L.bs_hbm_probe.argtypes = [i32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.bs_mfma_probe.argtypes = [i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        _LIB = L
    return _LIB


def source_build_id():
    """SHA-256 of the library sources beside this file (the stamp build.py compiles into
    bs_build_id); None when the sources are not present (an installed library)."""
    from .build import source_hash
    try:
        return source_hash()
    except FileNotFoundError:
        return None


def _check(rc):
    if rc != 0:
        raise BloomStageError(f"bloomstage error {rc}: {lib().bs_last_error().decode(errors='replace')}")


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    if hasattr(x, "data_ptr"):  # torch tensor
        return x.data_ptr()
    raise TypeError(f"cannot take a pointer of {type(x)}")


class Stage:
    """One pipeline stage (contiguous layer range) resident on one GPU."""

    def __init__(self, hidden, n_head, n_layer, vocab, layer_begin, layer_end, *, dtype="bf16", device=0,
                 max_batch=1, max_ctx=2048, max_tokens=0, seed=0, eps=1e-5, host_weights=None,
                 is_first=None, is_last=None, head_slice=None, int8_weights=False, weights_file=None, n_labels=0):
        """weights_file: a safetensors checkpoint (or its sharded *.index.json) of HF BLOOM tensors;
        the stage maps it and loads only its own layer range (bs_init_stage_file).
        n_labels > 0: a sequence-classification tail (BS_FLAG_CLASSIFIER, last stage): forwards return class ids
        and logits [batch][n_labels] instead of tokens and vocabulary logits."""
        if weights_file is not None and host_weights is not None:
            raise ValueError("pass host_weights or weights_file, not both")
        d = StageDesc()
        d.hidden, d.n_head, d.n_layer, d.vocab, d.ln_eps = hidden, n_head, n_layer, vocab, eps
        d.layer_begin, d.layer_end = layer_begin, layer_end
        d.is_first = int(layer_begin == 0 if is_first is None else is_first)
        d.is_last = int(layer_end == n_layer if is_last is None else is_last)
        d.dtype = BS_DT_BFLOAT16 if dtype in ("bf16", BS_DT_BFLOAT16) else BS_DT_FLOAT
        d.device, d.max_batch, d.max_ctx, d.max_tokens = device, max_batch, max_ctx, max_tokens
        d.seed = seed
        d.flags = BS_FLAG_INT8_WEIGHTS if int8_weights else 0  # bloom*-int8 variants (server.py:796-799)
        if n_labels:
            d.flags |= BS_FLAG_CLASSIFIER
            d.n_labels = n_labels
        if head_slice is not None:
            d.head_vocab_begin, d.head_vocab_end = head_slice
        self._weights_ref = None
        if host_weights is not None:
            w = np.ascontiguousarray(host_weights, dtype=np.float32).reshape(-1)
            self._weights_ref = w
            d.weight_source = BS_WEIGHTS_HOST
            d.host_weights = w.ctypes.data
            d.host_weight_count = w.size
        else:
            d.weight_source = BS_WEIGHTS_SYNTHETIC
        self.desc = d
        self.hidden, self.vocab = hidden, vocab
        self.n_labels = n_labels
        self.n_out = n_labels if n_labels else vocab  # logits per row of the last stage
        self.is_first, self.is_last = bool(d.is_first), bool(d.is_last)
        self.max_batch, self.max_ctx = max_batch, max_ctx
        h = ctypes.c_void_p()
        if weights_file is not None:
            _check(lib().bs_init_stage_file(ctypes.byref(d), os.fsencode(weights_file), ctypes.byref(h)))
        else:
            _check(lib().bs_init_stage(ctypes.byref(d), ctypes.byref(h)))
        self._h = h
        self._weights_ref = None  # uploaded; host copy no longer needed
        self._steps = {}  # decode fast path: re-used Step structs
        self._fwd = lib().bs_forward
        self.past = [0] * max_batch  # host mirror of cached positions per KV row

    def _step(self, batch, seq, slot, past_len, flags):
        """Step struct; past_len is an int (every row) or a sequence of per-row positions.
        Returns (step, per-row pasts)."""
        if past_len is None:
            past_len = self.past[slot:slot + batch] if 0 <= slot and slot + batch <= len(self.past) else 0
        if isinstance(past_len, int):  # the decode fast path: a Step per (batch, seq, slot, flags), re-used
            key = (batch, seq, slot, flags)
            st = self._steps.get(key)
            if st is None:
                st = self._steps[key] = Step(batch, seq, slot, past_len, flags, None)
            st.past_len = past_len
            return st, None
        if np.ndim(past_len) == 0:
            pasts = [int(past_len)] * batch
            st = Step(batch, seq, slot, int(past_len), flags, None)
        else:
            pasts = [int(p) for p in past_len]
            if len(pasts) != batch:
                raise BloomStageError(f"{len(pasts)} past lengths for {batch} rows")
            arr = (ctypes.c_int32 * batch)(*pasts)
            st = Step(batch, seq, slot, pasts[0], flags, arr)
            st._keep = arr
        return st, pasts

    # ---- fast path (device pointers, stream ordered)
    def forward(self, inp, out, batch, seq, slot=0, past_len=None, logits=None, stream=None):
        """past_len: positions already cached, one int for every row or one per row (None: the
        host mirror of each row's position)."""
        st, pasts = self._step(batch, seq, slot, past_len, BS_STEP_LOGITS if logits is not None else 0)
        _check(self._fwd(self._h, ctypes.byref(st), _ptr(inp), _ptr(out), _ptr(logits), stream))
        if pasts is None:
            self.past[slot:slot + batch] = [st.past_len + seq] * batch
        else:
            for i, r in enumerate(range(slot, slot + batch)):
                self.past[r] = pasts[i] + seq
        return out

    def set_sampling(self, top_k=1, temperature=1.0, seed=0):
        """Tail token pick (bs_set_sampling): greedy for top_k <= 1, else seeded top-k sampling in
        decoding.cpp:24-66's order (last stage only)."""
        _check(lib().bs_set_sampling(self._h, int(top_k), float(temperature), int(seed)))

    def set_graphs(self, on=True):
        """bs_set_graphs: replay captured decode graphs (default) or launch every step eagerly."""
        _check(lib().bs_set_graphs(self._h, 1 if on else 0))

    # ---- vocabulary-parallel head (device pointers, stream ordered)
    def head_norm(self, hidden, batch, seq, xn, stream=None):
        """ln_f of each row's last position -> xn [batch][hidden] (stage activation dtype)."""
        _check(lib().bs_head_norm(self._h, _ptr(hidden), batch, seq, _ptr(xn), stream))

    def head_slice(self, xn, batch, keys_in=None, keys_out=None, tokens=None, stream=None):
        """Argmax keys of this stage's vocabulary slice, merged with keys_in (uint64 [batch])."""
        _check(lib().bs_head_slice(self._h, _ptr(xn), batch, _ptr(keys_in), _ptr(keys_out), _ptr(tokens), stream))

    # ---- host I/O convenience (numpy in, numpy out)
    def forward_host(self, x, batch, seq, slot=0, past_len=None, want_logits=False):
        if self.is_first:
            x = np.ascontiguousarray(x, dtype=np.int32).reshape(batch, seq)
        else:
            x = np.ascontiguousarray(x, dtype=np.float32).reshape(batch, seq, self.hidden)
        out = np.empty(batch, np.int32) if self.is_last else np.empty((batch, seq, self.hidden), np.float32)
        logits = np.empty((batch, self.n_out), np.float32) if want_logits else None
        flags = BS_STEP_HOST_IO | (BS_STEP_LOGITS if want_logits else 0)
        st, pasts = self._step(batch, seq, slot, past_len, flags)
        _check(lib().bs_forward(self._h, ctypes.byref(st), x.ctypes.data, out.ctypes.data,
                                logits.ctypes.data if logits is not None else None, None))
        if pasts is None:
            self.past[slot:slot + batch] = [st.past_len + seq] * batch
        else:
            for i, r in enumerate(range(slot, slot + batch)):
                self.past[r] = pasts[i] + seq
        return (out, logits) if want_logits else out

    def reset(self, slot=-1):
        _check(lib().bs_reset_kv(self._h, slot))
        if slot < 0:
            self.past = [0] * self.max_batch
        else:
            self.past[slot] = 0

    def read_kv(self, layer, slot, pos0, npos):
        """KV row `slot` of local layer `layer`, positions [pos0, pos0+npos): fp32 [2 (K, V)][n_head][npos][hd]."""
        nh = self.desc.n_head
        out = np.empty((2, nh, npos, self.hidden // nh), np.float32)
        _check(lib().bs_read_kv(self._h, layer, slot, pos0, npos, out.ctypes.data))
        return out

    def info(self):
        d = StageDesc()
        wb, kb, sb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().bs_stage_info(self._h, ctypes.byref(d), ctypes.byref(wb), ctypes.byref(kb), ctypes.byref(sb)))
        return {"weight_bytes": wb.value, "kv_bytes": kb.value, "workspace_bytes": sb.value}

    def read_weights(self, offset=0, count=None):
        """Weights in canonical stage order (BS_WEIGHTS_HOST layout) as fp32."""
        if count is None:
            count = lib().bs_stage_weight_count(ctypes.byref(self.desc)) - offset
        out = np.empty(count, np.float32)
        _check(lib().bs_read_weights(self._h, offset, count, out.ctypes.data))
        return out

    def profile_enable(self, kernel_class):
        _check(lib().bs_profile_enable(self._h, kernel_class))

    @staticmethod
    def stream_delay(stream, microseconds):
        """Spin the stream for `microseconds` so the host can enqueue ahead of the GPU."""
        _check(lib().bs_stream_delay(stream, microseconds))

    def profile_read(self):
        ms, n, units = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_double()
        _check(lib().bs_profile_read(self._h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(units)))
        return ms.value, n.value, units.value

    def close(self):
        if getattr(self, "_h", None):
            lib().bs_release(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def prompt_ids(seed, batch, seq, vocab):
    """Synthetic prompt ids [batch][seq] (repo generator, computed by the library)."""
    out = np.empty((batch, seq), np.int32)
    _check(lib().bs_prompt_ids(seed, batch * seq, vocab, out.ctypes.data))
    return out


def hbm_probe(device=0, nbytes=2 << 30):
    """STREAM-like (read GB/s, copy GB/s) of a device (bs_hbm_probe)."""
    r, c = ctypes.c_double(), ctypes.c_double()
    _check(lib().bs_hbm_probe(device, nbytes, ctypes.byref(r), ctypes.byref(c)))
    return r.value, c.value


def mfma_probe(device=0):
    """Measured dense bf16 MFMA TFLOP/s of a device (bs_mfma_probe): (32x32x16 chains, 16x16x32 chains)."""
    a, b = ctypes.c_double(), ctypes.c_double()
    _check(lib().bs_mfma_probe(device, ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


def probe_weights_file(path):
    """(hidden, n_layer, vocab) a checkpoint implies (bs_weights_file_probe); -1 where unknown."""
    v = [ctypes.c_int32() for _ in range(3)]
    _check(lib().bs_weights_file_probe(os.fsencode(path), *[ctypes.byref(x) for x in v]))
    return tuple(x.value for x in v)


def weight_count(**kw):
    d = StageDesc()
    for k, v in kw.items():
        setattr(d, k, v)
    return lib().bs_stage_weight_count(ctypes.byref(d))


# ---------------------------------------------------------------------------------------
# Wire codec (utils.cpp:124-368) through the C library.
# ---------------------------------------------------------------------------------------
def serialize_tensors(arrays) -> bytes:
    """SerializeTensorVectorToBytes (utils.cpp:124-264)."""
    arrays = [np.asarray(a) for a in arrays]
    arrays = [a if a.flags.c_contiguous else a.copy(order="C") for a in arrays]  # keeps 0-d shapes
    views = (TensorView * max(1, len(arrays)))()
    for i, a in enumerate(arrays):
        if a.dtype not in NP_TO_DT:
            raise BloomStageError(f"dtype {a.dtype} is not carried by the reference wire codec")
        views[i].dtype = NP_TO_DT[a.dtype]
        views[i].ndim = a.ndim
        for k, s in enumerate(a.shape):
            views[i].dims[k] = s
        views[i].data = a.ctypes.data if a.size else None
    n = lib().bs_codec_serialize(views, len(arrays), None, 0)
    if n < 0:
        raise BloomStageError(f"serialize failed ({n})")
    buf = ctypes.create_string_buffer(n)
    m = lib().bs_codec_serialize(views, len(arrays), buf, n)
    if m != n:
        raise BloomStageError(f"serialize failed ({m})")
    return buf.raw


def deserialize_tensors(data: bytes):
    """DeserializeTensorVectorFromBytes (utils.cpp:266-368); returns copies as numpy arrays."""
    n = ctypes.c_int32()
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    rc = lib().bs_codec_deserialize(buf, len(data), None, 0, ctypes.byref(n))
    if rc != 0:
        raise BloomStageError(f"deserialize failed ({rc})")
    views = (TensorView * max(1, n.value))()
    _check(lib().bs_codec_deserialize(buf, len(data), views, n.value, ctypes.byref(n)))
    base = ctypes.addressof(buf)
    out = []
    for i in range(n.value):
        v = views[i]
        dt = np.dtype(DTYPES[v.dtype])
        shape = tuple(v.dims[k] for k in range(v.ndim))
        cnt = int(np.prod(shape)) if shape else 1
        off = (v.data or base) - base
        out.append(np.frombuffer(buf.raw, dtype=dt, count=cnt, offset=off).reshape(shape).copy())
    return out


def serialize_int(value: int) -> bytes:
    """SerializeInt (utils.cpp:11-15): 4 native little-endian bytes."""
    b = ctypes.create_string_buffer(4)
    lib().bs_serialize_int(value, b)
    return b.raw


def deserialize_int(data: bytes) -> int:
    """Java_..._deserializeInt (native-lib.cpp:1445-1471) / utils::DeserializeInt (utils.cpp:17-25)."""
    v = ctypes.c_int32()
    _check(lib().bs_deserialize_int(bytes(data), len(data), ctypes.byref(v)))
    return v.value


# ---------------------------------------------------------------------------------------
# JNI-mirror entry points (host I/O, one sample per session like the reference).
# ---------------------------------------------------------------------------------------
def create_session(model, layer_begin, layer_end, **kw) -> Stage:
    """createSession (native-lib.cpp:671-678): one module == one contiguous layer range of `model`
    (a BloomDims from .config) on a GPU."""
    return Stage(model.hidden, model.n_head, model.n_layer, model.vocab, layer_begin, layer_end, **kw)


def release_session(stage: Stage) -> None:
    """releaseSession (native-lib.cpp:1290-1303)."""
    stage.close()


def run_inference_master_residual(stage: Stage, input_ids, to_send_seq_indices=(0,), to_send_res_indices=()):
    """runInferenceMasterResidual (native-lib.cpp:942-1034): header stage on new token ids.
    Returns (seq_bytes, [residual_bytes...]) like the JNI Object[]{byte[], byte[][]}; this build
    forwards only the hidden state, so the residual list is empty."""
    if not stage.is_first:
        raise BloomStageError("master (header) entry called on a non-first stage")
    ids = np.asarray(input_ids, dtype=np.int32).reshape(1, -1)
    hidden = stage.forward_host(ids, 1, ids.shape[1])
    return serialize_tensors([hidden]), []


def run_inference_worker_residual(stage: Stage, seq_bytes: bytes, residuals=(), to_send_seq_indices=(0,),
                                  to_send_res_indices=()):
    """runInferenceWorkerResidual (native-lib.cpp:1036-1194): middle stage, wire bytes in/out."""
    tensors = deserialize_tensors(seq_bytes)
    x = tensors[0].astype(np.float32, copy=False)
    S = x.shape[-2]
    hidden = stage.forward_host(x, 1, S)
    return serialize_tensors([hidden]), []


def run_inference_worker_residual_last_generation(stage: Stage, seq_bytes: bytes, residuals=(), k: int = 1,
                                                  initial_temp: float = 1.0, seed: int = 0) -> bytes:
    """runInferenceWorkerResidualLastGeneration (native-lib.cpp:1368-1443): tail stage, returns the
    next token id as 4 little-endian bytes (utils::SerializeInt).  k <= 1: greedy argmax; k > 1:
    the device top-k pick of decoding::StaticDecoding (decoding.cpp:24-66, bs_set_sampling), seeded
    by `seed` and keyed by the row's position, so every step draws afresh.  Like the reference
    (decoding.cpp:51-52), initial_temp is accepted and not applied."""
    tensors = deserialize_tensors(seq_bytes)
    x = tensors[0].astype(np.float32, copy=False)
    S = x.shape[-2]
    pick = (max(1, int(k)), int(seed))
    if getattr(stage, "_pick", (1, 0)) != pick:
        stage.set_sampling(pick[0], 1.0, pick[1])
        stage._pick = pick
    tok = stage.forward_host(x, 1, S)
    return serialize_int(int(tok[0]))


def run_inference_worker_residual_last_classification(stage: Stage, seq_bytes: bytes, residuals=()) -> bytes:
    """runInferenceWorkerResidualLastClassification (native-lib.cpp:1305-1366): classifier tail stage
    (Stage(..., n_labels=...)), returns the class of the sample -- the first index of the largest score logit,
    inference::binary_classify (inference.cpp:57-69) -- as 4 little-endian bytes (utils::SerializeInt)."""
    if not stage.n_labels:
        raise BloomStageError("classification entry called on a stage without a classifier head")
    x = deserialize_tensors(seq_bytes)[0].astype(np.float32, copy=False)
    cls = stage.forward_host(x, 1, x.shape[-2])
    return serialize_int(int(cls[0]))


def binary_classify(data: bytes) -> int:
    """binaryClassify (native-lib.cpp:128-160): the first tensor of a wire buffer holds logits; the class is the
    first index of the larger of its first two floats (bs_binary_classify)."""
    v = ctypes.c_int32()
    _check(lib().bs_binary_classify(bytes(data), len(data), ctypes.byref(v)))
    return v.value


def unpack_int_be(data: bytes) -> int:
    """Java-side big-endian int codec (Utils.java:107-125), for the sample-id frames."""
    return struct.unpack(">i", data)[0]
