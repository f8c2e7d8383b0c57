"""oracle/oracle.py — TEST INFRASTRUCTURE: ctypes loader for the CPU checker
(oracle/liboracle.so, built by oracle/Makefile).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg import this; the product path never does.
"""
import ctypes
import os
import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(path)
        L.or_create.restype = ctypes.c_void_p
        L.or_create.argtypes = [ctypes.c_int] * 4 + [ctypes.c_float] + [ctypes.c_int] * 7 + [ctypes.c_uint64]
        L.or_destroy.argtypes = [ctypes.c_void_p]
        L.or_forward.restype = ctypes.c_int
        L.or_forward.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 4 + [ctypes.c_void_p] * 3
        L.or_gen_tensor.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
        L.or_prompt_ids.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.or_alibi_slopes.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.or_read_kv.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p]
        L.or_num_threads.restype = ctypes.c_int
        L.or_write_kv.restype = ctypes.c_int
        L.or_write_kv.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 4 + [ctypes.c_void_p]
        L.or_set_accum_double.argtypes = [ctypes.c_int]
        L.or_set_accum_mode.argtypes = [ctypes.c_int]
        L.or_set_emul_pv.argtypes = [ctypes.c_int]
        L.or_round_fp16.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.or_set_skip_round.argtypes = [ctypes.c_int]
        L.or_set_classifier.restype = ctypes.c_int
        L.or_set_classifier.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64]
        L.or_quantize_int8.restype = ctypes.c_int
        L.or_quantize_int8.argtypes = [ctypes.c_void_p]
        L.or_head_norm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.or_head_slice.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def gen_tensor(seed, layer, tid, n):
    out = np.empty(n, dtype=np.float32)
    lib().or_gen_tensor(seed, layer, tid, n, _p(out))
    return out


def prompt_ids(seed, batch, seq, vocab):
    out = np.empty(batch * seq, dtype=np.int32)
    lib().or_prompt_ids(seed, batch * seq, vocab, _p(out))
    return out.reshape(batch, seq)


def alibi_slopes(n_head):
    out = np.empty(n_head, dtype=np.float32)
    lib().or_alibi_slopes(n_head, _p(out))
    return out


def round_fp16(x):
    """The checker's fp32 -> fp16 rounding (or_set_emul_pv bit 1), for its test against numpy."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    lib().or_round_fp16(_p(x), _p(out), x.size)
    return out


class checker_mode:
    """Context manager: the checker's accumulation order (or_set_accum_mode) and P.V emulation
    (or_set_emul_pv) for the calls inside the block -- global knobs of liboracle."""

    def __init__(self, accum=0, emul_pv=0):
        self.accum, self.emul = accum, emul_pv

    def __enter__(self):
        lib().or_set_accum_mode(self.accum)
        lib().or_set_emul_pv(self.emul)
        return self

    def __exit__(self, *a):
        lib().or_set_accum_mode(0)
        lib().or_set_emul_pv(0)
        return False


# or_set_emul_pv bits that model the bf16 device library's P.V staging: bf16 hi + lo P against bf16 V, normalised
# after the product, in the prefill kernel (attn_prefill.hip); fp32 unnormalised P in the decode kernel (S = 1)
EMUL_DEVICE = 4 | 8


def num_threads():
    return lib().or_num_threads()


class OracleStage:
    """CPU checker for one pipeline stage; same call semantics as the product Stage."""

    def __init__(self, hidden, n_head, n_layer, vocab, layer_begin, layer_end, *, bf16=False,
                 max_batch=1, max_ctx=64, seed=0, eps=1e-5, is_first=None, is_last=None, int8=False, emul_pv=None,
                 n_labels=0):
        """n_labels > 0: a sequence-classification tail (or_set_classifier): the last stage emits class ids and
        fp32 logits [B][n_labels] instead of tokens and vocabulary logits."""
        self.hidden, self.vocab = hidden, vocab
        self.n_out = n_labels if n_labels else vocab
        self.emul = emul_pv  # None: the global knob as set (checker_mode); else this stage's own P.V mode per call
        self.is_first = layer_begin == 0 if is_first is None else is_first
        self.is_last = layer_end == n_layer if is_last is None else is_last
        self.h = lib().or_create(hidden, n_head, n_layer, vocab, eps, layer_begin, layer_end,
                                 int(self.is_first), int(self.is_last), int(bf16), max_batch, max_ctx, seed)
        if not self.h:
            raise ValueError("or_create failed (bad stage description)")
        if int8 and lib().or_quantize_int8(self.h) != 0:  # weight-only int8 (BS_FLAG_INT8_WEIGHTS)
            raise ValueError("or_quantize_int8 needs a bf16-mode stage")
        if n_labels and lib().or_set_classifier(self.h, n_labels, seed) != 0:
            raise ValueError("or_set_classifier needs a last stage and n_labels >= 1")

    def forward(self, x, B, S, slot=0, past_len=0, want_logits=False):
        if self.is_first:
            x = np.ascontiguousarray(x, dtype=np.int32).reshape(B, S)
        else:
            x = np.ascontiguousarray(x, dtype=np.float32).reshape(B, S, self.hidden)
        logits = np.empty((B, self.n_out), dtype=np.float32) if (self.is_last and want_logits) else None
        out = np.empty(B, dtype=np.int32) if self.is_last else np.empty((B, S, self.hidden), dtype=np.float32)
        if self.emul is None:
            rc = lib().or_forward(self.h, B, S, slot, past_len, _p(x), _p(out), _p(logits))
        else:
            lib().or_set_emul_pv(self.emul)
            try:
                rc = lib().or_forward(self.h, B, S, slot, past_len, _p(x), _p(out), _p(logits))
            finally:
                lib().or_set_emul_pv(0)
        if rc != 0:
            raise ValueError(f"or_forward failed rc={rc}")
        return (out, logits) if want_logits else out

    def head_norm(self, hidden, B, S):
        hidden = np.ascontiguousarray(hidden, dtype=np.float32).reshape(B, S, self.hidden)
        xn = np.empty((B, self.hidden), np.float32)
        if lib().or_head_norm(self.h, _p(hidden), B, S, _p(xn)) != 0:
            raise ValueError("or_head_norm needs a stage with the head (is_last)")
        return xn

    def head_slice(self, xn, B, v0, v1, keys_in=None):
        xn = np.ascontiguousarray(xn, dtype=np.float32).reshape(B, self.hidden)
        keys = np.empty(B, np.uint64)
        toks = np.empty(B, np.int32)
        kin = None if keys_in is None else np.ascontiguousarray(keys_in, dtype=np.uint64)
        if lib().or_head_slice(self.h, _p(xn), B, v0, v1, _p(kin), _p(keys), _p(toks)) != 0:
            raise ValueError("or_head_slice failed")
        return keys, toks

    def read_kv(self, layer_local, which, row, head, pos, head_dim):
        out = np.empty(head_dim, dtype=np.float32)
        lib().or_read_kv(self.h, layer_local, which, row, head, pos, _p(out))
        return out

    def write_kv(self, layer_local, row, pos0, kv):
        """Overwrite KV row `row` of local layer `layer_local` from kv fp32 [2][n_head][npos][hd] (e.g. a
        device cache read back with Stage.read_kv)."""
        kv = np.ascontiguousarray(kv, dtype=np.float32)
        if lib().or_write_kv(self.h, layer_local, row, pos0, kv.shape[2], _p(kv)) != 0:
            raise ValueError("or_write_kv: range outside the stage")

    def close(self):
        if self.h:
            lib().or_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
