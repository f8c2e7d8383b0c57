"""CPU tests: wire codec (byte-exact vs the utils.cpp restatement), stage placement
(server.py:893-905), and the C-ABI library's exports (no compute without a GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import codec_ref
from distributed_inference_demo_amd import stage as bs
from distributed_inference_demo_amd.placement import round_robin_module_arrangement, stage_ranges

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_codec_known_answer():
    # one fp32 [1,2] tensor of ones: n=1 | type 1 | ndim 2 | dims 1,2 | 2 floats
    want = bytes.fromhex("0100000000000000" "01000000" "0200000000000000" "0100000000000000"
                         "0200000000000000" "0000803f" "0000803f")
    assert bs.serialize_tensors([np.ones((1, 2), np.float32)]) == want
    assert codec_ref.serialize([np.ones((1, 2), np.float32)]) == want
    # the tail's 4-byte token (utils.cpp:11-15)
    assert bs.serialize_int(250879) == (250879).to_bytes(4, "little")
    assert bs.deserialize_int(bs.serialize_int(-7)) == -7


def test_codec_roundtrip_all_reference_dtypes():
    rng = np.random.default_rng(0)
    arrays = [rng.standard_normal((1, 5, 16)).astype(np.float32), np.arange(7, dtype=np.int64).reshape(1, 7),
              np.array([[1, 0, 1]], np.bool_), rng.integers(-100, 100, (3, 2, 2)).astype(np.int8),
              rng.integers(0, 255, (4,)).astype(np.uint8), np.arange(6, dtype=np.uint16),
              np.arange(6, dtype=np.int16), np.arange(6, dtype=np.int32), np.arange(3, dtype=np.float64),
              np.arange(3, dtype=np.uint32), np.arange(3, dtype=np.uint64), np.zeros((0, 4), np.float32),
              np.float32(3.5).reshape(())]
    wire = bs.serialize_tensors(arrays)
    assert wire == codec_ref.serialize(arrays)
    for a, b in zip(arrays, bs.deserialize_tensors(wire)):
        assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b)
    for a, b in zip(arrays, codec_ref.deserialize(wire)):
        assert np.array_equal(a, b)


def test_codec_empty_vector_and_errors():
    assert bs.serialize_tensors([]) == bytes(8)
    assert bs.deserialize_tensors(bytes(8)) == []
    wire = bs.serialize_tensors([np.ones((2, 3), np.float32)])
    with pytest.raises(bs.BloomStageError):
        bs.deserialize_tensors(wire[:-1])  # truncated payload
    with pytest.raises(bs.BloomStageError):
        bs.serialize_tensors([np.ones(3, np.float16)])  # not carried by the reference codec
    bad = bytearray(wire)
    bad[8:12] = (10).to_bytes(4, "little")  # FLOAT16 tag
    with pytest.raises(bs.BloomStageError):
        bs.deserialize_tensors(bytes(bad))
    with pytest.raises(bs.BloomStageError):
        bs.deserialize_int(b"\x01\x02\x03")


@pytest.mark.parametrize("dims", [(2 ** 62, 4), (2 ** 32, 2 ** 32), (2 ** 63 - 1, 2 ** 63 - 1, 2)])
def test_codec_rejects_wrapping_wire_shapes(dims):
    """A crafted header whose element count (or count x element size) wraps uint64 must be rejected,
    not handed back as a view whose dims describe more bytes than the buffer holds."""
    hdr = (1).to_bytes(8, "little") + (1).to_bytes(4, "little") + len(dims).to_bytes(8, "little")
    hdr += b"".join(int(d).to_bytes(8, "little") for d in dims)
    with pytest.raises(bs.BloomStageError):
        bs.deserialize_tensors(hdr + bytes(16))


@pytest.mark.parametrize("dev,mods", [(1, 24), (2, 24), (4, 30), (8, 30), (3, 2), (2, 2), (5, 3)])
def test_round_robin_matches_reference_semantics(dev, mods):
    arr = round_robin_module_arrangement(dev, mods)
    assert arr.shape == (dev, mods)
    assert (arr.sum(0) == 1).all()  # every module placed exactly once
    counts = arr.sum(1)
    per, extra = divmod(mods, dev)
    assert list(counts) == [per + (1 if i < extra else 0) for i in range(dev)]
    for row in arr:  # contiguous
        idx = np.flatnonzero(row)
        assert idx.size == 0 or (np.diff(idx) == 1).all()


def test_stage_ranges_survey_table():
    assert stage_ranges(2, 24) == [(0, 12), (12, 24)]
    assert stage_ranges(4, 30) == [(0, 8), (8, 16), (16, 23), (23, 30)]
    assert [b - a for a, b in stage_ranges(8, 30)] == [4, 4, 4, 4, 4, 4, 3, 3]


def test_library_exports_every_declared_symbol():
    header = open(os.path.join(ROOT, "include", "bloomstage.h")).read()
    header = re.sub(r"/\*.*?\*/", "", header, flags=re.S)  # drop comments
    header = re.sub(r"//[^\n]*", "", header)
    declared = set(re.findall(r"\b(bs_[a-z_0-9]+)\s*\(", header))
    assert declared, "no declarations parsed"
    L = bs.lib()
    for name in sorted(declared):
        assert hasattr(L, name), f"{name} declared in bloomstage.h but not exported"
    assert set(bs.EXPORTS) <= declared


def test_weight_count_matches_canonical_layout():
    h, V = 64, 512
    n = bs.weight_count(hidden=h, n_head=4, n_layer=4, vocab=V, ln_eps=1e-5, layer_begin=0, layer_end=2,
                        is_first=1, is_last=0, dtype=16, max_batch=1, max_ctx=8)
    assert n == V * h + 2 * h + 2 * (12 * h * h + 13 * h)
    n2 = bs.weight_count(hidden=h, n_head=4, n_layer=4, vocab=V, ln_eps=1e-5, layer_begin=2, layer_end=4,
                         is_first=0, is_last=1, dtype=16, max_batch=1, max_ctx=8)
    assert n2 == V * h + 2 * h + 2 * (12 * h * h + 13 * h)
    bad = bs.weight_count(hidden=65, n_head=4, n_layer=4, vocab=V, ln_eps=1e-5, layer_begin=0, layer_end=2,
                          is_first=1, is_last=0, dtype=16, max_batch=1, max_ctx=8)
    assert bad == 0


def test_weight_count_classifier_tail():
    """BS_FLAG_CLASSIFIER: a last-only classifier stage holds no word_embeddings, ln_f and score [n_labels][h];
    a whole-model classifier keeps the embedding (it is first).  Bad n_labels / non-last stages / head slices
    are rejected (count 0)."""
    h, V = 64, 512
    kw = dict(hidden=h, n_head=4, n_layer=4, vocab=V, ln_eps=1e-5, dtype=16, max_batch=1, max_ctx=8,
              flags=bs.BS_FLAG_CLASSIFIER)
    assert bs.weight_count(layer_begin=2, layer_end=4, is_first=0, is_last=1, n_labels=2, **kw) == \
        2 * (12 * h * h + 13 * h) + 2 * h + 2 * h
    assert bs.weight_count(layer_begin=0, layer_end=4, is_first=1, is_last=1, n_labels=3, **kw) == \
        V * h + 2 * h + 4 * (12 * h * h + 13 * h) + 2 * h + 3 * h
    assert bs.weight_count(layer_begin=2, layer_end=4, is_first=0, is_last=1, n_labels=0, **kw) == 0
    assert bs.weight_count(layer_begin=2, layer_end=4, is_first=0, is_last=1, n_labels=65, **kw) == 0
    assert bs.weight_count(layer_begin=0, layer_end=2, is_first=1, is_last=0, n_labels=2, **kw) == 0
    assert bs.weight_count(layer_begin=2, layer_end=4, is_first=0, is_last=1, n_labels=2, head_vocab_begin=0,
                           head_vocab_end=64, **kw) == 0


def test_binary_classify_on_wire_bytes():
    """binaryClassify (native-lib.cpp:128-160): first tensor = logits, first index of the larger of the first
    two floats (inference.cpp:57-69); ties keep index 0; errors instead of the reference's -1 / -2 / over-read."""
    assert bs.binary_classify(bs.serialize_tensors([np.array([[0.1, 0.7]], np.float32)])) == 1
    assert bs.binary_classify(bs.serialize_tensors([np.array([[0.7, 0.1, 9.0]], np.float32)])) == 0
    assert bs.binary_classify(bs.serialize_tensors([np.array([0.5, 0.5], np.float32), np.ones(3, np.int64)])) == 0
    assert bs.binary_classify(bs.serialize_tensors([np.array([-np.inf, -1e30], np.float32)])) == 1
    for bad in ([], [np.array([1.0], np.float32)], [np.array([1, 2], np.int32)]):
        with pytest.raises(bs.BloomStageError):
            bs.binary_classify(bs.serialize_tensors(bad))
    with pytest.raises(bs.BloomStageError):
        bs.binary_classify(b"\x01\x00")


def test_init_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(bs.BloomStageError):
        bs.Stage(64, 4, 4, 512, 0, 4, max_ctx=16)


def test_library_prompt_ids_match_generator():
    from oracle import gen_np
    assert np.array_equal(bs.prompt_ids(1234, 3, 40, 250880), gen_np.prompt_ids(1234, 3, 40, 250880))
