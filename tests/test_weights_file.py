"""Checkpoint-file stage init (bs_init_stage_file / bs_weights_file_probe), host side: the
safetensors reader and every check that runs before a device is touched.  createSession(model_path)
is the reference entry this replaces (native-lib.cpp:671-678, session_cache.h:26-35); the device
half (weights equal to the host-buffer and synthetic paths, forward parity) is in
tests/test_gpu_weights_file.py."""
import json
import os
import struct

import numpy as np
import pytest
import torch
from safetensors.torch import save_file

from distributed_inference_demo_amd.stage import BloomStageError, Stage, probe_weights_file
from oracle import gen_np

H, NH, L, V = 64, 4, 4, 512


def hf_tensors(seed=4, prefix=True, dtype=torch.float32):
    sd = gen_np.hf_state_dict(seed, H, L, V)
    out = {}
    for k, v in sd.items():
        if k == "lm_head.weight":
            continue  # tied: HF saves it once, as the embedding
        name = k if prefix else k.replace("transformer.", "", 1)
        out[name] = torch.from_numpy(np.ascontiguousarray(v)).to(dtype)
    return out


def write_sharded(tmp_path, tensors, n_shards=2):
    names = sorted(tensors)
    wm = {}
    for i in range(n_shards):
        part = {n: tensors[n] for n in names[i::n_shards]}
        fn = f"model-{i + 1:05d}-of-{n_shards:05d}.safetensors"
        save_file(part, str(tmp_path / fn))
        wm.update({n: fn for n in part})
    idx = tmp_path / "model.safetensors.index.json"
    idx.write_text(json.dumps({"metadata": {"total_size": 0}, "weight_map": wm}))
    return str(idx)


def test_probe_single_file_and_index(tmp_path):
    f = str(tmp_path / "model.safetensors")
    save_file(hf_tensors(prefix=False), f)
    assert probe_weights_file(f) == (H, L, V)
    assert probe_weights_file(write_sharded(tmp_path, hf_tensors())) == (H, L, V)


def test_probe_partial_checkpoint(tmp_path):
    """A middle-stage file (blocks only) says hidden and depth but not the vocabulary."""
    t = {k: v for k, v in hf_tensors().items() if ".h.1." in k or ".h.2." in k}
    f = str(tmp_path / "mid.safetensors")
    save_file(t, f)
    assert probe_weights_file(f) == (H, 3, -1)


def _stage_from(path, lb=0, le=L, **kw):
    return Stage(H, NH, L, V, lb, le, dtype="fp32", max_ctx=8, weights_file=path, **kw)


def test_missing_and_misshaped_tensors_fail_before_the_device(tmp_path):
    """These checks run before any HIP call, so they hold on a host without a GPU."""
    t = hf_tensors()
    f = str(tmp_path / "m.safetensors")
    save_file({k: v for k, v in t.items() if ".h.3." not in k}, f)
    with pytest.raises(BloomStageError, match=r"no tensor 'h\.3\.input_layernorm\.weight'"):
        _stage_from(f, 2, 4)
    t2 = dict(t)
    t2["transformer.h.1.mlp.dense_4h_to_h.weight"] = t2["transformer.h.1.mlp.dense_4h_to_h.weight"].t().contiguous()
    f2 = str(tmp_path / "m2.safetensors")
    save_file(t2, f2)
    with pytest.raises(BloomStageError, match=r"dense_4h_to_h\.weight' has shape \[256,64,\] but the stage needs \[64,256,\]"):
        _stage_from(f2, 0, 2)
    t3 = dict(t)
    t3["transformer.ln_f.bias"] = t3["transformer.ln_f.bias"].to(torch.int32)
    f3 = str(tmp_path / "m3.safetensors")
    save_file(t3, f3)
    with pytest.raises(BloomStageError, match="dtype I32"):
        _stage_from(f3, 2, 4)
    with pytest.raises(ValueError, match="not both"):
        Stage(H, NH, L, V, 0, L, dtype="fp32", weights_file=f, host_weights=np.zeros(4, np.float32))


def _raw(header: bytes, data: bytes = b"") -> bytes:
    return struct.pack("<Q", len(header)) + header + data


@pytest.mark.parametrize("blob,msg", [
    (b"\x05\x00", "too short"),
    (struct.pack("<Q", 1 << 40) + b"{}", "header length past the end"),
    (_raw(b'{"a": {"dtype": "F32", "shape": [2], "data_offsets": [0, 8]'), "malformed"),
    (_raw(b'{"a": {"dtype": "F32", "shape": [2], "data_offsets": [0, 8]}}', b"\0" * 4), "outside the data block"),
    (_raw(b'{"a": {"dtype": "F32", "shape": [3], "data_offsets": [0, 8]}}', b"\0" * 8), "disagree with its shape"),
    (_raw(b'{"a": {"dtype": "F32", "shape": [-2], "data_offsets": [0, 8]}}', b"\0" * 8), "bad shape"),
    (_raw(b'{"a": {"dtype": "Q4", "shape": [2], "data_offsets": [0, 8]}}', b"\0" * 8), "unknown dtype"),
    (_raw(b'{"a": {"dtype": "F32", "shape": [4294967296, 4294967296, 2], "data_offsets": [0, 8]}}', b"\0" * 8),
     "shape overflow"),
    (_raw(b'{"a": {"dtype": "F32", "shape": [2], "data_offsets": [8, 0]}}', b"\0" * 8), "outside the data block"),
    (_raw(b'{"a": {"dtype": "F32", "shape": [2]}}', b"\0" * 8), "bad tensor entry"),
])
def test_malformed_files_are_rejected(tmp_path, blob, msg):
    f = tmp_path / "bad.safetensors"
    f.write_bytes(blob)
    with pytest.raises(BloomStageError, match=msg):
        probe_weights_file(str(f))


def test_index_rejects_paths_outside_its_directory_and_missing_shards(tmp_path):
    idx = tmp_path / "m.index.json"
    idx.write_text(json.dumps({"weight_map": {"ln_f.weight": "../elsewhere.safetensors"}}))
    with pytest.raises(BloomStageError, match="bad shard name"):
        probe_weights_file(str(idx))
    save_file({"ln_f.weight": torch.zeros(H)}, str(tmp_path / "s.safetensors"))
    idx.write_text(json.dumps({"weight_map": {"ln_f.bias": "s.safetensors"}}))
    with pytest.raises(BloomStageError, match="does not hold it"):
        probe_weights_file(str(idx))
    with pytest.raises(BloomStageError, match="cannot open"):
        probe_weights_file(str(tmp_path / "absent.safetensors"))


def test_json_escapes_and_metadata(tmp_path):
    """Header strings with escapes and a __metadata__ block parse; names come back decoded."""
    hdr = json.dumps({"__metadata__": {"format": "pt", "note": "a\"b\\u00e9"},
                      "ln_f.weight": {"dtype": "BF16", "shape": [H], "data_offsets": [0, 2 * H]}}).encode()
    f = tmp_path / "e.safetensors"
    f.write_bytes(_raw(hdr, b"\0" * (2 * H)))
    assert probe_weights_file(str(f)) == (H, 0, -1)


def test_probe_reads_a_save_pretrained_checkpoint(tmp_path):
    """The names transformers itself writes (tied head dropped, sharded with an index)."""
    transformers = pytest.importorskip("transformers")
    cfg = transformers.BloomConfig(vocab_size=V, hidden_size=H, n_layer=L, n_head=NH)
    transformers.BloomForCausalLM(cfg).save_pretrained(str(tmp_path), safe_serialization=True, max_shard_size="200KB")
    idx = tmp_path / "model.safetensors.index.json"
    assert idx.exists()
    assert probe_weights_file(str(idx)) == (H, L, V)
