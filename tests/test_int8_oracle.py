"""CPU side of the weight-only int8 variant (BS_FLAG_INT8_WEIGHTS): the quantization rule's
properties, the oracle's int8 mode, and the C-ABI's argument checks (no GPU needed)."""
import numpy as np
import pytest

from distributed_inference_demo_amd.stage import BloomStageError, Stage
from oracle import gen_np
from oracle.oracle import OracleStage


def test_int8_rule_properties():
    w = gen_np.bf16_round(gen_np.tensor(3, 0, 8, (64, 256)))  # layer 0 fc1 rows
    w[5] = 0.0
    q, sc = gen_np.int8_rows(w)
    assert q.dtype == np.int8 and np.abs(q.astype(np.int32)).max() <= 127
    assert sc[5] == 1.0 and not q[5].any()
    nz = np.arange(64) != 5
    assert (np.abs(q[nz].astype(np.int32)).max(axis=1) == 127).all()
    err = np.abs(q.astype(np.float32) * sc[:, None] - w)
    assert (err <= sc[:, None] * 0.501).all()  # half a step, plus fp32 rounding of w / scale and q * scale


def test_oracle_int8_close_to_bf16_but_not_equal():
    h, nh, L, V = 128, 4, 2, 512
    ids = gen_np.prompt_ids(2, 1, 8, V).astype(np.int32)
    a = OracleStage(h, nh, L, V, 0, L, bf16=True, max_ctx=8, seed=4)
    b = OracleStage(h, nh, L, V, 0, L, bf16=True, max_ctx=8, seed=4, int8=True)
    _, la = a.forward(ids, 1, 8, want_logits=True)
    _, lb = b.forward(ids, 1, 8, want_logits=True)
    assert not np.array_equal(la, lb)
    assert np.abs(la - lb).max() <= 0.05 * np.abs(la).max()


def test_oracle_int8_needs_bf16_mode():
    with pytest.raises(ValueError):
        OracleStage(64, 4, 1, 256, 0, 1, bf16=False, max_ctx=4, int8=True)


def test_int8_flag_rejected_on_fp32_stage():
    with pytest.raises(BloomStageError, match="BFLOAT16"):
        Stage(64, 4, 1, 256, 0, 1, dtype="fp32", max_ctx=4, int8_weights=True)


def test_int8_model_names():
    """The reference's model request names (server.py:796-799): "bloom560m" / "bloom560m-int8"."""
    from distributed_inference_demo_amd import config
    a, b = config.get("bloom560m"), config.get("bloom560m-int8")
    assert (a.name, a.int8_weights) == ("bloom-560m", False)
    assert (b.name, b.int8_weights, b.hidden, b.n_layer) == ("bloom-560m-int8", True, 1024, 24)
    assert config.get("bloom-7b1-int8").int8_weights and not config.get("7b1").int8_weights
