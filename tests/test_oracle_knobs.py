"""The checker's diagnostic knobs used by the bf16 parity study (tools/parity_study.py): the fp16 rounding that
emulates the device's V staging, the alternative fp32 accumulation orders, and the P.V emulation modes.  CPU only."""
import numpy as np

from oracle.oracle import OracleStage, checker_mode, prompt_ids, round_fp16


def test_round_fp16_matches_numpy():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(20000).astype(np.float32) * s for s in (1e-6, 1e-4, 1.0, 100.0, 3e4)])
    x = np.concatenate([x, np.float32([0.0, -0.0, 65504.0, 65519.0, 65520.0, -70000.0, 6.1e-5, 2.0 ** -25,
                                       3 * 2.0 ** -26, 1 + 2.0 ** -11, 1 + 3 * 2.0 ** -11])])
    with np.errstate(over="ignore"):
        want = x.astype(np.float16).astype(np.float32)
    got = round_fp16(x)
    assert np.array_equal(got, want, equal_nan=True), x[got != want][:8]


def _logits(accum, emul, seed=3):
    h, nh, L, V, B, S = 128, 4, 2, 512, 2, 9
    o = OracleStage(h, nh, L, V, 0, L, bf16=True, max_batch=B, max_ctx=S, seed=seed)
    with checker_mode(accum, emul):
        _, lg = o.forward(prompt_ids(11, B, S, V), B, S, want_logits=True)
    o.close()
    return lg


def test_accumulation_orders_and_pv_emulation_stay_within_fp32_noise():
    ref = _logits(1, 0)  # float64 dot products
    for accum in (0, 2, 3):
        for emul in (0, 1 | 2, 4):
            d = float(np.abs(_logits(accum, emul) - ref).max())
            assert d < 2e-3, (accum, emul, d)
    assert np.array_equal(_logits(0, 0), _logits(0, 0))  # knobs reset after the block
