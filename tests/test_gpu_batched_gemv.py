"""Batched decode (4 < B <= 32 rows) through gemv_ldsw4 (kernels.hip: the weight stream read one 128-B
line per row per load and transposed through a per-wave LDS stage), bf16 and weight-only int8, against
the bf16-mode checker (oracle/bloom_oracle.c).  h = 1024 and 4h = 4096 make every block matrix a
multiple of the kernel's K parts (8 waves x 64 bf16 / 128 int8 columns), so all four GEMVs and the
argmax head run on it; ragged row counts (not a multiple of 16) exercise the clamped activation rows,
B > 16 the two-m-tile variant, and the N = h GEMVs its split-K (write-through partials + ticket).
The stage's parity bounds are tests/test_gpu_parity.py's (logits 2e-2 max-abs, ids by the checker's
top-2 margin); reference tail: inference.cpp:272-327."""
import numpy as np
import pytest

from oracle import gen_np

from test_gpu_int8 import pair8
from test_gpu_parity import assert_ids_match, check_logits, pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B", [5, 13, 17, 29])
@pytest.mark.parametrize("weights", ["bf16", "int8"])
def test_ldsw4_batched_decode_ragged_rows(B, weights):
    h, nh, L, V = 1024, 16, 2, 4096
    mk = pair8 if weights == "int8" else (lambda *a, **k: pair(*a[:6], "bf16", *a[6:], **k))
    gs, os_ = mk(h, nh, L, V, 0, L, seed=21, max_batch=B + 3, max_ctx=24, max_tokens=B * 4)
    ids = gen_np.prompt_ids(17, B, 4, V).astype(np.int32)
    gs.forward_host(ids, B, 4, slot=3, past_len=0)
    to = os_.forward(ids, B, 4, slot=3, past_len=0)
    for step in range(3):
        tg, lg = gs.forward_host(to.reshape(B, 1), B, 1, slot=3, past_len=4 + step, want_logits=True)
        to_n, lo = os_.forward(to.reshape(B, 1), B, 1, slot=3, past_len=4 + step, want_logits=True)
        check_logits(lg, lo, "bf16", f"{weights} B={B} decode step {step}")
        assert_ids_match(tg, to_n, lo, f"{weights} B={B} decode step {step}")
        to = to_n
    gs.close()
    os_.close()


@pytest.mark.parametrize("B", [8, 20])
def test_ldsw4_ragged_tile_columns(B):
    """bloom-3b widths (h = 2560): fc1 (N = 10240) runs 3-tile blocks, so its last block is ragged
    (10240 = 213 x 48 + 16), and fc2 (K = 10240) splits K in 2 (B <= 16) / 5 (B > 16) parts."""
    h, nh, L, V = 2560, 32, 1, 4096
    gs, os_ = pair(h, nh, L, V, 0, L, "bf16", seed=23, max_batch=B, max_ctx=16, max_tokens=B * 3)
    ids = gen_np.prompt_ids(29, B, 3, V).astype(np.int32)
    gs.forward_host(ids, B, 3, slot=0, past_len=0)
    to = os_.forward(ids, B, 3, slot=0, past_len=0)
    for step in range(2):
        tg, lg = gs.forward_host(to.reshape(B, 1), B, 1, slot=0, past_len=3 + step, want_logits=True)
        to_n, lo = os_.forward(to.reshape(B, 1), B, 1, slot=0, past_len=3 + step, want_logits=True)
        check_logits(lg, lo, "bf16", f"h=2560 B={B} decode step {step}")
        assert_ids_match(tg, to_n, lo, f"h=2560 B={B} decode step {step}")
        to = to_n
    gs.close()
    os_.close()


@pytest.mark.parametrize("B", [8, 32])
def test_batched_decode_middle_stage_offset_rows(B):
    """4 < B <= 32 (B <= 16: gemv_ldsw4 with the LayerNorm in its prologue; B > 16: ln_rows_wave_kernel + gemv_ldsw4): a 3-layer bloom-1b1-width middle stage fed hidden states
    with a large common offset (|mean| 20 x std: a plain one-pass sum-of-squares variance would cancel; the
    kernel's shifted sums must not) decodes 3 steps; every output within the wide-block bound."""
    h, nh, L, V = 1536, 16, 4, 2048
    gs, os_ = pair(h, nh, L, V, 1, 4, "bf16", seed=31, max_batch=B, max_ctx=16, max_tokens=B * 4, is_first=False,
                   is_last=False)
    rng = np.random.default_rng(7)
    x = (20.0 + rng.standard_normal((B, 4, h))).astype(np.float32)
    from test_gpu_parity import check_close
    check_close(gs.forward_host(x, B, 4, past_len=0), os_.forward(x, B, 4, past_len=0), "bf16", f"B={B} prefill")
    for step in range(3):
        x1 = (20.0 + rng.standard_normal((B, 1, h))).astype(np.float32)
        yg = gs.forward_host(x1, B, 1, past_len=4 + step)
        yo = os_.forward(x1, B, 1, past_len=4 + step)
        check_close(yg, yo, "bf16", f"B={B} offset-rows decode step {step}")
    gs.close()
    os_.close()


# bloom-7b1 width (h = 4096) hidden states of this 2-layer middle stage fed 5 + N(0, 1) rows (max |ref| ~18): constant
# bounds fixed from the committed multi-seed study (tools/parity_study_hidden.py, profiles/r06_parity_study_h4096_hidden.txt:
# 16 cases, B = 5 and 8, prefill + 3 decode steps).  Distances to the checker's default fp32 order: the device 0.043-0.064
# max-abs (mean-abs <= 0.0094), two other correct fp32 orders of the same rounded math 0.037-0.054, the float64 checker
# 0.032-0.048 -- the rounding noise of bf16 storage in any order; the 2e-2 + 2^-9 max|ref| formula was exceeded by one
# of the 16 cases (ratio 1.13), so at this width it gives way to:
H4096_HIDDEN_MAX_TOL = 8e-2   # 1.24x the device's largest distance in the study, 1.5x the CPU orders'
H4096_HIDDEN_MEAN_TOL = 1.25e-2


def check_h4096_hidden(got, ref, what):
    from test_gpu_parity import record_error
    err = record_error(what, got, ref, H4096_HIDDEN_MAX_TOL, "hidden bf16 (h=4096 study bound)")
    mean = float(np.abs(np.asarray(got, np.float64) - ref).mean())
    assert err <= H4096_HIDDEN_MAX_TOL and mean <= H4096_HIDDEN_MEAN_TOL, f"{what}: max-abs {err} mean-abs {mean}"


@pytest.mark.parametrize("h,nh", [(1024, 16), (2560, 32), (4096, 32)])
@pytest.mark.parametrize("B", [5, 7, 8])
def test_small_batch_decode_middle_stage_widths(h, nh, B):
    """4 < B <= 8 at the 560m / 3b / 7b1 widths (gemv_ldsw4 with the LayerNorm in its prologue at 560m / 3b; at 7b1 the
    K part is 8 stages per wave, beyond the prologue's register budget: ln_rows_wave_kernel first; split-K on the N = h GEMVs): a
    2-layer middle stage fed offset rows at a slot offset decodes 3 steps within the wide-block bound (h = 4096: the
    study's constant bound above)."""
    from test_gpu_parity import check_close as _cc
    check_close = (lambda g, o, dt, what: check_h4096_hidden(g, o, what)) if h == 4096 else _cc
    L, V = 3, 1024
    gs, os_ = pair(h, nh, L, V, 1, 3, "bf16", seed=41, max_batch=B + 1, max_ctx=16, max_tokens=B * 4, is_first=False,
                   is_last=False)
    rng = np.random.default_rng(9)
    x = (5.0 + rng.standard_normal((B, 4, h))).astype(np.float32)
    check_close(gs.forward_host(x, B, 4, slot=1, past_len=0), os_.forward(x, B, 4, slot=1, past_len=0), "bf16",
                f"h={h} B={B} prefill")
    for step in range(3):
        x1 = (5.0 + rng.standard_normal((B, 1, h))).astype(np.float32)
        check_close(gs.forward_host(x1, B, 1, slot=1, past_len=4 + step), os_.forward(x1, B, 1, slot=1, past_len=4 + step),
                    "bf16", f"h={h} B={B} decode step {step}")
    gs.close()
    os_.close()


@pytest.mark.parametrize("h,nh", [(2560, 32), (4096, 32)])
@pytest.mark.parametrize("B", [2, 3, 4])
def test_two_to_four_rows_decode_split_attention(h, nh, B):
    """2 <= B <= 4 at the 3b / 7b1 widths after a 260-token prefill (round-6 dispatch): the tile GEMV takes M = 3..4
    everywhere and M = 2 at these K; the split decode attention (2 splits at this cache size) merges its own partials
    at M = 3..4 and defers the merge to the dense rows GEMV at M = 2.  One middle layer, 3 decode steps."""
    from test_gpu_parity import check_close as _cc
    check_close = (lambda g, o, dt, what: check_h4096_hidden(g, o, what)) if h == 4096 else _cc
    L, V, P = 2, 1024, 260
    gs, os_ = pair(h, nh, L, V, 1, 2, "bf16", seed=43, max_batch=B, max_ctx=400, max_tokens=B * P, is_first=False,
                   is_last=False)
    rng = np.random.default_rng(11)
    x = (rng.standard_normal((B, P, h))).astype(np.float32)
    check_close(gs.forward_host(x, B, P, past_len=0), os_.forward(x, B, P, past_len=0), "bf16", f"h={h} B={B} prefill")
    for step in range(3):
        x1 = rng.standard_normal((B, 1, h)).astype(np.float32)
        check_close(gs.forward_host(x1, B, 1, past_len=P + step), os_.forward(x1, B, 1, past_len=P + step), "bf16",
                    f"h={h} B={B} decode step {step}")
    gs.close()
    os_.close()


@pytest.mark.parametrize("h,nh", [(1024, 16), (1536, 16), (2560, 32), (4096, 32)])
@pytest.mark.parametrize("B,S", [(3, 11), (2, 24), (1, 64), (4, 16)])
def test_short_prefill_four_m_tiles(h, nh, B, S):
    """33 <= B x S <= 64 tokens (a short prefill): fc2 (K = 4N) on the batched tile GEMV with four m-tiles (round 6;
    before, the prefill GEMM), split-K at bloom-1b1 / 3b / 7b1 widths; QKV / dense / fc1 on the prefill GEMMs.  Ragged
    row counts (33, 48), one row of 64 tokens, 4 rows of 16.  A 2-layer middle stage at a slot offset, then 2 decode
    steps of the same rows."""
    from test_gpu_parity import check_close as _cc
    check_close = (lambda g, o, dt, what: check_h4096_hidden(g, o, what)) if h == 4096 else _cc
    L, V = 3, 1024
    gs, os_ = pair(h, nh, L, V, 1, 3, "bf16", seed=47, max_batch=B + 1, max_ctx=S + 4, max_tokens=B * S,
                   is_first=False, is_last=False)
    rng = np.random.default_rng(13)
    x = (2.0 + rng.standard_normal((B, S, h))).astype(np.float32)
    check_close(gs.forward_host(x, B, S, slot=1, past_len=0), os_.forward(x, B, S, slot=1, past_len=0), "bf16",
                f"h={h} B={B} S={S} prefill")
    for step in range(2):
        x1 = (2.0 + rng.standard_normal((B, 1, h))).astype(np.float32)
        check_close(gs.forward_host(x1, B, 1, slot=1, past_len=S + step),
                    os_.forward(x1, B, 1, slot=1, past_len=S + step), "bf16", f"h={h} B={B} S={S} decode step {step}")
    gs.close()
    os_.close()
