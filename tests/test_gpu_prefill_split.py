"""GPU parity of the prefill attention's grid variants (attn_prefill.hip attn_prefill_tr_kernel).

When a prefill's (rows x heads x 64-query tiles) grid is under 256 blocks, each query tile's keys are
split over blocks of four 64-key tiles whose partial (max, sum, context) records the last-arriving block
merges in split order.  These cases run through that path and check the stage's hidden states against
the CPU checker (oracle/bloom_oracle.c, bf16 mode) at the wide-block bound, per row and per query tile:
  * head dims 64 / 96 / 128 (hidden 1024 / 1536 / 2048, 16 heads);
  * one row, 512 tokens from an empty cache (8 query tiles, 1..8 key tiles, 2 splits);
  * two rows continuing from different cached lengths (130 and 450 positions, per-row bs_step.past_lens):
    row 1's last query tile sees 11 key tiles (3 splits), row 0's at most 6, so its third split is empty;
  * short prompts (130 tokens: 3 key tiles, one block per query tile) that seed the continuation;
  * many rows (8 x 512 tokens, 16 heads: 512 blocks of 128 queries) -- two 16-query groups per wave.
"""
import numpy as np
import pytest

from distributed_inference_demo_amd.stage import Stage
from oracle.oracle import OracleStage

from test_gpu_parity import check_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("h", [1024, 1536, 2048])
def test_prefill_split_kv_one_row_512(h):
    nh, S = 16, 512
    gs = Stage(h, nh, 1, 512, 0, 1, dtype="bf16", max_batch=1, max_ctx=S, max_tokens=S, seed=101,
               is_first=False, is_last=False)
    os_ = OracleStage(h, nh, 1, 512, 0, 1, bf16=True, max_batch=1, max_ctx=S, seed=101, is_first=False,
                      is_last=False)
    x = np.random.default_rng(7).standard_normal((1, S, h)).astype(np.float32)
    yg = gs.forward_host(x, 1, S, past_len=0)
    yo = os_.forward(x, 1, S, past_len=0)
    err = check_close(yg, yo, "bf16", f"h={h} prefill 1x{S}")
    for t in range(0, S, 64):
        check_close(yg[:, t:t + 64], yo[:, t:t + 64], "bf16", f"h={h} query tile {t // 64}")
    print(f"h={h}: prefill 1x{S} max-abs {err:.3e}")
    gs.close()
    os_.close()


@pytest.mark.parametrize("h", [1024, 1536])
def test_prefill_split_kv_two_rows_continuing_from_different_lengths(h):
    nh, S2, L = 16, 200, 2
    lens = [130, 450]
    kw = dict(max_batch=2, max_ctx=1024, seed=103, is_first=False, is_last=False)
    gs = Stage(h, nh, L, 512, 0, L, dtype="bf16", max_tokens=2 * 512, **kw)
    os_ = OracleStage(h, nh, L, 512, 0, L, bf16=True, **kw)
    rng = np.random.default_rng(11)
    for r, n in enumerate(lens):
        x = rng.standard_normal((1, n, h)).astype(np.float32)
        yg = gs.forward_host(x, 1, n, slot=r, past_len=0)
        yo = os_.forward(x, 1, n, slot=r, past_len=0)
        check_close(yg, yo, "bf16", f"h={h} row {r} prompt {n}")
    x = rng.standard_normal((2, S2, h)).astype(np.float32)
    yg = gs.forward_host(x, 2, S2, past_len=lens)
    for r in range(2):
        yo = os_.forward(x[r:r + 1], 1, S2, slot=r, past_len=lens[r])
        err = check_close(yg[r:r + 1], yo, "bf16", f"h={h} row {r} continuation from {lens[r]}")
        for t in range(0, S2, 64):
            check_close(yg[r:r + 1, t:t + 64], yo[:, t:t + 64], "bf16", f"h={h} row {r} query tile {t // 64}")
        print(f"h={h} row {r}: continuation {S2} after {lens[r]} max-abs {err:.3e}")
    gs.close()
    os_.close()


@pytest.mark.parametrize("h", [1024, 1536, 2048])
def test_prefill_two_query_groups_many_rows(h):
    """8 rows x 512 tokens (16 heads): 8 x 16 x 4 = 512 blocks of 128 queries, so every wave takes two 16-query
    groups (each K fragment and transposed V read feeds two MFMAs).  Hidden states per row and per 64-query tile
    against the checker."""
    nh, B, S = 16, 8, 512
    gs = Stage(h, nh, 1, 512, 0, 1, dtype="bf16", max_batch=B, max_ctx=S + 256, max_tokens=B * S, seed=103,
               is_first=False, is_last=False)
    os_ = OracleStage(h, nh, 1, 512, 0, 1, bf16=True, max_batch=B, max_ctx=S + 256, seed=103, is_first=False,
                      is_last=False)
    rng = np.random.default_rng(11)
    x = rng.standard_normal((B, S, h)).astype(np.float32)
    yg = gs.forward_host(x, B, S, past_len=0)
    yo = os_.forward(x, B, S, past_len=0)
    err = check_close(yg, yo, "bf16", f"h={h} prefill {B}x{S}")
    for bi in (0, B - 1):
        for t in range(0, S, 64):
            check_close(yg[bi:bi + 1, t:t + 64], yo[bi:bi + 1, t:t + 64], "bf16", f"h={h} row {bi} query tile {t // 64}")
    print(f"h={h}: two-query-group prefill {B}x{S} max-abs {err:.3e}")
    gs.close()
    os_.close()


def test_prefill_256_tiles_bitwise_equal_to_128_tiles():
    """Big prefills (>= 512 whole 256 x 256 tiles, K <= 8192) run gemm_mfma3 on 256 x 256 tiles (round 6); every output
    element sums K in the same order as the 128 x 128 path, so a bloom-7b1-width layer over 16 rows x 512 tokens (QKV,
    dense, fc1 on 256 x 256 tiles: 1536 / 512 / 2048 tiles; fc2, K = 16384, stays on 128 x 128) gives the same bits
    with the big tiles switched off (BS_GEMM_BIG=0): hidden states and the K/V rows written by the QKV epilogue."""
    import os
    h, nh, B, S = 4096, 32, 16, 512
    x = (0.5 * np.random.default_rng(21).standard_normal((B, S, h))).astype(np.float32)
    out = {}
    for big in ("1", "0"):
        os.environ["BS_GEMM_BIG"] = big
        try:
            gs = Stage(h, nh, 1, 512, 0, 1, dtype="bf16", max_batch=B, max_ctx=S, max_tokens=B * S, seed=7,
                       is_first=False, is_last=False)
            y = gs.forward_host(x, B, S, past_len=0)
            kv = gs.read_kv(0, B - 1, 0, S)
            gs.close()
        finally:
            os.environ.pop("BS_GEMM_BIG", None)
        out[big] = (y, kv)
    assert np.isfinite(out["1"][0]).all()
    assert np.array_equal(out["1"][0].view(np.uint32), out["0"][0].view(np.uint32))
    assert np.array_equal(out["1"][1].view(np.uint32), out["0"][1].view(np.uint32))
