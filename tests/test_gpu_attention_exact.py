"""Attention kernels pinned element by element, free of the bf16 rounding-flip noise of whole-block checks.

A one-layer middle stage (bf16) gets host weights that make everything around the attention exact:
  * ln1 gamma = 1, beta = 0; the fused QKV weight is one-hot (HF per-head interleave [heads][3][hd]): q of head j =
    xn slice j, k of head j = xn slice j + 1, v of head j = xn slice j + 2 (mod n_head), zero bias -- the GEMM sums one
    exact product per output, so q / K / V are the device's own bf16 xn values, copied;
  * dense = identity, zero bias: the residual stream becomes a = x + ctx exactly (fp32 sum of ONE product);
  * fc1, fc2 and their biases zero: the MLP adds exactly 0, so the stage output is x + ctx.
So ctx = out - x (x ~ N(0, 0.01^2): the fp32 add loses < 1e-8), and the exact inputs of the attention are known from
the device's own KV cache (bs_read_kv): K_j and V_j directly, q_j = K_{j-1} at the query's position (the same xn slice,
the same bf16 rounding); V_j == K_{j+1} is checked bit for bit.  Reference: float64 HF BLOOM attention
(modeling_bloom.py:245-310: scores = alibi + q.k / sqrt(hd), causal mask, softmax, P.V) on those inputs.

Bound per element: |ctx_dev - ctx_ref| <= 0.5 ulp_bf16(ctx_ref) (the device rounds the context to bf16)
+ 2^-14 max|V| of the (row, head) (P through the MFMAs as bf16 hi + lo keeps ~16 bits; fp32 accumulation).  A wrong
key, mask, scale, split merge or XCD grouping moves elements by far more.

Grid variants (attn_prefill.hip attn_prefill_tr_launch / kernels.hip attention_decode_splits), one case each:
split-KV (1 row x 512, 16 heads, hd 64 / 96 / 128), two key groups (2 rows x 512, 16 heads: 256 one-block units),
two query groups (8 rows x 512, 16 heads), per-row past lengths (continuations from 130 and 450), hd 80 (padded to
96), and decode (S = 1) with the context split over blocks and merged in the dense GEMV's prologue (B = 1, 3).
"""
import numpy as np
import pytest

from distributed_inference_demo_amd.stage import Stage
from oracle.oracle import alibi_slopes

from test_gpu_parity import record_error

pytestmark = pytest.mark.gpu


def identity_attention_weights(h, nh):
    """BS_WEIGHTS_HOST layout of one middle-stage layer (tests/test_gpu_parity.py canonical_weights order)."""
    hd = h // nh
    wqkv = np.zeros((3 * h, h), np.float32)
    ar = np.arange(hd)
    for j in range(nh):
        for which, src in ((0, j), (1, (j + 1) % nh), (2, (j + 2) % nh)):
            wqkv[j * 3 * hd + which * hd + ar, src * hd + ar] = 1.0
    parts = [np.ones(h), np.zeros(h), wqkv, np.zeros(3 * h), np.eye(h, dtype=np.float32), np.zeros(h),
             np.ones(h), np.zeros(h), np.zeros((4 * h, h)), np.zeros(4 * h), np.zeros((h, 4 * h)), np.zeros(h)]
    return np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in parts])


def bf16_ulp(x):
    a = np.abs(x)
    e = np.floor(np.log2(np.maximum(a, 2.0 ** -126)))
    return 2.0 ** (e - 7)


class AttnStage:
    def __init__(self, h, nh, max_batch, max_ctx, max_tokens):
        self.h, self.nh, self.hd = h, nh, h // nh
        self.st = Stage(h, nh, 1, 512, 0, 1, dtype="bf16", max_batch=max_batch, max_ctx=max_ctx,
                        max_tokens=max_tokens, host_weights=identity_attention_weights(h, nh), is_first=False,
                        is_last=False)
        self.slopes = alibi_slopes(nh).astype(np.float64)
        self.inv_norm = float(np.float32(1.0) / np.sqrt(np.float32(self.hd)))

    def run_and_check(self, x, B, S, slot, pasts, what):
        """Forward x [B, S, h] at KV rows slot.. with per-row cached lengths; check every context element."""
        out = self.st.forward_host(x, B, S, slot=slot, past_len=list(pasts))
        ctx = (out.astype(np.float64) - x.astype(np.float64)).reshape(B, S, self.nh, self.hd)
        worst = 0.0
        for b in range(B):
            n = pasts[b] + S
            kv = self.st.read_kv(0, slot + b, 0, n).astype(np.float64)  # [2][nh][n][hd]
            K, V = kv[0], kv[1]
            assert np.array_equal(V, np.roll(K, -1, axis=0)), f"{what}: V_j != K_(j+1) in row {b}"
            for j in range(self.nh):
                q = K[(j - 1) % self.nh, pasts[b]:n]                     # [S][hd]
                s = self.inv_norm * (q @ K[j].T) + self.slopes[j] * np.arange(n)[None, :]
                s[np.arange(n)[None, :] > (pasts[b] + np.arange(S))[:, None]] = -np.inf
                p = np.exp(s - s.max(axis=1, keepdims=True))
                ref = (p @ V[j]) / p.sum(axis=1, keepdims=True)          # [S][hd]
                got = ctx[b, :, j, :]
                slack = 2.0 ** -14 * np.abs(V[j]).max() + 1e-7  # what the device may add to the half-ulp rounding
                over = (np.abs(got - ref) - 0.5 * bf16_ulp(ref)) / slack
                worst = max(worst, float(over.max()))
                bad = np.argwhere(over > 1.0)
                assert bad.size == 0, (f"{what}: row {b} head {j} query {bad[0][0]} dim {bad[0][1]}: "
                                       f"{got[tuple(bad[0])]} vs {ref[tuple(bad[0])]}")
        record_error(what + " [attention exact: worst (error - half ulp) / slack]", np.array([worst]), np.array([0.0]),
                     1.0, "attention exact")
        return worst


def _x(rng, B, S, h):
    return (0.01 * rng.standard_normal((B, S, h))).astype(np.float32)


@pytest.mark.parametrize("hd", [64, 96, 128])
def test_prefill_split_kv_exact(hd):
    """1 row x 512 tokens, 16 heads: 128 query-tile units < 256 -> each query tile's keys split over two blocks,
    merged by the last arriver."""
    nh, S = 16, 512
    a = AttnStage(nh * hd, nh, 1, S + 8, S)
    w = a.run_and_check(_x(np.random.default_rng(1), 1, S, nh * hd), 1, S, 0, [0], f"split-KV hd={hd} 1x{S}")
    print(f"hd={hd}: worst (error - half ulp) / slack {w:.3f}")


@pytest.mark.parametrize("hd", [96, 128])
def test_prefill_two_key_groups_exact(hd):
    """2 rows x 512 tokens, 16 heads: 256 unsplit units, >= 8 key tiles -> 8-wave blocks, two key groups merged in LDS."""
    nh, B, S = 16, 2, 512
    a = AttnStage(nh * hd, nh, B, S + 8, B * S)
    a.run_and_check(_x(np.random.default_rng(2), B, S, nh * hd), B, S, 0, [0, 0], f"two key groups hd={hd} {B}x{S}")


def test_prefill_two_query_groups_exact():
    """8 rows x 512 tokens, 16 heads: 512 blocks of 128 queries (two 16-query groups per wave)."""
    nh, hd, B, S = 16, 64, 8, 512
    a = AttnStage(nh * hd, nh, B, S + 8, B * S)
    a.run_and_check(_x(np.random.default_rng(3), B, S, nh * hd), B, S, 0, [0] * B, f"two query groups {B}x{S}")


def test_prefill_continuations_from_different_lengths_exact():
    """Two rows at KV rows 1, 2 holding 130 and 450 cached positions, 200 new tokens each (per-row past lengths):
    row 1's last query tile sees 11 key tiles (3 splits), row 0's at most 6."""
    nh, hd = 16, 96
    h = nh * hd
    a = AttnStage(h, nh, 3, 1024, 2 * 512)
    rng = np.random.default_rng(4)
    for r, n in enumerate((130, 450)):
        a.run_and_check(_x(rng, 1, n, h), 1, n, 1 + r, [0], f"prompt {n}")
    a.run_and_check(_x(rng, 2, 200, h), 2, 200, 1, [130, 450], "continuation 200 after 130 / 450")


def test_prefill_head_dim_80_exact():
    """hd 80 (bloom-3b) padded to 96 in LDS: lanes past hd re-read finite data multiplied by Q's zero dims."""
    nh, hd, S = 16, 80, 300
    a = AttnStage(nh * hd, nh, 1, S + 8, S)
    a.run_and_check(_x(np.random.default_rng(5), 1, S, nh * hd), 1, S, 0, [0], f"hd=80 1x{S}")


@pytest.mark.parametrize("B", [1, 3])
def test_decode_split_context_exact(B):
    """S = 1 after a 700-token prefill: the decode attention splits the context over blocks (few (row, head) pairs)
    and the dense GEMV merges the partials in its prologue (attn_merge.h); contexts 701..705 and one row at a
    different length."""
    nh, hd = 16, 96
    h = nh * hd
    P = 700
    a = AttnStage(h, nh, B, P + 16, B * P)
    rng = np.random.default_rng(6 + B)
    pasts = [P - 37 * r for r in range(B)]
    for r in range(B):
        a.run_and_check(_x(rng, 1, pasts[r], h), 1, pasts[r], r, [0], f"B={B} row {r} prompt {pasts[r]}")
    for step in range(5):
        a.run_and_check(_x(rng, B, 1, h), B, 1, 0, [p + step for p in pasts], f"B={B} decode step {step}")
