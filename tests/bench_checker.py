"""TEST INFRASTRUCTURE: the CPU checker (oracle/) as bench.py's pipeline stage executor, so the
N-rank launcher and the pipeline bench bookkeeping run on gloo ranks without a GPU
(`bench.py --backend gloo --executor bench_checker:make`).  Never used by a GPU run."""
import os

import numpy as np
import torch

from oracle.oracle import OracleStage


class CheckerExecutor:
    def __init__(self, model, seed, lb, le, first, last, max_batch, max_ctx, hslice=None):
        self.model, self.hslice = model, hslice
        self.st = OracleStage(model.hidden, model.n_head, model.n_layer, model.vocab, lb, le, max_batch=max_batch,
                              max_ctx=max_ctx, seed=seed, is_first=first, is_last=last)
        if hslice is not None:  # layer-free stage owning the tied head: ln_f + this rank's vocabulary slice
            self.head = OracleStage(model.hidden, model.n_head, model.n_layer, model.vocab, 0, 0, max_batch=max_batch,
                                    max_ctx=max_ctx, seed=seed, is_first=False, is_last=True)

    def forward(self, inp, out, batch, seq, slot, past_len):
        y = self.st.forward(inp.numpy(), batch, seq, slot=slot, past_len=past_len)
        out.copy_(torch.from_numpy(np.ascontiguousarray(y).reshape(-1)[: out.numel()]).view(out.shape))

    def head_norm(self, hidden, batch, seq, xn):
        h = self.model.hidden
        xn.copy_(torch.from_numpy(self.head.head_norm(hidden.numpy()[: batch * seq * h], batch, seq).reshape(-1)))

    def head_slice(self, xn, batch, keys_in, keys_out, tokens):
        kin = None if keys_in is None else keys_in.numpy().view(np.uint64)
        keys, toks = self.head.head_slice(xn.numpy(), batch, self.hslice[0], self.hslice[1], kin)
        if keys_out is not None:
            keys_out.copy_(torch.from_numpy(keys.view(np.int64)))
        if tokens is not None:
            tokens.copy_(torch.from_numpy(toks))


def make(model, dtype, seed):
    """bench.py --executor hook: build_rank's executor factory for `model` (fp32 checker stages)."""
    def factory(lb, le, first, last, max_batch, max_ctx, hslice):
        return CheckerExecutor(model, seed, lb, le, first, last, max_batch, max_ctx, hslice)
    return factory


def make_failing(model, dtype, seed):
    """As `make`, but rank 1's stage cannot be built: the launcher must exit non-zero."""
    if int(os.environ.get("RANK", "0")) == 1:
        raise RuntimeError("bench_checker: rank 1 fails on purpose")
    return make(model, dtype, seed)
