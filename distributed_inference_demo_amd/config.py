"""BLOOM family dimensions (HF BloomConfig fields; SURVEY.md §8 model table) and the
benchmark configurations of BASELINE.json."""
from dataclasses import dataclass, replace


@dataclass(frozen=True)
class BloomDims:
    name: str
    hidden: int
    n_layer: int
    n_head: int
    vocab: int = 250880
    eps: float = 1e-5
    int8_weights: bool = False  # "-int8" model names: weight-only int8 stages (BS_FLAG_INT8_WEIGHTS)

    @property
    def head_dim(self):
        return self.hidden // self.n_head

    def block_params(self):
        return 12 * self.hidden * self.hidden + 13 * self.hidden


MODELS = {
    "bloom-560m": BloomDims("bloom-560m", 1024, 24, 16),
    "bloom-1b1": BloomDims("bloom-1b1", 1536, 24, 16),
    "bloom-1b7": BloomDims("bloom-1b7", 2048, 24, 16),
    "bloom-3b": BloomDims("bloom-3b", 2560, 30, 32),
    "bloom-7b1": BloomDims("bloom-7b1", 4096, 30, 32),
    # small shapes for tests
    "tiny": BloomDims("tiny", 64, 4, 4, vocab=512),
}


def get(name: str) -> BloomDims:
    """Model by name: "bloom-560m", "560m", the reference's "bloom560m"; an "-int8" suffix
    ("bloom560m-int8", server.py:796-799) selects the weight-only int8 variant of the same dims."""
    int8 = name.endswith("-int8")
    base = name[:-5] if int8 else name
    if base.startswith("bloom") and not base.startswith("bloom-") and base not in MODELS:
        base = "bloom-" + base[5:]
    key = base if base.startswith("bloom-") or base in MODELS else f"bloom-{base}"
    m = MODELS[key]
    return replace(m, name=m.name + "-int8", int8_weights=True) if int8 else m


def decode_step_bytes(m: BloomDims, layers: int, batch: int, ctx: int, first: bool, last: bool,
                      w_bytes: int = 2, kv_bytes: int = 2, act_bytes: int = 4) -> float:
    """Algorithmic HBM bytes of one decode step of a stage (BASELINE.md / SURVEY §8d):
    sum_layers[(12h^2+13h)w + 2*B*ctx*h*k (KV read) + 2*B*h*k (KV write)]
    + [first](B*h*w + 4h*w... emb row gather + emb LN) + [last](V*h*w + 2h*w) + 2*B*h*act."""
    h = m.hidden
    b = layers * (m.block_params() * w_bytes + 2 * batch * ctx * h * kv_bytes + 2 * batch * h * kv_bytes)
    if first:
        b += batch * h * w_bytes + 4 * h * w_bytes
    if last:
        b += m.vocab * h * w_bytes + 2 * h * w_bytes
    b += 2 * batch * h * act_bytes
    return float(b)


def prefill_flops(m: BloomDims, layers: int, batch: int, seq: int, last: bool) -> float:
    """sum_l [2*B*S*12h^2 + 2*B*heads*S(S+1)*hd] + [last] 2*B*V*h  (SURVEY §8d)."""
    h = m.hidden
    f = layers * (2.0 * batch * seq * 12 * h * h + 2.0 * batch * m.n_head * seq * (seq + 1) * m.head_dim)
    if last:
        f += 2.0 * batch * m.vocab * h
    return f
