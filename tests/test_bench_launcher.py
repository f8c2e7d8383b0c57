"""bench.py's N-rank launcher and pipeline bench bookkeeping on CPU (gloo, the checker as stage).

`python bench.py --gpus N` run plainly (WORLD_SIZE unset) must start N rank processes itself -- before
any GPU call -- and print rank 0's one JSON line with N per-stage records; under torchrun the same
script is one rank.  Here the ranks are gloo processes whose stages are the CPU checker
(tests/bench_checker.py, via bench.py's --executor hook), so this runs without a GPU: the schedule,
the per-stage bytes/busy bookkeeping and the configs[3] / configs[4] records are the code the
driver's multi-GPU run executes."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--backend", "gloo", "--model", "tiny", "--configs-model", "tiny", "--prompt", "6", "--steps", "3",
        "--warmup", "1", "--configs3-mb", "3", "--configs3-prompt", "5", "--configs4-rows", "4",
        "--configs4-ctx", "12,16", "--cpu-baseline", "0", "--no-profile", "--dtype", "fp32"]


def _bench(n, executor="bench_checker:make", extra=()):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "tests")]), OMP_NUM_THREADS="1")
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--executor", executor]
                          + ARGS + list(extra), cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_starts_n_ranks(n):
    r = _bench(n)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and res["config"]["stages"] == n
    assert [s["rank"] for s in res["per_stage"]] == list(range(n))
    want = [(0, 2), (2, 4)] if n == 2 else [(0, 2), (2, 3), (3, 4)]  # server.py:893-903 on 4 layers
    assert [tuple(s["layers"]) for s in res["per_stage"]] == want
    assert res["config"]["batch"] == 2 * n and res["value"] > 0 and "scaling_ref" in res
    # strong: 16 rows over 2N micro-batches; N = 3 cannot split 16 evenly and says what it ran
    st = res["strong"]
    assert st["rows"] == (16 if n == 2 else 18) and ("do not split" in st["definition"]) == (n == 3)
    c3 = res["configs3"]
    assert c3["rows"] == 3 and c3["n_mb"] == 3 and c3["prompt"] == 5
    assert len(c3["prefill"]["stage_busy_frac"]) == n and c3["prefill"]["ideal_busy_frac"] == pytest.approx(3 / (3 + n - 1))
    assert all(0 < b <= 1.0 for b in c3["prefill"]["stage_busy_frac"])
    c4 = res["configs4"]["by_ctx"]
    assert sorted(c4, key=int) == ["12", "16"]
    for c, rec in c4.items():
        assert rec["decode_positions"][1] == int(c) and rec["value"] > 0 and len(rec["per_stage"]) == n


def test_bench_rank_failure_is_nonzero():
    r = _bench(2, executor="bench_checker:make_failing", extra=["--no-strong", "--no-configs"])
    assert r.returncode != 0


def test_bench_world_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + ARGS, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
