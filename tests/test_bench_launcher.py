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
        "--configs4-ctx", "4,12,16", "--configs2-model", "tiny", "--configs2-prompt", "5", "--configs2-steps", "2",
        "--cpu-baseline", "0", "--no-profile", "--dtype", "fp32"]


def _bench(n, executor="bench_checker:make", extra=()):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "tests")]), OMP_NUM_THREADS="1")
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--executor", executor]
                          + ARGS + list(extra), cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("n", [2, 3, 4])
def test_bench_gpus_n_starts_n_ranks(n):
    r = _bench(n)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and res["config"]["stages"] == n
    assert [s["rank"] for s in res["per_stage"]] == list(range(n))
    want = {2: [(0, 2), (2, 4)], 3: [(0, 2), (2, 3), (3, 4)], 4: [(0, 1), (1, 2), (2, 3), (3, 4)]}[n]  # server.py:893-903
    assert [tuple(s["layers"]) for s in res["per_stage"]] == want
    assert res["config"]["batch"] == 2 * n and res["value"] > 0 and "scaling_ref" in res
    # strong: 16 rows over 2N micro-batches; N = 3 cannot split 16 evenly and says what it ran
    st = res["strong"]
    assert st["rows"] == (18 if n == 3 else 16) and ("do not split" in st["definition"]) == (n == 3)
    c3 = res["configs3"]
    assert c3["rows"] == 3 and c3["n_mb"] == 3 and c3["prompt"] == 5
    assert len(c3["prefill"]["stage_busy_frac"]) == n and c3["prefill"]["ideal_busy_frac"] == pytest.approx(3 / (3 + n - 1))
    assert all(0 < b <= 1.0 for b in c3["prefill"]["stage_busy_frac"])
    c4 = res["configs4"]["by_ctx"]
    assert sorted(c4, key=int) == ["12", "16"]
    assert res["configs4"]["skipped_ctx"]["ctx"] == [4]  # 4 <= warmup + steps: skipped, not a crash
    for c, rec in c4.items():
        assert rec["decode_positions"][1] == int(c) and rec["value"] > 0 and len(rec["per_stage"]) == n
    # configs[2]: B = 1 and B = 8 on the round-robin split, n_mb = the largest divisor of B <= 2N
    c2 = res["configs2"]
    assert c2["B1"]["rows"] == 1 and c2["B1"]["n_mb"] == 1 and c2["B1"]["prompt"] == 5
    assert c2["B8"]["rows"] == 8 and c2["B8"]["n_mb"] == {2: 4, 3: 4, 4: 8}[n]
    for rec in (c2["B1"], c2["B8"]):
        assert rec["value"] > 0 and [tuple(s["layers"]) for s in rec["per_stage"]] == want
        assert all(s["achieved_GBps"] > 0 for s in rec["per_stage"])
    # replicas: the whole model on every rank, same total rows as the pipeline lines
    rep = res["replicas"]
    assert rep["weak"]["rows"] == 2 * n and rep["weak"]["per_gpu_rows"] == 2 and rep["weak"]["value"] > 0
    assert rep["strong"]["per_gpu_rows"] * n >= 16 and rep["strong"]["value"] > 0
    sr = res["scaling_ref"]
    assert sr["strong_value"] == st["value"] and sr["replicas_weak_value"] == rep["weak"]["value"]
    assert sr["weak_value"] == res["value"]


def test_bench_rank_failure_is_nonzero():
    r = _bench(2, executor="bench_checker:make_failing", extra=["--no-strong", "--no-configs"])
    assert r.returncode != 0


def test_bench_world_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + ARGS, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
