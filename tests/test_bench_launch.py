"""bench.py --gpus N without a launcher ("do this" 3): bench.py starts its own N
ranks (RANK / LOCAL_RANK / WORLD_SIZE, rendezvous at 127.0.0.1), refuses when fewer than N GPUs
are visible (unless the one-GPU gloo rehearsal is asked for) and never falls back to one rank.

CPU tests: the launcher with stand-in child programs, and the refusal on a host with no GPU.
The GPU test runs the real bench as a 2-rank gloo rehearsal on one GPU."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

CHILD = """
import json, os, sys
out = sys.argv[1]
keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys}, f)
if len(sys.argv) > 2 and os.environ["RANK"] == sys.argv[2]:
    sys.exit(3)
if len(sys.argv) > 2:
    import time
    time.sleep(60)   # the healthy ranks would wait for the failed one
"""


def _child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return p


def test_launch_ranks_env(tmp_path, monkeypatch):
    monkeypatch.delenv("MASTER_PORT", raising=False)
    code = bench.launch_ranks(3, [str(_child(tmp_path)), str(tmp_path)], visible=3)
    assert code == 0
    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1"
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_launch_ranks_failure_stops_the_rest(tmp_path):
    import time
    t0 = time.perf_counter()
    code = bench.launch_ranks(3, [str(_child(tmp_path)), str(tmp_path), "1"], visible=3)
    assert code == 3
    assert time.perf_counter() - t0 < 30  # the sleeping ranks were stopped, not waited for


def test_launch_refuses_without_gpus(tmp_path, monkeypatch):
    monkeypatch.delenv("IBTK_BENCH_BACKEND", raising=False)
    monkeypatch.delenv("IBTK_BENCH_DEVICE", raising=False)
    code = bench.launch_ranks(8, [str(_child(tmp_path)), str(tmp_path)], visible=1)
    assert code == 2
    assert not list(tmp_path.glob("rank*.json"))  # no rank was started


def test_launch_rehearsal_allows_one_gpu(tmp_path, monkeypatch):
    monkeypatch.setenv("IBTK_BENCH_BACKEND", "gloo")
    monkeypatch.setenv("IBTK_BENCH_DEVICE", "0")
    assert bench.launch_ranks(2, [str(_child(tmp_path)), str(tmp_path)], visible=1) == 0
    assert len(list(tmp_path.glob("rank*.json"))) == 2


def test_bench_gpus8_exits_nonzero_without_gpus():
    """The real entry point: --gpus 8 where fewer GPUs are visible exits non-zero with a message
    (this container has none; a one-GPU box likewise)."""
    import torch
    if torch.cuda.device_count() >= 8:
        pytest.skip("8 GPUs visible")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "IBTK_BENCH_BACKEND", "IBTK_BENCH_DEVICE")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs 8 visible GPUs" in r.stderr
    assert r.stdout.strip() == ""


@pytest.mark.gpu
def test_bench_gpus2_rehearsal_launches_two_ranks():
    """bench.py --gpus 2 with no launcher, as a one-GPU gloo rehearsal: two ranks run, rank 0
    prints one line with n_gpus 2, and the overlapped exchange passes its self-check."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(IBTK_BENCH_BACKEND="gloo", IBTK_BENCH_DEVICE="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--config", "cfg2",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    # (gloo itself prints a connection note on stdout; the record is the one JSON line)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "z-slab x2"
    assert rec["config"]["overlap_check"].startswith("bitwise equal")
