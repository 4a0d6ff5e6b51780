"""bench.py's N-rank plumbing on CPU: `--gpus N` outside torch.distributed starts N ranks as a
child (torch.distributed.run) and the line reports the ranks that ran; a rank count other than
--gpus, or RCCL ranks without a GPU each, fail instead of measuring one GPU.  `--dry-run` runs the
whole N-rank path except the GPU work (LPT shards, the variable-size gather to rank 0, the merge
in caller order) and compares the gathered records with one process's."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["BG_BENCH_BACKEND"] = "gloo"
    return env


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(out):
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [2, 3])
def test_gpus_n_spawns_n_ranks(gpus):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus), "--dry-run", "--pairs", "17",
                        "--len1", "300", "--len2", "200"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["ranks"] == gpus and d["gpus_arg"] == gpus
    assert d["gathered_pairs"] == 17 and len(d["shard_pairs"]) == gpus
    assert sum(d["shard_pairs"]) == 17
    assert d["gather_equals_single"] is True
    assert d["value"] is None


def test_one_rank_dry_run_matches():
    r = subprocess.run([sys.executable, BENCH, "--dry-run", "--pairs", "5", "--len1", "50",
                        "--len2", "60"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["ranks"] == 1 and d["gather_equals_single"] is True


def test_rank_count_other_than_gpus_fails():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), BENCH, "--gpus", "3",
           "--dry-run", "--pairs", "4", "--len1", "20", "--len2", "20"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert "--gpus 3" in r.stderr


def test_rccl_ranks_without_gpus_fail():
    torch = pytest.importorskip("torch")
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has GPUs for both ranks")
    env = _env()
    env["BG_BENCH_BACKEND"] = "nccl"
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--pairs", "4", "--len1", "20",
                        "--len2", "20", "--steps", "1", "--warmup", "0"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert "need 2 GPUs" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]
