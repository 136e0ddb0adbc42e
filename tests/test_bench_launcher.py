"""bench.py --gpus N without a launcher starts N rank processes itself
(VERDICT r03 item 2).  CPU-only: the rank environment, a gloo world-2
rendezvous through it, the exit-code plumbing and the --gpus / WORLD_SIZE
consistency check."""
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_rank_envs():
    envs = bench.rank_envs(4, 29555, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and
               e["MASTER_PORT"] == "29555" and e["PATH"] == "/bin" for e in envs)
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)


CHILD = r"""
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
assert r == int(os.environ["RANK"]) and w == int(os.environ["WORLD_SIZE"])
t = torch.tensor([float(r + 1)])
dist.all_reduce(t)
assert t.item() == w * (w + 1) / 2, t
open(os.path.join(sys.argv[1], f"rank{r}"), "w").write(f"{w} {t.item()}")
dist.destroy_process_group()
"""


def test_launch_ranks_gloo_world2(tmp_path):
    rc = bench.launch_ranks(2, [], cmd=[sys.executable, "-c", CHILD, str(tmp_path)])
    assert rc == 0
    assert sorted(os.listdir(tmp_path)) == ["rank0", "rank1"]
    assert all(open(tmp_path / f).read() == "2 3.0" for f in ("rank0", "rank1"))


def test_launch_ranks_reports_failure():
    code = "import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)"
    assert bench.launch_ranks(2, [], cmd=[sys.executable, "-c", code]) == 3


def test_launch_ranks_failure_ends_waiting_ranks():
    # rank 1 fails at once; rank 0 would wait (like a rank stuck in rendezvous):
    # the launcher terminates it and reports rank 1's code without waiting it out
    code = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1': sys.exit(5)\n"
            "time.sleep(120)\n")
    t = time.perf_counter()
    assert bench.launch_ranks(2, [], cmd=[sys.executable, "-c", code]) == 5
    assert time.perf_counter() - t < 60


def test_gpus_world_size_mismatch_exits():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=300)
    assert r.returncode != 0
    assert b"--gpus 2 but WORLD_SIZE = 1" in r.stdout
