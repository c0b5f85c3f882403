"""CPU: the multi-GPU launch path of bench.py (`python bench.py --gpus N` without a torchrun environment, as the
driver's scaling run may start it).

bench.py starts torchrun as a child process before torch or the HIP library is loaded, every rank runs bench.py
with the same arguments, rank 0 prints the one JSON line (the other ranks print none) and the parent exits with
torchrun's status.  Here the ranks run a stand-in script with bench.py's rank-side contract (read RANK /
WORLD_SIZE / LOCAL_RANK / MASTER_*, rank 0 prints one line), so the launcher itself -- argv, rendezvous on
127.0.0.1, stdout relay, exit status -- runs for real on CPU at N = 2 and 8.
"""
import argparse
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

RANK_SCRIPT = r'''
import json, os, sys
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["LOCAL_RANK"]) == rank
assert os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY") == "0"
fail = os.environ.get("FAIL_RANK")
if fail is not None and int(fail) == rank:
    sys.exit(3)
if rank == 0:
    print(json.dumps({"world": world, "argv": sys.argv[1:]}), flush=True)
'''


def test_torchrun_cmd():
    cmd = bench.torchrun_cmd(8, ["--gpus", "8", "--steps", "5"], 12345)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "12345"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5] == os.path.join(ROOT, "bench.py")


@pytest.mark.parametrize("gpus", [2, 8])
def test_spawn_relays_rank0_line(tmp_path, gpus):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    argv = ["--gpus", str(gpus), "--steps", "7"]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)  # spawn_ranks sets it for the ranks
    code = ("import argparse, sys, bench; "
            f"sys.exit(bench.spawn_ranks(argparse.Namespace(gpus={gpus}), {argv!r}, {str(script)!r}))")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0's line only
    assert json.loads(lines[0]) == {"world": gpus, "argv": argv}


def test_spawn_returns_failure_status(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", FAIL_RANK="1")
    code = ("import argparse, sys, bench; "
            f"sys.exit(bench.spawn_ranks(argparse.Namespace(gpus=2), [], {str(script)!r}))")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0


def test_main_spawns_before_loading_anything(monkeypatch):
    """--gpus N > 1 without WORLD_SIZE: main() hands over to the launcher first (no torch / HIP library work in the
    parent, whose GPU state a child process must not inherit) and exits with its status."""
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "spawn_ranks", lambda args, argv: calls.append((args.gpus, list(argv))) or 5)
    monkeypatch.setattr(bench, "bench_single", lambda *a: pytest.fail("the parent must not bench"))
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "4", "--steps", "3"])
    assert e.value.code == 5 and calls == [(4, ["--gpus", "4", "--steps", "3"])]
    assert bench.parse_args(["--gpus", "8"]).config == "c2"  # the driver's default: the headline C2, weak scaling
    assert isinstance(bench.parse_args([]), argparse.Namespace)
