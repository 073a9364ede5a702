"""bench.py's launcher contract (CPU): `python bench.py --gpus N` without WORLD_SIZE spawns N
ranks with the torch.distributed.run environment; a WORLD_SIZE that disagrees with --gpus is
an error; a failing rank fails the run.  The ranks here are a stub script (no GPU)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


class _Args:
    def __init__(self, gpus):
        self.gpus = gpus


def test_resolve_world(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.resolve_world(_Args(None)) == 1
    assert bench.resolve_world(_Args(4)) == 4
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.resolve_world(_Args(None)) == 2
    assert bench.resolve_world(_Args(2)) == 2
    with pytest.raises(SystemExit) as e:
        bench.resolve_world(_Args(8))
    assert e.value.code == 2


def test_spawn_ranks_env(tmp_path, capfd):
    stub = tmp_path / "stub.py"
    out = tmp_path / "ranks"
    out.mkdir()
    stub.write_text(textwrap.dedent(f"""
        import json, os, sys
        keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
        env = {{k: os.environ[k] for k in keys}}
        env["argv"] = sys.argv[1:]
        open(os.path.join({str(out)!r}, env["RANK"]), "w").write(json.dumps(env))
        if env["RANK"] == "0":
            print("LINE", flush=True)
    """))
    rc = bench.spawn_ranks(3, script=str(stub), argv=["--gpus", "3", "--steps", "2"])
    assert rc == 0
    got = [json.loads((out / str(r)).read_text()) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"]
    assert [g["LOCAL_RANK"] for g in got] == ["0", "1", "2"]
    assert {g["WORLD_SIZE"] for g in got} == {"3"}
    assert {g["MASTER_ADDR"] for g in got} == {"127.0.0.1"}
    assert len({g["MASTER_PORT"] for g in got}) == 1
    assert got[0]["argv"] == ["--gpus", "3", "--steps", "2"]
    assert "LINE" in capfd.readouterr().out  # rank 0's stdout passes through


def test_spawn_ranks_failure(tmp_path):
    stub = tmp_path / "stub.py"
    stub.write_text("import os, sys, time\n"
                    "sys.exit(3) if os.environ['RANK'] == '1' else time.sleep(30)\n")
    rc = bench.spawn_ranks(2, script=str(stub), argv=[])
    assert rc == 3  # rank 1's failure; rank 0 was stopped instead of waited for


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_bench_strong_split_checked_before_any_rank_starts():
    """The strong-scaling headline cuts n per class and the 64 shards over the ranks: a world
    size that does not divide them is refused up front (exit 2), before ranks are spawned."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"],
                       env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"},
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "do not split over 3 ranks" in r.stderr
