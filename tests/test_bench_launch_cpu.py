"""bench.py --gpus N starts N ranks itself when no launcher did (the driver's
SCALE command and a plain `python bench.py --gpus 8` must agree), and a
launcher whose WORLD_SIZE disagrees with --gpus is rejected.  CPU only: the
hidden --launch-probe flag makes every rank report its layout and stop
before any GPU work."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bench_self_launches_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-probe"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    import re
    lines = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert sorted(d["rank"] for d in lines) == [0, 1, 2]
    assert all(d["world"] == 3 for d in lines)
    assert sorted(d["local_rank"] for d in lines) == [0, 1, 2]


def test_bench_single_rank_needs_no_launcher():
    r = subprocess.run([sys.executable, BENCH, "--launch-probe"],
                       capture_output=True, text=True, timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"rank": 0, "world": 1,
                                                              "local_rank": 0}


def test_bench_rejects_world_size_mismatch():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-probe"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def _probe(n, *extra):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-probe", *extra],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    import re
    return sorted((json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)),
                  key=lambda d: d["rank"])


def test_bench_self_launches_eight_ranks():
    """The driver's N=8 line: ranks 0-7, one distinct LOCAL_RANK (= GPU)
    each, before any GPU work."""
    lines = _probe(8)
    assert [d["rank"] for d in lines] == list(range(8))
    assert all(d["world"] == 8 for d in lines)
    assert sorted(d["local_rank"] for d in lines) == list(range(8))


def test_bench_c4_z_slabs_at_world_4_and_8():
    """C4's 256-plane volume over 4 and 8 ranks: contiguous slabs covering
    every plane once, each boundary a multiple of 2^(z halvings) = 4 (z
    256 -> 128 -> 64), so no z pair or z group straddles two GPUs."""
    for n in (4, 8):
        lines = _probe(n, "--config", "c4")
        slabs = [tuple(d["z_slab"]) for d in lines]
        assert slabs[0][0] == 0 and slabs[-1][1] == 256
        assert all(a[1] == b[0] for a, b in zip(slabs, slabs[1:]))
        assert all(lo % 4 == 0 and hi % 4 == 0 and hi - lo == 256 // n for lo, hi in slabs)
