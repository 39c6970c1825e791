"""CPU checks of the host replay's walks (nakama_amd/csrc/replay_core.h, no GPU).

tools/replay_bench.cpp builds one pool of synthetic tickets in the store's
interleaved slot order and replays its complete hit list five ways — the
generic replay_pool (ReplayCore::row / fast_row), the dense walk over gathered
per-position copies (DenseRun::step / fast_step, slot -> position map), and
the identity walk the product takes when a pool's rows are its list (row j's
ticket at position j) — and exits 1 unless every output (records, group
entries) is identical.  Modes: C3's 5v5 parties (Min = Max = 10,
CountMultiple 5), C4's 1v1 solos over 64 interleaved pools, and mixed rows
(Min 4-10, CountMultiple 1 or 2, Intervals 0-2: the last-interval rule and
the CountMultiple trim).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def replay_bench(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("rpb") / "replay_bench")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe, os.path.join(ROOT, "tools", "replay_bench.cpp")],
                   check=True)
    return exe


@pytest.mark.parametrize("mode,pools,n", [("c3", 8, 40_000), ("solo2", 64, 60_000), ("mixed", 8, 40_000),
                                          ("mixed", 3, 5_000), ("c3", 1, 3_000)])
def test_walks_agree(replay_bench, mode, pools, n):
    env = dict(os.environ, RB_MODE=mode, RB_POOLS=str(pools))
    out = subprocess.run([replay_bench, str(n), "2", "0"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0 and "MATCH" in out.stdout, out.stdout + out.stderr
