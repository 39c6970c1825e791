"""CPU checks of the range walk (nakama_amd/csrc/range_walk.h, no GPU).

tools/range_bench.cpp replays one pool of C2-shaped skill-window searches two
ways — replay_pool (replay_core.h) over every row's full hit list in the
reference's order (score desc, created_at asc; matchmaker_process.go:86-130),
and RangeRun over a min tree of the value-sorted candidates with build_tiers'
tier lists — and exits 1 unless the records and group entries are identical.
Solo 1v1 rows, and mixed rows (parties, shared or exclusive sessions, Min < Max,
CountMultiple, Intervals, MUST_NOT and fractional-boost ranges, candidates
without a number in the field).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def range_bench(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("rb") / "range_bench")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "range_bench.cpp")], check=True)
    return exe


@pytest.mark.parametrize("n,mode,seed", [(3000, "solo", 1), (3000, "mixed", 1), (3000, "mixed", 2), (1200, "mixed", 7),
                                         (64, "mixed", 3), (1, "solo", 4), (3000, "mixedx", 1), (2000, "mixedx", 5)])
@pytest.mark.parametrize("body", ["fast", "exact"])
def test_range_walk_equals_list_replay(range_bench, n, mode, seed, body):
    """mixedx: exclusive sessions, so the fast body runs (bailing to the exact
    one at the CountMultiple trim); "exact" forces the exact body."""
    out = subprocess.run([range_bench, str(n), mode, str(seed), "ref", body], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0 and "MATCH" in out.stdout, out.stdout + out.stderr
