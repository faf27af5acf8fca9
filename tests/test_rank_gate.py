"""The failure semantics of the multi-device driver, on the CPU: the RankGate (skirt_amd/csrc/host/rank_gate.hpp)
that the device threads of skirt_sim_run_devices pass before every all-reduce. The reference's Parallel::call
stops every worker at the first exception (SKIRTcore/Parallel.cpp:181-193); here a rank that fails must leave
no peer waiting in a collective it will never join. tests/native/rank_gate_check.cpp runs the gate over
threads; a hang fails the test through the subprocess timeout."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "native", "rank_gate_check.cpp")


@pytest.fixture(scope="module")
def gate_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("gate") / "rank_gate_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-Wall", "-o", exe, SRC], check=True)
    return exe


def run(exe, ranks, colls, fail_rank, fail_after):
    out = subprocess.run([exe, str(ranks), str(colls), str(fail_rank), str(fail_after)], capture_output=True,
                         text=True, timeout=30, check=True).stdout.split("\n")
    logs = {int(l.split()[0]): (l.split() + [""])[1] for l in out if l and l[0].isdigit()}
    failed = [l for l in out if l.startswith("failed")][0]
    return logs, failed


def test_every_rank_passes_every_collective_without_a_failure(gate_check):
    logs, failed = run(gate_check, 8, 20, -1, 0)
    assert all(logs[r] == "1" * 20 for r in range(8))
    assert failed.startswith("failed 0")


@pytest.mark.parametrize("fail_rank", [0, 3, 7])
def test_a_rank_failing_before_its_first_collective_stops_every_other(gate_check, fail_rank):
    logs, failed = run(gate_check, 8, 20, fail_rank, 0)
    assert logs[fail_rank] == "F"
    for r in range(8):
        if r != fail_rank:
            assert logs[r] == "0", (r, logs[r])  # refused at its first collective, not left waiting
    assert failed == "failed 1 rank %d failed" % fail_rank


def test_a_rank_failing_between_collectives(gate_check):
    """rank 2 fails after 5 collectives: every other rank passes those 5 (all ranks arrived) and is refused at
    the sixth, the first failure's message kept"""
    for _ in range(20):  # thread timings vary from run to run
        logs, failed = run(gate_check, 4, 12, 2, 5)
        assert logs[2] == "11111F"
        for r in (0, 1, 3):
            assert logs[r] == "111110", (r, logs[r])
        assert failed == "failed 1 rank 2 failed"
