"""The C++ route to the cross-GPU sums (include/skirt_host.h, skirt_rccl_* and skirt_sim_run_devices; the
reference's MPI_Allreduce at the phase ends, PanDustSystem.cpp:394-404, Instrument.cpp:57-66): the CLI's
`-g N` mode drives one engine per device from its own thread and installs the RCCL all-reduce as the
engines' reducer. On the one-GPU test box N = 1 (a one-device communicator: the all-reduce runs, over one
rank): its outputs equal the single-device run of the same packets, every phase of the model included
(pan_cart16_sa: the stellar phase, self-absorption cycles whose convergence reads the reduced dust Labs, and
the dust emission phase). N > 1 is unmeasured on hardware here (the pool gives one GPU per call)."""
import os
import subprocess

import numpy as np
import pytest

import skirt_files as F

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "skirt_amd", "bin", "skirt-mi355x")
GOLD = os.path.join(REPO, "tests", "golden", "ski")


@pytest.mark.parametrize("name", ["pan_oct", "pan_cart16_sa"])
def test_rccl_one_device_equals_single_device_run(tmp_path, name):
    ski = os.path.join(GOLD, name + ".ski")
    one = str(tmp_path / "one")
    rccl = str(tmp_path / "rccl")
    r1 = subprocess.run([CLI, "-d", "0", "-p", "2000", "-o", one, ski], capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr
    r2 = subprocess.run([CLI, "-g", "1", "-p", "2000", "-o", rccl, ski], capture_output=True, text=True, timeout=300)
    assert r2.returncode == 0, r2.stderr
    assert "1 GPUs (RCCL all-reduce" in r2.stdout
    outs = sorted(f for f in os.listdir(tmp_path) if f.startswith("one_"))
    assert any(f.endswith("_sed.dat") for f in outs) and any(f.endswith(".fits") for f in outs)
    for f in outs:
        a, b = os.path.join(tmp_path, f), os.path.join(tmp_path, "rccl_" + f[4:])
        assert os.path.exists(b), f
        if f.endswith(".fits"):
            np.testing.assert_allclose(F.read_fits(b), F.read_fits(a), rtol=1e-6, atol=0)  # float32 frames
        else:
            ta = [t for row in F.read_text_tokens(a) for t in row]
            tb = [t for row in F.read_text_tokens(b) for t in row]
            assert len(ta) == len(tb), f
            for x, y in zip(ta, tb):
                try:
                    np.testing.assert_allclose(float(y), float(x), rtol=1e-6, atol=0)  # 7-9 printed digits
                except ValueError:
                    assert x == y, f


def test_a_failing_device_thread_returns_its_error(tmp_path):
    """The failure path of `-g N` (Parallel.cpp:181-193: the first failure stops every worker and is reported
    by the parent): SKIRT_AMD_FAIL_DEVICE=0 makes device 0's thread fail before its first phase. The call
    returns that error, without waiting in a collective, and writes no outputs. (The gate that keeps the
    other ranks out of their collectives is tested on the CPU, tests/test_rank_gate.py.)"""
    ski = os.path.join(GOLD, "pan_oct.ski")
    env = dict(os.environ, SKIRT_AMD_FAIL_DEVICE="0")
    r = subprocess.run([CLI, "-g", "1", "-p", "200", "-o", str(tmp_path / "f"), ski], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert "device 0: failure injected (SKIRT_AMD_FAIL_DEVICE)" in r.stderr, r.stderr
    assert not [f for f in os.listdir(tmp_path) if f.startswith("f_")]
