"""The setup's Mersenne twister (skirt_amd/csrc/host/mt_random.hpp, the reference's Random.cpp:41-126):
its SSE2 refill and batched words() against a plain one-word-at-a-time restatement, over several seeds
and request sizes crossing the 624-word refills (tools/mt_check.cpp); and a seed of 0, which leaves the
generator emitting rejected zeros forever, refused at load."""
import os
import subprocess

import pytest

import skirt_amd as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_batched_words_match_plain_generator(tmp_path):
    exe = str(tmp_path / "mt_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "skirt_amd", "csrc", "host"),
                    os.path.join(REPO, "tools", "mt_check.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout


def test_seed_zero_is_refused(tmp_path):
    if not os.path.exists(S.LIB_PATH):
        pytest.skip("engine library not built")
    with open(os.path.join(REPO, "tests", "golden", "ski", "pan_cart16.ski")) as f:
        text = f.read()
    path = str(tmp_path / "seed0.ski")
    with open(path, "w") as f:
        f.write(text.replace('<Random seed="4357"/>', '<Random seed="0"/>'))
    with pytest.raises(S.SkirtError, match="seed 0"):
        S.Simulation(path)
