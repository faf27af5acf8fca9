"""The compact Voronoi step's exactness argument, checked on the host (tools/vor_compact_check.cpp): rays
walked through a Plummer-site tessellation with the reference's step (double sites, VoronoiMesh.cpp:749-844)
and with the device's step (bounds from float offsets in double or single precision, the exact reference
expression for the winner, exact re-evaluation when the bounds cannot separate the candidates) cross the
same cells with bitwise equal segment lengths."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "skirt_amd", "libskirt_amd.so")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if not os.path.exists(LIB):
        pytest.skip("engine library not built")
    exe = str(tmp_path_factory.mktemp("vor") / "vor_compact_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tools", "vor_compact_check.cpp"), "-L", os.path.dirname(LIB), "-lskirt_amd",
                    "-Wl,-rpath," + os.path.dirname(LIB), "-o", exe], check=True)
    return exe


# the checker's modes: n -- double bounds; f -- the round-2 float bounds; x -- per-entry Cauchy-Schwarz
# terms; d -- the cell's largest terms from its header on the offsets n (round 3); r -- the device's step
# (engine.hip Grid<SKIRT_GRID_VORONOI>::bounds: entries m = n / |n|^2 and the cell's terms, both computed by
# the engine's own vor_terms.hpp); r+ / r- / r~ -- the device's step with its approximate reciprocal
# (v_rcp_f32, 1 ulp) emulated: every reciprocal one ulp up, down, or each by a random -1 / 0 / +1 ulp
@pytest.mark.parametrize("mode", ["n", "f", "x", "d", "r", "r+", "r-", "r~"],
                         ids=["f64", "f32_r2", "f32_entry", "f32_cell_terms", "device", "device_rcp_up",
                              "device_rcp_down", "device_rcp_random"])
def test_compact_voronoi_step_is_exact(checker, mode):
    r = subprocess.run([checker, "20000", "3000", mode], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout, r.stdout
    steps = int(r.stdout.split("steps ")[1].split(",")[0])
    assert steps > 50000
