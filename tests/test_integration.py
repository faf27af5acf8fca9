"""The maintainer-side binding (integration/GpuPhotonEngine.cpp) compiles against
the reference's own headers with the documented friend patch, and every engine symbol it calls is exported
by the built library. Needs /root/reference and the Qt5 headers of the build container; skipped elsewhere
(the GPU box has neither)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("SKIRT_REFERENCE", "/root/reference")
QT = os.environ.get("QT_INCLUDE", "/opt/conda/include/qt")


@pytest.mark.skipif(not (os.path.isdir(os.path.join(REF, "SKIRTcore")) and os.path.isdir(os.path.join(QT, "QtCore"))),
                    reason="reference headers or Qt5 headers not present")
def test_binding_compiles_against_the_reference_headers(tmp_path):
    lib = os.path.join(REPO, "skirt_amd", "libskirt_amd.so")
    if not os.path.exists(lib):
        pytest.skip("engine library not built")
    r = subprocess.run(["bash", os.path.join(REPO, "integration", "check_binding.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "skirt_mcrt_run_phase_shard" in r.stdout
