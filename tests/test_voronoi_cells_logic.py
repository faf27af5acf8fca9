"""The device Voronoi cells kernel's logic on the CPU (no GPU): tools/vor_cells_cpu.py compiles the device
functions of skirt_amd/csrc/device/voronoi_cells.hip as plain C++ beside the host construction
(host/voronoi.cpp) and requires every cell of uniform and Plummer site sets to equal the host's bit for bit
(cells beyond the kernel's capacities excepted: the host builds those). The kernel itself runs in
tests/test_gpu_setup.py."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_device_cell_logic_equals_host_on_cpu():
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "vor_cells_cpu.py"), "1500"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("N=1500")]
    assert len(lines) == 2 and all(" 0 cells differ" in l for l in lines), r.stdout
