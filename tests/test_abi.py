"""The drop-in boundary without a GPU: the C-ABI library loads, exports every function the headers in
include/ declare, its ctypes mirror matches the header structs, and the host-side setup (the .ski ->
model path that feeds the engine) runs and reports the reference's model sizes."""
import ctypes
import os
import re

import pytest

import skirt_amd as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h) for h in ("skirt_mcrt.h", "skirt_host.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names.update(re.findall(r"^[A-Za-z_][\w \*]*?\b(skirt_\w+)\s*\(", text, flags=re.M))
    return names


def test_library_exports_every_declared_function():
    decl = declared_functions()
    assert len(decl) >= 25
    assert decl == set(S.ABI_SYMBOLS), decl ^ set(S.ABI_SYMBOLS)
    lib = S.lib()
    missing = [n for n in decl if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version_and_stats_layout():
    assert S.lib().skirt_mcrt_abi_version() == 14 == S.ABI_VERSION
    assert "#define SKIRT_MCRT_ABI_VERSION %d" % S.ABI_VERSION in open(HEADERS[0]).read()
    text = open(HEADERS[0]).read()
    body = re.search(r"typedef struct \{([^}]*)\} SkirtStats;", text, flags=re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"(uint64_t|int32_t|double)\s+(\w+);", body)
    assert [n for _, n in fields] == [n for n, _ in S.SkirtStats._fields_]
    size = {"uint64_t": 8, "int32_t": 4, "double": 8}
    assert ctypes.sizeof(S.SkirtStats) == sum(size[t] for t, _ in fields)


def test_engine_creation_fails_loudly_without_a_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = S.lib()
    lib.skirt_mcrt_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    h = ctypes.c_void_p()
    assert lib.skirt_mcrt_create(0, ctypes.byref(h)) != 0
    assert not h.value


@pytest.mark.parametrize("name,pan,grid,ncells,nlambda", [
    ("c1_oligo16", 0, 0, 16 ** 3, 1),
    ("pan_cart16", 1, 0, 16 ** 3, None),
    ("pan_oct", 1, 1, None, None),
])
def test_host_setup_without_gpu(name, pan, grid, ncells, nlambda):
    sim = S.Simulation(os.path.join(REPO, "tests", "golden", "ski", name + ".ski"), packages=100)
    info = sim.info
    assert info.pan == pan and info.grid_kind == grid
    if ncells:
        assert info.ncells == ncells
    if nlambda:
        assert info.nlambda == nlambda
    assert info.total_packets == info.npp * info.nlambda
    assert info.ninstruments >= 1
    if grid == 1:
        assert info.nnodes > info.ncells


def test_missing_ski_is_an_error():
    with pytest.raises(S.SkirtError):
        S.Simulation(os.path.join(REPO, "no_such_model.ski"))
