"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this module.
"""
import ctypes
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(REPO, "oracle", "liboracle.so")
DATA_DIR = os.path.join(REPO, "skirt_amd", "data")

RNG_MT = 0
RNG_PHILOX = 1
PHASES_STELLAR, PHASES_DUST, PHASES_ALL = 1, 2, 3  # oracle_run's phase mask (oracle.h)

TALLY_LABS, TALLY_DUST_LABS = 0, 1  # ORACLE_TALLY_* (oracle.h)
# int (*)(void* user, int tally, double* data, size_t n): oracle_run_shard's host-array reduction
REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                             ctypes.c_size_t)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_run.restype = ctypes.c_void_p
        L.oracle_run.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                 ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p]
        L.oracle_run_shard.restype = ctypes.c_void_p
        L.oracle_run_shard.argtypes = L.oracle_run.argtypes + [ctypes.c_int, ctypes.c_int, REDUCE_FN, ctypes.c_void_p]
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_labs.restype = ctypes.POINTER(ctypes.c_double)
        L.oracle_labs.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.oracle_num_instruments.argtypes = [ctypes.c_void_p]
        L.oracle_instrument.argtypes = [ctypes.c_void_p, ctypes.c_int,
                                        ctypes.POINTER(ctypes.POINTER(ctypes.c_double)),
                                        ctypes.POINTER(ctypes.POINTER(ctypes.c_double)),
                                        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int)]
        L.oracle_seconds.restype = ctypes.c_double
        L.oracle_seconds.argtypes = [ctypes.c_void_p]
        L.oracle_packets.restype = ctypes.c_uint64
        L.oracle_packets.argtypes = [ctypes.c_void_p]
        L.oracle_segments.restype = ctypes.c_uint64
        L.oracle_segments.argtypes = [ctypes.c_void_p]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_set_engine_attenuation.argtypes = [ctypes.c_int]
        L.oracle_counts.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_crossed.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64))]
        L.oracle_labs_dust.restype = ctypes.POINTER(ctypes.c_double)
        L.oracle_labs_dust.argtypes = [ctypes.c_void_p]
        L.oracle_selfabs_cycles.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.POINTER(ctypes.c_double))]
        L.oracle_philox4x32_10.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.POINTER(ctypes.c_uint32)]
        _lib = L
    return _lib


class OracleResult:
    """Raw (uncalibrated) accumulators of one oracle run, copied into numpy arrays."""

    def __init__(self, handle):
        L = lib()
        nc, nl = ctypes.c_int(), ctypes.c_int()
        p = L.oracle_labs(handle, ctypes.byref(nc), ctypes.byref(nl))
        self.ncells, self.nlambda = nc.value, nl.value
        self.labs = (np.ctypeslib.as_array(p, shape=(self.ncells, self.nlambda)).copy() if p else None)
        self.frames, self.seds = [], []
        for i in range(L.oracle_num_instruments(handle)):
            fp, sp = ctypes.POINTER(ctypes.c_double)(), ctypes.POINTER(ctypes.c_double)()
            ns, nf, nlam = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            L.oracle_instrument(handle, i, ctypes.byref(fp), ctypes.byref(sp), ctypes.byref(ns), ctypes.byref(nf),
                                ctypes.byref(nlam))
            self.frames.append(np.ctypeslib.as_array(fp, shape=(ns.value, nlam.value, nf.value)).copy()
                               if fp else None)
            self.seds.append(np.ctypeslib.as_array(sp, shape=(ns.value, nlam.value)).copy() if sp else None)
        pd = L.oracle_labs_dust(handle)
        self.labs_dust = (np.ctypeslib.as_array(pd, shape=(self.ncells, self.nlambda)).copy() if pd else None)
        tp = ctypes.POINTER(ctypes.c_double)()
        n = L.oracle_selfabs_cycles(handle, ctypes.byref(tp))
        self.labs_dust_totals = [tp[i] for i in range(n)] if n else []
        self.seconds = L.oracle_seconds(handle)
        self.packets = L.oracle_packets(handle)
        self.segments = L.oracle_segments(handle)
        c = (ctypes.c_uint64 * 3)()
        L.oracle_counts(handle, c)
        # segments of the FILL paths and of the peel-off paths, Labs adds (the engine's statistics)
        self.segments_fill, self.segments_peel, self.absorb_adds = int(c[0]), int(c[1]), int(c[2])
        hp = ctypes.POINTER(ctypes.c_uint64)()
        n = L.oracle_crossed(handle, ctypes.byref(hp))
        # DustSystem's _crossed histogram: paths per number of segments
        self.crossed = np.ctypeslib.as_array(hp, shape=(n,)).copy() if n > 0 else np.zeros(0, np.uint64)


class engine_attenuation:
    """Context: the oracle evaluates the absorption's exp(-tau_{n-1}) as the engine does or did, to separate
    that arithmetic from everything else (oracle_set_engine_attenuation): mode 1 the running product of the
    engine until round 3, mode 2 the engine's carry since round 5 (the product while dtau < 0.5, exp(-tau)
    anew behind a thicker segment)."""

    def __init__(self, mode=1):
        self.mode = mode

    def __enter__(self):
        lib().oracle_set_engine_attenuation(self.mode)

    def __exit__(self, *exc):
        lib().oracle_set_engine_attenuation(0)


def run(ski, rng=RNG_MT, threads=1, packages=0.0, seed=0, packet_begin=0, packet_end=0, outprefix=None,
        phases=PHASES_STELLAR, rank=0, world=1, reduce=None):
    """Runs the oracle; by default only the stellar emission phase (phases=PHASES_ALL adds the dust
    self-absorption and dust emission phases of a Pan simulation with dust emission).

    With world > 1 (Philox mode) this is rank `rank`'s shard: its slice of every wavelength of every
    phase; reduce(tally, array) must sum the numpy array over the ranks in place (called for the stellar
    Labs and after every self-absorption cycle for the dust Labs)."""
    L = lib()
    args = [ski.encode(), DATA_DIR.encode(), rng, threads, float(packages), seed, packet_begin, packet_end, phases,
            outprefix.encode() if outprefix else None]
    if world == 1:
        h = L.oracle_run(*args)
    else:
        def cb(_user, tally, data, n):
            try:
                reduce(tally, np.ctypeslib.as_array(data, shape=(n,)))
                return 0
            except Exception:  # noqa: BLE001 -- reported to the C side as a failed reduction
                return 1

        fn = REDUCE_FN(cb) if reduce else ctypes.cast(None, REDUCE_FN)
        h = L.oracle_run_shard(*args, rank, world, fn, None)
    if not h:
        raise RuntimeError("oracle failed: " + L.oracle_last_error().decode())
    try:
        return OracleResult(h)
    finally:
        L.oracle_free(h)


def philox(ctr, key):
    L = lib()
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    L.oracle_philox4x32_10(c, k, o)
    return list(o)


def star_positions(ski, comp, n, seed=1):
    """n random positions of stellar component `comp` ([n, 3]) and the geometry's density there."""
    L = lib()
    L.oracle_star_positions.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_uint64, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_double)]
    out = np.zeros((n, 3))
    dens = np.zeros(n)
    rc = L.oracle_star_positions(ski.encode(), DATA_DIR.encode(), comp, n, seed,
                                 out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                 dens.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    if rc:
        raise RuntimeError("oracle failed: " + L.oracle_last_error().decode())
    return out, dens


def grid_paths(ski, rays, maxseg=4096):
    """DustGrid::path of the ski's dust grid for rays [n, 6] (position, direction): a list of
    (boxes [nseg, 6] (NaN rows before the grid), ds [nseg]) per ray, and the grid's cell count."""
    L = lib()
    L.oracle_grid_paths.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_int)]
    rays = np.ascontiguousarray(rays, dtype=np.float64)
    n = rays.shape[0]
    out = np.zeros((n, maxseg, 7))
    nseg = np.zeros(n, dtype=np.int32)
    nc = ctypes.c_int()
    rc = L.oracle_grid_paths(ski.encode(), DATA_DIR.encode(), n,
                             rays.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), maxseg,
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                             nseg.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), ctypes.byref(nc))
    if rc:
        raise RuntimeError("oracle failed: " + L.oracle_last_error().decode())
    return [(out[i, :nseg[i], :6], out[i, :nseg[i], 6]) for i in range(n)], nc.value


def dust_component(ski, comp=0):
    """(normalization factor, kappa_ext per wavelength, wavelengths) of dust component `comp`."""
    L = lib()
    L.oracle_dust_component.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
    nf, nl = ctypes.c_double(), ctypes.c_int()
    kext, lam = np.zeros(4096), np.zeros(4096)
    rc = L.oracle_dust_component(ski.encode(), DATA_DIR.encode(), comp, ctypes.byref(nf),
                                 kext.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                 lam.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), ctypes.byref(nl))
    if rc:
        raise RuntimeError("oracle failed: " + L.oracle_last_error().decode())
    return nf.value, kext[:nl.value].copy(), lam[:nl.value].copy()
