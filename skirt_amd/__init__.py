"""skirt_amd -- MI355X-native photon-packet engine for SKIRT's photon-shooting hot path.

The package is a thin Python face over the native library ``libskirt_amd.so`` (HIP kernels for gfx950
plus the C++ host driver): ``include/skirt_mcrt.h`` is the engine's C ABI, ``include/skirt_host.h``
the host driver (.ski -> model -> engine -> SKIRT-format outputs). Python is used only for plumbing
(tests, benchmarking, torch.distributed/RCCL reductions across GPUs); no compute happens here and
there is no CPU fallback: if the native library is missing, importing the engine fails loudly.

Mirrors the reference's simulation interface for this path:
    sim = Simulation("model.ski")            # Simulation::setup (SKIRTcore/Simulation.cpp:36-48)
    sim.attach(device=0)
    sim.run_stellar()                        # MonteCarloSimulation::runstellaremission (:251-261)
    sim.fetch(); sim.write("out/model")      # MonteCarloSimulation::write (:553-558)
"""
import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ABI_VERSION = 14  # SKIRT_MCRT_ABI_VERSION of include/skirt_mcrt.h
# SKIRT_AMD_LIB selects another build of the same library (e.g. a tuning variant built by
# tools/build_variant.sh next to the default one)
LIB_PATH = os.path.join(PKG_DIR, os.environ.get("SKIRT_AMD_LIB", "libskirt_amd.so"))
DATA_DIR = os.path.join(PKG_DIR, "data")

GRID_CARTESIAN, GRID_OCTREE, GRID_VORONOI = 0, 1, 2
# SkirtStats.grid_walk: the trace kernel's grid walk in the last run (SKIRT_WALK_*)
WALK_CARTESIAN, WALK_OCTREE_MAP, WALK_VORONOI, WALK_TREE_NODES, WALK_KDTREE_MAP, WALK_OCTREE_BOOKKEEPING = 0, 1, 2, 3, 4, 5


class SkirtError(RuntimeError):
    pass


class SkirtStats(ctypes.Structure):
    _fields_ = [("packets", ctypes.c_uint64), ("segments_fill", ctypes.c_uint64),
                ("segments_walk", ctypes.c_uint64), ("segments_peel", ctypes.c_uint64),
                ("detects", ctypes.c_uint64), ("absorb_adds", ctypes.c_uint64), ("lane_slots", ctypes.c_uint64),
                ("iterations", ctypes.c_uint64), ("kernel_ms", ctypes.c_double), ("trace_ms", ctypes.c_double),
                ("trace_launches", ctypes.c_uint64), ("grid_walk", ctypes.c_int32), ("map_level", ctypes.c_int32),
                ("labs_requests", ctypes.c_uint64), ("device_cells", ctypes.c_uint64),
                ("trace_blocks_per_cu", ctypes.c_uint64), ("packages", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class SkirtSimInfo(ctypes.Structure):
    _fields_ = [("pan", ctypes.c_int), ("ncells", ctypes.c_int), ("nlambda", ctypes.c_int), ("ncomp", ctypes.c_int),
                ("ninstruments", ctypes.c_int), ("grid_kind", ctypes.c_int), ("nnodes", ctypes.c_int),
                ("npp", ctypes.c_uint64), ("total_packets", ctypes.c_uint64), ("seed", ctypes.c_uint64),
                ("store_absorption", ctypes.c_int), ("has_dust", ctypes.c_int), ("setup_seconds", ctypes.c_double)]


# every symbol declared by include/skirt_mcrt.h and include/skirt_host.h
ABI_SYMBOLS = [
    "skirt_mcrt_abi_version", "skirt_mcrt_create", "skirt_mcrt_set_stream", "skirt_mcrt_upload_grid",
    "skirt_mcrt_upload_media", "skirt_mcrt_upload_sources", "skirt_mcrt_set_instruments",
    "skirt_mcrt_tally_sizes", "skirt_mcrt_bind_tallies", "skirt_mcrt_zero_tallies", "skirt_mcrt_run_stellar",
    "skirt_mcrt_synchronize", "skirt_mcrt_download", "skirt_mcrt_stats", "skirt_mcrt_configure",
    "skirt_mcrt_last_error", "skirt_mcrt_destroy", "skirt_mcrt_run_phase", "skirt_mcrt_upload_cell_sources",
    "skirt_mcrt_bind_dust_labs", "skirt_mcrt_zero_dust_labs", "skirt_mcrt_download_dust_labs",
    "skirt_mcrt_upload_emissivity", "skirt_mcrt_compute_cell_sources", "skirt_mcrt_dust_labs_total",
    "skirt_sim_load", "skirt_sim_info", "skirt_sim_attach", "skirt_sim_engine", "skirt_sim_run_stellar",
    "skirt_sim_fetch", "skirt_sim_labs", "skirt_sim_instrument", "skirt_sim_set_tallies", "skirt_sim_write",
    "skirt_sim_error", "skirt_sim_free", "skirt_sim_run_dust", "skirt_sim_labs_dust", "skirt_sim_selfabs_totals",
    "skirt_mcrt_run_phase_shard", "skirt_mcrt_shard_slice", "skirt_mcrt_set_reducer", "skirt_mcrt_reduce_instruments",
    "skirt_sim_run_stellar_shard", "skirt_sim_run_dust_shard", "skirt_sim_set_photon_seed",
    "skirt_host_voronoi_build", "skirt_host_voronoi_describe", "skirt_host_voronoi_free",
    "skirt_sim_load_ex", "skirt_mcrt_sample_density", "skirt_sim_density",
    "skirt_mcrt_set_crossed", "skirt_mcrt_download_crossed", "skirt_mcrt_column_densities",
    "skirt_rccl_create", "skirt_rccl_wrap", "skirt_rccl_rank", "skirt_rccl_reducer", "skirt_rccl_abort", "skirt_rccl_destroy", "skirt_sim_describe", "skirt_host_write_descriptors",
    "skirt_sim_run_devices", "skirt_mcrt_voronoi_cells", "skirt_host_voronoi_build_ex", "skirt_host_voronoi_cells",
]

_lib = None
# SKIRT_TALLY_*: what the engine's reducer is asked to sum
TALLY_LABS, TALLY_DUST_LABS, TALLY_INSTRUMENTS = 0, 1, 2
# int (*)(void* user, int tally, double* d_buf, size_t n, void* hip_stream): skirt_mcrt_set_reducer's callback
REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                             ctypes.c_void_p)


def lib():
    """The native library; raises SkirtError when it has not been built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SkirtError("native library %s is missing: run `make -C skirt_amd/csrc` "
                             "(or __graft_entry__.build())" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        # the structs below follow include/skirt_mcrt.h at ABI_VERSION; a library built from another header
        # would read or write them at other offsets (a tuning build chosen by SKIRT_AMD_LIB may be older)
        v = L.skirt_mcrt_abi_version()
        if v != ABI_VERSION and "SKIRT_AMD_LIB" not in os.environ:
            raise SkirtError("native library %s has C ABI %d, this binding expects %d: rebuild it" % (LIB_PATH, v, ABI_VERSION))
        vp, c_int, c_u64, c_dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_double
        L.skirt_sim_load.restype = vp
        L.skirt_sim_load.argtypes = [ctypes.c_char_p, ctypes.c_char_p, c_dbl, c_u64]
        L.skirt_sim_load_ex.restype = vp
        L.skirt_sim_load_ex.argtypes = [ctypes.c_char_p, ctypes.c_char_p, c_dbl, c_u64, c_int]
        L.skirt_sim_info.argtypes = [vp, ctypes.POINTER(SkirtSimInfo)]
        L.skirt_sim_attach.argtypes = [vp, c_int]
        L.skirt_sim_engine.restype = vp
        L.skirt_sim_engine.argtypes = [vp]
        L.skirt_sim_run_stellar.argtypes = [vp, c_u64, c_u64]
        L.skirt_sim_fetch.argtypes = [vp]
        L.skirt_sim_run_dust.argtypes = [vp]
        L.skirt_sim_set_photon_seed.argtypes = [vp, c_u64]
        L.skirt_sim_run_stellar_shard.argtypes = [vp, c_int, c_int]
        L.skirt_sim_run_dust_shard.argtypes = [vp, c_int, c_int]
        L.skirt_mcrt_set_reducer.argtypes = [vp, REDUCE_FN, vp]
        L.skirt_mcrt_reduce_instruments.argtypes = [vp]
        L.skirt_mcrt_shard_slice.restype = None
        L.skirt_mcrt_shard_slice.argtypes = [c_u64, c_int, c_int, ctypes.POINTER(c_u64), ctypes.POINTER(c_u64)]
        L.skirt_mcrt_bind_dust_labs.argtypes = [vp, vp]
        L.skirt_sim_labs_dust.restype = ctypes.POINTER(c_dbl)
        L.skirt_sim_labs_dust.argtypes = [vp]
        L.skirt_sim_selfabs_totals.argtypes = [vp, ctypes.POINTER(ctypes.POINTER(c_dbl))]
        L.skirt_sim_labs.restype = ctypes.POINTER(c_dbl)
        L.skirt_sim_density.restype = ctypes.POINTER(c_dbl)
        L.skirt_sim_density.argtypes = [vp]
        L.skirt_sim_labs.argtypes = [vp]
        L.skirt_sim_instrument.restype = ctypes.POINTER(c_dbl)
        L.skirt_sim_instrument.argtypes = [vp, c_int] + [ctypes.POINTER(c_int)] * 4
        L.skirt_sim_set_tallies.argtypes = [vp, ctypes.POINTER(c_dbl), ctypes.POINTER(c_dbl)]
        L.skirt_sim_write.argtypes = [vp, ctypes.c_char_p]
        L.skirt_sim_describe.argtypes = [vp, ctypes.c_char_p]
        L.skirt_sim_error.restype = ctypes.c_char_p
        L.skirt_sim_free.argtypes = [vp]
        L.skirt_mcrt_stats.argtypes = [vp, ctypes.POINTER(SkirtStats)]
        L.skirt_mcrt_last_error.restype = ctypes.c_char_p
        L.skirt_mcrt_last_error.argtypes = [vp]
        L.skirt_mcrt_set_stream.argtypes = [vp, vp]
        L.skirt_mcrt_tally_sizes.argtypes = [vp, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
        L.skirt_mcrt_bind_tallies.argtypes = [vp, vp, vp]
        L.skirt_mcrt_zero_tallies.argtypes = [vp]
        L.skirt_mcrt_synchronize.argtypes = [vp]
        L.skirt_mcrt_configure.argtypes = [vp, c_int, c_int, c_int]
        L.skirt_mcrt_set_crossed.argtypes = [vp, c_int]
        L.skirt_mcrt_download_crossed.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), c_int]
        L.skirt_mcrt_column_densities.argtypes = [vp, ctypes.POINTER(ctypes.c_double), c_int,
                                                  ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


class Simulation:
    """One SKIRT simulation (a .ski file) driven through the native host library."""

    def __init__(self, ski, packages=0.0, seed=0, datadir=None, setup_device=None):
        """setup_device: a HIP device for the setup's density sampling (tree subdivision, cell densities);
        None keeps the setup on the host, bit-identical to the reference."""
        L = lib()
        self._h = L.skirt_sim_load_ex(os.fspath(ski).encode(), (datadir or DATA_DIR).encode(), float(packages),
                                      int(seed), -1 if setup_device is None else int(setup_device))
        if not self._h:
            raise SkirtError(L.skirt_sim_error().decode())
        info = SkirtSimInfo()
        L.skirt_sim_info(self._h, ctypes.byref(info))
        self.info = info
        self.attached = False

    def set_photon_seed(self, seed):
        """Seed of the photon phases' random streams; the grid and other setup draws keep the setup seed."""
        self._check(lib().skirt_sim_set_photon_seed(self._h, int(seed)))
        self.info.seed = int(seed)

    def _check(self, rc):
        if rc != 0:
            raise SkirtError(lib().skirt_sim_error().decode())

    @property
    def engine(self):
        return lib().skirt_sim_engine(self._h)

    def attach(self, device=0):
        self._check(lib().skirt_sim_attach(self._h, device))
        self.attached = True

    def configure(self, slots=0, grid=0, threshold=0):
        """Engine knobs (0 = default): packet slots in flight, trace-kernel workgroups, and the number
        of idle lanes that makes a wave pull new rays."""
        self._check_engine(lib().skirt_mcrt_configure(self.engine, slots, grid, threshold))

    def _check_engine(self, rc):
        if rc != 0:
            raise SkirtError(lib().skirt_mcrt_last_error(self.engine).decode())

    def set_stream(self, stream_ptr):
        self._check_engine(lib().skirt_mcrt_set_stream(self.engine, ctypes.c_void_p(stream_ptr)))

    def tally_sizes(self):
        a, b = ctypes.c_size_t(), ctypes.c_size_t()
        lib().skirt_mcrt_tally_sizes(self.engine, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def bind_tallies(self, labs_ptr, instr_ptr):
        self._check_engine(lib().skirt_mcrt_bind_tallies(self.engine, ctypes.c_void_p(labs_ptr),
                                                         ctypes.c_void_p(instr_ptr)))

    def zero_tallies(self):
        self._check_engine(lib().skirt_mcrt_zero_tallies(self.engine))

    def run_stellar(self, first=0, count=0):
        self._check(lib().skirt_sim_run_stellar(self._h, first, count))

    def _collective(self, check, rc):
        """check(rc) for a call that may reach the reducer: when it fails on this rank, a reducer with an
        abort() (TallyReducer) tells the other ranks at their next reduction, so that none waits for this
        one in a collective (the reference's Parallel::call: the first failure stops every worker)"""
        try:
            check(rc)
        except SkirtError as e:
            fn = getattr(self, "_reducer_fn", None)
            if fn is not None and hasattr(fn, "abort"):
                fn.abort(str(e))
            raise

    def run_stellar_shard(self, rank, world):
        """This rank's slice of every wavelength of the stellar phase (IdenticalAssigner); with world > 1
        the reducer (set_reducer) sums the stellar Labs at the phase end."""
        self._collective(self._check, lib().skirt_sim_run_stellar_shard(self._h, rank, world))

    def run_dust(self, rank=0, world=1):
        """Self-absorption cycles (if enabled) and the dust emission phase (PanMonteCarloSimulation::runSelf).
        With world > 1 this rank shoots its slice of every wavelength of every phase, and the reducer
        (set_reducer) sums the dust Labs after every self-absorption cycle."""
        self._collective(self._check, lib().skirt_sim_run_dust_shard(self._h, rank, world))

    def set_reducer(self, fn):
        """fn(tally, device_ptr, n, hip_stream) sums the engine's device buffer over all processes in place
        (skirt_mcrt_set_reducer); e.g. skirt_amd.sharding.TallyReducer over the bound tally tensors.
        None removes it."""
        if fn is None:
            self._reducer = None
            self._check_engine(lib().skirt_mcrt_set_reducer(self.engine, ctypes.cast(None, REDUCE_FN), None))
            return

        def cb(_user, tally, ptr, n, stream):
            try:
                return 1 if fn(tally, ptr, n, stream) else 0  # a callable may return non-zero for a failure
            except Exception as e:  # noqa: BLE001 -- reported to the C side as a failed reduction
                self.reducer_error = e
                return 1

        self._reducer = REDUCE_FN(cb)  # kept alive as long as the engine may call it
        self._reducer_fn = fn
        self._check_engine(lib().skirt_mcrt_set_reducer(self.engine, self._reducer, None))

    def reduce_instruments(self):
        """Instrument::sumResults: sums the instrument tallies over the processes (once per simulation)."""
        self._collective(self._check_engine, lib().skirt_mcrt_reduce_instruments(self.engine))

    def bind_dust_labs(self, ptr):
        """Make the engine accumulate the dust Labs in caller device memory (tally_sizes()[0] doubles)."""
        self._check_engine(lib().skirt_mcrt_bind_dust_labs(self.engine, ctypes.c_void_p(ptr)))

    def labs_dust(self):
        p = lib().skirt_sim_labs_dust(self._h)
        if not p:
            return None
        return np.ctypeslib.as_array(p, shape=(self.info.ncells, self.info.nlambda)).copy()

    def selfabs_totals(self):
        tp = ctypes.POINTER(ctypes.c_double)()
        n = lib().skirt_sim_selfabs_totals(self._h, ctypes.byref(tp))
        return [tp[i] for i in range(n)] if n > 0 else []

    def synchronize(self):
        self._check_engine(lib().skirt_mcrt_synchronize(self.engine))

    def describe(self, path):
        """Writes the descriptors attach() would upload (grid, media, sources, instruments) to `path` in the
        canonical form of skirt_host_write_descriptors; no device needed (tests of the maintainer binding)."""
        self._check(lib().skirt_sim_describe(self._h, os.fspath(path).encode()))

    def fetch(self):
        """waits and copies the tallies to the host (summing the instruments over the ranks first)"""
        self._collective(self._check, lib().skirt_sim_fetch(self._h))

    def set_crossed(self, bins=16384):
        """Turn on DustSystem's cells-crossed histogram (writeCellsCrossed) for the following phases:
        every FILL and peel-off path counts in bin min(segments, bins - 1); 0 turns it off."""
        self._check_engine(lib().skirt_mcrt_set_crossed(self.engine, int(bins)))

    def crossed(self, bins=16384):
        """The cells-crossed histogram: paths per number of segments (waits for the device)."""
        h = np.zeros(int(bins), dtype=np.uint64)
        self._check_engine(lib().skirt_mcrt_download_crossed(self.engine, h.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                                             int(bins)))
        return h

    def column_densities(self, rays):
        """Column densities (kg/m2) of the grid along rays (n x 6: origin, direction), over the photon
        paths' walk (DustSystem::writeconvergence's DustGridPath::opticalDepth with the cell densities)."""
        r = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        out = np.zeros(len(r))
        dp = ctypes.POINTER(ctypes.c_double)
        self._check_engine(lib().skirt_mcrt_column_densities(self.engine, r.ctypes.data_as(dp), len(r),
                                                             out.ctypes.data_as(dp)))
        return out

    def stats(self):
        s = SkirtStats()
        self._check_engine(lib().skirt_mcrt_stats(self.engine, ctypes.byref(s)))
        return s.as_dict()

    def density(self):
        """The setup's cell densities [ncells, ncomp] (None without dust)."""
        p = lib().skirt_sim_density(self._h)
        if not p:
            return None
        return np.ctypeslib.as_array(p, shape=(self.info.ncells, self.info.ncomp)).copy()

    def labs(self):
        p = lib().skirt_sim_labs(self._h)
        if not p:
            return None
        return np.ctypeslib.as_array(p, shape=(self.info.ncells, self.info.nlambda)).copy()

    def instrument(self, i):
        """(frames [nslots, nlambda, nframe] or None, seds [nslots, nlambda] or None)"""
        ns, nf, hf, hs = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        p = lib().skirt_sim_instrument(self._h, i, ctypes.byref(ns), ctypes.byref(nf), ctypes.byref(hf),
                                       ctypes.byref(hs))
        if not p:
            raise SkirtError("no instrument %d" % i)
        nl = self.info.nlambda
        n_frames = ns.value * nl * nf.value if hf.value else 0
        arr = np.ctypeslib.as_array(p, shape=(n_frames + (ns.value * nl if hs.value else 0),)).copy()
        frames = arr[:n_frames].reshape(ns.value, nl, nf.value) if hf.value else None
        seds = arr[n_frames:].reshape(ns.value, nl) if hs.value else None
        return frames, seds

    def set_tallies(self, labs=None, instr=None):
        P = ctypes.POINTER(ctypes.c_double)
        la = np.ascontiguousarray(labs, dtype=np.float64) if labs is not None else None
        ia = np.ascontiguousarray(instr, dtype=np.float64) if instr is not None else None
        self._check(lib().skirt_sim_set_tallies(self._h, la.ctypes.data_as(P) if la is not None else None,
                                                ia.ctypes.data_as(P) if ia is not None else None))

    def write(self, prefix):
        self._check(lib().skirt_sim_write(self._h, os.fspath(prefix).encode()))

    def close(self):
        if getattr(self, "_h", None):
            lib().skirt_sim_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
