"""Multi-GPU sharding of the photon phases: one process per GPU, every rank shooting its slice of every
wavelength, the tallies summed over the ranks at the reference's reduction points.

The reference numbers a phase's chunks wavelength-fastest (`ell = index % Nlambda`,
SKIRTcore/MonteCarloSimulation.cpp:267) and its IdenticalAssigner gives every process a block of chunks
at EVERY wavelength (IdenticalAssigner.cpp:37-58, through a SequentialAssigner over the chunks,
SequentialAssigner.cpp:37-59). The engine does the same with chunks of one packet:
skirt_mcrt_run_phase_shard shoots packets [lo, lo + count) of each wavelength, lo and count from
shard_slice below. Every packet draws from its own Philox stream keyed by its global index
(wavelength * npp + packet), so the union of the ranks' packets is one unsharded run.

The sums are the reference's PanDustSystem::sumResults (the stellar Labs after the stellar phase, the
dust Labs after every self-absorption cycle) and Instrument::sumResults (once, before output). The engine
calls its reducer (skirt_mcrt_set_reducer) at those points; TallyReducer implements it with
torch.distributed (RCCL over xGMI on the GPUs, gloo in the CPU tests).
"""


def shard_slice(npp, rank, world):
    """(lo, count) of rank `rank`: packets [lo, lo + count) of every wavelength of a phase with npp packets
    per wavelength (skirt_mcrt_shard_slice; SequentialAssigner's balanced contiguous blocks)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank %d outside a world of %d" % (rank, world))
    lo = npp * rank // world
    hi = npp * (rank + 1) // world
    return lo, hi - lo


def shard_packets(npp, nlambda, rank, world):
    """The global packet indices of rank `rank` (wavelength ell has packets ell*npp ... ell*npp + npp - 1),
    in the engine's order: for a small check of which packets a shard covers."""
    lo, n = shard_slice(npp, rank, world)
    return [ell * npp + lo + j for ell in range(nlambda) for j in range(n)]


def allreduce_tallies(*tensors):
    """Sums tally tensors over all ranks, in place."""
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return
    for t in tensors:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)


class TallyReducer:
    """The engine's reducer over torch.distributed: sums the device buffer the engine names (one of the
    tensors bound with bind_tallies / bind_dust_labs) over all ranks, in place, on the engine's stream.

    The engine passes the buffer's address; the reducer sums the bound tensor that starts there, after
    the work already queued on the engine's HIP stream (a collective waits for the current stream).

    Failure semantics (the reference's Parallel::call stops every worker at the first exception,
    SKIRTcore/Parallel.cpp:181-193; its MPI ranks would abort): before each sum the ranks agree, in a one-int
    all-reduce, that none has failed. A rank whose buffer lookup fails, or which failed outside the reducer
    and calls abort() (Simulation does so when one of its phases raises), contributes a failure there, and
    then every rank returns non-zero from that reduction instead of entering a collective that some rank
    will never join. A rank that has seen a failure makes no further collective calls."""

    def __init__(self, *tensors, via_host=False, agree=True):
        self.by_ptr = {t.data_ptr(): t for t in tensors}
        self.via_host = via_host  # stage device buffers through host memory (gloo ranks sharing one GPU)
        self.agree = agree  # the failure agreement before each sum
        self.device = tensors[0].device if tensors else None
        self.calls = []  # (tally, n) of every reduction, for tests and logs
        self.error = None  # why the reductions stopped (this rank's failure or another rank's)

    @staticmethod
    def _world():
        import torch.distributed as dist

        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1

    def _all_ok(self, ok):
        """every rank's verdict: True when no rank reports a failure"""
        import torch
        import torch.distributed as dist

        dev = self.device if (dist.get_backend() == "nccl" and self.device is not None) else "cpu"
        flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.SUM)
        return int(flag.item()) == 0

    def abort(self, why="a phase failed on this rank"):
        """this rank failed outside the reducer: the other ranks learn it at their next reduction, and fail it
        too, instead of waiting in a collective this rank will never join"""
        if self.error is not None:
            return
        self.error = why
        if self.agree and self._world() > 1:
            self._all_ok(False)

    def __call__(self, tally, ptr, n, stream):
        """0 when the tally was summed; 1 when this rank or another one failed (no collective entered)"""
        import torch
        import torch.distributed as dist

        if self.error is not None:
            return 1
        t = self.by_ptr.get(ptr)
        ok = t is not None and t.numel() >= n
        world = self._world()
        if self.agree and world > 1 and not self._all_ok(ok):
            self.error = "the engine asked to reduce a buffer that is not a bound tensor" if not ok else \
                "another rank failed"
            return 1
        if not ok:
            self.error = "the engine asked to reduce a buffer that is not a bound tensor"
            return 1
        self.calls.append((tally, n))
        if world == 1:
            return 0
        view = t[:n]
        if t.is_cuda and self.via_host:
            if stream:
                torch.cuda.ExternalStream(stream, device=t.device).synchronize()
            torch.cuda.synchronize(t.device)
            host = view.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM)
            view.copy_(host)
            torch.cuda.synchronize(t.device)
        elif t.is_cuda and stream:
            with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=t.device)):
                dist.all_reduce(view, op=dist.ReduceOp.SUM)
        else:
            dist.all_reduce(view, op=dist.ReduceOp.SUM)
        return 0
