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
    the work already queued on the engine's HIP stream (a collective waits for the current stream)."""

    def __init__(self, *tensors, via_host=False):
        self.by_ptr = {t.data_ptr(): t for t in tensors}
        self.via_host = via_host  # stage device buffers through host memory (gloo ranks sharing one GPU)
        self.calls = []  # (tally, n) of every reduction, for tests and logs

    def __call__(self, tally, ptr, n, stream):
        import torch
        import torch.distributed as dist

        t = self.by_ptr.get(ptr)
        if t is None or t.numel() < n:
            raise ValueError("the engine asked to reduce a buffer that is not a bound tensor")
        self.calls.append((tally, n))
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return
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
