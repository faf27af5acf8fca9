"""Multi-GPU sharding of a photon phase: one process per GPU, contiguous packet ranges, one tally
reduction per phase.

The reference splits a phase's chunk index space over MPI processes (IdenticalAssigner /
SequentialAssigner, SKIRTcore/IdenticalAssigner.cpp:37-58, SequentialAssigner.cpp:37-59) and sums the
tallies at phase end (PanDustSystem::sumResults, Instrument::sumResults). Here every packet draws from
its own Philox stream keyed by its global index, so any split of [0, total) gives the same packets;
the reduction is one all-reduce per tally buffer over torch.distributed (RCCL over xGMI on the GPUs,
gloo in the CPU tests).
"""


def shard_range(total, rank, world):
    """(first, count) of rank `rank` in a contiguous, balanced split of [0, total) over `world` ranks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("rank %d outside a world of %d" % (rank, world))
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi - lo


def allreduce_tallies(*tensors):
    """Sums tally tensors (Labs, instrument frames and SEDs) over all ranks, in place."""
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return
    for t in tensors:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
