"""The multi-GPU path's sharding and reduction, exercised with torch.distributed over gloo on the CPU
(world size 2): each rank shoots its shard_range slice of the packet index space (with the oracle in
Philox mode standing in for the engine, since the packet streams are identical), the tallies are
all-reduced with allreduce_tallies exactly as bench.py does on the GPUs, and the result equals one
unsharded run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
from skirt_amd.sharding import allreduce_tallies, shard_range

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SKI = os.path.join(GOLD, "ski", "pan_cart16.ski")
PACKAGES = 300


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tallies(res):
    parts = [res.labs.ravel()] + [f.ravel() for f in res.frames if f is not None] + \
            [s.ravel() for s in res.seds if s is not None]
    return np.concatenate(parts)


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        total = O.run(SKI, rng=O.RNG_PHILOX, packages=PACKAGES, packet_begin=0, packet_end=1).nlambda * PACKAGES
        first, count = shard_range(total, rank, world)
        res = O.run(SKI, rng=O.RNG_PHILOX, threads=2, packages=PACKAGES, packet_begin=first,
                    packet_end=first + count)
        t = torch.from_numpy(_tallies(res))
        n = torch.tensor([float(res.packets)], dtype=torch.float64)
        allreduce_tallies(t, n)
        if rank == 0:
            np.save(os.path.join(outdir, "reduced.npy"), t.numpy())
            np.save(os.path.join(outdir, "packets.npy"), n.numpy())
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions_exactly():
    for total in (0, 1, 7, 1000, 10 ** 9 + 7):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(c for _, c in spans) == total
            for (f0, c0), (f1, _) in zip(spans, spans[1:]):
                assert f0 + c0 == f1
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_two_rank_gloo_sharding_equals_single_run(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    reduced = np.load(os.path.join(tmp_path, "reduced.npy"))
    packets = np.load(os.path.join(tmp_path, "packets.npy"))[0]
    full = O.run(SKI, rng=O.RNG_PHILOX, threads=2, packages=PACKAGES)
    assert packets == full.packets
    ref = _tallies(full)
    np.testing.assert_allclose(reduced, ref, rtol=1e-12, atol=1e-300)
    assert ref.sum() > 0
