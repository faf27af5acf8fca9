"""The multi-GPU path's sharding and reductions, exercised with torch.distributed over gloo on the CPU.

Each rank shoots its slice of every wavelength of every phase (the reference's IdenticalAssigner,
IdenticalAssigner.cpp:37-58; skirt_mcrt_run_phase_shard on the GPUs), with the oracle in Philox mode
standing in for the engine, since the packet streams are identical. The oracle calls its reducer where
the engine calls its own (the stellar Labs after the stellar phase, the dust Labs after every
self-absorption cycle); the reducer sums with torch.distributed exactly as TallyReducer does on the GPUs.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
from skirt_amd.sharding import allreduce_tallies, shard_packets, shard_slice

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKI_SA = os.path.join(GOLD, "ski", "pan_cart16_sa.ski")
SKI_C3 = os.path.join(REPO, "benchmarks", "c3_oct128.ski")
PACKAGES = 300


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tallies(res):
    parts = [res.labs.ravel()] + [f.ravel() for f in res.frames if f is not None] + \
            [s.ravel() for s in res.seds if s is not None]
    return np.concatenate(parts)


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _sum(_tally, arr):
    t = torch.from_numpy(arr)  # shares the oracle's host array: summed in place
    dist.all_reduce(t)


def _worker_all_phases(rank, world, port, outdir):
    _init(rank, world, port)
    try:
        res = O.run(SKI_SA, rng=O.RNG_PHILOX, threads=2, packages=PACKAGES, phases=O.PHASES_ALL, rank=rank,
                    world=world, reduce=_sum)
        t = torch.from_numpy(np.concatenate([f.ravel() for f in res.frames] + [s.ravel() for s in res.seds]))
        n = torch.tensor([float(res.packets)], dtype=torch.float64)
        allreduce_tallies(t, n)  # Instrument::sumResults, once at the end
        if rank == 0:
            np.save(os.path.join(outdir, "instr.npy"), t.numpy())
            np.save(os.path.join(outdir, "packets.npy"), n.numpy())
            np.save(os.path.join(outdir, "labs.npy"), res.labs)
            np.save(os.path.join(outdir, "dust.npy"), res.labs_dust)
            np.save(os.path.join(outdir, "totals.npy"), np.array(res.labs_dust_totals))
    finally:
        dist.destroy_process_group()


def _worker_balance(rank, world, port, outdir, packages):
    _init(rank, world, port)
    try:
        res = O.run(SKI_C3, rng=O.RNG_PHILOX, threads=1, packages=packages, rank=rank, world=world)
        seg = torch.tensor([float(res.segments), float(res.packets)], dtype=torch.float64)
        out = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(out, seg)
        if rank == 0:
            np.save(os.path.join(outdir, "work.npy"), torch.stack(out).numpy())
    finally:
        dist.destroy_process_group()


def test_shard_slices_cover_every_wavelength_exactly():
    for npp in (1, 7, 1000, 10 ** 9 + 7):
        for world in (1, 2, 3, 8):
            spans = [shard_slice(npp, r, world) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(c for _, c in spans) == npp
            for (f0, c0), (f1, _) in zip(spans, spans[1:]):
                assert f0 + c0 == f1
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    # the union of the ranks' global packets is the phase, each once, and every rank has every wavelength
    npp, nl, world = 11, 5, 3
    got = sorted(p for r in range(world) for p in shard_packets(npp, nl, r, world))
    assert got == list(range(npp * nl))
    for r in range(world):
        assert sorted({p // npp for p in shard_packets(npp, nl, r, world)}) == list(range(nl))
    with pytest.raises(ValueError):
        shard_slice(10, 2, 2)


def test_shard_slice_matches_the_engine_abi():
    import skirt_amd as S
    import ctypes

    lo, n = ctypes.c_uint64(), ctypes.c_uint64()
    for npp, r, w in ((1000, 0, 8), (1000, 7, 8), (10 ** 12 + 3, 5, 7), (3, 2, 8)):
        S.lib().skirt_mcrt_shard_slice(npp, r, w, ctypes.byref(lo), ctypes.byref(n))
        assert (lo.value, n.value) == shard_slice(npp, r, w)


def test_two_rank_gloo_shards_with_self_absorption_equal_single_run(tmp_path):
    """Stellar phase, self-absorption cycles (convergence-driven schedule, the dust Labs summed after each)
    and dust emission, over 2 ranks: the summed tallies and the per-cycle totals equal one run."""
    mp.spawn(_worker_all_phases, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    load = lambda n: np.load(os.path.join(tmp_path, n + ".npy"))  # noqa: E731
    full = O.run(SKI_SA, rng=O.RNG_PHILOX, threads=2, packages=PACKAGES, phases=O.PHASES_ALL)
    assert load("packets")[0] == full.packets
    np.testing.assert_allclose(load("totals"), full.labs_dust_totals, rtol=1e-12)
    np.testing.assert_allclose(load("labs"), full.labs, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(load("dust"), full.labs_dust, rtol=1e-12, atol=1e-300)
    ref = np.concatenate([f.ravel() for f in full.frames] + [s.ravel() for s in full.seds])
    np.testing.assert_allclose(load("instr"), ref, rtol=1e-12, atol=1e-300)
    assert len(full.labs_dust_totals) > 1 and ref.sum() > 0


def test_eight_rank_gloo_shards_balance_the_c3_work(tmp_path):
    """C3 (the 128^3 octree, 25 wavelengths, 5 of them without stellar luminosity) over 8 ranks: every
    rank shoots every wavelength, so the ranks' grid segments (the trace kernel's work) agree to within
    5 % of the mean. The contiguous split of the wavelength-slowest packet space used before gave a
    max/mean of 2.16, one rank holding only wavelengths without luminosity."""
    packages = 1600
    mp.spawn(_worker_balance, args=(8, _free_port(), str(tmp_path), packages), nprocs=8, join=True)
    work = np.load(os.path.join(tmp_path, "work.npy"))
    segs, pkts = work[:, 0], work[:, 1]
    assert np.all(pkts == pkts[0]) and pkts[0] > 0
    print("C3 segments per rank:", segs.astype(int).tolist(), "max/mean %.4f" % (segs.max() / segs.mean()))
    assert segs.max() / segs.mean() <= 1.05, segs


def _worker_reducer_failure(rank, world, port, outdir, mode):
    from skirt_amd.sharding import TallyReducer

    _init(rank, world, port)
    try:
        t = torch.ones(8, dtype=torch.float64)
        red = TallyReducer(t)
        res = [red(0, t.data_ptr(), 8, 0)]  # every rank healthy: summed
        if rank == 1 and mode == "lookup":
            res.append(red(0, t.data_ptr() + 8, 8, 0))  # a buffer that is not a bound tensor
        elif rank == 1 and mode == "abort":
            red.abort("rank 1: the photon phase failed")  # failed outside the reducer
            res.append(-1)
        else:
            res.append(red(0, t.data_ptr(), 8, 0))
        res.append(red(0, t.data_ptr(), 8, 0))  # after a failure: refused without a collective
        np.save(os.path.join(outdir, "r%d.npy" % rank), np.array(res + [t.sum().item()], dtype=np.float64))
        with open(os.path.join(outdir, "e%d.txt" % rank), "w") as f:
            f.write(str(red.error))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("mode", ["lookup", "abort"])
def test_reducer_failure_reaches_every_rank_without_a_hang(tmp_path, mode):
    """TallyReducer's failure agreement (the reference's Parallel::call: the first failure stops every worker,
    Parallel.cpp:181-193). Rank 1 of 3 fails at the second reduction, either in the reducer (a buffer lookup)
    or outside it (abort(), as Simulation calls it when a phase raises). Every rank's second reduction then
    returns 1 instead of entering an all-reduce rank 1 never joins, the third is refused at once, and only the
    first sum happened (a hang fails the test through its timeout)."""
    world = 3
    mp.spawn(_worker_reducer_failure, args=(world, _free_port(), str(tmp_path), mode), nprocs=world, join=True)
    for r in range(world):
        res = np.load(os.path.join(tmp_path, "r%d.npy" % r))
        second = -1 if (r == 1 and mode == "abort") else 1
        assert res.tolist() == [0, second, 1, 8 * world], (r, res)
        err = open(os.path.join(tmp_path, "e%d.txt" % r)).read()
        if r == 1:
            assert ("rank 1: the photon phase failed" if mode == "abort" else "not a bound tensor") in err
        else:
            assert err == "another rank failed"
