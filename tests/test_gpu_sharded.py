"""Multi-rank photon phases on the GPU: two processes share the box's GPU, each shooting its slice of
every wavelength of every phase (stellar emission, self-absorption cycles, dust emission;
skirt_mcrt_run_phase_shard), with the engine's reducer summing the tallies where the reference sums them
(bench.py reduces over RCCL; here gloo on host copies, since both ranks sit on one device). The result
must equal one unsharded run.

Two reducer paths run: staged through host copies, and the stream-ordered one bench.py uses -- the
collective on CUDA tensors inside torch.cuda.stream(ExternalStream(engine stream)), so it is ordered
after the phase's kernels without a host synchronisation (sharding.py, TallyReducer's ExternalStream
branch; gloo's CUDA all-reduce here, RCCL in bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import skirt_amd as S
from skirt_amd.sharding import TallyReducer

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SKI = os.path.join(GOLD, "ski", "pan_cart16_sa.ski")
PACKAGES = 1000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir, via_host):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        sim = S.Simulation(SKI, packages=PACKAGES)
        sim.attach(0)
        stream = torch.cuda.current_stream()
        sim.set_stream(stream.cuda_stream)
        n_labs, n_instr = sim.tally_sizes()
        labs = torch.zeros(n_labs, dtype=torch.float64, device="cuda")
        instr = torch.zeros(n_instr, dtype=torch.float64, device="cuda")
        dust = torch.zeros(n_labs, dtype=torch.float64, device="cuda")
        sim.bind_tallies(labs.data_ptr(), instr.data_ptr())
        sim.bind_dust_labs(dust.data_ptr())
        red = TallyReducer(labs, instr, dust, via_host=via_host)
        sim.set_reducer(red)
        sim.zero_tallies()
        sim.run_stellar_shard(rank, world)  # + Labs summed at the phase end
        sim.run_dust(rank, world)           # + dust Labs summed after every cycle
        sim.fetch()                         # + instruments summed once
        tallies = [c[0] for c in red.calls]
        assert tallies[0] == S.TALLY_LABS and tallies[-1] == S.TALLY_INSTRUMENTS, tallies
        assert tallies.count(S.TALLY_DUST_LABS) == len(sim.selfabs_totals()) > 0, tallies
        if rank == 0:
            np.save(os.path.join(outdir, "labs.npy"), sim.labs())
            np.save(os.path.join(outdir, "dust.npy"), sim.labs_dust())
            np.save(os.path.join(outdir, "totals.npy"), np.array(sim.selfabs_totals()))
            frames, seds = sim.instrument(0)
            np.save(os.path.join(outdir, "seds.npy"), seds)
            np.save(os.path.join(outdir, "frames.npy"), frames)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("via_host", [True, False], ids=["host_staged", "stream_ordered"])
def test_two_ranks_equal_one_run(tmp_path, via_host):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), via_host), nprocs=2, join=True)
    full = S.Simulation(SKI, packages=PACKAGES)
    full.attach(0)
    full.run_stellar()
    full.run_dust()
    full.fetch()
    load = lambda n: np.load(os.path.join(tmp_path, n + ".npy"))  # noqa: E731
    np.testing.assert_allclose(load("totals"), full.selfabs_totals(), rtol=1e-9)
    np.testing.assert_allclose(load("labs"), full.labs(), rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(load("dust").sum(axis=0), full.labs_dust().sum(axis=0), rtol=1e-9)
    frames, seds = full.instrument(0)
    np.testing.assert_allclose(load("seds"), seds, rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(load("frames").sum(axis=2), frames.sum(axis=2), rtol=1e-9, atol=1e-300)


def test_crossed_histograms_of_the_shards_sum_to_the_whole():
    """ds_crossed is per process, as in the reference (DustSystem::write writes the root process's own
    _crossed, DustSystem.cpp:1004-1024; TextOutFile writes on the root only): each shard's histogram counts
    the paths of its own slice, and the shards' histograms add up to the unsharded run's, bin for bin."""
    ski = os.path.join(GOLD, "ski", "pan_oct.ski")
    full = S.Simulation(ski, packages=600)
    full.attach(0)
    full.set_crossed()
    full.run_stellar()
    whole = full.crossed()
    parts = []
    for r in range(3):
        sim = S.Simulation(ski, packages=600)
        sim.attach(0)
        sim.set_crossed()
        sim.set_reducer(lambda tally, ptr, n, stream: None)  # one process: nothing to sum
        sim.run_stellar_shard(r, 3)
        parts.append(sim.crossed())
        assert 0 < parts[-1].sum() < whole.sum()
    assert np.array_equal(sum(parts), whole)
