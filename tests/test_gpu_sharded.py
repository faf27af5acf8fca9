"""Multi-rank photon phases on the GPU: two processes share the box's GPU, each shooting its
shard_range slice of every phase (stellar emission, self-absorption cycles, dust emission), with the
tallies summed between phases exactly where the multi-GPU run sums them (bench.py uses RCCL; here gloo
on host copies, since both ranks sit on one device). The result must equal one unsharded run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import skirt_amd as S
from skirt_amd.sharding import shard_range

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SKI = os.path.join(GOLD, "ski", "pan_cart16_sa.ski")
PACKAGES = 1000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _host_allreduce(t):
    c = t.cpu()
    dist.all_reduce(c)
    t.copy_(c)


def _worker(rank, world, port, outdir):
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
        sim.zero_tallies()
        first, count = shard_range(sim.info.total_packets, rank, world)
        sim.run_stellar(first, count)
        sim.synchronize()
        _host_allreduce(labs)  # PanDustSystem::sumResults before the dust phases
        sim.run_dust(rank, world, lambda: (torch.cuda.synchronize(), _host_allreduce(dust)))
        sim.synchronize()
        _host_allreduce(instr)
        sim.fetch()
        if rank == 0:
            np.save(os.path.join(outdir, "labs.npy"), sim.labs())
            np.save(os.path.join(outdir, "dust.npy"), sim.labs_dust())
            np.save(os.path.join(outdir, "totals.npy"), np.array(sim.selfabs_totals()))
            frames, seds = sim.instrument(0)
            np.save(os.path.join(outdir, "seds.npy"), seds)
            np.save(os.path.join(outdir, "frames.npy"), frames)
    finally:
        dist.destroy_process_group()


def test_two_ranks_equal_one_run(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
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
