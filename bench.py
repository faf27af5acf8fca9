#!/usr/bin/env python3
"""Photon packets per second of SKIRT's stellar emission phase on MI355X (BASELINE.json metric).

One "step" is one stellar-emission phase (MonteCarloSimulation::runstellaremission,
SKIRTcore/MonteCarloSimulation.cpp:251-261) over a fixed number of primary photon packets per GPU on the
C3 workload: Pan simulation, 128^3-resolution octree (levels 3-7, Saftly mass-fraction refinement), 25
wavelengths, peel-off to a 250x250 FullInstrument, Plummer stars + dust (benchmarks/c3_oct128.ski).
C3 shoots 4e7 packets per wavelength (1e9 in all) on 8 GPUs, so a step is one rank's share of it:
5e6 packets per wavelength, 1.25e8 packets. Weak scaling: every rank shoots its own slice of the global packet index space and, for N > 1, the
phase ends with the reference's reductions (Labs all-reduce, instrument all-reduce) done by RCCL.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5]
       (N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
       --dist-backend gloo runs the same sharded path over gloo (ranks may then share one GPU: rank r uses
       device LOCAL_RANK mod the visible device count), to rehearse N > 1 on a one-GPU box;
       --digest adds the summed tallies (Labs per wavelength, instrument totals) to the line, so that an
       N-rank run can be checked against one rank shooting the same global packets.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# Bytes one grid segment of the trace kernel actually reads in this engine's layouts,
# beside SURVEY 8(d)'s figure: octree leaf map 16 (one entry {node, cell|level, rho0}); Cartesian 8 (rho,
# the mesh is in LDS); Voronoi 48 + 16 k (the cell's header {exact site, rho0, id, count} and one 16-byte
# entry per neighbour, k = 15.5 on the C4 mesh)
ENGINE_SEGMENT_BYTES = {0: 8.0, 1: 16.0, 2: 48.0 + 16.0 * 15.5}

CONFIGS = {
    # name: (ski, packets per wavelength per rank, segment geometry bytes, description)
    # C3 is 4e7 packets per wavelength (1e9 in all) over 8 GPUs: 5e6 per wavelength per rank
    "c3": ("benchmarks/c3_oct128.ski", 5000000, 56, "C3 octree 128^3 (levels 3-7, mass fraction 1e-6), 25 lambda, peel-off"),
    # C2 is 1e8 packets over 10 wavelengths on one GPU: 1e7 per wavelength (rounds 1-3 ran 1e6)
    "c2": ("benchmarks/c2_cart64.ski", 10000000, 0, "C2 Cartesian 64^3, 10 lambda, peel-off"),
    # C4 is 1e9 packets over 25 wavelengths on 8 GPUs, like C3: 5e6 per wavelength per rank (rounds 1-3
    # ran 2e5, whose phase tail -- the last few long-lived packets -- then weighed 25x more per packet)
    "c4": ("benchmarks/c4_vor1e5.ski", 5000000, 438,
           "C4 Voronoi 1e5 sites (DustDensity), 25 lambda, peel-off"),
    # C5 at its per-GPU share of the 1e9-packet configuration, like C3 (round 2 ran 4e5 per wavelength)
    "c5": ("benchmarks/c5_oct128_sa.ski", 5000000, 56,
           "C5 = C3 + dust self-absorption (3 cycles) + dust emission, all phases per step"),
}
DUST_CONFIGS = ("c5",)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)
# f64 atomic requests per second (one scattered add per 64-byte request), measured chip-wide
# (tools/atomic_bench.hip, profiles/r01_atomic_bench.txt); requests carrying 2-8 adds of one line cost the same
ATOMIC_PEAK_REQUESTS = 2.36e10


# The chip's SIMDs and XCDs (MI355X_MICROARCH.md): the VALU-busy fraction is the gfx94x VALUBusy formula
# (ROCm 7.2 applies it to gfx950, MI355X_MICROARCH.md "rocprofv3 PMC slots"): SQ_ACTIVE_INST_VALU counts the
# quad-cycles (4 cycles) in which a wave issues a VALU instruction, summed over waves, over the SIMD-cycles of
# the launch; GRBM_GUI_ACTIVE is summed over the 8 XCDs (per XCD it times the launch at the 2.37 GHz the
# chip holds: profiles/r05_rocprof_*.txt)
SIMDS = 256 * 4
XCDS = 8


def pmc_traffic(config):
    """Per trace-kernel launch, from the committed rocprofv3 PMC passes of this same bench command
    (tools/pmc_traffic.py writes profiles/pmc_<config>.json): HBM bytes (FETCH_SIZE + WRITE_SIZE) and, where
    their passes ran, VALU wave-instructions; None when absent."""
    path = os.path.join(REPO, "profiles", "pmc_%s.json" % config)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    out = {"bytes_per_launch": d["traffic_bytes_per_launch"], "source": d["source"],
           "valu_per_launch": d.get("valu_insts_per_launch")}
    grbm = d.get("grbm_gui_active_per_launch")
    if grbm and d.get("valu_active_quads_per_launch"):
        simd_cycles = SIMDS * grbm / XCDS
        out["valu_busy"] = 4 * d["valu_active_quads_per_launch"] / simd_cycles
        if d.get("inst_active_quads_per_launch"):
            # any instruction issued, summed over the waves of a SIMD (types issue in parallel: may pass 1)
            out["inst_busy"] = 4 * d["inst_active_quads_per_launch"] / simd_cycles
    return out


def bound_of(hbm_frac, atomic_frac, valu_busy=None):
    """The trace kernel's limiter: whichever of HBM bandwidth, the f64 atomic request rate and the VALU (the
    PMC VALU-busy fraction, where the passes exist) it uses the largest fraction of, if that is at least half;
    else latency."""
    fracs = {"hbm": hbm_frac, "atomic": atomic_frac, "valu": valu_busy if valu_busy is not None else 0.0}
    best = max(fracs, key=fracs.get)
    return best if fracs[best] >= 0.5 else "latency"


def algorithmic_bytes(stats, geom_bytes, ncomp):
    """per segment the cell geometry (octree: 48 B box + 8 B index/neighbour;
    Voronoi: 4 + 28 k B for k ~ 15.5 neighbours; Cartesian: 0, the mesh lives in LDS) plus 8*Ncomp B of density; 16 B read-modify-write per absorbed
    segment (Labs) and per frame pixel update of a detection."""
    segs = stats["segments_fill"] + stats["segments_walk"] + stats["segments_peel"]
    return segs * (geom_bytes + 8 * ncomp) + stats["absorb_adds"] * 16 + stats["detects"] * 16


def cpu_baseline(ski, target_seconds=20.0):
    """The CPU oracle (a C++ restatement of the reference's photon loop, std::thread over packets with
    lock-free tallies like the reference's Parallel + LockFree::add) on this host's cores, on a bounded
    sample of the same workload: fewer packets per wavelength, all wavelengths. A short probe sizes the
    sample to about `target_seconds`. Returns (packets/s, threads, sample description)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib

    threads = max(1, min(16, os.cpu_count() or 1))  # the GPU box grants 16 CPUs per GPU
    # the probe's rate in the sample's own unit (packages x wavelengths, launched or not), from enough packets
    # that the threads' start-up does not dominate it (200 packages gave samples of ~7 s for a 20 s target)
    probe_pk = 1000
    probe = oracle_lib.run(ski, rng=oracle_lib.RNG_PHILOX, threads=threads, packages=probe_pk)
    nl = probe.nlambda
    rate = probe_pk * nl / max(probe.seconds, 1e-6)
    per = int(max(probe_pk, min(1e6, rate * target_seconds / nl)))
    r = oracle_lib.run(ski, rng=oracle_lib.RNG_PHILOX, threads=threads, packages=per)
    # counted like the GPU line: packages x wavelengths (wavelengths without source luminosity launch none)
    return per * nl / r.seconds, threads, "%d packets/wavelength x %d wavelengths = %d packets (%d launched) in %.1f s" % (
        per, nl, per * nl, r.packets, r.seconds)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--packets-per-lambda", type=int, default=0, help="per rank; default per config")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--threshold", type=int, default=0, help="idle lanes before a wave pulls rays (0 = engine default)")
    ap.add_argument("--slots", type=int, default=0, help="packet slots in flight (0 = engine default)")
    ap.add_argument("--trace-grid", type=int, default=0, help="trace kernel workgroups (0 = occupancy-derived)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI)")
    ap.add_argument("--digest", action="store_true", help="report the reduced tallies' sums")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = local
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            # gloo: ranks may share a device (rehearsal of the N > 1 path on a one-GPU box)
            device = local % max(1, torch.cuda.device_count())
            dist.init_process_group("gloo")
    torch.cuda.set_device(device)

    import skirt_amd
    from skirt_amd.sharding import TallyReducer, shard_slice

    ski_rel, ppl_default, geom_bytes, desc = CONFIGS[args.config]
    ski = os.path.join(REPO, ski_rel)
    ppl = args.packets_per_lambda or ppl_default
    t_setup = time.perf_counter()
    sim = skirt_amd.Simulation(ski, packages=float(ppl * world))
    setup_s = time.perf_counter() - t_setup  # host model setup: grid, densities (outside the timed region)
    info = sim.info
    # weak scaling: the phase has ppl packets per wavelength per rank; rank r shoots its slice of every
    # wavelength (the reference's IdenticalAssigner, skirt_mcrt_run_phase_shard)
    share = shard_slice(ppl * world, rank, world)[1] * info.nlambda
    sim.attach(device)
    if args.threshold or args.slots or args.trace_grid:
        sim.configure(slots=args.slots, grid=args.trace_grid, threshold=args.threshold)
    stream = torch.cuda.current_stream()
    sim.set_stream(stream.cuda_stream)
    n_labs, n_instr = sim.tally_sizes()
    labs = torch.zeros(max(1, n_labs), dtype=torch.float64, device="cuda")
    instr = torch.zeros(max(1, n_instr), dtype=torch.float64, device="cuda")
    sim.bind_tallies(labs.data_ptr(), instr.data_ptr())
    dust_phases = args.config in DUST_CONFIGS
    bound = [labs, instr]
    if dust_phases:
        dust = torch.zeros(max(1, n_labs), dtype=torch.float64, device="cuda")
        sim.bind_dust_labs(dust.data_ptr())
        bound.append(dust)
    # the reference's reductions (PanDustSystem::sumResults, Instrument::sumResults) as RCCL all-reduces,
    # called by the engine at the phase ends (skirt_mcrt_set_reducer)
    sim.set_reducer(TallyReducer(*bound))

    def step():
        # one simulation's photon phases from zeroed tallies, as the reference runs each phase once
        sim.zero_tallies()
        sim.run_stellar_shard(rank, world)  # + the Labs summed over the ranks at the phase end
        if dust_phases:
            # PanMonteCarloSimulation::runSelf: self-absorption cycles (dust Labs summed after each) and
            # dust emission, every phase sharded over the ranks' slices of every wavelength
            sim.run_dust(rank, world)
        sim.reduce_instruments()  # Instrument::sumResults

    for _ in range(args.warmup):
        step()
        sim.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    s0 = sim.stats()
    kernel_ms = []
    per_step = []  # every step zeroes the tallies and counters: collect each step's counters
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        sim.synchronize()
        st = sim.stats()
        kernel_ms.append(st["kernel_ms"])
        per_step.append(st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    s1 = sim.stats()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    delta = {k: sum(st[k] for st in per_step) for k in ("packets", "segments_fill", "segments_walk", "segments_peel",
                                                        "detects", "absorb_adds", "lane_slots", "labs_requests",
                                                        "packages")}
    delta["trace_ms"] = s1["trace_ms"] - s0["trace_ms"]
    delta["trace_launches"] = s1["trace_launches"] - s0["trace_launches"]
    trace_ms, trace_launches = delta["trace_ms"], delta["trace_launches"]
    # one unit for every config, SURVEY 8(d)'s: the packages x wavelengths of every phase the step ran (stellar;
    # C5 also its self-absorption cycles and dust emission), launched or not, over all ranks; the packets
    # actually launched (wavelengths and cells without luminosity launch none) are reported beside it
    n = torch.tensor([float(delta["packages"])], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(n)
    packets_all = float(n.item())
    if packets_all == 0 and not dust_phases:  # a library from before SkirtStats::packages (A/B against old builds)
        packets_all = float(ppl * world * info.nlambda * args.steps)
    value = packets_all / elapsed
    launched = torch.tensor([float(delta["packets"])], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(launched)
    launched_rate = float(launched.item()) / elapsed
    avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    segs = delta["segments_fill"] + delta["segments_walk"] + delta["segments_peel"]
    # the dominant kernel: traceKernel. Its algorithmic bytes per launch (without the
    # detections, which the detect kernel performs) over its average launch time (HIP events)
    trace_bytes = algorithmic_bytes(delta, geom_bytes, info.ncomp) - 16 * delta["detects"]
    launch_s = trace_ms / max(1, trace_launches) / 1e3
    bytes_per_launch = trace_bytes / max(1, trace_launches)
    achieved = bytes_per_launch / launch_s / 1e9
    # the PMC passes were taken on this config's own bench command (its default packets per rank); another
    # launch size would misprice them
    traffic = pmc_traffic(args.config) if ppl == ppl_default else None
    hbm_frac = achieved / HBM_PEAK_GBS
    traffic_frac = traffic["bytes_per_launch"] / launch_s / 1e9 / HBM_PEAK_GBS if traffic else None
    # instruction issue: the fraction of SIMD cycles the VALU is busy (PMC, cycle-based)
    valu_busy = traffic.get("valu_busy") if traffic else None
    # the same launch priced at the bytes this engine's layouts read (ENGINE_SEGMENT_BYTES)
    engine_bytes = (segs * ENGINE_SEGMENT_BYTES[info.grid_kind] + delta["absorb_adds"] * 16) / max(1, trace_launches)
    requests_per_s = delta["labs_requests"] / max(1e-9, trace_ms / 1e3)
    atomic_frac = requests_per_s / ATOMIC_PEAK_REQUESTS

    result = {
        "metric": "photon packets/sec (whole node), 128^3 octree, 1/2/4/8 MI355X + HBM%",
        "value": value,
        "unit": "photon packets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Plummer stars + Plummer dust model of the reference's survey probes; no datasets)",
        "config": {
            "workload": desc,
            "ski": ski_rel,
            "cells": info.ncells,
            "octree_nodes": info.nnodes,
            "device_cells": s1["device_cells"],
            "wavelengths": info.nlambda,
            "packets_per_step_per_gpu": share,
            # value counts packages x wavelengths of every phase; the
            # stellar SED emits nothing at the longest wavelengths, whose packets the reference
            # (dostellaremissionchunk) and the engine skip alike. The rate of packets actually launched:
            "launched_packets_per_s": launched_rate,
            "packages_per_step": packets_all / args.steps,
            "parallelism": "dp%d (packet sharding, RCCL all-reduce of Labs + instrument tallies per phase)" % world,
            "segments_per_packet": segs / max(1, delta["packets"]),
            "lane_use": (delta["segments_fill"] + delta["segments_walk"] + delta["segments_peel"]) / max(1, delta["lane_slots"]),
            "iterations": s1["iterations"],
            "trace_blocks_per_cu": s1["trace_blocks_per_cu"],
            "host_setup_s": round(setup_s, 3),
            "per_packet": {k: delta[k] / max(1, delta["packets"]) for k in
                           ("segments_fill", "segments_walk", "segments_peel", "absorb_adds", "detects")},
        },
        "roofline": {
            # the limiter: whichever of HBM bytes, the chip's f64 atomic request rate (the Labs adds) and the
            # VALU (PMC VALU-busy) the trace kernel uses the largest fraction of -- HBM as measured (PMC traffic)
            # when the passes exist, since a cached working set (the C4 Voronoi mesh, 30 MB, in the MALL) makes
            # the SURVEY bytes exceed what HBM delivers -- or "latency" when none is above half its peak
            # 
            "bound": bound_of(hbm_frac if traffic is None else traffic_frac, atomic_frac, valu_busy),
            # SURVEY 8(d)'s bytes over the launch time; where they exceed the HBM peak (a cache-resident
            # working set: the C4 mesh lives in the MALL) they are no roofline, and frac is the measured
            # HBM traffic's fraction instead
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": hbm_frac if (hbm_frac <= 1.0 or traffic_frac is None) else traffic_frac,
            "frac_basis": "algorithmic bytes (SURVEY 8(d))" if (hbm_frac <= 1.0 or traffic_frac is None) else
                          "measured HBM traffic (the SURVEY bytes model a cache-resident working set: %.2f of peak)" % hbm_frac,
            "atomic_frac": atomic_frac,
            "valu_busy": valu_busy,
            "inst_busy": traffic.get("inst_busy") if traffic else None,
            "traffic": traffic["bytes_per_launch"] if traffic else None,
            "kernel": {0: "traceKernel<cartesian>", 1: "traceKernel<octree leaf map>", 2: "traceKernel<voronoi>"}[info.grid_kind],
            "launch_ms_avg": launch_s * 1e3,
            "launches_per_step": trace_launches / args.steps,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "engine_bytes_per_launch": engine_bytes,
            "engine_gbs": engine_bytes / launch_s / 1e9,
            "engine_frac": engine_bytes / launch_s / 1e9 / HBM_PEAK_GBS,
            "traffic_source": traffic["source"] if traffic else None,
            "traffic_gbs": traffic["bytes_per_launch"] / launch_s / 1e9 if traffic else None,
            "traffic_frac": traffic_frac,
            # Labs adds are scattered f64 atomics, executed memory-side in 64-byte requests at a fixed
            # chip-wide request rate (tools/atomic_bench.hip, profiles/r01_atomic_bench.txt); adds of one
            # wave instruction that fall in one line share a request
            "labs_atomic_adds_per_s": delta["absorb_adds"] / max(1e-9, trace_ms / 1e3),
            "labs_requests_per_s": requests_per_s,
            "labs_adds_per_request": delta["absorb_adds"] / max(1, delta["labs_requests"]),
            "atomic_request_peak_measured": ATOMIC_PEAK_REQUESTS,
        },
        "phase_ms_avg": avg_kernel_s * 1e3,
    }
    if world > 1:
        # every rank's share of the work (its slice of every wavelength): segments and packets per rank
        mine = torch.tensor([float(delta["packets"]), float(segs), elapsed], dtype=torch.float64, device="cuda")
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        result["per_rank"] = [{"rank": r, "packets": int(e[0].item()), "segments": int(e[1].item()),
                               "elapsed_s": float(e[2].item())} for r, e in enumerate(every)]
        result["config"]["dist_backend"] = args.dist_backend
        if args.dist_backend != "nccl":
            result["config"]["note"] = "gloo rehearsal: ranks share %d device(s); not a hardware scaling number" % (
                torch.cuda.device_count())
    if args.digest:
        # the last step's tallies, already summed over the ranks by the engine's reducer
        sim.fetch()
        labs_l = sim.labs().sum(axis=0)
        frames, seds = sim.instrument(0)
        result["tally_digest"] = {"labs_per_lambda": [float(x) for x in labs_l],
                                  "labs_total": float(labs_l.sum()),
                                  "sed_total": float(seds.sum()) if seds is not None else None,
                                  "frame_total": float(frames.sum()) if frames is not None else None}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        v, cores, sample = cpu_baseline(ski)
        result["cpu_baseline"] = {"value": v, "unit": "photon packets/s", "cores": cores, "kind": "port",
                                  "sample": sample}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
