"""How much the Voronoi walk's per-step cost depends on the mesh's cache footprint (GPU, timing only).

C4's model with the Voronoi grid at several site counts: the cells shrink as the count grows, but a step's
work (a cell's header and ~15.5 entries, its bounds, one segment) stays the same, so the trace kernel's time
per lane-step tracks how well the mesh (48 B + 16 B per neighbour per cell: 3 MB at 1e4 sites, 30 MB at
1e5, 90 MB at 3e5) is served by the L2s (4 MB per XCD) and the MALL. DESIGN.md section 3, "Voronoi walk".
usage (GPU box): python3 tools/vor_l2_probe.py [packets per wavelength]
"""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import skirt_amd

    ppl = float(sys.argv[1]) if len(sys.argv) > 1 else 1e6
    text = open(os.path.join(REPO, "benchmarks", "c4_vor1e5.ski")).read()
    assert 'numParticles="100000"' in text
    for sites in (10000, 30000, 100000, 300000):
        with tempfile.TemporaryDirectory() as d:
            ski = os.path.join(d, "c4_probe.ski")
            open(ski, "w").write(text.replace('numParticles="100000"', 'numParticles="%d"' % sites))
            sim = skirt_amd.Simulation(ski, packages=ppl)
            sim.attach(0)
            sim.run_stellar()  # warm-up
            sim.synchronize()
            s0 = sim.stats()  # (zero_tallies resets the counts; the trace time accumulates, as in bench.py)
            sim.zero_tallies()
            sim.run_stellar()
            sim.synchronize()
            s1 = sim.stats()
            seg = sum(s1[k] for k in ("segments_fill", "segments_walk", "segments_peel"))
            lanes = s1["lane_slots"]
            tms = s1["trace_ms"] - s0["trace_ms"]
            print("sites %7d  cells %7d  trace %.1f ms  segments %.3e  lane use %.3f  ns per 1e3 lane-steps %.3f" % (
                sites, sim.info.ncells, tms, seg, seg / max(1, lanes), tms * 1e6 / max(1.0, lanes) * 1e3), flush=True)
            del sim


if __name__ == "__main__":
    main()
