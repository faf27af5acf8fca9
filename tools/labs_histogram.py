"""Distribution of Labs atomic adds over (cell, wavelength): run with a counting build
(SKIRT_AMD_LIB=libskirt_amd_count.so adds 1.0 per absorbing segment instead of the luminosity)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import skirt_amd as S

ski = sys.argv[1] if len(sys.argv) > 1 else "benchmarks/c3_oct128.ski"
sim = S.Simulation(ski, packages=float(sys.argv[2]) if len(sys.argv) > 2 else 40000.0)
sim.attach(0)
sim.run_stellar()
sim.fetch()
counts = sim.labs()  # [cell, lambda]
flat = np.sort(counts.ravel())[::-1]
tot = flat.sum()
print("total adds %.4g over %d (cell,lambda) entries, %d nonzero" % (tot, flat.size, (flat > 0).sum()))
for k in (1024, 4096, 8192, 16384, 65536, 262144):
    print("top %7d entries: %.3f of adds" % (k, flat[:k].sum() / tot))
percell = np.sort(counts.sum(axis=1))[::-1]
for k in (256, 1024, 4096, 16384):
    print("top %7d cells: %.3f of adds" % (k, percell[:k].sum() / tot))
