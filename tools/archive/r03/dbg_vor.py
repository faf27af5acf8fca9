# round 3 debug: engine vs oracle path histograms on vor_pan (which paths lose segments)
import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import oracle_lib as O
import skirt_amd as S
path = "tests/golden/ski/vor_pan.ski"
for pk in (1000, 100):
    sim = S.Simulation(path, packages=pk)
    sim.attach(0)
    sim.set_crossed(4096)
    sim.zero_tallies()
    sim.run_stellar()
    sim.fetch()
    st = sim.stats()
    h = sim.crossed(4096)
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=pk)
    print(pk, "engine", st["segments_fill"], st["segments_peel"], "oracle", orc.segments_fill, orc.segments_peel,
          "paths", int(h.sum()), int(orc.crossed.sum()))
    n = max(len(orc.crossed), int(np.nonzero(h)[0].max()) + 1)
    oc = np.zeros(n, np.int64); oc[:len(orc.crossed)] = orc.crossed
    d = h[:n].astype(np.int64) - oc
    idx = np.nonzero(d)[0]
    print("bins differing:", [(int(i), int(d[i])) for i in idx[:40]])
