"""diagnostic: the 128^3 Cartesian model at several wavelength counts, engine vs oracle outliers (tool only)"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle_lib as O
import skirt_amd as S
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "ski")
for pts, glob_ in ((257, "0"), (200, "0"), (200, "1")):
    os.environ["SKIRT_AMD_LABS_GLOBAL"] = glob_
    text = open(os.path.join(GOLD, "pan_cart16.ski")).read()
    for n in ("X", "Y", "Z"):
        text = text.replace('<mesh%s type="MoveableMesh"><LinMesh numBins="16"/></mesh%s>' % (n, n),
                            '<mesh%s type="MoveableMesh"><LinMesh numBins="128"/></mesh%s>' % (n, n))
    text = text.replace('points="10"', 'points="%d"' % pts)
    path = "/tmp/cart_big_%d.ski" % pts
    open(path, "w").write(text)
    sim = S.Simulation(path, packages=20)
    sim.attach(0); sim.run_stellar(); sim.fetch()
    a = sim.labs()
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=20)
    b = orc.labs
    scale = np.maximum(np.abs(a), np.abs(b)); top = scale.max()
    rel = np.where(scale > 1e-15 * top, np.abs(a - b) / np.where(scale > 0, scale, 1), 0)
    idx = np.argwhere(rel > 1e-9)
    print("points", pts, "global", glob_, "packets", sim.stats()["packets"], orc.packets, "n>1e-9:", len(idx), "max", rel.max())
    for c, l in idx[:12]:
        print("   cell", c, "ell", l, "engine %.17g oracle %.17g rel %.3g  (cell/top %.3g)" % (a[c, l], b[c, l], rel[c, l], scale[c, l] / top))
    del a, b, orc, sim
