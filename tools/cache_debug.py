"""Debug of the cached trace kernel: Labs totals and counts against the oracle per SKIRT_AMD_CACHE_DEBUG mode
(0 cache, 1 every add straight to Labs, 2 unsorted FILL rays, 3 both) and with the cache off
(SKIRT_AMD_LABS_CACHE=0). Runs in a subprocess per mode. Tool only."""
import json, os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))

def one(name, packages):
    import numpy as np
    import skirt_amd as S
    import tree_models as T
    import tempfile
    d = tempfile.mkdtemp()
    path = T.write(name, d) if not name.endswith(".ski") else name
    sim = S.Simulation(path, packages=packages)
    sim.attach(0)
    sim.run_stellar()
    sim.fetch()
    st = sim.stats()
    labs = sim.labs()
    print(json.dumps({"labs": float(labs.sum()), "packets": st["packets"], "fill": st["segments_fill"],
                      "walk": st["segments_walk"], "peel": st["segments_peel"], "adds": st["absorb_adds"]}))

if __name__ == "__main__":
    if sys.argv[1] == "one":
        one(sys.argv[2], int(sys.argv[3])); sys.exit(0)
    name, packages = sys.argv[1], int(sys.argv[2])
    import oracle_lib as O
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import tree_models as T, tempfile
    path = T.write(name, tempfile.mkdtemp()) if not name.endswith(".ski") else name
    orc = O.run(path, rng=O.RNG_PHILOX, threads=16, packages=packages)
    print("oracle labs %.9e packets %d counts %s" % (orc.labs.sum(), orc.packets, O.counts(orc) if hasattr(O, "counts") else ""))
    for env in ({"SKIRT_AMD_LABS_CACHE": "0"}, {"SKIRT_AMD_CACHE_DEBUG": "0"}, {"SKIRT_AMD_CACHE_DEBUG": "1"},
                {"SKIRT_AMD_CACHE_DEBUG": "2"}, {"SKIRT_AMD_CACHE_DEBUG": "3"}):
        e = dict(os.environ); e.update(env)
        out = subprocess.run([sys.executable, __file__, "one", path, str(packages)], env=e, capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(env, line[-1] if line else out.stderr[-500:])
