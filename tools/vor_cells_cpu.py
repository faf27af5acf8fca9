"""CPU check of the device Voronoi cells kernel's logic (skirt_amd/csrc/device/voronoi_cells.hip): its device
functions, compiled as plain C++ next to the host construction (host/voronoi.cpp) in one translation unit, run
for every cell of random site sets and are compared with the host build bit for bit (neighbour lists, bounding
boxes, volumes, centroids). The GPU test (tests/test_gpu_setup.py) repeats this with the kernel on the device.
Usage: python tools/vor_cells_cpu.py [nsites ...]"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MAIN = r'''
#include <cstdio>
#include <random>
int main(int argc, char** argv) {
    const int N = atoi(argv[1]);
    const int kind = atoi(argv[2]);
    std::mt19937_64 rng(12345 + N + kind);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::vector<double> sites;
    const double h = 1.0;
    while ((int)sites.size() < 3 * N) {
        double x, y, z;
        if (kind == 0) { x = U(rng) * 2 - 1; y = U(rng) * 2 - 1; z = U(rng) * 2 - 1; }
        else {  // Plummer, c = 0.1, clipped to the box
            const double t = std::cbrt(U(rng));
            const double r = 0.1 * t / std::sqrt((1 - t) * (1 + t));
            const double ct = 2 * U(rng) - 1, ph = 6.283185307179586 * U(rng), st = std::sqrt(1 - ct * ct);
            x = r * st * std::cos(ph); y = r * st * std::sin(ph); z = r * ct;
            if (std::fabs(x) > h || std::fabs(y) > h || std::fabs(z) > h) continue;
        }
        sites.push_back(x); sites.push_back(y); sites.push_back(z);
    }
    skirt::VoronoiGrid g;
    skirt::buildVoronoi(g, sites, -h, h, -h, h, -h, h);
    const skirt::SiteTree tree(sites);
    const int maxIds = 96;
    std::vector<int> ids((size_t)N * maxIds), nids(N);
    std::vector<double> bbox(6 * (size_t)N), vol(N), cen(3 * (size_t)N);
    VorArgs A{};
    A.site = sites.data(); A.n = N;
    double box[6] = {-h, -h, -h, h, h, h};
    for (int q = 0; q < 6; q++) A.box[q] = box[q];
    const double wx = 2 * h, wy = 2 * h, wz = 2 * h;
    A.L = std::sqrt(wx * wx + wy * wy + wz * wz);
    A.nodes = reinterpret_cast<const SkirtKdNode*>(tree.nodes().data());
    A.perm = tree.perm().data();
    A.maxIds = maxIds; A.ids = ids.data(); A.nids = nids.data(); A.bbox = bbox.data(); A.volume = vol.data();
    A.centroid = cen.data();
    Work* W = new Work;
    int over = 0, bad = 0;
    for (int i = 0; i < N; i++) {
        if (!cellOf(A, *W, i)) { over++; continue; }
        bool ok = nids[i] == g.nbrOffset[i + 1] - g.nbrOffset[i];
        for (int q = 0; ok && q < nids[i]; q++) ok = ids[(size_t)i * maxIds + q] == g.nbrList[g.nbrOffset[i] + q];
        for (int q = 0; ok && q < 6; q++) ok = bbox[6 * (size_t)i + q] == g.bbox[6 * (size_t)i + q];
        ok = ok && vol[i] == g.volume[i];
        for (int q = 0; ok && q < 3; q++) ok = cen[3 * (size_t)i + q] == g.centroid[3 * (size_t)i + q];
        if (!ok && bad++ < 5) printf("cell %d differs: nids %d vs %d, vol %.17g vs %.17g\n", i, nids[i],
                                     g.nbrOffset[i + 1] - g.nbrOffset[i], vol[i], g.volume[i]);
    }
    printf("N=%d kind=%d: %d cells differ, %d out of the device capacities\n", N, kind, bad, over);
    return bad ? 1 : 0;
}
'''


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [2000, 20000]
    src = open(os.path.join(REPO, "skirt_amd", "csrc", "device", "voronoi_cells.hip")).read()
    body = src[src.index("namespace {"):src.index("}  // namespace")]
    body = re.sub(r"__global__.*?\n}\n", "", body, flags=re.S)  # the kernel itself
    host = open(os.path.join(REPO, "skirt_amd", "csrc", "host", "voronoi.cpp")).read()
    host = host.replace('#include "voronoi.hpp"', '#include "%s/skirt_amd/csrc/host/voronoi.hpp"' % REPO)
    host = host.replace('#include "mt_random.hpp"', '#include "%s/skirt_amd/csrc/host/mt_random.hpp"' % REPO)
    tu = "\n".join([
        "#include <cfloat>", "#include <cmath>", "#include <cstdint>", "#include <cstdlib>",
        "#define __device__", "#define __forceinline__ inline",
        '#include "%s/include/skirt_mcrt.h"' % REPO,
        host.replace("}  // namespace\n\nvoid VoronoiGrid::blockIndices", "SiteTree* dummy_;\n}  // namespace\n\nvoid VoronoiGrid::blockIndices"),
        "using namespace std;",
        body + "}\n",
        "namespace skirt { using ::skirt::SiteTree; }",
        MAIN,
    ])
    d = tempfile.mkdtemp(prefix="vorcells_")
    cpp, exe = os.path.join(d, "t.cpp"), os.path.join(d, "t")
    open(cpp, "w").write(tu)
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe, cpp, "-lpthread"], check=True)
    rc = 0
    for n in sizes:
        for kind in (0, 1):
            rc |= subprocess.run([exe, str(n), str(kind)]).returncode
    sys.exit(rc)


if __name__ == "__main__":
    main()
