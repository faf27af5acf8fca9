// Locality study of the Labs adds: how many 64-byte memory-side atomic requests
// would the trace kernel issue for one launch's FILL rays under different ray orders and merge schemes?
//
// The FILL paths come from the oracle (Philox streams, the engine's packets) through oracle_set_fill_hook;
// cells are renumbered as the engine numbers device cells (engine.hip: depth-first octant order, groups of
// 8 sibling leaves aligned to one 64-byte line of a Labs row). Then a model of the persistent trace kernel
// (W waves of 64 lanes, one segment per lane-step, 64-ray pull chunks handed round robin to the waves,
// kLabsBuf = 16 adds buffered per lane) counts requests for:
//   run     consecutive adds of one ray in one line share a request (the engine's own count, 1.85 on C3)
//   instr   the transposed drain: one wave instruction per step carries 16 adds of 4 lanes; distinct lines
//   window  a per-wave merge over 16 steps (every add the wave buffered): distinct lines per window
//   cacheC  a workgroup-wide (4 waves) LDS cache of C lines, 8-way set associative LRU: requests = evictions
// and for a domain decomposition the region changes along each ray (regions = contiguous device-cell
// ranges of equal add counts).
//
// Build: g++ -O2 -std=c++17 -o /tmp/labs_locality tools/labs_locality.cpp -Ioracle -Iskirt_amd/csrc/host \
//          -Loracle -loracle -Wl,-rpath,$PWD/oracle -lpthread
// Run:   /tmp/labs_locality benchmarks/c3_oct128.ski skirt_amd/data <packages per lambda> <ell> [threads]
// Tool only: not part of the product or the tests.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <mutex>
#include <numeric>
#include <random>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "model.hpp"
#include "oracle.h"

namespace {

struct Ray {
    float r[3], k[3];
    uint32_t begin, n;
};

struct Store {
    std::mutex mu;
    std::vector<Ray> rays;
    std::vector<int> cells;  // reference cell numbers, then device lines
    int ell = -1;
};

void hook(void* user, int ell, const double r[3], const double k[3], const int* cells, int n) {
    Store* s = static_cast<Store*>(user);
    if (ell != s->ell || n == 0) return;
    std::lock_guard<std::mutex> g(s->mu);
    Ray y;
    for (int i = 0; i < 3; i++) { y.r[i] = (float)r[i]; y.k[i] = (float)k[i]; }
    y.begin = (uint32_t)s->cells.size();
    y.n = (uint32_t)n;
    s->cells.insert(s->cells.end(), cells, cells + n);
    s->rays.push_back(y);
}

// engine.hip's octree device numbering (upload of SKIRT_GRID_OCTREE)
std::vector<int> deviceCells(const skirt::OctreeGrid& g, int ncells) {
    std::vector<int> dev(ncells, -1);
    std::vector<int> stack{0};
    int next = 0;
    while (!stack.empty()) {
        const int l = stack.back();
        stack.pop_back();
        const int fc = g.firstChild[l];
        if (fc < 0) { dev[g.cellnumber[l]] = next++; continue; }
        bool leaves = true;
        for (int k = 0; k < 8 && leaves; k++) leaves = g.firstChild[fc + k] < 0;
        if (leaves) {
            next = (next + 7) & ~7;
            for (int k = 0; k < 8; k++) dev[g.cellnumber[fc + k]] = next++;
        } else {
            for (int k = 7; k >= 0; k--) stack.push_back(fc + k);
        }
    }
    return dev;
}

struct Result {
    double adds = 0, run = 0, instr = 0, window = 0;
    std::vector<double> cache, epoch;
};

// set-associative LRU cache of lines (8 ways); returns misses that evict (requests), flushes at the end
struct LineCache {
    int sets, ways = 8;
    int policy = 0;  // 0 LRU, 1 FIFO (round robin victim per set), 2 a victim chosen by the line's hash
    std::vector<unsigned> rr;
    std::vector<long long> tag;
    std::vector<unsigned> age;
    unsigned clock = 0;
    double requests = 0;
    explicit LineCache(int lines, int pol = 0) : policy(pol), rr(std::max(1, lines / 8), 0), sets(std::max(1, lines / 8)), tag((size_t)sets * 8, -1), age((size_t)sets * 8, 0) {}
    void touch(long long line) {
        const size_t s = (size_t)(((unsigned long long)line * 0x9E3779B97F4A7C15ull) >> 40) % (size_t)sets;
        long long* t = &tag[s * 8];
        unsigned* a = &age[s * 8];
        clock++;
        int victim = 0;
        bool empty = false;
        for (int w = 0; w < ways; w++) {
            if (t[w] == line) { if (policy == 0) a[w] = clock; return; }
            if (t[w] < 0) { victim = w; a[victim] = 0; empty = true; break; }
            if (a[w] < a[victim]) victim = w;
        }
        if (!empty && policy == 1) victim = (int)(rr[s]++ % 8);
        if (!empty && policy == 2) victim = (int)(((unsigned long long)line * 0xD6E8FEB86659FD93ull) >> 61);
        if (t[victim] >= 0) requests += 1;
        t[victim] = line;
        a[victim] = clock;
    }
    void flush() {
        for (long long x : tag)
            if (x >= 0) requests += 1;
        std::fill(tag.begin(), tag.end(), -1);
    }
};

// fill-only cache flushed every K steps (the workgroup's barrier): an add hits a cached line, or takes an
// empty way of its set, or goes out directly (through the per-lane buffers: consecutive direct adds of a
// lane in one line share a request)
// cold = true: at the barrier only the lines no add touched since the last barrier leave (an LRU of period K)
struct EpochCache {
    int sets;
    bool cold;
    std::vector<long long> tag;
    std::vector<char> used;
    double requests = 0;
    EpochCache(int lines, bool c) : sets(std::max(1, lines / 8)), cold(c), tag((size_t)sets * 8, -1), used((size_t)sets * 8, 0) {}
    bool touch(long long line) {
        const size_t s = (size_t)(((unsigned long long)line * 0x9E3779B97F4A7C15ull) >> 40) % (size_t)sets;
        long long* t = &tag[s * 8];
        for (int w = 0; w < 8; w++) {
            if (t[w] == line) { used[s * 8 + w] = 1; return true; }
            if (t[w] < 0) { t[w] = line; used[s * 8 + w] = 1; return true; }
        }
        return false;
    }
    void flush(bool all = false) {
        for (size_t i = 0; i < tag.size(); i++) {
            if (tag[i] >= 0 && (all || !cold || !used[i])) { requests += 1; tag[i] = -1; }
            used[i] = 0;
        }
    }
};

Result simulate(const std::vector<Ray>& rays, const std::vector<int>& lines, const std::vector<uint32_t>& order,
                int W, const std::vector<int>& cacheSizes, int kWavesPerWG, bool randomPulls, int K, bool coldFlush, bool missMerge, int policy) {
    constexpr int kChunk = 64, kBuf = 16, kLanes = 64;
    Result res;
    res.cache.assign(cacheSizes.size(), 0.0);
    res.epoch.assign(cacheSizes.size(), 0.0);
    const size_t nchunks = (order.size() + kChunk - 1) / kChunk;
    for (int g = 0; g < W / kWavesPerWG; g++) {
        std::vector<LineCache> caches;
        for (int c : cacheSizes) caches.emplace_back(c, policy);
        std::vector<EpochCache> ecaches;
        for (int c : cacheSizes) ecaches.emplace_back(c, coldFlush);
        std::vector<std::vector<long long>> lastDirect(cacheSizes.size(), std::vector<long long>((size_t)kWavesPerWG * kLanes, -1));
        long long gstep = 0;
        struct Wave {
            std::vector<uint32_t> q;
            size_t qi = 0;
            int ray[kLanes];
            uint32_t pos[kLanes];
            std::vector<long long> buf[kLanes];
            std::unordered_set<long long> win;
            long long lastLine[kLanes];
            int step = 0;
        };
        std::vector<Wave> waves(kWavesPerWG);
        for (int v = 0; v < kWavesPerWG; v++) {
            const int w = g * kWavesPerWG + v;
            for (size_t c0 = w; c0 < nchunks; c0 += W) {
                // random pulls: the chunk a wave gets is anywhere in the window of W chunks in flight
                const size_t c = randomPulls ? (c0 - c0 % W) + (size_t)(((c0 % W) * 2654435761ull) % (unsigned long long)W) : c0;
                if (c >= nchunks) continue;
                for (size_t i = c * kChunk; i < std::min(order.size(), (c + 1) * kChunk); i++) waves[v].q.push_back(order[i]);
            }
            for (int l = 0; l < kLanes; l++) { waves[v].ray[l] = -1; waves[v].lastLine[l] = -1; }
        }
        bool any = true;
        while (any) {
            any = false;
            if (++gstep % K == 0)
                for (auto& e : ecaches) e.flush();
            for (auto& wv : waves) {
                bool live = false;
                for (int l = 0; l < kLanes; l++) {
                    if (wv.ray[l] < 0 && wv.qi < wv.q.size()) { wv.ray[l] = (int)wv.q[wv.qi++]; wv.pos[l] = 0; wv.lastLine[l] = -1; }
                    if (wv.ray[l] < 0) continue;
                    live = true;
                    const Ray& y = rays[wv.ray[l]];
                    const long long line = lines[y.begin + wv.pos[l]];
                    res.adds += 1;
                    if (line != wv.lastLine[l]) res.run += 1;
                    wv.lastLine[l] = line;
                    wv.buf[l].push_back(line);
                    wv.win.insert(line);
                    for (auto& c : caches) c.touch(line);
                    for (size_t q = 0; q < ecaches.size(); q++) {
                        long long& ld = lastDirect[q][(size_t)(&wv - &waves[0]) * kLanes + l];
                        if (!ecaches[q].touch(line)) {
                            // a miss leaves at once, one request per add (LOC_MISS_MERGE=1: consecutive misses of
                            // a lane into one line share one)
                            if (!missMerge || ld != line) ecaches[q].requests += 1;
                            ld = line;
                        } else {
                            ld = -1;
                        }
                    }
                    if (++wv.pos[l] == y.n) wv.ray[l] = -1;
                }
                if (!live && wv.qi >= wv.q.size()) {
                    // drain what is left
                    for (int l = 0; l < kLanes; l += 4) {
                        std::unordered_set<long long> s;
                        for (int j = 0; j < 4; j++) { s.insert(wv.buf[l + j].begin(), wv.buf[l + j].end()); wv.buf[l + j].clear(); }
                        res.instr += (double)s.size();
                    }
                    res.window += (double)wv.win.size();
                    wv.win.clear();
                    continue;
                }
                any = true;
                // the transposed drain: instruction i = step % 16 carries lanes 4i..4i+3
                const int i = wv.step % kBuf;
                std::unordered_set<long long> s;
                for (int j = 0; j < 4; j++) { s.insert(wv.buf[4 * i + j].begin(), wv.buf[4 * i + j].end()); wv.buf[4 * i + j].clear(); }
                res.instr += (double)s.size();
                if (++wv.step % kBuf == 0) { res.window += (double)wv.win.size(); wv.win.clear(); }
            }
        }
        for (size_t c = 0; c < caches.size(); c++) {
            caches[c].flush();
            res.cache[c] += caches[c].requests;
            ecaches[c].flush(true);
            res.epoch[c] += ecaches[c].requests;
        }
    }
    return res;
}

// cube-map direction bin: face (6) x N x N
int dirBin(const float k[3], int N) {
    const float ax = std::fabs(k[0]), ay = std::fabs(k[1]), az = std::fabs(k[2]);
    int face;
    float u, v, m;
    if (ax >= ay && ax >= az) { face = k[0] > 0 ? 0 : 1; m = ax; u = k[1]; v = k[2]; }
    else if (ay >= az) { face = k[1] > 0 ? 2 : 3; m = ay; u = k[0]; v = k[2]; }
    else { face = k[2] > 0 ? 4 : 5; m = az; u = k[0]; v = k[1]; }
    int iu = std::min(N - 1, (int)((u / m * 0.5f + 0.5f) * N));
    int iv = std::min(N - 1, (int)((v / m * 0.5f + 0.5f) * N));
    return (face * N + iu) * N + iv;
}

unsigned morton3(unsigned x, unsigned y, unsigned z, int bits) {
    unsigned m = 0;
    for (int b = bits - 1; b >= 0; b--) m = (m << 3) | (((x >> b) & 1) << 2) | (((y >> b) & 1) << 1) | ((z >> b) & 1);
    return m;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s ski datadir packages_per_lambda ell [threads]\n", argv[0]);
        return 2;
    }
    const char* ski = argv[1];
    const char* datadir = argv[2];
    const double packages = std::atof(argv[3]);
    const int ell = std::atoi(argv[4]);
    const int threads = argc > 5 ? std::atoi(argv[5]) : 8;

    Store st;
    st.ell = ell;
    const std::string cacheFile = "/tmp/labs_locality_rays_" + std::to_string(ell) + "_" + argv[3] + ".bin";
    if (FILE* f = std::fopen(cacheFile.c_str(), "rb")) {
        size_t nr = 0, nc = 0;
        if (std::fread(&nr, sizeof nr, 1, f) != 1 || std::fread(&nc, sizeof nc, 1, f) != 1) return 1;
        st.rays.resize(nr);
        st.cells.resize(nc);
        if (std::fread(st.rays.data(), sizeof(Ray), nr, f) != nr || std::fread(st.cells.data(), 4, nc, f) != nc) return 1;
        std::fclose(f);
    } else {
        oracle_set_fill_hook(hook, &st);
        const uint64_t npp = (uint64_t)std::ceil(packages);
        OracleRun* run = oracle_run(ski, datadir, ORACLE_RNG_PHILOX, threads, packages, 0, npp * ell, npp * (ell + 1),
                                    ORACLE_PHASES_STELLAR, nullptr);
        if (!run) { std::fprintf(stderr, "oracle: %s\n", oracle_last_error()); return 1; }
        oracle_set_fill_hook(nullptr, nullptr);
        oracle_free(run);
        if (FILE* g = std::fopen(cacheFile.c_str(), "wb")) {
            size_t nr = st.rays.size(), nc = st.cells.size();
            std::fwrite(&nr, sizeof nr, 1, g);
            std::fwrite(&nc, sizeof nc, 1, g);
            std::fwrite(st.rays.data(), sizeof(Ray), nr, g);
            std::fwrite(st.cells.data(), 4, nc, g);
            std::fclose(g);
        }
    }

    skirt::MTRandom mt(4357);
    skirt::Model M = skirt::loadSki(ski, mt, datadir);
    const std::vector<int> dev = deviceCells(M.grid.tree, M.ncells());
    std::vector<int> lines(st.cells.size());
    for (size_t i = 0; i < st.cells.size(); i++) lines[i] = dev[st.cells[i]] >> 3;
    const size_t nr = st.rays.size();
    std::printf("lambda %d: %zu FILL rays, %zu adds (%.1f per ray), %d cells\n", ell, nr, st.cells.size(),
                (double)st.cells.size() / nr, M.ncells());

    const double ext = M.grid.tree.xmax - M.grid.tree.xmin;
    auto cellOf = [&](const Ray& y, int bits) {
        const int n = 1 << bits;
        auto c = [&](float x, double lo) { return (unsigned)std::min(n - 1, std::max(0, (int)((x - lo) / ext * n))); };
        return morton3(c(y.r[0], M.grid.tree.xmin), c(y.r[1], M.grid.tree.ymin), c(y.r[2], M.grid.tree.zmin), bits);
    };
    auto octant = [](const Ray& y) { return (y.k[0] > 0) | ((y.k[1] > 0) << 1) | ((y.k[2] > 0) << 2); };

    struct Order {
        std::string name;
        std::vector<unsigned long long> key;
    };
    std::vector<Order> orders;
    {
        Order o{"random", std::vector<unsigned long long>(nr)};
        std::mt19937_64 g(1);
        for (auto& x : o.key) x = g();
        orders.push_back(std::move(o));
    }
    auto add = [&](const std::string& name, auto f) {
        Order o{name, std::vector<unsigned long long>(nr)};
        for (size_t i = 0; i < nr; i++) o.key[i] = f(st.rays[i]);
        orders.push_back(std::move(o));
    };
    add("region8^3+octant", [&](const Ray& y) { return ((unsigned long long)cellOf(y, 3) << 3) | octant(y); });
    add("region16^3+octant", [&](const Ray& y) { return ((unsigned long long)cellOf(y, 4) << 3) | octant(y); });
    add("octant+region32^3", [&](const Ray& y) { return ((unsigned long long)octant(y) << 15) | cellOf(y, 5); });
    add("dir6x4^2+region16^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 4) << 12) | cellOf(y, 4); });
    add("dir6x4^2+region32^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 4) << 15) | cellOf(y, 5); });
    add("dir6x4^2+region4^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 4) << 6) | cellOf(y, 2); });
    add("dir6x4^2+region2^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 4) << 3) | cellOf(y, 1); });
    add("dir6x4^2+region8^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 4) << 9) | cellOf(y, 3); });
    add("dir6x2^2+region16^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 2) << 12) | cellOf(y, 4); });
    add("dir6x3^2+region16^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 3) << 12) | cellOf(y, 4); });
    add("dir6x8^2+region8^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 8) << 9) | cellOf(y, 3); });
    add("dir6x8^2+region32^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 8) << 15) | cellOf(y, 5); });
    add("dir6x8^2+region64^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 8) << 18) | cellOf(y, 6); });
    add("dir6x4^2+region64^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 4) << 18) | cellOf(y, 6); });
    add("dir6x2^2+region64^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 2) << 18) | cellOf(y, 6); });
    add("dir6x8^2+region16^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 8) << 12) | cellOf(y, 4); });
    add("dir6x16^2+region16^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 16) << 12) | cellOf(y, 4); });
    add("dir6x32^2+region16^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 32) << 12) | cellOf(y, 4); });
    add("dir6x64^2+region8^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 64) << 9) | cellOf(y, 3); });
    add("dir6x32^2+region64^3", [&](const Ray& y) { return ((unsigned long long)dirBin(y.k, 32) << 18) | cellOf(y, 6); });

    auto env = [](const char* n, int d) { const char* v = getenv(n); return v ? std::atoi(v) : d; };
    const int W = env("LOC_WAVES", 3072);
    const int G = env("LOC_GROUP", 4);
    const bool randomPulls = env("LOC_RANDOM_PULLS", 0) != 0;
    const int K = env("LOC_EPOCH", 64);
    std::vector<int> cacheSizes{512, 1024, 2048, 8192};
    if (const char* c = getenv("LOC_CACHES")) {
        cacheSizes.clear();
        for (const char* p = c; *p;) { cacheSizes.push_back(std::atoi(p)); while (*p && *p != ',') p++; if (*p) p++; }
    }
    const std::string only = getenv("LOC_ORDERS") ? getenv("LOC_ORDERS") : "";
    std::printf("waves %d, waves per cache %d, %s pulls, epoch %d steps\n", W, G, randomPulls ? "random" : "group-coherent", K);
    std::printf("%-24s %8s %8s %8s %8s", "order", "run", "instr", "window", "");
    for (int c : cacheSizes) std::printf(" lru%-6d", c);
    for (int c : cacheSizes) std::printf(" ep%-7d", c);
    std::printf("   (adds per 64-B request)\n");
    for (auto& o : orders) {
        if (!only.empty() && ("," + only + ",").find("," + o.name + ",") == std::string::npos) continue;
        std::vector<uint32_t> idx(nr);
        std::iota(idx.begin(), idx.end(), 0u);
        std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return o.key[a] < o.key[b]; });
        Result r = simulate(st.rays, lines, idx, W, cacheSizes, G, randomPulls, K, env("LOC_COLD", 1) != 0, env("LOC_MISS_MERGE", 0) != 0, env("LOC_POLICY", 0));
        std::printf("%-24s %8.3f %8.3f %8.3f %8s", o.name.c_str(), r.adds / r.run, r.adds / r.instr, r.adds / r.window, "");
        for (double c : r.cache) std::printf(" %9.3f", r.adds / c);
        for (double c : r.epoch) std::printf(" %9.3f", r.adds / c);
        std::printf("\n");
        std::fflush(stdout);
    }

    // domain decomposition: regions of contiguous device lines with equal add counts
    if (env("LOC_DOMAINS", 0)) {
        const int nlines = (*std::max_element(dev.begin(), dev.end()) >> 3) + 1;
        std::vector<double> hist(nlines, 0);
        for (int l : lines) hist[l] += 1;
        for (int R : {64, 256, 1024, 4096}) {
            std::vector<int> region(nlines);
            double acc = 0, total = (double)lines.size();
            for (int l = 0; l < nlines; l++) {
                region[l] = std::min(R - 1, (int)(acc / total * R));
                acc += hist[l];
            }
            double changes = 0;
            std::vector<int> span(R, 0);
            for (int l = 0; l < nlines; l++) span[region[l]]++;
            for (const Ray& y : st.rays)
                for (uint32_t i = 1; i < y.n; i++)
                    if (region[lines[y.begin + i]] != region[lines[y.begin + i - 1]]) changes += 1;
            const int maxSpan = *std::max_element(span.begin(), span.end());
            std::printf("regions %5d: %.2f region changes per FILL ray, %.1f adds per change; largest region %d lines (%d KB per lambda)\n",
                        R, changes / nr, total / std::max(1.0, changes), maxSpan, maxSpan * 64 / 1024);
        }
    }
    return 0;
}
