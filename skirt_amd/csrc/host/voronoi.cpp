// Voronoi tessellation restricted to a box, by convex-cell clipping; see voronoi.hpp.
#include "voronoi.hpp"

#include <algorithm>
#include <array>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>

#include "mt_random.hpp"

namespace skirt {

namespace {

using V3 = std::array<double, 3>;

inline double dot(const V3& a, const V3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline V3 sub(const V3& a, const V3& b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
inline V3 cross(const V3& a, const V3& b) {
    return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}

struct Face {
    int id;                // neighbour cell or wall (-1 .. -6)
    std::vector<V3> pts;   // convex polygon, in order around the face
};

// A convex cell: its faces. Clipping keeps the half space dot(n, x) <= c.
struct Cell {
    std::vector<Face> faces;

    double maxDist2(const V3& s) const {
        double r = 0;
        for (const Face& f : faces)
            for (const V3& p : f.pts) r = std::max(r, dot(sub(p, s), sub(p, s)));
        return r;
    }

    // the point where edge (a, b) crosses the plane, computed from the lexicographically smaller end so
    // that the two faces sharing the edge produce the same bits
    static V3 crossing(const V3& a0, const V3& b0, const V3& n, double c) {
        const bool swap = b0 < a0;
        const V3& a = swap ? b0 : a0;
        const V3& b = swap ? a0 : b0;
        const double da = dot(n, a) - c, db = dot(n, b) - c;
        const double t = da / (da - db);
        return {a[0] + t * (b[0] - a[0]), a[1] + t * (b[1] - a[1]), a[2] + t * (b[2] - a[2])};
    }

    // clips by dot(n, x) <= c; the new face gets `id`. Returns whether the cell changed.
    bool clip(const V3& n, double c, double tol, int id) {
        double dmax = -DBL_MAX;
        for (const Face& f : faces)
            for (const V3& p : f.pts) dmax = std::max(dmax, dot(n, p) - c);
        if (dmax <= tol) return false;  // entirely inside: the plane does not cut
        std::vector<V3> cap;
        std::vector<Face> out;
        out.reserve(faces.size() + 1);
        for (const Face& f : faces) {
            const int m = (int)f.pts.size();
            Face g{f.id, {}};
            for (int k = 0; k < m; k++) {
                const V3& a = f.pts[k];
                const V3& b = f.pts[(k + 1) % m];
                const double da = dot(n, a) - c, db = dot(n, b) - c;
                const bool ina = da <= tol, inb = db <= tol;
                if (ina) {
                    g.pts.push_back(a);
                    if (da >= -tol) cap.push_back(a);  // on the plane: also a vertex of the new face
                }
                if (ina != inb && std::fabs(da) > tol && std::fabs(db) > tol) {
                    V3 q = crossing(a, b, n, c);
                    g.pts.push_back(q);
                    cap.push_back(q);
                }
            }
            if (g.pts.size() >= 3) out.push_back(std::move(g));
        }
        // the new face: the distinct cut points ordered by angle around their centre
        std::sort(cap.begin(), cap.end());
        cap.erase(std::unique(cap.begin(), cap.end()), cap.end());
        if (cap.size() >= 3) {
            V3 ctr{0, 0, 0};
            for (const V3& p : cap)
                for (int q = 0; q < 3; q++) ctr[q] += p[q];
            for (int q = 0; q < 3; q++) ctr[q] /= (double)cap.size();
            // in-plane basis of equal lengths: u and n^ x u (n normalized, or the angles would be stretched)
            const double nl = std::sqrt(dot(n, n));
            const V3 nh{n[0] / nl, n[1] / nl, n[2] / nl};
            V3 u = sub(cap[0], ctr);
            V3 v = cross(nh, u);
            std::vector<std::pair<double, V3>> ang;
            for (const V3& p : cap) {
                const V3 d = sub(p, ctr);
                ang.push_back({std::atan2(dot(d, v), dot(d, u)), p});
            }
            std::sort(ang.begin(), ang.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
            Face nf{id, {}};
            for (auto& a : ang) nf.pts.push_back(a.second);
            out.push_back(std::move(nf));
        }
        faces = std::move(out);
        return true;
    }
};


// A k-d tree over the sites (leaves of at most 8, split at the median of the widest axis) answering
// "the k nearest sites to p other than `self`, in (squared distance, index) order".
class SiteTree {
public:
    explicit SiteTree(const std::vector<double>& s) : site_(s), idx_(s.size() / 3) {
        for (size_t q = 0; q < idx_.size(); q++) idx_[q] = (int)q;
        if (!idx_.empty()) build(0, (int)idx_.size());
    }

    void nearest(const V3& p, int self, int k, std::vector<std::pair<double, int>>& out) const {
        out.clear();
        if (nodes_.empty()) return;
        // max-heap of the best k by (d2, index)
        auto worse = [](const std::pair<double, int>& x, const std::pair<double, int>& y) { return x < y; };
        std::vector<int> stack{0};
        while (!stack.empty()) {
            const Node& nd = nodes_[stack.back()];
            stack.pop_back();
            if ((int)out.size() == k && boxDist2(nd, p) > out.front().first) continue;
            if (nd.left < 0) {
                for (int q = nd.lo; q < nd.hi; q++) {
                    const int j = idx_[q];
                    if (j == self) continue;
                    const double dx = site_[3 * j] - p[0], dy = site_[3 * j + 1] - p[1], dz = site_[3 * j + 2] - p[2];
                    const std::pair<double, int> c{dx * dx + dy * dy + dz * dz, j};
                    if ((int)out.size() < k) {
                        out.push_back(c);
                        std::push_heap(out.begin(), out.end(), worse);
                    } else if (c < out.front()) {
                        std::pop_heap(out.begin(), out.end(), worse);
                        out.back() = c;
                        std::push_heap(out.begin(), out.end(), worse);
                    }
                }
            } else {
                // nearer child last, so that it is visited first
                const bool leftFirst = p[nd.dim] < nd.split;
                stack.push_back(leftFirst ? nd.right : nd.left);
                stack.push_back(leftFirst ? nd.left : nd.right);
            }
        }
        std::sort_heap(out.begin(), out.end(), worse);
    }

    const std::vector<KdNode>& nodes() const { return nodes_; }
    const std::vector<int>& perm() const { return idx_; }

private:
    using Node = KdNode;
    const std::vector<double>& site_;
    std::vector<int> idx_;
    std::vector<Node> nodes_;

    static double boxDist2(const Node& nd, const V3& p) {
        double d2 = 0;
        for (int q = 0; q < 3; q++) {
            const double d = p[q] < nd.bmin[q] ? nd.bmin[q] - p[q] : p[q] > nd.bmax[q] ? p[q] - nd.bmax[q] : 0.;
            d2 += d * d;
        }
        return d2;
    }

    int build(int lo, int hi) {
        const int me = (int)nodes_.size();
        nodes_.push_back(Node{lo, hi, -1, -1, 0, 0.0, {}, {}});
        Node nd{lo, hi, -1, -1, 0, 0.0, {}, {}};
        for (int q = 0; q < 3; q++) { nd.bmin[q] = DBL_MAX; nd.bmax[q] = -DBL_MAX; }
        for (int t = lo; t < hi; t++)
            for (int q = 0; q < 3; q++) {
                nd.bmin[q] = std::min(nd.bmin[q], site_[3 * (size_t)idx_[t] + q]);
                nd.bmax[q] = std::max(nd.bmax[q], site_[3 * (size_t)idx_[t] + q]);
            }
        if (hi - lo > 8) {
            int dim = 0;
            for (int q = 1; q < 3; q++)
                if (nd.bmax[q] - nd.bmin[q] > nd.bmax[dim] - nd.bmin[dim]) dim = q;
            const int mid = (lo + hi) / 2;
            std::nth_element(idx_.begin() + lo, idx_.begin() + mid, idx_.begin() + hi, [&](int x, int y) {
                const double a = site_[3 * (size_t)x + dim], b = site_[3 * (size_t)y + dim];
                return a < b || (a == b && x < y);
            });
            nd.dim = dim;
            nd.split = site_[3 * (size_t)idx_[mid] + dim];
            nd.left = build(lo, mid);
            nd.right = build(mid, hi);
        }
        nodes_[me] = nd;
        return me;
    }
};

}  // namespace

void VoronoiGrid::blockIndices(double x, double y, double z, int& i, int& j, int& k) const {
    i = std::max(0, std::min(nb - 1, static_cast<int>(nb * (x - xmin) / (xmax - xmin))));
    j = std::max(0, std::min(nb - 1, static_cast<int>(nb * (y - ymin) / (ymax - ymin))));
    k = std::max(0, std::min(nb - 1, static_cast<int>(nb * (z - zmin) / (zmax - zmin))));
}

int VoronoiGrid::cellIndex(double x, double y, double z) const {
    if (!(x >= xmin && x <= xmax && y >= ymin && y <= ymax && z >= zmin && z <= zmax)) return -1;
    int i, j, k;
    blockIndices(x, y, z, i, j, k);
    const int b = i * nb * nb + j * nb + k;
    int m = -1;
    double best = DBL_MAX;
    for (int q = blockOffset[b]; q < blockOffset[b + 1]; q++) {
        const int c = blockList[q];
        const double dx = x - site[3 * c], dy = y - site[3 * c + 1], dz = z - site[3 * c + 2];
        const double d = dx * dx + dy * dy + dz * dz;  // Vec::norm2 of (r - site)
        if (d < best) { best = d; m = c; }
    }
    return m;
}

bool VoronoiGrid::isPointClosestTo(double x, double y, double z, int m) const {
    auto d2 = [&](int c) {
        const double dx = x - site[3 * c], dy = y - site[3 * c + 1], dz = z - site[3 * c + 2];
        return dx * dx + dy * dy + dz * dz;
    };
    const double target = d2(m);
    for (int q = nbrOffset[m]; q < nbrOffset[m + 1]; q++) {
        const int id = nbrList[q];
        if (id >= 0 && d2(id) < target) return false;
    }
    return true;
}

void buildVoronoi(VoronoiGrid& g, const std::vector<double>& sites, double xmin, double xmax, double ymin, double ymax,
                  double zmin, double zmax, const VoronoiCellsFn* cells, int* hostCells) {
    g.xmin = xmin; g.xmax = xmax; g.ymin = ymin; g.ymax = ymax; g.zmin = zmin; g.zmax = zmax;
    const double wx = xmax - xmin, wy = ymax - ymin, wz = zmax - zmin;
    const double L = std::sqrt(wx * wx + wy * wy + wz * wz);
    g.eps = 1e-12 * L;
    g.site = sites;
    const int N = g.ncells();
    if (N < 1) throw std::runtime_error("a Voronoi grid needs sites");

    // SKIRT_AMD_SETUP_TIMES: the stages' wall times
    static const bool timing = std::getenv("SKIRT_AMD_SETUP_TIMES") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto stage = [&](const char* what) {
        if (!timing) return;
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[setup] voronoi %-18s %.3f s\n", what, std::chrono::duration<double>(t1 - t0).count());
        t0 = t1;
    };
    // candidate neighbours come nearest first from a k-d tree over the sites (the sites of a
    // DustDensity grid cluster by orders of magnitude, which a uniform bucket grid cannot follow)
    const SiteTree tree(sites);
    stage("k-d tree");
    g.bbox.assign(6 * (size_t)N, 0);
    g.volume.assign(N, 0);
    g.centroid.assign(3 * (size_t)N, 0);
    std::vector<std::vector<int>> cellIds(N);
    // the cells are independent: computed by worker threads over chunks of cell indices
    auto buildCell = [&](int i, std::vector<std::pair<double, int>>& cand) {
        const V3 s{sites[3 * i], sites[3 * i + 1], sites[3 * i + 2]};
        // the domain box, faces labelled with the wall ids of the reference (Voro++ walls)
        const V3 c000{xmin, ymin, zmin}, c100{xmax, ymin, zmin}, c010{xmin, ymax, zmin}, c110{xmax, ymax, zmin};
        const V3 c001{xmin, ymin, zmax}, c101{xmax, ymin, zmax}, c011{xmin, ymax, zmax}, c111{xmax, ymax, zmax};
        Cell cell;
        cell.faces = {{-1, {c000, c001, c011, c010}}, {-2, {c100, c110, c111, c101}},
                      {-3, {c000, c100, c101, c001}}, {-4, {c010, c011, c111, c110}},
                      {-5, {c000, c010, c110, c100}}, {-6, {c001, c101, c111, c011}}};
        double R2 = cell.maxDist2(s);
        // the k nearest sites in (distance, index) order; each larger query extends the previous one
        size_t done = 0;
        for (int k = 32;; k *= 2) {
            tree.nearest(s, i, k, cand);
            bool stop = false;
            for (size_t q = done; q < cand.size(); q++) {
                const auto& cj = cand[q];
                if (cj.first >= 4 * R2) { stop = true; break; }  // too far to cut (|pj - s| / 2 >= farthest vertex)
                const int j = cj.second;
                const V3 pj{sites[3 * j], sites[3 * j + 1], sites[3 * j + 2]};
                const V3 n = sub(pj, s);
                const V3 mid{0.5 * (pj[0] + s[0]), 0.5 * (pj[1] + s[1]), 0.5 * (pj[2] + s[2])};
                const double tol = 1e-12 * std::sqrt(cj.first) * L;
                if (cell.clip(n, dot(n, mid), tol, j)) R2 = cell.maxDist2(s);
            }
            if (stop || (int)cand.size() < k) break;  // cut off, or every other site seen
            done = cand.size();
        }
        // neighbours, bounding box, volume and centroid of the finished cell
        std::vector<int>& ids = cellIds[i];
        double bmin[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, bmax[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        double vol = 0, cx = 0, cy = 0, cz = 0;
        for (const Face& f : cell.faces) {
            ids.push_back(f.id);
            for (const V3& p : f.pts)
                for (int q = 0; q < 3; q++) { bmin[q] = std::min(bmin[q], p[q]); bmax[q] = std::max(bmax[q], p[q]); }
            for (size_t k = 1; k + 1 < f.pts.size(); k++) {
                const V3 a = sub(f.pts[0], s), bq = sub(f.pts[k], s), cq = sub(f.pts[k + 1], s);
                const double v = std::fabs(dot(a, cross(bq, cq))) / 6.0;
                vol += v;
                cx += v * (s[0] + (f.pts[0][0] + f.pts[k][0] + f.pts[k + 1][0] - 3 * s[0]) / 4.0);
                cy += v * (s[1] + (f.pts[0][1] + f.pts[k][1] + f.pts[k + 1][1] - 3 * s[1]) / 4.0);
                cz += v * (s[2] + (f.pts[0][2] + f.pts[k][2] + f.pts[k + 1][2] - 3 * s[2]) / 4.0);
            }
        }
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
        for (int q = 0; q < 3; q++) { g.bbox[6 * (size_t)i + q] = bmin[q]; g.bbox[6 * (size_t)i + 3 + q] = bmax[q]; }
        g.volume[i] = vol;
        g.centroid[3 * (size_t)i] = vol > 0 ? cx / vol : s[0];
        g.centroid[3 * (size_t)i + 1] = vol > 0 ? cy / vol : s[1];
        g.centroid[3 * (size_t)i + 2] = vol > 0 ? cz / vol : s[2];
    };
    // the cells on the device first (where they fit its capacities); the host builds the rest. The device
    // returns up to kIds neighbour ids per cell in one N x kIds table on each side (1e7 sites: 3.8 GB), so
    // tessellations above kMaxDeviceSites stay on the host, and so does one whose device run fails (e.g. its
    // work areas do not fit): the host's cells are the same, bit for bit
    std::vector<int> todo;
    constexpr int kIds = 96;                    // neighbour ids per cell the device returns
    constexpr int kMaxDeviceSites = 4 << 20;    // 1.6 GB of ids on each side
    bool onDevice = false;
    if (cells && N <= kMaxDeviceSites) {
        try {
            std::vector<int> ids((size_t)N * kIds), nids(N);
            const double box[6] = {xmin, ymin, zmin, xmax, ymax, zmax};
            (*cells)(sites, box, tree.nodes(), tree.perm(), kIds, ids.data(), nids.data(), g.bbox.data(),
                     g.volume.data(), g.centroid.data());
            for (int i = 0; i < N; i++) {
                if (nids[i] < 0 || nids[i] > kIds) {
                    todo.push_back(i);
                    continue;
                }
                cellIds[i].assign(ids.begin() + (size_t)i * kIds, ids.begin() + (size_t)i * kIds + nids[i]);
            }
            onDevice = true;
        } catch (std::exception& e) {
            std::fprintf(stderr, "Voronoi cells on the device failed (%s): every cell on the host\n", e.what());
            todo.clear();
            for (auto& c : cellIds) c.clear();
        }
    }
    if (!onDevice) {
        todo.resize(N);
        for (int i = 0; i < N; i++) todo[i] = i;
    }
    if (onDevice) stage("device cells");
    if (hostCells) *hostCells = (int)todo.size();
    {
        const int T = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
        const int NT = (int)todo.size();
        std::atomic<int> next{0};
        std::vector<std::thread> th;
        std::vector<std::string> errs(T);
        for (int w = 0; w < T; w++)
            th.emplace_back([&, w] {
                try {
                    std::vector<std::pair<double, int>> cand;
                    for (int c0; (c0 = next.fetch_add(64)) < NT;)
                        for (int q = c0; q < std::min(NT, c0 + 64); q++) buildCell(todo[q], cand);
                } catch (std::exception& e) {
                    errs[w] = e.what();
                }
            });
        for (auto& t : th) t.join();
        for (auto& e : errs)
            if (!e.empty()) throw std::runtime_error(e);
    }
    stage("host cells");
    g.nbrOffset.assign(N + 1, 0);
    g.nbrList.clear();
    for (int i = 0; i < N; i++) {
        g.nbrList.insert(g.nbrList.end(), cellIds[i].begin(), cellIds[i].end());
        g.nbrOffset[i + 1] = (int)g.nbrList.size();
    }

    // block lists (VoronoiMesh::buildMesh): nb = max(3, min(1000, int(3 N^(1/3)))) blocks per axis
    g.nb = std::max(3, std::min(1000, static_cast<int>(3. * std::pow(N, 1. / 3.))));
    const int nb = g.nb;
    const size_t nb2 = (size_t)nb * nb, nb3 = nb2 * nb;
    std::vector<int> range(6 * (size_t)N);  // block index range of every cell's eps-widened box
    for (int m = 0; m < N; m++) {
        const double* bx = &g.bbox[6 * (size_t)m];
        int* r = &range[6 * (size_t)m];
        g.blockIndices(bx[0] - g.eps, bx[1] - g.eps, bx[2] - g.eps, r[0], r[1], r[2]);
        g.blockIndices(bx[3] + g.eps, bx[4] + g.eps, bx[5] + g.eps, r[3], r[4], r[5]);
    }
    // CSR over the blocks, each list in cell order; worker threads own slabs of the first block index
    std::vector<size_t> count(nb3 + 1, 0);
    const int T = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    auto slabs = [&](auto&& fn) {
        std::vector<std::thread> th;
        for (int w = 0; w < T; w++)
            th.emplace_back([&, w] {
                const int i0 = (int)((long long)nb * w / T), i1 = (int)((long long)nb * (w + 1) / T);
                for (int m = 0; m < N; m++) {
                    const int* r = &range[6 * (size_t)m];
                    for (int i = std::max(r[0], i0); i <= std::min(r[3], i1 - 1); i++)
                        for (int j = r[1]; j <= r[4]; j++)
                            for (int k = r[2]; k <= r[5]; k++) fn((size_t)i * nb2 + (size_t)j * nb + k, m);
                }
            });
        for (auto& t : th) t.join();
    };
    slabs([&](size_t b, int) { count[b + 1]++; });
    for (size_t b = 0; b < nb3; b++) count[b + 1] += count[b];
    if (count[nb3] > (size_t)INT32_MAX) throw std::runtime_error("Voronoi block lists too long");
    g.blockOffset.assign(count.begin(), count.end());
    g.blockList.assign(count[nb3], 0);
    std::vector<int> fill(g.blockOffset.begin(), g.blockOffset.end() - 1);
    slabs([&](size_t b, int m) { g.blockList[fill[b]++] = m; });
    stage("neighbours, blocks");
}

void voronoiRandomPosition(const VoronoiGrid& g, UniformSource& rng, int m, double& x, double& y, double& z) {
    const double* b = &g.bbox[6 * (size_t)m];
    for (int i = 0; i < 10000; i++) {
        // Random::position(box) then Box::fracpos
        double fx = rng.uniform();
        double fy = rng.uniform();
        double fz = rng.uniform();
        x = b[0] + fx * (b[3] - b[0]);
        y = b[1] + fy * (b[4] - b[1]);
        z = b[2] + fz * (b[5] - b[2]);
        if (g.isPointClosestTo(x, y, z, m)) return;
    }
    throw std::runtime_error("Can't find random position in cell");
}

}  // namespace skirt
