// The cells of a Voronoi dust grid's tessellation on the device (skirt_mcrt_voronoi_cells, include/skirt_mcrt.h):
// the host's construction (host/voronoi.cpp, buildVoronoi) with one cell per thread. The reference computes the
// cells with its vendored Voro++ (VoronoiMesh.cpp:310-376); the host restates them as the domain box clipped by
// the bisector planes of the nearest sites, nearest first ((squared distance, index) order from a k-d tree,
// k = 32, 64, ... nearest), until no farther site can cut the cell. This kernel runs that loop with the same
// double-precision operations in the same order (no FMA contraction: the Makefile's -ffp-contract=off), so the
// neighbour lists, bounding boxes, volumes and centroids equal the host's bit for bit; the only library call
// is atan2, which orders a new face's vertices around it (an ulp changes that order only for two vertices at
// the same angle, which a convex face does not have). A cell outgrowing the fixed capacities below (faces,
// vertices, cut points, nearest sites per query) is left to the host (nids < 0).
//
// Layout: the sites, the k-d tree (nodes, permutation) and the outputs in HBM; each thread a private work area
// in HBM (two face lists it clips from one into the other, the cut points, the nearest-site heap), threads
// striding over the cells. Setup work outside the photon phases: latency-bound, not tuned to a roofline.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "../../../include/skirt_mcrt.h"

namespace {

constexpr int kFaces = 96;   // faces of a cell
constexpr int kPts = 1024;   // vertices of a cell's faces, over all its faces
constexpr int kCap = 128;    // cut points of one clip (before duplicates go)
constexpr int kMaxK = 2048;  // nearest sites of one query (a thread's heap: more is slower than the host)
constexpr int kStack = 128;  // k-d tree traversal stack
constexpr int kThreads = 64;
constexpr int kMaxThreads = 16384;  // concurrent cells: work areas of 81 KB, 1.3 GB (65,536: 5.3 GB, no faster)

struct V3 {
    double x, y, z;
};

// the host's V3 arithmetic (std::array<double, 3>), operation for operation
__device__ __forceinline__ double dot(const V3& a, const V3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 sub(const V3& a, const V3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 cross(const V3& a, const V3& b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// std::array's operator< (lexicographic) and operator==
__device__ __forceinline__ bool lexLess(const V3& a, const V3& b) {
    if (a.x < b.x) return true;
    if (b.x < a.x) return false;
    if (a.y < b.y) return true;
    if (b.y < a.y) return false;
    return a.z < b.z;
}
__device__ __forceinline__ bool same(const V3& a, const V3& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
__device__ __forceinline__ double stdMax(double a, double b) { return a < b ? b : a; }  // std::max
__device__ __forceinline__ double stdMin(double a, double b) { return b < a ? b : a; }  // std::min
// std::pair<double, int>'s operator<
__device__ __forceinline__ bool pairLess(double da, int ja, double db, int jb) {
    return da < db || (!(db < da) && ja < jb);
}

struct Work {
    V3 pts[2][kPts];  // the face vertices of the current and the next face list
    int fid[2][kFaces], fstart[2][kFaces], fcnt[2][kFaces];
    V3 cap[kCap];
    double ang[kCap];
    double hd[kMaxK];  // nearest-site max-heap: squared distance, site
    int hj[kMaxK];
};

struct VorArgs {
    const double* site;
    int n;
    double box[6];  // xmin ymin zmin xmax ymax zmax
    double L;       // the box's diagonal
    const SkirtKdNode* nodes;
    const int* perm;
    int maxIds;
    int* ids;
    int* nids;
    double* bbox;
    double* volume;
    double* centroid;
    Work* work;
    int nthreads;
};

__device__ __forceinline__ V3 siteOf(const VorArgs& A, int j) {
    return {A.site[3 * (size_t)j], A.site[3 * (size_t)j + 1], A.site[3 * (size_t)j + 2]};
}

// max-heap on (d2, j) of cnt entries
__device__ void heapUp(Work& W, int c) {
    while (c > 0) {
        const int p = (c - 1) / 2;
        if (!pairLess(W.hd[p], W.hj[p], W.hd[c], W.hj[c])) break;
        const double td = W.hd[p]; W.hd[p] = W.hd[c]; W.hd[c] = td;
        const int tj = W.hj[p]; W.hj[p] = W.hj[c]; W.hj[c] = tj;
        c = p;
    }
}
__device__ void heapDown(Work& W, int c, int cnt) {
    for (;;) {
        const int l = 2 * c + 1, r = l + 1;
        int m = c;
        if (l < cnt && pairLess(W.hd[m], W.hj[m], W.hd[l], W.hj[l])) m = l;
        if (r < cnt && pairLess(W.hd[m], W.hj[m], W.hd[r], W.hj[r])) m = r;
        if (m == c) break;
        const double td = W.hd[m]; W.hd[m] = W.hd[c]; W.hd[c] = td;
        const int tj = W.hj[m]; W.hj[m] = W.hj[c]; W.hj[c] = tj;
        c = m;
    }
}

__device__ double boxDist2(const SkirtKdNode& nd, const V3& p) {
    const double pc[3] = {p.x, p.y, p.z};
    double d2 = 0;
    for (int q = 0; q < 3; q++) {
        const double d = pc[q] < nd.bmin[q] ? nd.bmin[q] - pc[q] : pc[q] > nd.bmax[q] ? pc[q] - nd.bmax[q] : 0.;
        d2 += d * d;
    }
    return d2;
}

// SiteTree::nearest: the k nearest sites to p other than `self`, ascending in (d2, index) into W.hd / W.hj;
// their count, or -1 if the traversal stack overflowed. The set is unique, so any traversal order gives the
// host's list.
__device__ int nearest(const VorArgs& A, Work& W, const V3& p, int self, int k) {
    int stack[kStack];
    int sp = 0, cnt = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const SkirtKdNode nd = A.nodes[stack[--sp]];
        if (cnt == k && boxDist2(nd, p) > W.hd[0]) continue;
        if (nd.left < 0) {
            for (int q = nd.lo; q < nd.hi; q++) {
                const int j = A.perm[q];
                if (j == self) continue;
                const double dx = A.site[3 * (size_t)j] - p.x, dy = A.site[3 * (size_t)j + 1] - p.y,
                             dz = A.site[3 * (size_t)j + 2] - p.z;
                const double d2 = dx * dx + dy * dy + dz * dz;
                if (cnt < k) {
                    W.hd[cnt] = d2;
                    W.hj[cnt] = j;
                    heapUp(W, cnt);
                    cnt++;
                } else if (pairLess(d2, j, W.hd[0], W.hj[0])) {
                    W.hd[0] = d2;
                    W.hj[0] = j;
                    heapDown(W, 0, cnt);
                }
            }
        } else {
            if (sp + 2 > kStack) return -1;
            const double pd = nd.dim == 0 ? p.x : nd.dim == 1 ? p.y : p.z;
            const bool leftFirst = pd < nd.split;
            stack[sp++] = leftFirst ? nd.right : nd.left;
            stack[sp++] = leftFirst ? nd.left : nd.right;
        }
    }
    // heap sort: ascending
    for (int e = cnt - 1; e > 0; e--) {
        const double td = W.hd[0]; W.hd[0] = W.hd[e]; W.hd[e] = td;
        const int tj = W.hj[0]; W.hj[0] = W.hj[e]; W.hj[e] = tj;
        heapDown(W, 0, e);
    }
    return cnt;
}

struct CellState {
    int cur, nf;
};

__device__ double maxDist2(const Work& W, const CellState& c, const V3& s) {
    double r = 0;
    for (int f = 0; f < c.nf; f++) {
        const int b = W.fstart[c.cur][f], m = W.fcnt[c.cur][f];
        for (int t = 0; t < m; t++) r = stdMax(r, dot(sub(W.pts[c.cur][b + t], s), sub(W.pts[c.cur][b + t], s)));
    }
    return r;
}

// Cell::crossing: from the lexicographically smaller end, so that the two faces sharing the edge agree
__device__ V3 crossing(const V3& a0, const V3& b0, const V3& n, double c) {
    const bool swap = lexLess(b0, a0);
    const V3& a = swap ? b0 : a0;
    const V3& b = swap ? a0 : b0;
    const double da = dot(n, a) - c, db = dot(n, b) - c;
    const double t = da / (da - db);
    return {a.x + t * (b.x - a.x), a.y + t * (b.y - a.y), a.z + t * (b.z - a.z)};
}

// Cell::clip by dot(n, x) <= c, the new face labelled `id`: 1 changed, 0 not cut, -1 out of capacity
__device__ int clip(Work& W, CellState& cs, const V3& n, double c, double tol, int id) {
    const int cur = cs.cur, nx = 1 - cs.cur;
    double dm = -DBL_MAX;
    for (int f = 0; f < cs.nf; f++) {
        const int b = W.fstart[cur][f], m = W.fcnt[cur][f];
        for (int t = 0; t < m; t++) dm = stdMax(dm, dot(n, W.pts[cur][b + t]) - c);
    }
    if (dm <= tol) return 0;
    int np = 0, nnf = 0, ncap = 0;
    for (int f = 0; f < cs.nf; f++) {
        const int b = W.fstart[cur][f], m = W.fcnt[cur][f];
        const int st = np;
        for (int k = 0; k < m; k++) {
            const V3 a = W.pts[cur][b + k];
            const V3 e = W.pts[cur][b + (k + 1) % m];
            const double da = dot(n, a) - c, db = dot(n, e) - c;
            const bool ina = da <= tol, inb = db <= tol;
            if (ina) {
                if (np >= kPts) return -1;
                W.pts[nx][np++] = a;
                if (da >= -tol) {
                    if (ncap >= kCap) return -1;
                    W.cap[ncap++] = a;
                }
            }
            if (ina != inb && fabs(da) > tol && fabs(db) > tol) {
                const V3 q = crossing(a, e, n, c);
                if (np >= kPts || ncap >= kCap) return -1;
                W.pts[nx][np++] = q;
                W.cap[ncap++] = q;
            }
        }
        if (np - st >= 3) {
            if (nnf >= kFaces) return -1;
            W.fid[nx][nnf] = W.fid[cur][f];
            W.fstart[nx][nnf] = st;
            W.fcnt[nx][nnf] = np - st;
            nnf++;
        } else {
            np = st;
        }
    }
    // the new face: the distinct cut points (std::sort, std::unique) ordered by angle around their centre
    for (int i = 1; i < ncap; i++) {
        const V3 v = W.cap[i];
        int j = i - 1;
        while (j >= 0 && lexLess(v, W.cap[j])) {
            W.cap[j + 1] = W.cap[j];
            j--;
        }
        W.cap[j + 1] = v;
    }
    int w = 0;
    for (int r = 0; r < ncap; r++)
        if (w == 0 || !same(W.cap[r], W.cap[w - 1])) W.cap[w++] = W.cap[r];
    ncap = w;
    if (ncap >= 3) {
        V3 ctr{0, 0, 0};
        for (int i = 0; i < ncap; i++) {
            ctr.x += W.cap[i].x;
            ctr.y += W.cap[i].y;
            ctr.z += W.cap[i].z;
        }
        ctr.x /= (double)ncap;
        ctr.y /= (double)ncap;
        ctr.z /= (double)ncap;
        const double nl = sqrt(dot(n, n));
        const V3 nh{n.x / nl, n.y / nl, n.z / nl};
        const V3 u = sub(W.cap[0], ctr);
        const V3 v = cross(nh, u);
        for (int i = 0; i < ncap; i++) {
            const V3 d = sub(W.cap[i], ctr);
            W.ang[i] = atan2(dot(d, v), dot(d, u));
        }
        // by angle, stable (std::sort on at most 16 elements is an insertion sort)
        for (int i = 1; i < ncap; i++) {
            const double ka = W.ang[i];
            const V3 kp = W.cap[i];
            int j = i - 1;
            while (j >= 0 && ka < W.ang[j]) {
                W.ang[j + 1] = W.ang[j];
                W.cap[j + 1] = W.cap[j];
                j--;
            }
            W.ang[j + 1] = ka;
            W.cap[j + 1] = kp;
        }
        if (nnf >= kFaces || np + ncap > kPts) return -1;
        W.fid[nx][nnf] = id;
        W.fstart[nx][nnf] = np;
        W.fcnt[nx][nnf] = ncap;
        nnf++;
        for (int i = 0; i < ncap; i++) W.pts[nx][np++] = W.cap[i];
    }
    cs.cur = nx;
    cs.nf = nnf;
    return 1;
}

// buildVoronoi's buildCell for cell i; false: out of capacity (the host builds it)
__device__ bool cellOf(const VorArgs& A, Work& W, int i) {
    const V3 s = siteOf(A, i);
    const double xmin = A.box[0], ymin = A.box[1], zmin = A.box[2], xmax = A.box[3], ymax = A.box[4], zmax = A.box[5];
    const V3 c000{xmin, ymin, zmin}, c100{xmax, ymin, zmin}, c010{xmin, ymax, zmin}, c110{xmax, ymax, zmin};
    const V3 c001{xmin, ymin, zmax}, c101{xmax, ymin, zmax}, c011{xmin, ymax, zmax}, c111{xmax, ymax, zmax};
    const V3 box[6][4] = {{c000, c001, c011, c010}, {c100, c110, c111, c101}, {c000, c100, c101, c001},
                          {c010, c011, c111, c110}, {c000, c010, c110, c100}, {c001, c101, c111, c011}};
    CellState cs{0, 6};
    for (int f = 0; f < 6; f++) {
        W.fid[0][f] = -1 - f;
        W.fstart[0][f] = 4 * f;
        W.fcnt[0][f] = 4;
        for (int t = 0; t < 4; t++) W.pts[0][4 * f + t] = box[f][t];
    }
    double R2 = maxDist2(W, cs, s);
    int done = 0;
    for (int k = 32;; k *= 2) {
        if (k > kMaxK) return false;
        const int cnt = nearest(A, W, s, i, k);
        if (cnt < 0) return false;
        bool stop = false;
        for (int q = done; q < cnt; q++) {
            const double d2 = W.hd[q];
            if (d2 >= 4 * R2) {  // too far to cut
                stop = true;
                break;
            }
            const int j = W.hj[q];
            const V3 pj = siteOf(A, j);
            const V3 n = sub(pj, s);
            const V3 mid{0.5 * (pj.x + s.x), 0.5 * (pj.y + s.y), 0.5 * (pj.z + s.z)};
            const double tol = 1e-12 * sqrt(d2) * A.L;
            const int r = clip(W, cs, n, dot(n, mid), tol, j);
            if (r < 0) return false;
            if (r) R2 = maxDist2(W, cs, s);
        }
        if (stop || cnt < k) break;
        done = cnt;
    }
    if (cs.nf > A.maxIds) return false;
    // neighbours (sorted, distinct), bounding box, volume and centroid
    int* ids = A.ids + (size_t)i * A.maxIds;
    double bmin[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, bmax[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    double vol = 0, cx = 0, cy = 0, cz = 0;
    const int cur = cs.cur;
    for (int f = 0; f < cs.nf; f++) {
        ids[f] = W.fid[cur][f];
        const V3* P = &W.pts[cur][W.fstart[cur][f]];
        const int m = W.fcnt[cur][f];
        for (int t = 0; t < m; t++) {
            bmin[0] = stdMin(bmin[0], P[t].x); bmax[0] = stdMax(bmax[0], P[t].x);
            bmin[1] = stdMin(bmin[1], P[t].y); bmax[1] = stdMax(bmax[1], P[t].y);
            bmin[2] = stdMin(bmin[2], P[t].z); bmax[2] = stdMax(bmax[2], P[t].z);
        }
        for (int k = 1; k + 1 < m; k++) {
            const V3 a = sub(P[0], s), bq = sub(P[k], s), cq = sub(P[k + 1], s);
            const double v = fabs(dot(a, cross(bq, cq))) / 6.0;
            vol += v;
            cx += v * (s.x + (P[0].x + P[k].x + P[k + 1].x - 3 * s.x) / 4.0);
            cy += v * (s.y + (P[0].y + P[k].y + P[k + 1].y - 3 * s.y) / 4.0);
            cz += v * (s.z + (P[0].z + P[k].z + P[k + 1].z - 3 * s.z) / 4.0);
        }
    }
    int nid = cs.nf;
    for (int a = 1; a < nid; a++) {  // std::sort + std::unique
        const int v = ids[a];
        int b = a - 1;
        while (b >= 0 && v < ids[b]) {
            ids[b + 1] = ids[b];
            b--;
        }
        ids[b + 1] = v;
    }
    int w = 0;
    for (int r = 0; r < nid; r++)
        if (w == 0 || ids[r] != ids[w - 1]) ids[w++] = ids[r];
    A.nids[i] = w;
    for (int q = 0; q < 3; q++) {
        A.bbox[6 * (size_t)i + q] = bmin[q];
        A.bbox[6 * (size_t)i + 3 + q] = bmax[q];
    }
    A.volume[i] = vol;
    A.centroid[3 * (size_t)i] = vol > 0 ? cx / vol : s.x;
    A.centroid[3 * (size_t)i + 1] = vol > 0 ? cy / vol : s.y;
    A.centroid[3 * (size_t)i + 2] = vol > 0 ? cz / vol : s.z;
    return true;
}

__global__ __launch_bounds__(kThreads) void voronoiCellsKernel(VorArgs A) {
    const int t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= A.nthreads) return;
    Work& W = A.work[t];
    for (int i = t; i < A.n; i += A.nthreads)
        if (!cellOf(A, W, i)) A.nids[i] = -1;
}

}  // namespace

extern "C" int skirt_mcrt_voronoi_cells(int device, const double* sites, int nsites, const double extent[6],
                                        const SkirtKdNode* nodes, int nnodes, const int* perm, int max_ids, int* ids,
                                        int* nids, double* bbox, double* volume, double* centroid) {
    if (!sites || nsites < 1 || !extent || !nodes || nnodes < 1 || !perm || max_ids < 1 || !ids || !nids || !bbox ||
        !volume || !centroid)
        return SKIRT_ERR_ARG;
    // the tree must be one the traversal can walk without leaving its arrays: permutation entries are
    // sites, leaves hold ranges of the permutation, children come after their parent
    for (int q = 0; q < nsites; q++)
        if (perm[q] < 0 || perm[q] >= nsites) return SKIRT_ERR_ARG;
    for (int b = 0; b < nnodes; b++) {
        const SkirtKdNode& nd = nodes[b];
        if (nd.lo < 0 || nd.hi < nd.lo || nd.hi > nsites) return SKIRT_ERR_ARG;
        if (nd.left >= 0 && (nd.left <= b || nd.left >= nnodes || nd.right <= b || nd.right >= nnodes ||
                             nd.dim < 0 || nd.dim > 2))
            return SKIRT_ERR_ARG;
    }
    if ((size_t)nsites * (size_t)max_ids > 0x7fffffffull * 4) return SKIRT_ERR_UNSUPPORTED;
    if (hipSetDevice(device) != hipSuccess) return SKIRT_ERR_HIP;
    const int T = nsites < kMaxThreads ? nsites : kMaxThreads;
    const size_t nSite = 3 * (size_t)nsites * sizeof(double), nNode = (size_t)nnodes * sizeof(SkirtKdNode);
    const size_t nPerm = (size_t)nsites * sizeof(int), nIds = (size_t)nsites * max_ids * sizeof(int);
    const size_t nOut = (size_t)nsites * (6 + 1 + 3) * sizeof(double);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t oSite = 0, oNode = oSite + al(nSite), oPerm = oNode + al(nNode), oIds = oPerm + al(nPerm);
    const size_t oNid = oIds + al(nIds), oOut = oNid + al((size_t)nsites * sizeof(int)), oWork = oOut + al(nOut);
    const size_t total = oWork + (size_t)T * sizeof(Work);
    char* buf = nullptr;
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return SKIRT_ERR_HIP;
    if (hipMalloc(&buf, total) != hipSuccess) {
        (void)hipStreamDestroy(st);
        return SKIRT_ERR_HIP;
    }
    VorArgs A{};
    A.site = reinterpret_cast<const double*>(buf + oSite);
    A.n = nsites;
    for (int q = 0; q < 6; q++) A.box[q] = extent[q];
    // VoronoiMesh's extent diagonal, as the host computes it
    const double wx = extent[3] - extent[0], wy = extent[4] - extent[1], wz = extent[5] - extent[2];
    A.L = std::sqrt(wx * wx + wy * wy + wz * wz);
    A.nodes = reinterpret_cast<const SkirtKdNode*>(buf + oNode);
    A.perm = reinterpret_cast<const int*>(buf + oPerm);
    A.maxIds = max_ids;
    A.ids = reinterpret_cast<int*>(buf + oIds);
    A.nids = reinterpret_cast<int*>(buf + oNid);
    A.bbox = reinterpret_cast<double*>(buf + oOut);
    A.volume = A.bbox + 6 * (size_t)nsites;
    A.centroid = A.volume + nsites;
    A.work = reinterpret_cast<Work*>(buf + oWork);
    A.nthreads = T;
    int rc = SKIRT_OK;
    if (hipMemcpyAsync(buf + oSite, sites, nSite, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(buf + oNode, nodes, nNode, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(buf + oPerm, perm, nPerm, hipMemcpyHostToDevice, st) != hipSuccess) {
        rc = SKIRT_ERR_HIP;
    } else {
        hipLaunchKernelGGL(voronoiCellsKernel, dim3((unsigned)((T + kThreads - 1) / kThreads)), dim3(kThreads), 0, st,
                           A);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(ids, A.ids, nIds, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(nids, A.nids, (size_t)nsites * sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(bbox, A.bbox, 6 * (size_t)nsites * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(volume, A.volume, (size_t)nsites * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(centroid, A.centroid, 3 * (size_t)nsites * sizeof(double), hipMemcpyDeviceToHost, st) !=
                hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = SKIRT_ERR_HIP;
    }
    (void)hipStreamSynchronize(st);
    (void)hipFree(buf);
    (void)hipStreamDestroy(st);
    return rc;
}
