// Host check of the compact Voronoi step (float neighbour offsets + exact winner), the arithmetic that
// Grid<SKIRT_GRID_VORONOI>::step in engine.hip runs: walks random rays through a tessellation twice,
// once with the reference's step (VoronoiMesh::path, VoronoiMesh.cpp:749-844, double sites) and once with
// the compact step (interval bounds from float offsets, the exact reference expression for the winner,
// exact re-evaluation of every possible winner when the bounds cannot separate them), and requires the
// same cells and bitwise equal segment lengths. Reports how often the exact re-evaluation was needed.
//   g++ -O2 -std=c++17 -ffp-contract=off -I include tools/vor_compact_check.cpp -L skirt_amd -lskirt_amd \
//       -Wl,-rpath,$PWD/skirt_amd -o /tmp/vor_compact_check && /tmp/vor_compact_check 100000 20000 d
// (mode r: the device's bounds on reciprocal entries m = n / |n|^2; d: round 3's bounds on the offsets n;
// x: per-entry terms; f / e / c: round-2 float variants; none: double bounds). The device takes 1/(m.k)
// from v_rcp_f32 (__builtin_amdgcn_rcpf), accurate to 1 ulp: mode r+ / r- nudges every reciprocal one ulp
// up / down, mode r~ each one by a pseudo-random -1, 0 or +1 ulp, so that the margin the device relies on
// is what the walk checks.
#include "../skirt_amd/csrc/device/vor_terms.hpp"
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "skirt_host.h"

namespace {
constexpr double kEps = 1.0 / (1 << 21);  // bound factor: 8x the float rounding of the offsets

struct Mesh {
    SkirtGridDesc g;
    std::vector<float> off;  // per list entry: float(site_nbr - site_own), 3 per entry
    std::vector<float> nmax;  // per cell: the longest scaled offset of its list
    std::vector<float> eA, eB;  // per cell: the device's error terms (vor_terms.hpp)
};

double wallDist(const SkirtGridDesc& g, int mi, const double r[3], const double k[3]) {
    switch (mi) {
    case -1: return (g.extent[0] - r[0]) / k[0];
    case -2: return (g.extent[3] - r[0]) / k[0];
    case -3: return (g.extent[1] - r[1]) / k[1];
    case -4: return (g.extent[4] - r[1]) / k[1];
    case -5: return (g.extent[2] - r[2]) / k[2];
    default: return (g.extent[5] - r[2]) / k[2];
    }
}

// the reference's distance to the bisector plane with neighbour mi (0 when the ray moves away from it)
double exactDist(const SkirtGridDesc& g, int m, int mi, const double r[3], const double k[3]) {
    if (mi < 0) return wallDist(g, mi, r, k);
    const double* pr = g.site + 3 * (size_t)m;
    const double* pi = g.site + 3 * (size_t)mi;
    const double nx = pi[0] - pr[0], ny = pi[1] - pr[1], nz = pi[2] - pr[2];
    const double ndotk = nx * k[0] + ny * k[1] + nz * k[2];
    if (!(ndotk > 0)) return 0;
    const double px = 0.5 * (pi[0] + pr[0]), py = 0.5 * (pi[1] + pr[1]), pz = 0.5 * (pi[2] + pr[2]);
    return (nx * (px - r[0]) + ny * (py - r[1]) + nz * (pz - r[2])) / ndotk;
}

// reference step: (exit neighbour or -99, distance)
int refStep(const SkirtGridDesc& g, int m, const double r[3], const double k[3], double& sq) {
    sq = DBL_MAX;
    int mq = -99;
    for (int q = g.cell_nbr_offset[m]; q < g.cell_nbr_offset[m + 1]; q++) {
        const int mi = g.cell_nbr_list[q];
        const double si = exactDist(g, m, mi, r, k);
        if (si > 0 && si < sq) { sq = si; mq = mi; }
    }
    return mq;
}

// the same bounds in single precision on coordinates scaled by 1/L (the device's f32 variant): every float
// operation adds at most a few 2^-24 of the sum of absolute terms, covered by kEpsF
constexpr float kEpsF = 1.0f / (1 << 20);
float gScale = 1.0f;
bool gCell = false, gEntry = false;  // per-cell / per-entry-norm error bounds instead of the round-2 device's
bool gPerEntry = false;  // mode x: the first round-3 device step (per-entry terms)
bool gDevice = false;                // the round-3 device step: per-entry Cauchy-Schwarz error terms
bool gRecip = false;                 // mode r: the entries hold m = n / |n|^2 (the device's final step)
int gRcpUlp = 0;                     // mode r+ / r- / r~: the approximate reciprocal's error (+1, -1, 2 = random)
uint32_t gRcpState = 12345u;
long gSignFallbacks = 0;  // re-evaluations with an entry whose n.k sign is uncertain
long gWholeList = 0;      // re-evaluations over the whole list (more than 4 possible winners)
float gLo[4096];          // the step's lower bounds, per list entry

// compact step: the same result from float offsets, exact only for the winner (or all possible winners)
int compactStep(const Mesh& M, int m, const double r[3], const double k[3], double& sq, long& fallbacks) {
    const SkirtGridDesc& g = M.g;
    const double* pr = g.site + 3 * (size_t)m;
    const double D[3] = {pr[0] - r[0], pr[1] - r[1], pr[2] - r[2]};
    double U = DBL_MAX, L1 = DBL_MAX, L2 = DBL_MAX;
    int w1 = -99;
    for (int q = g.cell_nbr_offset[m]; q < g.cell_nbr_offset[m + 1]; q++) {
        const int mi = g.cell_nbr_list[q];
        double lo, hi;
        if (mi < 0) {
            const double si = wallDist(g, mi, r, k);
            if (!(si > 0)) continue;
            lo = hi = si;
        } else {
            const double nx = M.off[3 * (size_t)q] / gScale, ny = M.off[3 * (size_t)q + 1] / gScale,
                         nz = M.off[3 * (size_t)q + 2] / gScale;
            const double den = nx * k[0] + ny * k[1] + nz * k[2];
            const double eA = kEps * (fabs(nx * k[0]) + fabs(ny * k[1]) + fabs(nz * k[2]));
            if (den <= -eA) continue;  // moving away for certain: si = 0
            const double tx = D[0] + 0.5 * nx, ty = D[1] + 0.5 * ny, tz = D[2] + 0.5 * nz;
            const double num = nx * tx + ny * ty + nz * tz;
            const double eB = kEps * (fabs(nx * tx) + fabs(ny * ty) + fabs(nz * tz) + 0.5 * (nx * nx + ny * ny + nz * nz));
            if (den > 2 * eA) {
                const double inv = 1.0 / den;
                const double s = num * inv;
                const double err = 2.0 * (eB + fabs(s) * eA) * inv;
                lo = s - err;
                hi = s + err;
                if (hi <= 0) continue;  // si <= 0 for certain
            } else {
                lo = -DBL_MAX;  // the sign of ndotk is uncertain
                hi = DBL_MAX;
            }
        }
        if (lo > 0 && hi < U) U = hi;
        if (lo < L1) { L2 = L1; L1 = lo; w1 = mi; }
        else if (lo < L2) L2 = lo;
    }
    if (L1 == DBL_MAX) { sq = DBL_MAX; return -99; }  // no exit for certain
    if (L2 > U) {  // one possible winner: its exact distance
        sq = exactDist(g, m, w1, r, k);
        return w1;
    }
    // several possible winners: the reference's rule over them, exactly, in list order
    fallbacks++;
    sq = DBL_MAX;
    int mq = -99;
    for (int q = g.cell_nbr_offset[m]; q < g.cell_nbr_offset[m + 1]; q++) {
        const int mi = g.cell_nbr_list[q];
        const double si = exactDist(g, m, mi, r, k);
        if (si > 0 && si < sq) { sq = si; mq = mi; }
    }
    return mq;
}
}  // namespace

// the device's step (Grid<SKIRT_GRID_VORONOI>::step): every entry, walls included (stored as the bisector
// plane with the site's mirror image), through the same branch-free bounds
static int compactStepF(const Mesh& M, int m, const double r[3], const double k[3], double& sq, long& fallbacks) {
    const SkirtGridDesc& g = M.g;
    const double* pr = g.site + 3 * (size_t)m;
    const float Dx = (float)((pr[0] - r[0]) * gScale), Dy = (float)((pr[1] - r[1]) * gScale),
                Dz = (float)((pr[2] - r[2]) * gScale);
    const float kx = (float)k[0], ky = (float)k[1], kz = (float)k[2];
    float U = FLT_MAX, L1 = FLT_MAX, L2 = FLT_MAX;
    int w1 = -99;
    // per-cell bounds (Cauchy-Schwarz over the longest offset of the cell)
    const float nm = M.nmax.empty() ? 0.f : M.nmax[m];
    const float eAc = kEpsF * nm, eBc = kEpsF * nm * (fabsf(Dx) + fabsf(Dy) + fabsf(Dz) + nm);
    for (int q = g.cell_nbr_offset[m]; q < g.cell_nbr_offset[m + 1]; q++) {
        const int mi = g.cell_nbr_list[q];
        const float nx = M.off[3 * (size_t)q], ny = M.off[3 * (size_t)q + 1], nz = M.off[3 * (size_t)q + 2];
        if (gDevice) {
            // Grid<SKIRT_GRID_VORONOI>::bounds (engine.hip) operation for operation: the error terms from
            // the cell's largest |n|_1 and |n|^2 (the header's eA, eB; mode x: per entry, as in round 3's
            // first version)
            const float Dn = fabsf(Dx) + fabsf(Dy) + fabsf(Dz);
            const float n2 = fmaf(nz, nz, fmaf(ny, ny, nx * nx));
            const float den = fmaf(nz, kz, fmaf(ny, ky, nx * kx));
            // mode r (engine.hip bounds()): (m.D + 1/2) / (m.k), the entries being m
            const float num = gRecip ? fmaf(nz, Dz, fmaf(ny, Dy, fmaf(nx, Dx, 0.5f)))
                                     : fmaf(n2, 0.5f, fmaf(nz, Dz, fmaf(ny, Dy, nx * Dx)));
            const float eA = gPerEntry ? kEpsF * (fabsf(nx) + fabsf(ny) + fabsf(nz)) : M.eA[m];
            const float eB = gPerEntry ? fmaf(eA, Dn, kEpsF * n2) : fmaf(eA, Dn, M.eB[m]);
            float inv = 1.0f / den;
            if (gRcpUlp) {  // the device's v_rcp_f32 errs by up to 1 ulp
                int u = gRcpUlp;
                if (u == 2) { gRcpState = gRcpState * 1664525u + 1013904223u; u = (int)(gRcpState >> 30) % 3 - 1; }
                if (u > 0) inv = nextafterf(inv, INFINITY);
                if (u < 0) inv = nextafterf(inv, -INFINITY);
            }
            const float sa = num * inv;
            const float err = fmaf(fmaf(fabsf(sa), 2.0f * eA, 2.0f * eB), inv, fabsf(sa) * kEpsF);
            (void)n2;
            const float lov = sa - err, hiv = sa + err;
            const bool sure = den > 2.0f * eA;
            const bool maybe = den > -eA;  // (den = 0 for a degenerate wall's m = 0: uncertain)
            // (an interval wholly behind the ray, hiv <= 0, stays a possible exit: the exact evaluation drops it;
            // inside the cell a plane ahead of the ray is never behind it, so it happens only at rounding level)
            const float lo = sure ? lov : (maybe ? -FLT_MAX : FLT_MAX);
            const float ucand = (sure && lov > 0.f) ? hiv : FLT_MAX;
            gLo[q - g.cell_nbr_offset[m]] = lo;
            U = fminf(U, ucand);
            w1 = lo < L1 ? mi : w1;
            L2 = fmaxf(fminf(L1, L2), fminf(fmaxf(L1, L2), lo));
            L1 = fminf(L1, lo);
            continue;
        }
        const float ne = sqrtf(nx * nx + ny * ny + nz * nz);
        const float px = nx * kx, py = ny * ky, pz = nz * kz;
        const float den = px + py + pz;
        const float eA = gEntry ? kEpsF * ne : gCell ? eAc : kEpsF * (fabsf(px) + fabsf(py) + fabsf(pz));
        const float tx = Dx + 0.5f * nx, ty = Dy + 0.5f * ny, tz = Dz + 0.5f * nz;
        const float qx = nx * tx, qy = ny * ty, qz = nz * tz;
        const float num = qx + qy + qz;
        const float eB = gEntry ? kEpsF * ne * (fabsf(Dx) + fabsf(Dy) + fabsf(Dz) + ne)
                         : gCell ? eBc
                                 : kEpsF * (fabsf(qx) + fabsf(qy) + fabsf(qz) + 0.5f * (nx * nx + ny * ny + nz * nz));
        const float inv = 1.0f / den;
        const float sa = num * inv;
        const float err = 2.0f * (eB + fabsf(sa) * eA) * inv + fabsf(sa) * kEpsF;
        const bool sure = den > 2.0f * eA;
        const bool none = den <= -eA || (sure && !(sa + err > 0.f));
        const float lo = none ? FLT_MAX : sure ? sa - err : -FLT_MAX;
        const float hi = (none || !sure) ? FLT_MAX : sa + err;
        gLo[q - g.cell_nbr_offset[m]] = lo;
        U = fminf(U, lo > 0.f ? hi : FLT_MAX);
        w1 = lo < L1 ? mi : w1;
        L2 = fmaxf(fminf(L1, L2), fminf(fmaxf(L1, L2), lo));  // median of L1 <= L2 and lo
        L1 = fminf(L1, lo);
    }
    if (L1 == FLT_MAX) { sq = DBL_MAX; return -99; }
    if (L2 > U) {
        sq = exactDist(g, m, w1, r, k);
        return w1;
    }
    fallbacks++;
    if (L1 == -FLT_MAX) gSignFallbacks++;
    // the possible winners (lower bound <= U), exactly, in list order; more than 4: the whole list
    std::vector<int> cand;
    for (int q = g.cell_nbr_offset[m]; q < g.cell_nbr_offset[m + 1]; q++)
        if (gLo[q - g.cell_nbr_offset[m]] < FLT_MAX && gLo[q - g.cell_nbr_offset[m]] <= U) cand.push_back(g.cell_nbr_list[q]);
    if (cand.size() > 4) { gWholeList++; return refStep(g, m, r, k, sq); }
    sq = DBL_MAX;
    int mq = -99;
    for (int mi : cand) {
        const double si = exactDist(g, m, mi, r, k);
        if (si > 0 && si < sq) { sq = si; mq = mi; }
    }
    return mq;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 100000;
    const int R = argc > 2 ? atoi(argv[2]) : 20000;
    std::mt19937_64 rng(4357);
    std::uniform_real_distribution<double> U01(0.0, 1.0);
    const double L = 1.5428387e19;  // 500 pc in m
    // Plummer-distributed sites (c = 100 pc) inside the box, like VoronoiDustGrid's DustDensity sites
    std::vector<double> sites;
    while ((int)sites.size() < 3 * N) {
        const double u = U01(rng);
        const double rr = 0.2 * L / sqrt(pow(u, -2.0 / 3.0) - 1.0);
        const double ct = 2 * U01(rng) - 1, ph = 2 * M_PI * U01(rng), st = sqrt(1 - ct * ct);
        const double x = rr * st * cos(ph), y = rr * st * sin(ph), z = rr * ct;
        if (fabs(x) < L && fabs(y) < L && fabs(z) < L) { sites.push_back(x); sites.push_back(y); sites.push_back(z); }
    }
    const double ext[6] = {-L, -L, -L, L, L, L};
    gScale = (float)(1.0 / L);
    const bool f32 = argc > 3 && (argv[3][0] == 'f' || argv[3][0] == 'c' || argv[3][0] == 'e' || argv[3][0] == 'd' ||
                                  argv[3][0] == 'x' || argv[3][0] == 'r');
    gDevice = argc > 3 && (argv[3][0] == 'd' || argv[3][0] == 'x' || argv[3][0] == 'r');
    gRecip = argc > 3 && argv[3][0] == 'r';
    if (gRecip && argv[3][1]) gRcpUlp = argv[3][1] == '+' ? 1 : argv[3][1] == '-' ? -1 : 2;
    gPerEntry = argc > 3 && argv[3][0] == 'x';
    gCell = argc > 3 && argv[3][0] == 'c';
    gEntry = argc > 3 && argv[3][0] == 'e';
    if (gEntry) gCell = true;
    SkirtVoronoi* v = skirt_host_voronoi_build(sites.data(), N, ext);
    if (!v) { fprintf(stderr, "voronoi: %s\n", skirt_sim_error()); return 1; }
    Mesh M{};
    skirt_host_voronoi_describe(v, &M.g);
    const SkirtGridDesc& g = M.g;
    const int nn = g.cell_nbr_offset[N];
    for (int m = 0; m < N; m++)
        if (g.cell_nbr_offset[m + 1] - g.cell_nbr_offset[m] > 4096) { fprintf(stderr, "neighbour list too long\n"); return 1; }
    M.off.assign(3 * (size_t)nn, 0.f);
    // scaled float offsets as the device stores them (engine.hip, Voronoi upload): walls as the offset to
    // the site's mirror image
    for (int m = 0; m < N; m++)
        for (int q = g.cell_nbr_offset[m]; q < g.cell_nbr_offset[m + 1]; q++) {
            const int mi = g.cell_nbr_list[q];
            const double* sm = g.site + 3 * (size_t)m;
            if (mi < 0) {
                const int axis = (-mi - 1) / 2;
                const double lim = (-mi - 1) % 2 ? g.extent[3 + axis] : g.extent[axis];
                const double w = lim - sm[axis];
                for (int d = 0; d < 3; d++) M.off[3 * (size_t)q + d] = 0.f;
                M.off[3 * (size_t)q + axis] = w != 0.0 ? (float)(2.0 * w * gScale) : 0.0f;  // degenerate: n = 0, den = 0, sign uncertain
                if (gRecip) {  // as the engine's Voronoi upload: m = n / |n|^2 (vor_terms.hpp)
                    double n[3] = {0.0, 0.0, 0.0};
                    n[axis] = w != 0.0 ? 2.0 * w * gScale : NAN;
                    vorRecipOffset(n[0], n[1], n[2], &M.off[3 * (size_t)q]);
                }
                continue;
            }
            for (int d = 0; d < 3; d++) M.off[3 * (size_t)q + d] = (float)((g.site[3 * (size_t)mi + d] - sm[d]) * gScale);
            if (gRecip)
                vorRecipOffset((g.site[3 * (size_t)mi] - sm[0]) * (double)gScale, (g.site[3 * (size_t)mi + 1] - sm[1]) * (double)gScale,
                               (g.site[3 * (size_t)mi + 2] - sm[2]) * (double)gScale, &M.off[3 * (size_t)q]);
        }
    M.nmax.assign(N, 0.f);
    for (int m = 0; m < N; m++)
        for (int q = g.cell_nbr_offset[m]; q < g.cell_nbr_offset[m + 1]; q++) {
            const float x = M.off[3 * (size_t)q], y = M.off[3 * (size_t)q + 1], z = M.off[3 * (size_t)q + 2];
            M.nmax[m] = fmaxf(M.nmax[m], sqrtf(x * x + y * y + z * z) * (1.0f + 4 * FLT_EPSILON));
        }
    // the header's per-cell error terms as the engine's Voronoi upload computes them
    M.eA.assign(N, 0.f);
    M.eB.assign(N, 0.f);
    for (int m = 0; m < N; m++) {
        const int q0 = g.cell_nbr_offset[m], q1 = g.cell_nbr_offset[m + 1];
        if (gRecip) vorRecipErrorTerms(M.off.data() + 3 * (size_t)q0, q1 - q0, 3, &M.eA[m], &M.eB[m]);
        else vorErrorTerms(M.off.data() + 3 * (size_t)q0, q1 - q0, 3, &M.eA[m], &M.eB[m]);
    }
    long steps = 0, fallbacks = 0, mismatches = 0;
    for (int i = 0; i < R; i++) {
        // a random start site's cell and an isotropic direction (positions start at the site)
        int m = (int)(U01(rng) * N);
        double r[3] = {g.site[3 * (size_t)m], g.site[3 * (size_t)m + 1], g.site[3 * (size_t)m + 2]};
        const double ct = 2 * U01(rng) - 1, ph = 2 * M_PI * U01(rng), st = sqrt(1 - ct * ct);
        const double k[3] = {st * cos(ph), st * sin(ph), ct};
        for (int s = 0; s < 100000 && m >= 0; s++) {
            double sa, sb;
            const int a = refStep(g, m, r, k, sa);
            const int b = f32 ? compactStepF(M, m, r, k, sb, fallbacks) : compactStep(M, m, r, k, sb, fallbacks);
            steps++;
            if (a != b || sa != sb) { mismatches++; break; }
            if (a == -99) break;
            for (int d = 0; d < 3; d++) r[d] += (sa + g.eps) * k[d];
            m = a;
        }
    }
    if (gRcpUlp) printf("reciprocals nudged: %s\n", gRcpUlp == 1 ? "+1 ulp" : gRcpUlp == -1 ? "-1 ulp" : "random -1/0/+1 ulp");
    printf("%s: sites %d, rays %d, steps %ld, exact re-evaluations %ld (%.3g per step), mismatches %ld\n",
           gRecip ? "f32 device bounds on reciprocal entries m = n/|n|^2 (per-cell terms)" :
           gPerEntry ? "f32 per-entry Cauchy-Schwarz bounds (round 3, first)" :
           gDevice ? "f32 device bounds (per-cell Cauchy-Schwarz terms)" : gEntry ? "f32 per-entry norm bounds" : gCell ? "f32 per-cell bounds" : f32 ? "f32 bounds" : "f64 bounds", N, R, steps,
           fallbacks, (double)fallbacks / steps, mismatches);
    if (f32) printf("  of which with an uncertain n.k sign: %ld; over the whole list: %ld\n", gSignFallbacks, gWholeList);
    skirt_host_voronoi_free(v);
    return mismatches ? 1 : 0;
}
