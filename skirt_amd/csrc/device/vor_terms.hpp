// The stored neighbour entries and per-cell error terms of the compact Voronoi step's single-precision bounds
// (engine.hip, Grid<SKIRT_GRID_VORONOI>::bounds), shared by the engine's Voronoi upload and the host
// exactness check (tools/vor_compact_check.cpp).
//
// For a neighbour offset n (scaled, rounded to float), the float evaluation of n.k and of n.D + |n|^2/2
// errs by at most a few 2^-24 of sum |n_i k_i| <= |n|_1 and of |n|_1 |D|_1 + |n|^2. The bounds take
// eA = kVorEpsF |n|_1 and kVorEpsF |n|^2 at the largest value over the cell's list (a per-cell Cauchy-
// Schwarz term: wider than per entry, so more steps fall back to the exact evaluation, but no entry
// pays for computing its own term).
#pragma once

#include <cmath>

// bound factor of the approximate (single-precision) plane distances: 16 x 2^-24
constexpr float kVorEpsF = 1.0f / (1 << 20);

// off: n offsets, each 3 floats at a stride of `stride` floats; NaN offsets (a degenerate wall, evaluated
// exactly by the step) are skipped. eA = kVorEpsF max |n|_1, eB = kVorEpsF max |n|^2, rounded up.
inline void vorErrorTerms(const float* off, int n, int stride, float* eA, float* eB) {
    double a = 0.0, b = 0.0;
    for (int q = 0; q < n; q++) {
        const double x = off[(long)q * stride], y = off[(long)q * stride + 1], z = off[(long)q * stride + 2];
        if (std::isnan(x) || std::isnan(y) || std::isnan(z)) continue;
        a = std::fmax(a, std::fabs(x) + std::fabs(y) + std::fabs(z));
        b = std::fmax(b, x * x + y * y + z * z);
    }
    *eA = std::nextafter((float)(kVorEpsF * a), INFINITY);
    *eB = std::nextafter((float)(kVorEpsF * b), INFINITY);
}

// Round 3 (final): the entries hold m = n / |n|^2 instead of n. The plane distance
// s = (n.D + |n|^2/2) / (n.k), numerator and denominator divided by |n|^2, is s = (m.D + 1/2) / (m.k):
// no |n|^2 to form per entry. Rounding m to float errs by 2^-24 |m_i| per component, as rounding n did, so
// the same Cauchy-Schwarz terms hold with m in place of n and the constant 1/2 in place of |n|^2/2:
// eA = kVorEpsF max |m|_1 and eB = kVorEpsF / 2 (the numerator's error <= eA |D|_1 + eB).
// n: the scaled offset in double; out: m in float, 0 for a degenerate offset (a site on a wall): its m.k is
// 0 for every direction, so the bounds call the entry's sign uncertain and the step evaluates the cell's
// list exactly. (NaN marks the padding after a cell's list instead: no exit.)
inline void vorRecipOffset(double nx, double ny, double nz, float out[3]) {
    const double q = nx * nx + ny * ny + nz * nz;
    if (!(q > 0.0) || !std::isfinite(q)) {
        out[0] = out[1] = out[2] = 0.0f;
        return;
    }
    out[0] = (float)(nx / q);
    out[1] = (float)(ny / q);
    out[2] = (float)(nz / q);
}

inline void vorRecipErrorTerms(const float* off, int n, int stride, float* eA, float* eB) {
    double a = 0.0;
    for (int q = 0; q < n; q++) {
        const double x = off[(long)q * stride], y = off[(long)q * stride + 1], z = off[(long)q * stride + 2];
        if (std::isnan(x) || std::isnan(y) || std::isnan(z)) continue;
        a = std::fmax(a, std::fabs(x) + std::fabs(y) + std::fabs(z));
    }
    *eA = std::nextafter((float)(kVorEpsF * a), INFINITY);
    *eB = std::nextafter((float)(kVorEpsF * 0.5), INFINITY);
}
