// The per-cell error terms of the compact Voronoi step's single-precision bounds
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
