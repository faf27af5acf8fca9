// MI355X photon-packet engine: persistent-wavefront HIP kernels + the C ABI of include/skirt_mcrt.h.
//
// One kernel launch runs one photon phase over a contiguous range of global packet indices. Every
// lane of every wavefront is a photon "slot" that runs the reference's per-packet life cycle
// (MonteCarloSimulation.cpp:265-301 launch -> peel-off -> fill/absorb -> propagate -> peel-off ->
// scatter) as a state machine whose expensive part -- walking a ray through the dust grid -- is one
// uniform loop body for all lanes. Ray kinds:
//   PEEL  optical depth to the grid edge towards an instrument (DustSystem::opticaldepth,
//         DustGridPath::opticalDepth, DustGridPath.hpp:97-108), then Instrument::detect;
//   FILL  fillOpticalDepth + simulateescapeandabsorption fused into one streaming pass (absorption of
//         segment n needs only tau_{n-1} and dtau_n, MonteCarloSimulation.cpp:447-470), f64 atomics
//         into Labs;
//   WALK  the same path walked again up to the sampled optical depth, replacing the stored segment
//         vector + NR::locate of DustGridPath::pathlength (DustGridPath.cpp:162-173) -- no per-lane
//         path buffer ever touches HBM.
// Lanes whose ray ended wait until enough lanes of the wave are waiting (ballot count >= threshold),
// then all of them run their event code together (launch, detect, sampling, scattering) and start
// their next ray, so the divergent event code is amortized over many lanes. New packets are claimed
// 64 at a time with one atomic per wave (ballot + mbcnt).
// Arithmetic follows the reference operation by operation (IEEE f64 division, exp/expm1/log), so a
// packet's history matches the CPU oracle's Philox mode to rounding.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/skirt_mcrt.h"
#include "philox.hpp"

using skirt_dev::PacketRng;

namespace {

constexpr double kDblMax = 1.7976931348623157e308;
constexpr int kBlock = 256;

// ------------------------------------------------------------------ device-side descriptors
struct DevInstr {
    int kind, nx, ny, nslots, levels, sedOff;  // sedOff: offset of this instrument's SEDs in LDS accumulator
    long long frameBase;                        // offset of frames in the global instrument tally
    long long sedBase;                          // offset of SEDs in the global instrument tally
    double kobs[3];
    double sinphi, cosphi, sintheta, costheta, sinpa, cospa;
    double xpmin, xpsiz, ypmin, ypsiz;
};

struct Args {
    // grid
    int nx, ny, nz, ncells;
    const double* xv;            // nx+1 | ny+1 | nz+1 concatenated (copied to LDS)
    double gx0, gx1, gy0, gy1, gz0, gz1;
    const double* box;           // octree
    const int* firstChild;
    const int* cellnumber;
    const int* nbrOffset;
    const int* nbrList;
    double eps;
    int search;
    // media
    int ncomp, nlambda;
    const double* rho;
    const double* optics;        // [4][ncomp][nlambda]: kext, ksca, albedo, g (copied to LDS)
    // sources
    int nstar;
    const int* geomKind;
    const double* geomParam;
    const double* lum;
    const double* lumtot;
    const double* cdf;
    double emissionBias;
    // instruments
    int ninstr;
    const DevInstr* instr;       // copied to LDS
    int nsed;                    // total SED accumulator doubles (LDS)
    // phase
    unsigned long long npp, first, end, seed;
    unsigned int tag;
    double minWeightReduction;
    int minScatt;
    double xi;
    int store, hasDust;
    // tallies
    double* labs;                // [nlambda][ncells]
    double* tally;               // instrument tallies
    unsigned long long* counter; // packet claim counter (relative to first)
    unsigned int* error;
    unsigned long long* stats;   // packets, seg_fill, seg_walk, seg_peel, detects, absorbs
    int threshold;
    int ldsMeshOff, ldsOptOff, ldsInstrOff, ldsSedOff;  // in doubles
};

enum RayMode : int { RAY_NONE = 0, RAY_PEEL = 1, RAY_FILL = 2, RAY_WALK = 3 };
enum State : int { S_NEW = 0, S_PEEL = 1, S_FILL = 2, S_WALK = 3, S_DONE = 4 };

__device__ inline void atomicAddF64(double* p, double v) {
    // explicit global address space: global_atomic_add_f64 instead of a flat atomic
    __hip_atomic_fetch_add((__attribute__((address_space(1))) double*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ per-lane photon slot
struct Slot {
    // photon package (PhotonPackage.hpp: _L, _ell, _nscatt, _stellar, _bfr, _bfk)
    double rx, ry, rz, kx, ky, kz, L, Lthreshold;
    int ell, nscatt, stellar, state;
    int peelScatter, instr;  // peel-off bookkeeping
    // current ray
    double x, y, z, dx, dy, dz;
    double tau, s, target;
    double ptau, ps, ptau2, ps2;  // WALK history (last two segment ends)
    double Lsca;                  // FILL with several dust components
    double bx0, by0, bz0, bx1, by1, bz1;  // octree: box of the current node
    int ci, cj, ck;               // Cartesian cell indices / octree node in ci
    int nseg, mode;
    PacketRng rng;
    // statistics
    unsigned int segFill, segWalk, segPeel, detects, absorbs, packets;
};

// ------------------------------------------------------------------ grid access helpers
template <int GRID>
struct Grid;

// Cartesian grid: CartesianDustGrid.cpp:136-283 (mesh borders staged in LDS)
template <>
struct Grid<SKIRT_GRID_CARTESIAN> {
    // returns false for an empty path; appends the up-to-three m=-1 entry segments through `seg`
    template <class SegFn>
    __device__ static inline bool begin(const Args& a, const double* __restrict__ mesh, Slot& sl, SegFn seg) {
        const double* xv = mesh;
        const double* yv = mesh + a.nx + 1;
        const double* zv = yv + a.ny + 1;
        double kx = sl.dx, ky = sl.dy, kz = sl.dz, x = sl.x, y = sl.y, z = sl.z;
        double d0 = 0, d1 = 0, d2 = 0;  // pending outside segments
        if (x < a.gx0) {
            if (kx <= 0.0) return false;
            d0 = (a.gx0 - x) / kx;
            x = a.gx0 + 1e-8 * (xv[1] - xv[0]); y += ky * d0; z += kz * d0;
        } else if (x > a.gx1) {
            if (kx >= 0.0) return false;
            d0 = (a.gx1 - x) / kx;
            x = a.gx1 - 1e-8 * (xv[a.nx] - xv[a.nx - 1]); y += ky * d0; z += kz * d0;
        }
        if (y < a.gy0) {
            if (ky <= 0.0) return false;
            d1 = (a.gy0 - y) / ky;
            x += kx * d1; y = a.gy0 + 1e-8 * (yv[1] - yv[0]); z += kz * d1;
        } else if (y > a.gy1) {
            if (ky >= 0.0) return false;
            d1 = (a.gy1 - y) / ky;
            x += kx * d1; y = a.gy1 - 1e-8 * (yv[a.ny] - yv[a.ny - 1]); z += kz * d1;
        }
        if (z < a.gz0) {
            if (kz <= 0.0) return false;
            d2 = (a.gz0 - z) / kz;
            x += kx * d2; y += ky * d2; z = a.gz0 + 1e-8 * (zv[1] - zv[0]);
        } else if (z > a.gz1) {
            if (kz >= 0.0) return false;
            d2 = (a.gz1 - z) / kz;
            x += kx * d2; y += ky * d2; z = a.gz1 - 1e-8 * (zv[a.nz] - zv[a.nz - 1]);
        }
        if (x < a.gx0 || x > a.gx1 || y < a.gy0 || y > a.gy1 || z < a.gz0 || z > a.gz1) return false;
        if (d0 > 0) seg(-1, d0);
        if (d1 > 0) seg(-1, d1);
        if (d2 > 0) seg(-1, d2);
        sl.x = x; sl.y = y; sl.z = z;
        sl.ci = locateClip(xv, a.nx + 1, x);
        sl.cj = locateClip(yv, a.ny + 1, y);
        sl.ck = locateClip(zv, a.nz + 1, z);
        return true;
    }

    __device__ static inline int locateClip(const double* v, int n, double q) {  // NR::locate_clip
        if (q < v[0]) return 0;
        int jl = -1, ju = n - 1;
        while (ju - jl > 1) {
            int jm = (ju + jl) >> 1;
            if (q < v[jm]) ju = jm;
            else jl = jm;
        }
        return jl;
    }

    // one DDA step: emits (m, ds) through `seg`; returns false when the ray left the grid
    template <class SegFn>
    __device__ static inline bool step(const Args& a, const double* __restrict__ mesh, Slot& sl, SegFn seg) {
        const double* xv = mesh;
        const double* yv = mesh + a.nx + 1;
        const double* zv = yv + a.ny + 1;
        const double kx = sl.dx, ky = sl.dy, kz = sl.dz;
        const int i = sl.ci, j = sl.cj, k = sl.ck;
        const int m = k + a.nz * j + a.nz * a.ny * i;
        const double xE = (kx < 0.0) ? xv[i] : xv[i + 1];
        const double yE = (ky < 0.0) ? yv[j] : yv[j + 1];
        const double zE = (kz < 0.0) ? zv[k] : zv[k + 1];
        const double dsx = (fabs(kx) > 1e-15) ? (xE - sl.x) / kx : kDblMax;
        const double dsy = (fabs(ky) > 1e-15) ? (yE - sl.y) / ky : kDblMax;
        const double dsz = (fabs(kz) > 1e-15) ? (zE - sl.z) / kz : kDblMax;
        if (dsx <= dsy && dsx <= dsz) {
            if (!seg(m, dsx)) return false;
            const int ni = i + ((kx < 0.0) ? -1 : 1);
            if (ni >= a.nx || ni < 0) return false;
            sl.ci = ni; sl.x = xE; sl.y += ky * dsx; sl.z += kz * dsx;
        } else if (dsy < dsx && dsy <= dsz) {
            if (!seg(m, dsy)) return false;
            const int nj = j + ((ky < 0.0) ? -1 : 1);
            if (nj >= a.ny || nj < 0) return false;
            sl.cj = nj; sl.x += kx * dsy; sl.y = yE; sl.z += kz * dsy;
        } else if (dsz < dsx && dsz < dsy) {
            if (!seg(m, dsz)) return false;
            const int nk = k + ((kz < 0.0) ? -1 : 1);
            if (nk >= a.nz || nk < 0) return false;
            sl.ck = nk; sl.x += kx * dsz; sl.y += ky * dsz; sl.z = zE;
        } else {
            return false;  // NaN direction; the reference would loop forever
        }
        return true;
    }

    __device__ static inline int whichcell(const Args& a, const double* __restrict__ mesh, double x, double y, double z) {
        const double* xv = mesh;
        const double* yv = mesh + a.nx + 1;
        const double* zv = yv + a.ny + 1;
        int i = locateFail(xv, a.nx + 1, x), j = locateFail(yv, a.ny + 1, y), k = locateFail(zv, a.nz + 1, z);
        if (i < 0 || j < 0 || k < 0) return -1;
        return k + a.nz * j + a.nz * a.ny * i;
    }
    __device__ static inline int locateFail(const double* v, int n, double q) {
        if (q > v[n - 1]) return -1;
        int jl = -1, ju = n - 1;
        while (ju - jl > 1) {
            int jm = (ju + jl) >> 1;
            if (q < v[jm]) ju = jm;
            else jl = jm;
        }
        return jl;
    }
};

// Octree grid: TreeDustGrid.cpp:390-521 (TopDown and Neighbor search), DustGridPath::moveInside
template <>
struct Grid<SKIRT_GRID_OCTREE> {
    __device__ static inline void loadBox(const Args& a, int l, double& x0, double& y0, double& z0, double& x1,
                                          double& y1, double& z1) {
        const double2* b = reinterpret_cast<const double2*>(a.box + 6 * (size_t)l);
        double2 p = b[0], q = b[1], r = b[2];
        x0 = p.x; y0 = p.y; z0 = q.x; x1 = q.y; y1 = r.x; z1 = r.y;
    }

    // TreeNode::whichnode from the root: returns the leaf node containing (x,y,z) or -1
    __device__ static inline int rootWhichnode(const Args& a, double x, double y, double z, Slot& sl) {
        if (!(x >= a.gx0 && x <= a.gx1 && y >= a.gy0 && y <= a.gy1 && z >= a.gz0 && z <= a.gz1)) return -1;
        int l = 0;
        int c0 = a.firstChild[0];
        while (c0 >= 0) {
            // OctTreeNode::child(r): split point = rmax of child 0
            const double* cb = a.box + 6 * (size_t)c0;
            l = c0 + (x < cb[3] ? 0 : 1) + (y < cb[4] ? 0 : 2) + (z < cb[5] ? 0 : 4);
            c0 = a.firstChild[l];
        }
        loadBox(a, l, sl.bx0, sl.by0, sl.bz0, sl.bx1, sl.by1, sl.bz1);
        return l;
    }

    template <class SegFn>
    __device__ static inline bool begin(const Args& a, const double* __restrict__, Slot& sl, SegFn seg) {
        const double kx = sl.dx, ky = sl.dy, kz = sl.dz, eps = a.eps;
        double rx = sl.x, ry = sl.y, rz = sl.z, d0 = 0, d1 = 0, d2 = 0;
        if (rx <= a.gx0) {
            if (kx <= 0.0) return false;
            d0 = (a.gx0 - rx) / kx; rx = a.gx0 + eps; ry += ky * d0; rz += kz * d0;
        } else if (rx >= a.gx1) {
            if (kx >= 0.0) return false;
            d0 = (a.gx1 - rx) / kx; rx = a.gx1 - eps; ry += ky * d0; rz += kz * d0;
        }
        if (ry <= a.gy0) {
            if (ky <= 0.0) return false;
            d1 = (a.gy0 - ry) / ky; rx += kx * d1; ry = a.gy0 + eps; rz += kz * d1;
        } else if (ry >= a.gy1) {
            if (ky >= 0.0) return false;
            d1 = (a.gy1 - ry) / ky; rx += kx * d1; ry = a.gy1 - eps; rz += kz * d1;
        }
        if (rz <= a.gz0) {
            if (kz <= 0.0) return false;
            d2 = (a.gz0 - rz) / kz; rx += kx * d2; ry += ky * d2; rz = a.gz0 + eps;
        } else if (rz >= a.gz1) {
            if (kz >= 0.0) return false;
            d2 = (a.gz1 - rz) / kz; rx += kx * d2; ry += ky * d2; rz = a.gz1 - eps;
        }
        int node = rootWhichnode(a, rx, ry, rz, sl);
        if (node < 0) return false;
        if (d0 > 0) seg(-1, d0);
        if (d1 > 0) seg(-1, d1);
        if (d2 > 0) seg(-1, d2);
        sl.x = rx; sl.y = ry; sl.z = rz;
        sl.ci = node;
        return true;
    }

    template <class SegFn>
    __device__ static inline bool step(const Args& a, const double* __restrict__, Slot& sl, SegFn seg) {
        const double kx = sl.dx, ky = sl.dy, kz = sl.dz;
        const int node = sl.ci;
        const double xnext = (kx < 0.0) ? sl.bx0 : sl.bx1;
        const double ynext = (ky < 0.0) ? sl.by0 : sl.by1;
        const double znext = (kz < 0.0) ? sl.bz0 : sl.bz1;
        const double dsx = (fabs(kx) > 1e-15) ? (xnext - sl.x) / kx : kDblMax;
        const double dsy = (fabs(ky) > 1e-15) ? (ynext - sl.y) / ky : kDblMax;
        const double dsz = (fabs(kz) > 1e-15) ? (znext - sl.z) / kz : kDblMax;
        double ds;
        int wall;
        if (dsx <= dsy && dsx <= dsz) { ds = dsx; wall = (kx < 0.0) ? 0 : 1; }
        else if (dsy <= dsx && dsy <= dsz) { ds = dsy; wall = (ky < 0.0) ? 2 : 3; }
        else { ds = dsz; wall = (kz < 0.0) ? 4 : 5; }
        if (!seg(a.cellnumber[node], ds)) return false;
        double x = sl.x + (ds + a.eps) * kx;
        double y = sl.y + (ds + a.eps) * ky;
        double z = sl.z + (ds + a.eps) * kz;
        int next = -1;
        if (a.search == SKIRT_TREE_NEIGHBOR) {
            const int q = 6 * node + wall;
            const int nb = a.nbrOffset[q], ne = a.nbrOffset[q + 1];
            for (int n = nb; n < ne; n++) {
                const int c = a.nbrList[n];
                double x0, y0, z0, x1, y1, z1;
                loadBox(a, c, x0, y0, z0, x1, y1, z1);
                if (x >= x0 && x <= x1 && y >= y0 && y <= y1 && z >= z0 && z <= z1) {
                    next = c;
                    sl.bx0 = x0; sl.by0 = y0; sl.bz0 = z0; sl.bx1 = x1; sl.by1 = y1; sl.bz1 = z1;
                    break;
                }
            }
        }
        if (next < 0) next = rootWhichnode(a, x, y, z, sl);
        if (next == node) {
            // stuck: advance to the next representable coordinates (TreeDustGrid.cpp:502-519)
            x = nextafter(x, (kx < 0.0) ? -kDblMax : kDblMax);
            y = nextafter(y, (ky < 0.0) ? -kDblMax : kDblMax);
            z = nextafter(z, (kz < 0.0) ? -kDblMax : kDblMax);
            next = rootWhichnode(a, x, y, z, sl);
            if (next == node) return false;
        }
        sl.x = x; sl.y = y; sl.z = z;
        sl.ci = next;
        return next >= 0;
    }

    __device__ static inline int whichcell(const Args& a, const double* __restrict__, double x, double y, double z) {
        if (!(x >= a.gx0 && x <= a.gx1 && y >= a.gy0 && y <= a.gy1 && z >= a.gz0 && z <= a.gz1)) return -1;
        int l = 0;
        int c0 = a.firstChild[0];
        while (c0 >= 0) {
            const double* cb = a.box + 6 * (size_t)c0;
            l = c0 + (x < cb[3] ? 0 : 1) + (y < cb[4] ? 0 : 2) + (z < cb[5] ? 0 : 4);
            c0 = a.firstChild[l];
        }
        return a.cellnumber[l];
    }
};

// ------------------------------------------------------------------ the kernel
template <int GRID, bool ONECOMP>
__global__ void __launch_bounds__(kBlock) stellarKernel(const Args a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* mesh = lds + a.ldsMeshOff;
    double* opt = lds + a.ldsOptOff;
    DevInstr* instr = reinterpret_cast<DevInstr*>(lds + a.ldsInstrOff);
    double* sedAcc = lds + a.ldsSedOff;

    // stage the mesh, the optical tables and the instruments in LDS
    {
        const int nmesh = (GRID == SKIRT_GRID_CARTESIAN) ? (a.nx + a.ny + a.nz + 3) : 0;
        for (int q = threadIdx.x; q < nmesh; q += blockDim.x) mesh[q] = a.xv[q];
        const int nopt = 4 * a.ncomp * a.nlambda;
        for (int q = threadIdx.x; q < nopt; q += blockDim.x) opt[q] = a.optics[q];
        const int ninw = a.ninstr * (int)(sizeof(DevInstr) / sizeof(double));
        const double* isrc = reinterpret_cast<const double*>(a.instr);
        double* idst = reinterpret_cast<double*>(instr);
        for (int q = threadIdx.x; q < ninw; q += blockDim.x) idst[q] = isrc[q];
        for (int q = threadIdx.x; q < a.nsed; q += blockDim.x) sedAcc[q] = 0.0;
        __syncthreads();
    }
    const double* kextT = opt;
    const double* kscaT = opt + a.ncomp * a.nlambda;
    const double* albT = opt + 2 * a.ncomp * a.nlambda;
    const double* gT = opt + 3 * a.ncomp * a.nlambda;

    const int lane = threadIdx.x & 63;
    Slot sl;
    sl.state = S_NEW;
    sl.mode = RAY_NONE;
    sl.segFill = sl.segWalk = sl.segPeel = sl.detects = sl.absorbs = sl.packets = 0;
    const unsigned long long total = a.end - a.first;

    // kappa*rho summed over components (DustSystem.cpp:465-491 KappaRho)
    auto kapparho = [&](int m, int ell) __attribute__((always_inline)) -> double {
        if (m < 0) return 0.0;
        if (ONECOMP) return 0.0 + kextT[ell] * a.rho[m];
        double r = 0;
        for (int h = 0; h < a.ncomp; h++) r += kextT[h * a.nlambda + ell] * a.rho[(size_t)m * a.ncomp + h];
        return r;
    };

    // per-segment work of the three ray kinds; returns false to stop the ray (WALK found its point)
    auto segment = [&](int m, double ds) __attribute__((always_inline)) -> bool {
        if (!(ds > 0)) return true;  // DustGridPath::addSegment skips ds <= 0
        sl.s += ds;
        sl.nseg++;
        const double dtau = kapparho(m, sl.ell) * ds;
        const double taustart = sl.tau;
        sl.tau = taustart + dtau;
        if (sl.mode == RAY_FILL) {
            sl.segFill++;
            if (m != -1) {
                if (ONECOMP) {
                    if (a.store) {
                        const double expfactorm = -expm1(-dtau);
                        const double Lintm = sl.L * exp(-taustart) * expfactorm;
                        const double Labsm = (1.0 - albT[sl.ell]) * Lintm;
                        atomicAddF64(a.labs + (size_t)sl.ell * a.ncells + m, Labsm);
                        sl.absorbs++;
                    }
                } else {
                    double ksca = 0.0, kext = 0.0;
                    for (int h = 0; h < a.ncomp; h++) {
                        const double rho = a.rho[(size_t)m * a.ncomp + h];
                        ksca += rho * kscaT[h * a.nlambda + sl.ell];
                        kext += rho * kextT[h * a.nlambda + sl.ell];
                    }
                    const double albedo = (kext > 0.0) ? ksca / kext : 0.0;
                    const double expfactorm = -expm1(-dtau);
                    const double Lintm = sl.L * exp(-taustart) * expfactorm;
                    sl.Lsca += albedo * Lintm;
                    if (a.store) {
                        atomicAddF64(a.labs + (size_t)sl.ell * a.ncells + m, (1.0 - albedo) * Lintm);
                        sl.absorbs++;
                    }
                }
            }
        } else if (sl.mode == RAY_WALK) {
            sl.segWalk++;
            if (sl.tau > sl.target) return false;  // interaction point lies in this segment
            sl.ptau2 = sl.ptau; sl.ps2 = sl.ps;
            sl.ptau = sl.tau; sl.ps = sl.s;
        } else {
            sl.segPeel++;
        }
        return true;
    };

    // starts a ray from the packet position; returns false if the path is empty
    auto startRay = [&](int mode, double dx, double dy, double dz) __attribute__((always_inline)) -> bool {
        sl.mode = mode;
        sl.x = sl.rx; sl.y = sl.ry; sl.z = sl.rz;
        sl.dx = dx; sl.dy = dy; sl.dz = dz;
        sl.tau = 0; sl.s = 0; sl.nseg = 0;
        sl.ptau = 0; sl.ps = 0; sl.ptau2 = 0; sl.ps2 = 0;
        sl.Lsca = 0;
        bool ok = Grid<GRID>::begin(a, mesh, sl, segment);
        if (!ok) { sl.mode = RAY_NONE; sl.tau = 0; sl.s = 0; sl.nseg = 0; sl.ptau = sl.ps = sl.ptau2 = sl.ps2 = 0; }
        return ok;
    };

    // Instrument::detect (FullInstrument.cpp:107-174, Simple/SED/Frame variants)
    auto detect = [&](const DevInstr& ins, double Lp, int nscatt, double taupath) __attribute__((always_inline)) {
        int l = -1;
        if (ins.kind != SKIRT_INSTR_SED) {
            const double x = sl.rx, y = sl.ry, z = sl.rz;
            const double xpp = -ins.sinphi * x + ins.cosphi * y;
            const double ypp = -ins.cosphi * ins.costheta * x - ins.sinphi * ins.costheta * y + ins.sintheta * z;
            const double xp = ins.cospa * xpp - ins.sinpa * ypp;
            const double yp = ins.sinpa * xpp + ins.cospa * ypp;
            const int i = static_cast<int>(floor((xp - ins.xpmin) / ins.xpsiz));
            const int j = static_cast<int>(floor((yp - ins.ypmin) / ins.ypsiz));
            l = (i < 0 || i >= ins.nx || j < 0 || j >= ins.ny) ? -1 : i + ins.nx * j;
        }
        const double extf = exp(-taupath);
        const double Lextf = Lp * extf;
        const int nl = a.nlambda;
        const long long nframe = (long long)ins.nx * ins.ny;
        sl.detects++;
        auto add = [&](int slot, double v) __attribute__((always_inline)) {
            if (ins.kind != SKIRT_INSTR_FRAME) atomicAdd(&sedAcc[ins.sedOff + slot * nl + sl.ell], v);
            if (l >= 0 && ins.kind != SKIRT_INSTR_SED)
                atomicAddF64(a.tally + ins.frameBase + ((long long)slot * nl + sl.ell) * nframe + l, v);
        };
        if (ins.kind != SKIRT_INSTR_FULL) { add(0, Lextf); return; }
        if (sl.stellar >= 0) {
            if (nscatt == 0) {
                add(0, Lp);
                if (a.hasDust) add(1, Lextf);
            } else {
                add(2, Lextf);
                if (nscatt <= ins.levels) add(5 + nscatt - 1, Lextf);
            }
        } else {
            add(nscatt == 0 ? 3 : 4, Lextf);
        }
    };

    // component weights of the peel-off phase functions (MonteCarloSimulation.cpp:325-339)
    auto peelWv = [&](double* wv) __attribute__((always_inline)) {
        if (ONECOMP) return;
        const int m = Grid<GRID>::whichcell(a, mesh, sl.rx, sl.ry, sl.rz);
        double sum = 0;
        for (int h = 0; h < a.ncomp; h++) wv[h] = kscaT[h * a.nlambda + sl.ell] * a.rho[(size_t)m * a.ncomp + h];
        for (int h = 0; h < a.ncomp; h++) sum += wv[h];
        for (int h = 0; h < a.ncomp; h++) wv[h] /= sum;
    };

    // peel-off weight of instrument `ins` for the current scattering (MonteCarloSimulation.cpp:319-363)
    auto peelWeight = [&](const DevInstr& ins, const double* wv) __attribute__((always_inline)) -> double {
        double I = 0;
        for (int h = 0; h < (ONECOMP ? 1 : a.ncomp); h++) {
            const double cosalpha = sl.kx * ins.kobs[0] + sl.ky * ins.kobs[1] + sl.kz * ins.kobs[2];
            const double g = gT[h * a.nlambda + sl.ell];
            const double t = 1.0 + g * g - 2 * g * cosalpha;
            const double w = (ONECOMP ? 1.0 : wv[h]) * ((1.0 - g) * (1.0 + g) / sqrt(t * t * t));
            I += w * 1.0;
        }
        return I;
    };

    // starts the next peel-off ray for instruments from sl.instr on; returns true if a ray was started,
    // false if all remaining instruments were handled (detected without traversal or skipped)
    auto nextPeel = [&]() __attribute__((always_inline)) -> bool {
        while (sl.instr < a.ninstr) {
            const DevInstr& ins = instr[sl.instr];
            if (ins.kind == SKIRT_INSTR_FRAME) {
                // FrameInstrument::detect computes tau only for packets that land on the frame
                const double x = sl.rx, y = sl.ry, z = sl.rz;
                const double xpp = -ins.sinphi * x + ins.cosphi * y;
                const double ypp = -ins.cosphi * ins.costheta * x - ins.sinphi * ins.costheta * y + ins.sintheta * z;
                const double xp = ins.cospa * xpp - ins.sinpa * ypp;
                const double yp = ins.sinpa * xpp + ins.cospa * ypp;
                const int i = static_cast<int>(floor((xp - ins.xpmin) / ins.xpsiz));
                const int j = static_cast<int>(floor((yp - ins.ypmin) / ins.ypsiz));
                if (i < 0 || i >= ins.nx || j < 0 || j >= ins.ny) { sl.instr++; continue; }
            }
            if (a.hasDust && startRay(RAY_PEEL, ins.kobs[0], ins.kobs[1], ins.kobs[2])) return true;
            // empty path or no dust: tau = 0
            double wv[8];
            if (sl.peelScatter) peelWv(wv);
            const double Lp = sl.peelScatter ? sl.L * peelWeight(ins, wv) : sl.L;
            detect(ins, Lp, sl.peelScatter ? sl.nscatt + 1 : 0, 0.0);
            sl.instr++;
        }
        return false;
    };

    // DustMix::scatteringDirectionAndPolarization (HG, DustMix.cpp:609-613) + Random::direction(k, costheta)
    auto scatter = [&]() __attribute__((always_inline)) {
        int hmix = 0;
        if (!ONECOMP) {
            // DustSystem::randomMixForPosition: NR::cdf over kappasca*rho, then NR::locate_clip
            const int m = Grid<GRID>::whichcell(a, mesh, sl.rx, sl.ry, sl.rz);
            if (m >= 0) {
                double Xv[9];
                Xv[0] = 0.0;
                for (int h = 0; h < a.ncomp; h++) Xv[h + 1] = Xv[h] + kscaT[h * a.nlambda + sl.ell] * a.rho[(size_t)m * a.ncomp + h];
                const double norm = Xv[a.ncomp];
                for (int h = 0; h <= a.ncomp; h++) Xv[h] /= norm;
                const double X = sl.rng.uniform();
                int sel = 0;
                for (int h = 1; h < a.ncomp; h++)
                    if (Xv[h] <= X) sel = h;
                hmix = sel;
            }
        }
        const double g = gT[hmix * a.nlambda + sl.ell];
        double nx, ny, nz;
        if (fabs(g) < 1e-6) {
            const double theta = acos(2.0 * sl.rng.uniform() - 1.0);
            const double phi = 2.0 * M_PI * sl.rng.uniform();
            if (theta <= 1e-8) { nx = 0; ny = 0; nz = 1; }
            else if (theta >= M_PI - 1e-8) { nx = 0; ny = 0; nz = -1; }
            else { const double st = sin(theta); nx = st * cos(phi); ny = st * sin(phi); nz = cos(theta); }
        } else {
            const double f = ((1.0 - g) * (1.0 + g)) / (1.0 - g + 2.0 * g * sl.rng.uniform());
            const double costheta = (1.0 + g * g - f * f) / (2.0 * g);
            const double phi = 2.0 * M_PI * sl.rng.uniform();
            const double cosphi = cos(phi), sinphi = sin(phi);
            const double sintheta = sqrt(fabs((1.0 - costheta) * (1.0 + costheta)));
            const double kx = sl.kx, ky = sl.ky, kz = sl.kz;
            if (kz > 0.99999) { nx = cosphi * sintheta; ny = sinphi * sintheta; nz = costheta; }
            else if (kz < -0.99999) { nx = cosphi * sintheta; ny = sinphi * sintheta; nz = -costheta; }
            else {
                const double root = sqrt((1.0 - kz) * (1.0 + kz));
                nx = sintheta / root * (-kx * kz * cosphi + ky * sinphi) + kx * costheta;
                ny = -sintheta / root * (ky * kz * cosphi + kx * sinphi) + ky * costheta;
                nz = root * sintheta * cosphi + kz * costheta;
            }
        }
        sl.nscatt++;
        sl.kx = nx; sl.ky = ny; sl.kz = nz;
    };

    // after a peel-off round of a scattering event: scatter and start the next FILL ray
    auto scatterAndFill = [&]() __attribute__((always_inline)) {
        scatter();
        sl.state = S_FILL;
        if (!startRay(RAY_FILL, sl.kx, sl.ky, sl.kz)) sl.mode = RAY_NONE;  // empty path: FILL ends at once
    };

    // WALK end: propagate and begin the peel-off round of this scattering (or scatter directly)
    auto propagateAndPeel = [&](double s) __attribute__((always_inline)) {
        sl.rx = sl.rx + s * sl.kx;
        sl.ry = sl.ry + s * sl.ky;
        sl.rz = sl.rz + s * sl.kz;
        bool ok = a.ninstr > 0;
        if (ok && !ONECOMP) {
            const int m = Grid<GRID>::whichcell(a, mesh, sl.rx, sl.ry, sl.rz);
            if (m == -1) ok = false;
            else {
                double sum = 0;
                for (int h = 0; h < a.ncomp; h++) sum += kscaT[h * a.nlambda + sl.ell] * a.rho[(size_t)m * a.ncomp + h];
                if (sum <= 0) ok = false;
            }
        }
        if (ok) {
            sl.state = S_PEEL;
            sl.peelScatter = 1;
            sl.instr = 0;
            if (nextPeel()) return;
        }
        scatterAndFill();
    };

    // ---------------------------------------------------------- event code: one packet transition
    // Runs for a lane whose ray ended (or that needs a new packet); leaves it with a new ray, or in
    // S_NEW (packet finished), or S_DONE.
    auto transition = [&]() __attribute__((always_inline)) {
        switch (sl.state) {
        case S_PEEL: {
            const DevInstr& ins = instr[sl.instr];
            double Lp = sl.L;
            if (sl.peelScatter) {
                double wv[8];
                peelWv(wv);
                Lp = sl.L * peelWeight(ins, wv);
            }
            detect(ins, Lp, sl.peelScatter ? sl.nscatt + 1 : 0, sl.tau);
            sl.instr++;
            if (nextPeel()) return;
            if (sl.peelScatter) { scatterAndFill(); return; }
            if (a.hasDust) {
                sl.state = S_FILL;
                if (!startRay(RAY_FILL, sl.kx, sl.ky, sl.kz)) sl.mode = RAY_NONE;
                return;
            }
            sl.state = S_NEW;
            return;
        }
        case S_FILL: {
            // ray finished (or empty): simulateescapeandabsorption + termination + propagation sampling
            const double taupath = sl.tau;
            if (taupath < 0.0 || isnan(taupath) || isinf(taupath)) {
                atomicOr(a.error, 1u);
                sl.state = S_NEW;
                return;
            }
            if (ONECOMP) {
                const double albedo = albT[sl.ell];
                const double expfactor = -expm1(-taupath);
                sl.L = sl.L * albedo * expfactor;
            } else {
                sl.L = sl.Lsca;
            }
            if (sl.L <= 0 || (sl.L <= sl.Lthreshold && sl.nscatt >= a.minScatt)) { sl.state = S_NEW; return; }
            if (taupath == 0.0) { propagateAndPeel(0.0); return; }
            double tauint;
            if (a.xi == 0.0) tauint = -1.0;
            else {
                const double X = sl.rng.uniform();
                tauint = (X < a.xi) ? sl.rng.uniform() * taupath : -1.0;
            }
            if (tauint < 0.0) {
                // Random::exponcutoff (Random.cpp:162-175)
                if (taupath < 1e-10) tauint = sl.rng.uniform() * taupath;
                else {
                    double x = -log(1.0 - sl.rng.uniform() * (1.0 - exp(-taupath)));
                    while (x > taupath) x = -log(1.0 - sl.rng.uniform() * (1.0 - exp(-taupath)));
                    tauint = x;
                }
            }
            if (a.xi != 0.0) {
                const double p = -exp(-tauint) / expm1(-taupath);
                const double q = (1.0 - a.xi) * p + a.xi / taupath;
                const double weight = p / q;
                sl.L = sl.L * weight;
            }
            sl.state = S_WALK;
            sl.target = tauint;
            if (!(tauint > 0) || !startRay(RAY_WALK, sl.kx, sl.ky, sl.kz)) { sl.mode = RAY_NONE; sl.nseg = 0; }
            return;
        }
        case S_WALK: {
            // DustGridPath::pathlength: the interaction segment was found (ray stopped) or the path ended
            double s = 0;
            const double tauint = sl.target;
            if (sl.nseg > 0 && tauint > 0) {
                if (sl.tau > tauint) {
                    s = sl.ps + ((tauint - sl.ptau) / (sl.tau - sl.ptau)) * (sl.s - sl.ps);
                } else if (sl.ptau < tauint || sl.nseg == 1) {
                    s = sl.ps;  // last segment end
                } else {
                    s = sl.ps2 + ((tauint - sl.ptau2) / (sl.ptau - sl.ptau2)) * (sl.ps - sl.ps2);
                }
            }
            propagateAndPeel(s);
            return;
        }
        default:
            return;
        }
    };

    // launch a new packet: StellarSystem::launch + GeometricStellarComp::launch (Plummer)
    auto launch = [&](unsigned long long p) __attribute__((always_inline)) {
        const int ell = (int)(p / a.npp);
        const double L0 = a.lumtot[ell] / (double)a.npp;
        if (!(L0 > 0)) { sl.state = S_NEW; return; }  // dostellaremissionchunk skips such wavelengths
        sl.packets++;
        sl.Lthreshold = L0 / a.minWeightReduction;
        sl.rng.start(a.seed, a.tag, p);
        sl.ell = ell;
        int h = 0;
        double L = L0;
        const int N = a.nstar;
        if (N > 1) {
            const double X = sl.rng.uniform();
            const double xi = a.emissionBias;
            if (X < xi) h = max(0, min(N - 1, static_cast<int>(N * X / xi)));
            else {
                const double* Xv = a.cdf + (size_t)ell * (N + 1);
                const double q = (X - xi) / (1.0 - xi);
                if (q < Xv[0]) h = 0;
                else {
                    int lo = -1, hi = N;
                    while (hi - lo > 1) { int jm = (hi + lo) >> 1; if (q < Xv[jm]) hi = jm; else lo = jm; }
                    h = lo;
                }
            }
            const double Lh = a.lum[(size_t)h * a.nlambda + ell];
            if (Lh > 0) {
                const double Lmean = a.lumtot[ell] / N;
                const double weight = 1.0 / (1.0 - xi + xi * Lmean / Lh);
                L = L0 * weight;
            } else {
                sl.state = S_NEW;  // launched with zero luminosity
                return;
            }
        }
        const double c = a.geomParam[4 * h];
        // PlummerGeometry::randomradius, SpheGeometry::generatePosition, Random::direction() twice
        const double t = pow(sl.rng.uniform(), 1.0 / 3.0);
        const double r = c * t / sqrt((1.0 - t) * (1.0 + t));
        double dx, dy, dz;
        {
            const double theta = acos(2.0 * sl.rng.uniform() - 1.0);
            const double phi = 2.0 * M_PI * sl.rng.uniform();
            if (theta <= 1e-8) { dx = 0; dy = 0; dz = 1; }
            else if (theta >= M_PI - 1e-8) { dx = 0; dy = 0; dz = -1; }
            else { const double st = sin(theta); dx = st * cos(phi); dy = st * sin(phi); dz = cos(theta); }
        }
        sl.rx = r * dx; sl.ry = r * dy; sl.rz = r * dz;
        {
            const double theta = acos(2.0 * sl.rng.uniform() - 1.0);
            const double phi = 2.0 * M_PI * sl.rng.uniform();
            if (theta <= 1e-8) { dx = 0; dy = 0; dz = 1; }
            else if (theta >= M_PI - 1e-8) { dx = 0; dy = 0; dz = -1; }
            else { const double st = sin(theta); dx = st * cos(phi); dy = st * sin(phi); dz = cos(theta); }
        }
        sl.kx = dx; sl.ky = dy; sl.kz = dz;
        sl.L = L;
        sl.nscatt = 0;
        sl.stellar = h;
        // peeloffemission
        sl.state = S_PEEL;
        sl.peelScatter = 0;
        sl.instr = 0;
        if (nextPeel()) return;
        if (a.hasDust) {
            sl.state = S_FILL;
            if (!startRay(RAY_FILL, sl.kx, sl.ky, sl.kz)) sl.mode = RAY_NONE;
            return;
        }
        sl.state = S_NEW;
    };

    // ---------------------------------------------------------- main loop
    while (true) {
        const bool waiting = (sl.mode == RAY_NONE) && (sl.state != S_DONE);
        const unsigned long long wmask = __ballot(waiting);
        const unsigned long long rmask = __ballot(sl.mode != RAY_NONE);
        if (wmask == 0 && rmask == 0) break;  // every lane is done
        if (wmask != 0 && (rmask == 0 || __popcll(wmask) >= a.threshold)) {
            bool inH = waiting;
            while (true) {
                // lanes that need a packet claim consecutive indices with one atomic per wave
                const bool need = inH && sl.state == S_NEW;
                const unsigned long long nmask = __ballot(need);
                if (nmask) {
                    const int cnt = __popcll(nmask);
                    const int leader = __ffsll((long long)nmask) - 1;
                    unsigned long long base = 0;
                    if (lane == leader) base = atomicAdd(a.counter, (unsigned long long)cnt);
                    base = __shfl(base, leader);
                    if (need) {
                        const unsigned long long rank = __popcll(nmask & ((1ull << lane) - 1ull));
                        const unsigned long long idx = base + rank;
                        if (idx >= total) sl.state = S_DONE;
                        else launch(a.first + idx);
                    }
                }
                if (inH && !need && sl.state != S_DONE && sl.state != S_NEW) transition();
                inH = inH && sl.state != S_DONE && sl.mode == RAY_NONE;
                if (!__ballot(inH)) break;
            }
        }
        // advance every active ray by a few segments
#pragma unroll 1
        for (int it = 0; it < 4; it++) {
            if (sl.mode != RAY_NONE) {
                if (!Grid<GRID>::step(a, mesh, sl, segment)) sl.mode = RAY_NONE;
            }
        }
    }

    // flush per-workgroup SED accumulators and statistics
    __syncthreads();
    for (int q = threadIdx.x; q < a.nsed; q += blockDim.x) {
        const double v = sedAcc[q];
        if (v != 0.0) {
            // map the LDS accumulator index back to the global SED tally
            int ii = 0;
            while (ii + 1 < a.ninstr && instr[ii + 1].sedOff <= q) ii++;
            atomicAddF64(a.tally + instr[ii].sedBase + (q - instr[ii].sedOff), v);
        }
    }
    unsigned long long vals[6] = {sl.packets, sl.segFill, sl.segWalk, sl.segPeel, sl.detects, sl.absorbs};
#pragma unroll
    for (int q = 0; q < 6; q++) {
        unsigned long long v = vals[q];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0 && v) atomicAdd(a.stats + q, v);
    }
}

}  // namespace

// ====================================================================== host side: the C ABI

struct SkirtMcrt {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    // grid
    int gridKind = -1, ncells = 0, nx = 0, ny = 0, nz = 0, nnodes = 0, search = 1;
    double eps = 0, gx0 = 0, gx1 = 0, gy0 = 0, gy1 = 0, gz0 = 0, gz1 = 0;
    double* dMesh = nullptr;
    double* dBox = nullptr;
    int *dFirstChild = nullptr, *dCellnumber = nullptr, *dNbrOffset = nullptr, *dNbrList = nullptr;
    // media
    int ncomp = 0, nlambda = 0;
    double *dRho = nullptr, *dOptics = nullptr;
    // sources
    int nstar = 0;
    int* dGeomKind = nullptr;
    double *dGeomParam = nullptr, *dLum = nullptr, *dLumtot = nullptr, *dCdf = nullptr;
    double emissionBias = 0.5;
    // instruments
    std::vector<DevInstr> instr;
    DevInstr* dInstr = nullptr;
    size_t nInstrTally = 0;
    int nsed = 0;
    // tallies
    double *dLabs = nullptr, *dTally = nullptr;
    bool ownLabs = true, ownTally = true;
    unsigned long long *dCounter = nullptr, *dStats = nullptr;
    unsigned int* dError = nullptr;
    // config
    int block = kBlock, grid = 0, threshold = 16;
    double lastMs = 0;
    size_t maxLds = 0;
    int numCUs = 0;
};

namespace {

int fail(SkirtMcrt* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHECK(ctx, call)                                                                    \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess) return fail(ctx, SKIRT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class T>
int upload(SkirtMcrt* c, T*& dst, const T* src, size_t n) {
    if (dst) { (void)hipFree(dst); dst = nullptr; }
    if (n == 0) return SKIRT_OK;
    if (!src) return fail(c, SKIRT_ERR_ARG, "null host array");
    HIPCHECK(c, hipMalloc(&dst, n * sizeof(T)));
    HIPCHECK(c, hipMemcpy(dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    return SKIRT_OK;
}

}  // namespace

extern "C" {

int skirt_mcrt_abi_version(void) { return SKIRT_MCRT_ABI_VERSION; }

int skirt_mcrt_create(int device, SkirtMcrt** out) {
    if (!out) return SKIRT_ERR_ARG;
    *out = nullptr;
    auto* c = new SkirtMcrt();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc(&c->dCounter, sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->dStats, 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->dError, sizeof(unsigned int)) != hipSuccess) {
        delete c;
        return SKIRT_ERR_HIP;
    }
    c->stream = c->own;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
        c->maxLds = prop.sharedMemPerBlock;
        c->numCUs = prop.multiProcessorCount;
    }
    (void)hipMemset(c->dStats, 0, 8 * sizeof(unsigned long long));
    (void)hipMemset(c->dError, 0, sizeof(unsigned int));
    *out = c;
    return SKIRT_OK;
}

int skirt_mcrt_set_stream(SkirtMcrt* c, void* s) {
    if (!c) return SKIRT_ERR_ARG;
    c->stream = s ? (hipStream_t)s : c->own;
    return SKIRT_OK;
}

int skirt_mcrt_configure(SkirtMcrt* c, int block, int grid, int threshold) {
    if (!c) return SKIRT_ERR_ARG;
    if (block) {
        if (block != kBlock) return fail(c, SKIRT_ERR_ARG, "only 256-thread blocks are compiled");
    }
    c->grid = grid;
    if (threshold) c->threshold = std::max(1, std::min(64, threshold));
    return SKIRT_OK;
}

int skirt_mcrt_upload_grid(SkirtMcrt* c, const SkirtGridDesc* g) {
    if (!c || !g) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    c->ncells = g->ncells;
    if (g->kind == SKIRT_GRID_CARTESIAN) {
        if (g->nx < 1 || g->ny < 1 || g->nz < 1 || !g->xv || !g->yv || !g->zv) return fail(c, SKIRT_ERR_ARG, "bad Cartesian grid");
        if ((long long)g->nx * g->ny * g->nz != g->ncells) return fail(c, SKIRT_ERR_ARG, "ncells != nx*ny*nz");
        std::vector<double> mesh;
        mesh.insert(mesh.end(), g->xv, g->xv + g->nx + 1);
        mesh.insert(mesh.end(), g->yv, g->yv + g->ny + 1);
        mesh.insert(mesh.end(), g->zv, g->zv + g->nz + 1);
        for (int i = 0; i < g->nx; i++) if (!(g->xv[i] < g->xv[i + 1])) return fail(c, SKIRT_ERR_ARG, "x mesh not increasing");
        for (int i = 0; i < g->ny; i++) if (!(g->yv[i] < g->yv[i + 1])) return fail(c, SKIRT_ERR_ARG, "y mesh not increasing");
        for (int i = 0; i < g->nz; i++) if (!(g->zv[i] < g->zv[i + 1])) return fail(c, SKIRT_ERR_ARG, "z mesh not increasing");
        c->nx = g->nx; c->ny = g->ny; c->nz = g->nz;
        c->gx0 = g->xv[0]; c->gx1 = g->xv[g->nx];
        c->gy0 = g->yv[0]; c->gy1 = g->yv[g->ny];
        c->gz0 = g->zv[0]; c->gz1 = g->zv[g->nz];
        int rc = upload(c, c->dMesh, mesh.data(), mesh.size());
        if (rc) return rc;
    } else if (g->kind == SKIRT_GRID_OCTREE) {
        if (g->nnodes < 1 || !g->box || !g->first_child || !g->cellnumber || !g->nbr_offset)
            return fail(c, SKIRT_ERR_ARG, "bad octree grid");
        // validate the index arrays so that the kernel never reads out of bounds
        int nleaf = 0;
        for (int l = 0; l < g->nnodes; l++) {
            int fc = g->first_child[l];
            if (fc >= 0 && (fc + 8 > g->nnodes || fc <= l)) return fail(c, SKIRT_ERR_ARG, "octree child index out of range");
            if (fc < 0) {
                if (g->cellnumber[l] < 0 || g->cellnumber[l] >= g->ncells) return fail(c, SKIRT_ERR_ARG, "octree cell number out of range");
                nleaf++;
            }
        }
        if (nleaf != g->ncells) return fail(c, SKIRT_ERR_ARG, "octree leaf count != ncells");
        int nnbr = g->nbr_offset[6 * (size_t)g->nnodes];
        for (size_t q = 0; q < 6 * (size_t)g->nnodes; q++)
            if (g->nbr_offset[q] < 0 || g->nbr_offset[q] > g->nbr_offset[q + 1]) return fail(c, SKIRT_ERR_ARG, "bad neighbor offsets");
        for (int q = 0; q < nnbr; q++)
            if (g->nbr_list[q] < 0 || g->nbr_list[q] >= g->nnodes) return fail(c, SKIRT_ERR_ARG, "neighbor index out of range");
        c->nnodes = g->nnodes;
        c->eps = g->eps;
        c->search = g->search;
        c->gx0 = g->box[0]; c->gy0 = g->box[1]; c->gz0 = g->box[2];
        c->gx1 = g->box[3]; c->gy1 = g->box[4]; c->gz1 = g->box[5];
        int rc;
        if ((rc = upload(c, c->dBox, g->box, 6 * (size_t)g->nnodes))) return rc;
        if ((rc = upload(c, c->dFirstChild, g->first_child, (size_t)g->nnodes))) return rc;
        if ((rc = upload(c, c->dCellnumber, g->cellnumber, (size_t)g->nnodes))) return rc;
        if ((rc = upload(c, c->dNbrOffset, g->nbr_offset, 6 * (size_t)g->nnodes + 1))) return rc;
        std::vector<int> dummy(1, 0);
        if ((rc = upload(c, c->dNbrList, nnbr ? g->nbr_list : dummy.data(), nnbr ? (size_t)nnbr : 1))) return rc;
    } else {
        return fail(c, SKIRT_ERR_UNSUPPORTED, "unsupported grid kind");
    }
    c->gridKind = g->kind;
    return SKIRT_OK;
}

int skirt_mcrt_upload_media(SkirtMcrt* c, const SkirtMediaDesc* m) {
    if (!c || !m) return SKIRT_ERR_ARG;
    if (c->gridKind < 0) return fail(c, SKIRT_ERR_STATE, "upload the grid before the media");
    if (m->ncells != c->ncells || m->ncomp < 1 || m->ncomp > 8 || m->nlambda < 1)
        return fail(c, SKIRT_ERR_ARG, "media sizes do not match the grid (1 <= ncomp <= 8)");
    HIPCHECK(c, hipSetDevice(c->device));
    c->ncomp = m->ncomp;
    c->nlambda = m->nlambda;
    size_t nt = (size_t)m->ncomp * m->nlambda;
    std::vector<double> opt(4 * nt);
    std::memcpy(opt.data(), m->kext, nt * sizeof(double));
    std::memcpy(opt.data() + nt, m->ksca, nt * sizeof(double));
    std::memcpy(opt.data() + 2 * nt, m->albedo, nt * sizeof(double));
    std::memcpy(opt.data() + 3 * nt, m->g, nt * sizeof(double));
    int rc;
    if ((rc = upload(c, c->dRho, m->rho, (size_t)m->ncells * m->ncomp))) return rc;
    if ((rc = upload(c, c->dOptics, opt.data(), opt.size()))) return rc;
    return SKIRT_OK;
}

int skirt_mcrt_upload_sources(SkirtMcrt* c, const SkirtSourceDesc* s) {
    if (!c || !s) return SKIRT_ERR_ARG;
    if (s->ncomp < 1 || s->nlambda < 1) return fail(c, SKIRT_ERR_ARG, "bad source sizes");
    for (int h = 0; h < s->ncomp; h++)
        if (s->geom_kind[h] != SKIRT_GEOM_PLUMMER) return fail(c, SKIRT_ERR_UNSUPPORTED, "unsupported source geometry");
    HIPCHECK(c, hipSetDevice(c->device));
    c->nstar = s->ncomp;
    c->emissionBias = s->emission_bias;
    if (c->nlambda && c->nlambda != s->nlambda) return fail(c, SKIRT_ERR_ARG, "sources and media disagree on nlambda");
    c->nlambda = s->nlambda;
    int rc;
    if ((rc = upload(c, c->dGeomKind, s->geom_kind, (size_t)s->ncomp))) return rc;
    if ((rc = upload(c, c->dGeomParam, s->geom_param, 4 * (size_t)s->ncomp))) return rc;
    if ((rc = upload(c, c->dLum, s->lum, (size_t)s->ncomp * s->nlambda))) return rc;
    if ((rc = upload(c, c->dLumtot, s->lumtot, (size_t)s->nlambda))) return rc;
    if ((rc = upload(c, c->dCdf, s->cdf, (size_t)s->nlambda * (s->ncomp + 1)))) return rc;
    return SKIRT_OK;
}

int skirt_mcrt_set_instruments(SkirtMcrt* c, const SkirtInstrDesc* in, int n) {
    if (!c || n < 0 || (n > 0 && !in)) return SKIRT_ERR_ARG;
    if (c->nlambda < 1) return fail(c, SKIRT_ERR_STATE, "upload sources or media before instruments");
    HIPCHECK(c, hipSetDevice(c->device));
    c->instr.clear();
    long long off = 0;
    int sedOff = 0;
    for (int i = 0; i < n; i++) {
        DevInstr d{};
        d.kind = in[i].kind;
        if (d.kind < SKIRT_INSTR_FULL || d.kind > SKIRT_INSTR_FRAME) return fail(c, SKIRT_ERR_ARG, "bad instrument kind");
        d.nx = in[i].nx;
        d.ny = in[i].ny;
        if (d.kind != SKIRT_INSTR_SED && (d.nx < 1 || d.ny < 1)) return fail(c, SKIRT_ERR_ARG, "bad instrument frame size");
        if (d.kind == SKIRT_INSTR_SED) { d.nx = 0; d.ny = 0; }
        d.levels = d.kind == SKIRT_INSTR_FULL ? in[i].scattering_levels : 0;
        d.nslots = d.kind == SKIRT_INSTR_FULL ? 5 + d.levels : 1;
        for (int q = 0; q < 3; q++) d.kobs[q] = in[i].kobs[q];
        d.sinphi = in[i].sinphi; d.cosphi = in[i].cosphi; d.sintheta = in[i].sintheta; d.costheta = in[i].costheta;
        d.sinpa = in[i].sinpa; d.cospa = in[i].cospa;
        d.xpmin = in[i].xpmin; d.xpsiz = in[i].xpsiz; d.ypmin = in[i].ypmin; d.ypsiz = in[i].ypsiz;
        d.frameBase = off;
        long long nframes = (d.kind == SKIRT_INSTR_SED) ? 0 : (long long)d.nslots * c->nlambda * d.nx * d.ny;
        off += nframes;
        d.sedBase = off;
        long long nseds = (d.kind == SKIRT_INSTR_FRAME) ? 0 : (long long)d.nslots * c->nlambda;
        off += nseds;
        d.sedOff = sedOff;
        sedOff += (int)nseds;
        c->instr.push_back(d);
    }
    c->nInstrTally = (size_t)off;
    c->nsed = sedOff;
    int rc = upload(c, c->dInstr, c->instr.data(), c->instr.size());
    if (rc) return rc;
    // (re)allocate owned tallies lazily at run time
    if (c->ownTally && c->dTally) { (void)hipFree(c->dTally); c->dTally = nullptr; }
    return SKIRT_OK;
}

int skirt_mcrt_tally_sizes(SkirtMcrt* c, size_t* nl, size_t* ni) {
    if (!c) return SKIRT_ERR_ARG;
    if (nl) *nl = (size_t)c->ncells * c->nlambda;
    if (ni) *ni = c->nInstrTally;
    return SKIRT_OK;
}

static int ensureTallies(SkirtMcrt* c) {
    size_t nl = (size_t)c->ncells * c->nlambda;
    if (!c->dLabs && nl) {
        HIPCHECK(c, hipMalloc(&c->dLabs, nl * sizeof(double)));
        HIPCHECK(c, hipMemsetAsync(c->dLabs, 0, nl * sizeof(double), c->stream));
        c->ownLabs = true;
    }
    if (!c->dTally && c->nInstrTally) {
        HIPCHECK(c, hipMalloc(&c->dTally, c->nInstrTally * sizeof(double)));
        HIPCHECK(c, hipMemsetAsync(c->dTally, 0, c->nInstrTally * sizeof(double), c->stream));
        c->ownTally = true;
    }
    return SKIRT_OK;
}

int skirt_mcrt_bind_tallies(SkirtMcrt* c, double* dl, double* di) {
    if (!c) return SKIRT_ERR_ARG;
    if (dl) {
        if (c->ownLabs && c->dLabs) (void)hipFree(c->dLabs);
        c->dLabs = dl;
        c->ownLabs = false;
    }
    if (di) {
        if (c->ownTally && c->dTally) (void)hipFree(c->dTally);
        c->dTally = di;
        c->ownTally = false;
    }
    return SKIRT_OK;
}

int skirt_mcrt_zero_tallies(SkirtMcrt* c) {
    if (!c) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    int rc = ensureTallies(c);
    if (rc) return rc;
    size_t nl = (size_t)c->ncells * c->nlambda;
    if (c->dLabs && nl) HIPCHECK(c, hipMemsetAsync(c->dLabs, 0, nl * sizeof(double), c->stream));
    if (c->dTally && c->nInstrTally) HIPCHECK(c, hipMemsetAsync(c->dTally, 0, c->nInstrTally * sizeof(double), c->stream));
    HIPCHECK(c, hipMemsetAsync(c->dStats, 0, 8 * sizeof(unsigned long long), c->stream));
    HIPCHECK(c, hipMemsetAsync(c->dError, 0, sizeof(unsigned int), c->stream));
    return SKIRT_OK;
}

int skirt_mcrt_run_stellar(SkirtMcrt* c, uint64_t npp, uint64_t first, uint64_t count, uint64_t seed,
                           const SkirtPhaseParams* p) {
    if (!c || !p) return SKIRT_ERR_ARG;
    if (c->gridKind < 0 && p->has_dust) return fail(c, SKIRT_ERR_STATE, "no grid uploaded");
    if (!c->dLumtot) return fail(c, SKIRT_ERR_STATE, "no sources uploaded");
    if (p->has_dust && !c->dRho) return fail(c, SKIRT_ERR_STATE, "no media uploaded");
    if (npp == 0) return fail(c, SKIRT_ERR_ARG, "npp must be positive");
    if (first + count > npp * (uint64_t)c->nlambda) return fail(c, SKIRT_ERR_ARG, "packet range exceeds npp*nlambda");
    if (p->min_weight_reduction <= 0 || p->scatt_bias < 0 || p->scatt_bias > 1) return fail(c, SKIRT_ERR_ARG, "bad phase parameters");
    HIPCHECK(c, hipSetDevice(c->device));
    int rc = ensureTallies(c);
    if (rc) return rc;
    if (count == 0) { c->lastMs = 0; return SKIRT_OK; }

    Args a{};
    a.ncells = c->ncells;
    a.nx = c->nx; a.ny = c->ny; a.nz = c->nz;
    a.xv = c->dMesh;
    a.gx0 = c->gx0; a.gx1 = c->gx1; a.gy0 = c->gy0; a.gy1 = c->gy1; a.gz0 = c->gz0; a.gz1 = c->gz1;
    a.box = c->dBox; a.firstChild = c->dFirstChild; a.cellnumber = c->dCellnumber;
    a.nbrOffset = c->dNbrOffset; a.nbrList = c->dNbrList; a.eps = c->eps; a.search = c->search;
    a.ncomp = std::max(1, c->ncomp); a.nlambda = c->nlambda;
    a.rho = c->dRho;
    // a dust-free simulation still needs (zero) optical tables for the LDS staging
    if (!c->dOptics) {
        std::vector<double> z(4 * (size_t)c->nlambda, 0.0);
        if ((rc = upload(c, c->dOptics, z.data(), z.size()))) return rc;
    }
    a.optics = c->dOptics;
    a.nstar = c->nstar; a.geomKind = c->dGeomKind; a.geomParam = c->dGeomParam; a.lum = c->dLum;
    a.lumtot = c->dLumtot; a.cdf = c->dCdf; a.emissionBias = c->emissionBias;
    a.ninstr = (int)c->instr.size(); a.instr = c->dInstr; a.nsed = c->nsed;
    a.npp = npp; a.first = first; a.end = first + count; a.seed = seed; a.tag = SKIRT_PHASE_STELLAR;
    a.minWeightReduction = p->min_weight_reduction; a.minScatt = p->min_scatt_events; a.xi = p->scatt_bias;
    a.store = p->store_absorption ? 1 : 0;
    a.hasDust = p->has_dust ? 1 : 0;
    if (a.store && !c->dLabs) return fail(c, SKIRT_ERR_STATE, "no Labs buffer");
    a.labs = c->dLabs; a.tally = c->dTally;
    a.counter = c->dCounter; a.error = c->dError; a.stats = c->dStats;
    a.threshold = c->threshold;
    // LDS layout (doubles)
    int off = 0;
    a.ldsMeshOff = off;
    off += (c->gridKind == SKIRT_GRID_CARTESIAN) ? (c->nx + c->ny + c->nz + 3) : 0;
    off = (off + 1) & ~1;
    a.ldsOptOff = off;
    off += 4 * a.ncomp * a.nlambda;
    off = (off + 1) & ~1;
    a.ldsInstrOff = off;
    off += a.ninstr * (int)(sizeof(DevInstr) / sizeof(double));
    a.ldsSedOff = off;
    off += c->nsed;
    size_t lds = (size_t)off * sizeof(double);
    if (lds > 160 * 1024) return fail(c, SKIRT_ERR_UNSUPPORTED, "tables do not fit in LDS (" + std::to_string(lds) + " bytes)");

    HIPCHECK(c, hipMemsetAsync(c->dCounter, 0, sizeof(unsigned long long), c->stream));
    int grid = c->grid;
    if (grid <= 0) {
        int per = 0;
        auto kfn = (c->gridKind == SKIRT_GRID_OCTREE)
                       ? (a.ncomp == 1 ? (const void*)stellarKernel<SKIRT_GRID_OCTREE, true> : (const void*)stellarKernel<SKIRT_GRID_OCTREE, false>)
                       : (a.ncomp == 1 ? (const void*)stellarKernel<SKIRT_GRID_CARTESIAN, true> : (const void*)stellarKernel<SKIRT_GRID_CARTESIAN, false>);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kfn, kBlock, lds) != hipSuccess || per < 1) per = 4;
        grid = std::max(1, c->numCUs) * per;
        // never more lanes than packets (each lane claims at least one packet)
        unsigned long long maxBlocks = (count + kBlock - 1) / kBlock;
        if ((unsigned long long)grid > maxBlocks) grid = (int)maxBlocks;
    }
    HIPCHECK(c, hipEventRecord(c->ev0, c->stream));
    int gk = (c->gridKind == SKIRT_GRID_OCTREE) ? SKIRT_GRID_OCTREE : SKIRT_GRID_CARTESIAN;
    if (gk == SKIRT_GRID_OCTREE) {
        if (a.ncomp == 1) hipLaunchKernelGGL((stellarKernel<SKIRT_GRID_OCTREE, true>), dim3(grid), dim3(kBlock), lds, c->stream, a);
        else hipLaunchKernelGGL((stellarKernel<SKIRT_GRID_OCTREE, false>), dim3(grid), dim3(kBlock), lds, c->stream, a);
    } else {
        if (a.ncomp == 1) hipLaunchKernelGGL((stellarKernel<SKIRT_GRID_CARTESIAN, true>), dim3(grid), dim3(kBlock), lds, c->stream, a);
        else hipLaunchKernelGGL((stellarKernel<SKIRT_GRID_CARTESIAN, false>), dim3(grid), dim3(kBlock), lds, c->stream, a);
    }
    HIPCHECK(c, hipGetLastError());
    HIPCHECK(c, hipEventRecord(c->ev1, c->stream));
    return SKIRT_OK;
}

int skirt_mcrt_synchronize(SkirtMcrt* c) {
    if (!c) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) c->lastMs = ms;
    unsigned int e = 0;
    HIPCHECK(c, hipMemcpy(&e, c->dError, sizeof e, hipMemcpyDeviceToHost));
    if (e) return fail(c, SKIRT_ERR_NUMERIC, "the optical depth along the path is not a positive number");
    return SKIRT_OK;
}

int skirt_mcrt_download(SkirtMcrt* c, double* labs, double* instr) {
    if (!c) return SKIRT_ERR_ARG;
    int rc = skirt_mcrt_synchronize(c);
    if (rc) return rc;
    size_t nl = (size_t)c->ncells * c->nlambda;
    if (labs && nl) {
        if (!c->dLabs) return fail(c, SKIRT_ERR_STATE, "no Labs buffer");
        std::vector<double> t(nl);
        HIPCHECK(c, hipMemcpy(t.data(), c->dLabs, nl * sizeof(double), hipMemcpyDeviceToHost));
        for (int ell = 0; ell < c->nlambda; ell++)
            for (int m = 0; m < c->ncells; m++) labs[(size_t)m * c->nlambda + ell] = t[(size_t)ell * c->ncells + m];
    }
    if (instr && c->nInstrTally) {
        if (!c->dTally) return fail(c, SKIRT_ERR_STATE, "no instrument buffer");
        HIPCHECK(c, hipMemcpy(instr, c->dTally, c->nInstrTally * sizeof(double), hipMemcpyDeviceToHost));
    }
    return SKIRT_OK;
}

int skirt_mcrt_stats(SkirtMcrt* c, SkirtStats* out) {
    if (!c || !out) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    unsigned long long v[8];
    HIPCHECK(c, hipMemcpy(v, c->dStats, sizeof v, hipMemcpyDeviceToHost));
    out->packets = v[0];
    out->segments_fill = v[1];
    out->segments_walk = v[2];
    out->segments_peel = v[3];
    out->detects = v[4];
    out->absorb_adds = v[5];
    out->kernel_ms = c->lastMs;
    return SKIRT_OK;
}

const char* skirt_mcrt_last_error(SkirtMcrt* c) { return c ? c->err.c_str() : "null context"; }

void skirt_mcrt_destroy(SkirtMcrt* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->dMesh, c->dBox, c->dFirstChild, c->dCellnumber, c->dNbrOffset, c->dNbrList, c->dRho,
                    c->dOptics, c->dGeomKind, c->dGeomParam, c->dLum, c->dLumtot, c->dCdf, c->dInstr,
                    c->dCounter, c->dStats, c->dError};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (c->ownLabs && c->dLabs) (void)hipFree(c->dLabs);
    if (c->ownTally && c->dTally) (void)hipFree(c->dTally);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

}  // extern "C"
