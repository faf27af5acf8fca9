// MI355X photon-packet engine: HIP kernels for gfx950 + the C ABI of include/skirt_mcrt.h.
//
// A photon phase (MonteCarloSimulation::dostellaremissionchunk, MonteCarloSimulation.cpp:265-301)
// runs as a wavefront pipeline over a pool of packet slots resident in HBM:
//
//   eventKernel  one thread per active slot: consumes the result of the slot's last ray and runs the
//                packet's event code in the reference's order -- launch (StellarSystem::launch),
//                escape/absorption bookkeeping and termination (simulateescapeandabsorption),
//                interaction sampling (simulatepropagation), propagation, peel-off weights
//                (peeloffscattering) and scattering (simulatescattering) -- then queues the packet's
//                next rays: its next FILL or WALK ray plus one PEEL ray per instrument. A finished
//                slot claims the next global packet index at once.
//   traceKernel  persistent: every lane pulls rays from the queue (one atomic per wave, ballot +
//                mbcnt) and walks them through the dust grid, one uniform loop body for all lanes:
//     FILL  DustSystem::fillOpticalDepth + the absorption of simulateescapeandabsorption fused in one
//           streaming pass (segment n needs only exp(-tau_{n-1}) and dtau_n,
//           MonteCarloSimulation.cpp:447-470), f64 atomics into Labs; result: tau of the path;
//     WALK  the same path again up to the sampled optical depth, interpolating inside the crossing
//           segment like DustGridPath::pathlength (DustGridPath.cpp:162-173); result: the distance;
//     PEEL  optical depth to the grid edge towards an instrument (DustSystem::opticaldepth), then
//           Instrument::detect into LDS-privatized SED sums and f64 frame atomics.
// Peel-off detections only add to tallies, so they run concurrently with the packet's next FILL ray;
// the random-number sequence of every packet is exactly the reference's. The trace kernel holds only
// the ray in registers (the heavy event code lives in the other kernel), which keeps its occupancy
// high enough to hide the latency of the density / tree gathers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "vor_terms.hpp"
#include "../../../include/skirt_mcrt.h"
#include "philox.hpp"

using skirt_dev::PacketRng;

namespace {

constexpr double kDblMax = 1.7976931348623157e308;
constexpr int kBlock = 256;
constexpr int kSegWords = 3 * (kBlock / 64) * 4 / 8;  // the trace kernel's per-wave segment counts, in doubles
#ifndef SKIRT_LABS_BUF
#define SKIRT_LABS_BUF 16
#endif
constexpr int kLabsBuf = SKIRT_LABS_BUF;  // buffered Labs adds per trace lane (LDS)
#ifndef SKIRT_VOR_DRAIN2
#define SKIRT_VOR_DRAIN2 1
#endif
constexpr int kStepsPerPull = 4;  // grid steps between two ray pulls of a trace wave
// The slot pool runs as one or two independent pipelines ("halves", SkirtMcrt::halves): with two, one
// half's event and detect kernels run beside the other half's trace kernel, on CUs of their own (CU-masked
// streams, see runPhase).
constexpr int kMaxHalves = 2;
// device counters per pipeline half (Args::ctr): 16, each on a 128-byte line of its own (kCtrStride words
// apart). The event kernel's block reservations add to four of them every round; packed in one line, those
// atomics serialized on it: C3 +2.1 %, C2 +6.9 %, C4 +0.5 % apart (profiles/r05_ctr_lines_ab.txt)
constexpr int kCtrStride = 32;
constexpr int kCtrWords = 16 * kCtrStride;
#define CTR(base, k) ((base)[(k) * kCtrStride])
#define CTRP(base, k) ((base) + (k) * kCtrStride)
constexpr int kSersicTable = 202;  // SersicFunction: 101 radii, then 101 cumulative masses
constexpr int kDetectCopies = 8;   // most LDS copies of the SED sums in the detect kernel (one per 8 lanes)
constexpr int kPollEvery = 1;      // iterations between two counter copies of a half
constexpr int kPollRing = 3;       // copies in flight per half (the host reads each kPollRing copies late)
// occupancy of the trace kernel: 3 waves per SIMD, i.e. at most 168 VGPRs (the grid entry on the pull
// path would otherwise take the octree kernel to 175 and 2 waves; C3 1.91e8 -> 2.15e8 pkt/s at 3). The
// Voronoi walk has its own kernel and attribute below.
#ifndef SKIRT_TRACE_WAVES  // (variant builds: tools/build_variant.sh TAG -DSKIRT_TRACE_WAVES=4)
#define SKIRT_TRACE_WAVES 3
#endif
#define SKIRT_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(SKIRT_TRACE_WAVES)))
#define SKIRT_NOSTORE_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(4)))
// the Voronoi trace kernel at 2 waves per SIMD: its branch-free bounds keep several entries in flight
// and run without spills in 256 VGPRs (C4 5.72e7 pkt/s at 3 waves, 6.08e7 at 2)
#ifndef SKIRT_VOR_TRACE_WAVES  // (variant builds)
#define SKIRT_VOR_TRACE_WAVES 2
#endif
#define SKIRT_VOR_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(SKIRT_VOR_TRACE_WAVES)))
// the event kernel at 2 waves per SIMD: the Voronoi instantiation (cellIndex on the grid entry of every
// queued ray) would otherwise take 256 VGPRs + AGPRs and run at 1
#ifndef SKIRT_EVENT_WAVES  // (variant builds)
#define SKIRT_EVENT_WAVES 2
#endif
#define SKIRT_EVENT_ATTR __attribute__((amdgpu_waves_per_eu(SKIRT_EVENT_WAVES)))

// ------------------------------------------------------------------ descriptors
struct DevInstr {
    int kind, nx, ny, nslots, levels, sedOff;  // sedOff: offset of this instrument's SEDs in the LDS sums
    int slotStride, pad;                        // frames: slots per pixel, padded (see frameAt)
    long long frameBase;                        // offset of the frames in the global instrument tally
    long long sedBase;                          // offset of the SEDs in the global instrument tally
    double kobs[3];
    double sinphi, cosphi, sintheta, costheta, sinpa, cospa;
    double xpmin, xpsiz, ypmin, ypsiz;
};

enum RayMode : unsigned { RAY_NONE = 0, RAY_PEEL = 1, RAY_FILL = 2, RAY_WALK = 3 };
enum State : int { S_NEW = 0, S_FILL = 2, S_WALK = 3 };
// peel-off categories (which FullInstrument arrays a detection adds to, FullInstrument.cpp:115-171)
enum PeelCat : unsigned { CAT_STAR_DIRECT = 0, CAT_STAR_SCATTERED = 1, CAT_DUST_DIRECT = 2, CAT_DUST_SCATTERED = 3 };

// one queued ray, 80 bytes = 5 x 16-byte chunks, written by the event kernel. The trace kernel enters the
// grid when it pulls the ray (the path before the grid, the first cell): that lookup then overlaps with the
// other lanes' steps instead of stalling the event kernel, whose waves are few (2 per SIMD) and long.
// Voronoi rays are entered by the event kernel (kEnterInEvent): s0 then holds the path length before the
// grid, ci/cj the first cell. The reciprocal direction is recomputed by the trace kernel (three divisions
// per ray, against 24 bytes more per record written and read).
struct __attribute__((aligned(16))) RayRec {
    double x, y, z;        // c0-c1: start point
    double dx, dy, dz;     // c1-c2: direction
    double s0;             // c3: path length before the grid (Voronoi) or 0
    double param;          // c3: FILL: packet luminosity L; WALK: optical depth to reach; PEEL: peel-off L
    int idx;               // c4: FILL/WALK: slot; PEEL: detection record
    unsigned flags;        // c4: mode | cat << 2 | instrument << 4 | scattering level << 10 | ell << 18
    int ci, cj;            // c4: Voronoi: first cell and where its block starts
};
static_assert(sizeof(RayRec) == 80, "ray record layout");

// continuous scattering (MonteCarloSimulation::continuouspeeloffscattering): the dust segments of a FILL
// ray's path as DustGridPath holds them -- where the segment starts along the path (s, tau) and its
// lengths (ds, dtau) -- recorded by the trace kernel for the peel-off kernel, at most kPathCap per path
struct PathRec {
    double s0, ds, tau0, dtau;
    int m, pad;
};
constexpr int kPathCap = 2048;
constexpr int kContSlots = 1 << 15;  // packet slots in flight with continuous scattering (ray queue sizing)
enum ErrorBits : unsigned { ERR_TAU = 1u, ERR_PATH_CAP = 2u, ERR_QUEUE = 4u };
template <int GRID>
constexpr bool kEnterInEvent = GRID == SKIRT_GRID_VORONOI;
// Voronoi cellIndex: block-list candidates loaded per round trip. Round 3 chose 4; with the round-4
// registers 2 lets the Voronoi event kernel run 3 waves/SIMD (165 VGPRs): event 2.59 -> 2.26 ms, C4
// 1.0225e8 -> 1.0345e8 (8: 1.021e8), profiles/r04_cellindex_group.txt
constexpr int kCellIndexGroup = 2;  // Voronoi cellIndex: block-list candidates per load round
constexpr int kNoCell = -2;  // a cached cell index not known yet (-1 is a located point without a cell)
// a ray entered by the event kernel carries the number of its segments before the grid in the top bits
// of its first cell (Voronoi device cells < 2^28)
constexpr int kOutsideShift = 28;
constexpr int kCellMaskOut = (1 << kOutsideShift) - 1;
// most segments one Grid<GRID>::step adds (the Voronoi step may add a pending and a new segment)
template <int GRID>
constexpr int kSegsPerStep = GRID == SKIRT_GRID_VORONOI ? 2 : 1;

// the detection of one peel-off ray, in a compact array of its own (the detect kernel reads only these,
// contiguously, instead of scanning every ray record): written by the event kernel, tau by the trace
// kernel
struct __attribute__((aligned(16))) DetRec {
    double Lp;             // peel-off luminosity
    double tau;            // optical depth to the grid edge
    int l;                 // frame pixel (-1: none)
    unsigned flags;        // as the ray's flags
};
static_assert(sizeof(DetRec) == 24 || sizeof(DetRec) == 32, "detection record layout");
__device__ __forceinline__ unsigned rayMode(unsigned f) { return f & 3u; }
__device__ __forceinline__ unsigned rayCat(unsigned f) { return (f >> 2) & 3u; }
__device__ __forceinline__ int rayInstr(unsigned f) { return (int)((f >> 4) & 63u); }
__device__ __forceinline__ int rayLevel(unsigned f) { return (int)((f >> 10) & 255u); }
__device__ __forceinline__ int rayEll(unsigned f) { return (int)(f >> 18); }

struct LeafEntry;

// Voronoi cells on the device: per cell a block of 16-byte slots, contiguous, in device cell order: a
// 48-byte header {exact site x, y | z, rho of component 0 | device cell number, neighbour count, the
// bounds' error terms eA, eB (vor_terms.hpp)} followed by one 16-byte slot per neighbour, in the reference's
// list order: the neighbour's site relative to the cell's site, scaled by Args::vorScale and rounded to
// float (an approximate bisector plane), and where the neighbour's block starts (walls: -1 xmin .. -6
// zmax). The entries are stored in pairs, component-interleaved: slots {ox0, ox1, oy0, oy1} and {oz0, oz1,
// next0, next1}, so that the two 16-byte loads of a pair hand the packed (v_pk_*) arithmetic its operand
// pairs directly; a list of odd length ends in an unused half pair. A step bounds every plane distance from
// the float offsets, and evaluates the reference's exact expression only for the winner (from the winner's
// header, which is the next step's first load) or, when the bounds cannot single one out, for every
// possible winner.
// one entry of a Voronoi block list (Box::cellindices): the device cell and its exact site, so that cellIndex
// reads a candidate in one round trip (two 16-byte loads) instead of the list entry, then the site
struct alignas(16) BlockSite {
    double x, y, z;
    int id, pad;
};
static_assert(sizeof(BlockSite) == 32, "block site layout");

struct alignas(16) VorEntry {
    float ox, oy, oz;
    int next;
};
constexpr int kVorHead = 3;  // header slots

// entry q of the list of the cell whose block starts at B
__device__ __forceinline__ VorEntry vorEntry(const VorEntry* B, int q) {
    const float* P = reinterpret_cast<const float*>(B + kVorHead + (q & ~1));
    const int h = q & 1;
    return VorEntry{P[h], P[2 + h], P[4 + h], __float_as_int(P[6 + h])};
}

// entries q0 .. q0 + N - 1 (q0 even), two 16-byte loads per pair
template <int N>
__device__ __forceinline__ void vorEntries(const VorEntry* B, int q0, VorEntry (&e)[N]) {
#pragma unroll
    for (int p = 0; p < N / 2; p++) {
        const float4 x = *reinterpret_cast<const float4*>(B + kVorHead + q0 + 2 * p);
        const int4 y = *reinterpret_cast<const int4*>(B + kVorHead + q0 + 2 * p + 1);
        e[2 * p] = VorEntry{x.x, x.z, __int_as_float(y.x), y.z};
        e[2 * p + 1] = VorEntry{x.y, x.w, __int_as_float(y.y), y.w};
    }
}
// Voronoi walk: entries per load group, even (pairs); with exp(-tau) per FILL segment 4 is best (C4 7.30e7;
// 6: 7.26e7 with 28 B/lane spilled; one group of 8: 7.25e7; profiles/r03_vor_pipe.txt, r03_exact_attenuation.txt)
// FILL segments: exp(-tau) carried as a product while the segments' optical depths stay below this
constexpr double kCarryTau = 0.5;
#ifndef SKIRT_POLY_EXPM1
#define SKIRT_POLY_EXPM1 1
#endif
// 1 - exp(-x) = -expm1(-x) for 0 <= x < kCarryTau (the FILL segments' absorbed fraction,
// MonteCarloSimulation.cpp:458-462) as x + x^2 q(x), q a degree-9 polynomial fitted at Chebyshev nodes of
// [0, 0.5] (approximation error 0.04 ulp): within 1 ulp of glibc's expm1 over 2e7 arguments, as ocml's is,
// in 11 VALU operations and 18 register moves against ocml's ~53 (range reduction, ldexp, the constants'
// moves): C2, C4, C5 +0.4 %, C3 +0.1 % (the trace kernels are not VALU-bound; profiles/r06_poly_expm1_ab.txt)
__device__ __forceinline__ double oneMinusExpNeg(double x) {
    double q = 2.0367415268789147e-08;
    q = fma(q, x, -2.7077568604087168e-07);
    q = fma(q, x, 2.7529604741385112e-06);
    q = fma(q, x, -2.4800612392596861e-05);
    q = fma(q, x, 0.00019841248533674491);
    q = fma(q, x, -0.0013888888604734388);
    q = fma(q, x, 0.0083333333311535578);
    q = fma(q, x, -0.04166666666658167);
    q = fma(q, x, 0.16666666666666538);
    q = fma(q, x, -0.5);
    return fma(x, x * q, x);
}
constexpr int kVorUnroll = 4;
// groups of entries in flight per step: loaded with the header, each reloaded once consumed. 3: C4 trace
// launch 23.64 -> 23.19 ms, 9.64e7 -> 9.89e7 pkt/s, profiles/r04_ktrace_groups_nolicm.txt; 4 with each
// cell's list padded to whole groups with NaN entries (no per-entry count check): 1.0155e8 -> 1.0243e8
// (profiles/r04_vor_groups4.txt). Measured and removed (git history): the neighbour-parallel drain step
// (profiles/r03_vor_wide.txt), the drain split around the step's loads (profiles/r04_c4_variants.txt).
#ifndef SKIRT_VOR_GROUPS
#define SKIRT_VOR_GROUPS 4
#endif
constexpr int kVorGroups = SKIRT_VOR_GROUPS;
constexpr int kVorFallbackGroup = 2;  // neighbour sites loaded together by the exact re-evaluation (<= kVorUnroll)
constexpr int kVorCand = 4;  // possible winners the exact re-evaluation collects before it takes the whole list
// slots after the last cell's block: a step loads whole groups of entries past its list
constexpr int kVorPad = (kVorGroups + 2) * kVorUnroll;

// grid kinds of the kernels: SKIRT_GRID_CARTESIAN, SKIRT_GRID_OCTREE (leaf-map walk), the k-d tree
// through its leaf map, and any tree walked through the node arrays (trees deeper than the leaf maps
// allow or not split at box centres, e.g. barycentric subdivision)
constexpr int kOctreeNodes = 16;
constexpr int kBinTreeMap = 17;
constexpr int kOctreeBookkeeping = 18;  // octree, Bookkeeping search (node arrays)

struct Args {
    // grid
    int nx, ny, nz, ncells;
    int brick;                   // Cartesian: device cells numbered in 2x2x2 bricks (see Grid<CARTESIAN>::dev)
    int labsStride;              // Labs row length (device cells, padded to a 64-byte line)
    const double* mesh;          // Cartesian borders x | y | z (staged in LDS)
    double gx0, gx1, gy0, gy1, gz0, gz1;
    const double* box;           // octree
    const int* firstChild;
    const signed char* splitDir;  // binary trees: split axis per node (null for octrees)
    const int* father;            // octree, Bookkeeping search: father of every node (-1 for the root)
    const int* cellnumber;
    const int* nbrOffset;
    const int* nbrList;
    double eps;
    int search;
    const double* site;          // Voronoi, device cell order: 3 per cell
    const int* vorStart;         // Voronoi: where each device cell's block of slots starts
    const VorEntry* vorSlots;    // Voronoi: headers and neighbour entries
    float vorScale;              // Voronoi: 1 / (largest half-width of the domain), the entries' offset unit
    const double* cellBbox;      // Voronoi: enclosing box per cell
    const int* devCell;          // reference cell -> device cell (Voronoi launches)
    int vnb;                     // Voronoi block grid: blocks per axis
    const int* blockOffset;
    const struct BlockSite* blockSites;  // Voronoi: the block lists, each entry with its cell's exact site
    const LeafEntry* leafMap;       // octree leaf map: Morton-ordered finest-level cells -> leaf
    const double* treeT;         // octree split coordinates per axis, 3 x (mapN + 1) (staged in LDS)
    int mapL, mapN;              // leaf map depth and 2^depth
    double mapInvX, mapInvY, mapInvZ;
    double mapX0, mapY0, mapZ0;  // T[0] of each axis (the root box's lower corner)
    // media
    int ncomp, nlambda;
    const double* rho;
    const double* optics;        // [4][ncomp][nlambda]: kext, ksca, albedo, g
    // sources
    int nstar;
    const double* geomParam;
    const double* geomTable;     // per component kSersicTable words: SersicFunction s_i, then M_i
    const double* lum;
    const double* lumtot;
    const double* cdf;
    double emissionBias;
    // dust-phase cell sources (PanMonteCarloSimulation.cpp:193-205, 273-294), reference cell order
    const double* cellLv;        // [nlambda][ncells]
    const double* cellCdf;       // [nlambda][ncells + 1]
    const int* cellGuide;        // [nlambda][ncells + 1]: the CDF index at k / ncells (cellGuideKernel)
    const double* cellLtot;      // [nlambda]
    double cellBias;             // PanDustSystem::emissionBias (dust emission phase)
    const int* cellNode;         // octree: the leaf node of every reference cell
    int phase, peel;             // SKIRT_PHASE_*; peel-off on
    // instruments
    int ninstr;
    const DevInstr* instr;
    int nsed;
    // phase
    unsigned long long npp, first, end, seed;
    // the per-wavelength slice [sliceLo, sliceLo + sliceCnt) of a sharded phase (sliceCnt == npp: the
    // whole phase); first/end index the slice's packets, wavelength-slowest (see globalPacket)
    unsigned long long sliceLo, sliceCnt;
    unsigned int tag;
    double minWeightReduction;
    int minScatt;
    double xi;
    int store, hasDust;
    // tallies
    double* labs;                // [nlambda][labsStride], device cell order
    unsigned labsBytes;          // its size (< 4 GiB: the trace kernel addresses it through a buffer descriptor)
    int labsGlobal;              // 1: a table of 4 GiB or more, added to with global atomics (no descriptor)
    int labsHi;                  // 1: a table of 2^32 elements or more (32 GiB): the buffered adds keep the
                                 //    element index's high bits in pendHi (implies labsGlobal)
    int labsCopies;              // > 1: `labs` holds that many replicas labsCopyStride bytes apart, wave w adding
    unsigned labsCopyStride;     //   into replica w % labsCopies (folded into the table at the phase end)
    double* tally;
    unsigned int* error;
    unsigned long long* stats;   // packets, seg_fill, seg_walk, seg_peel, detects, absorbs, lane slots
    // DustSystem's _crossed histogram (DustSystem.cpp:959-1000), or null: per FILL and PEEL path one count in
    // bin min(segments, crossedBins - 1), kCrossedCopies copies (by wave) against same-address contention
    unsigned long long* crossed;
    int crossedBins;
    // slot pool (structure of arrays) and queues
    int nslots;
    double *srx, *sry, *srz, *skx, *sky, *skz, *sL, *sLth;
    int *sell, *snscatt, *sstellar, *sstate;
    int* svcell;                 // Voronoi: the cell of the packet's position (cellIndex), kNoCell if not known
    uint32_t *splo, *sphi, *sblock, *sw2, *sw3, *shave;
    double *resA, *resB;         // per slot: FILL -> tau, Lsca | WALK -> distance
    RayRec* rays;
    DetRec* det;                 // detection records of the peel-off rays
    int* act[2];                 // active slot lists (double buffered)
    unsigned long long* claim;   // next packet index (relative to first)
    unsigned int* ctr;           // [0,1] ray counts, [2,3] active counts, [4] trace pull counter,
                                 // [5,6] detection record counts
    int parity, init, threshold;
    int walkBack;                // WALK rays queued from the top of the ray queue, so they are pulled last
    // continuous scattering: per slot the dust segments of its last FILL path and their number
    int continuous, rayCap;
    PathRec* pathBuf;            // [slot][kPathCap]
    int* pathCnt;
    int ldsMeshOff, ldsOptOff, ldsInstrOff, ldsSedOff;  // in doubles
    int detCopies;  // detect kernel: LDS copies of the SED sums (8, 4, 2, 1), 0 = SEDs straight to the tally
};

// One finest-level cell of the octree leaf map: the leaf node that covers it, that leaf's dust cell
// number and level, and the leaf's density of dust component 0 (the one-component kernels need no
// other gather per segment). 16 bytes, one global_load_dwordx4.
struct __attribute__((aligned(16))) LeafEntry {
    int node;
    unsigned cl;  // cell | level << 27
    double rho0;
};
constexpr int kLeafLevelShift = 27;
constexpr unsigned kLeafCellMask = (1u << kLeafLevelShift) - 1u;
constexpr int kMaxMapLevel = 9;  // 512^3 x 16 B = 2 GiB of HBM at most
// k-d tree leaf map entries: cl = cell | (shift x | shift y << 3 | shift z << 6) << kBinCellBits, the
// leaf's extent along each axis being 2^shift finest cells (binary trees split one axis at a time)
constexpr int kBinCellBits = 23;
constexpr unsigned kBinCellMask = (1u << kBinCellBits) - 1u;
constexpr int kMaxBinMapLevel = 7;

// Leaf map order of the finest-level cells of an N^3 map (N = 2^L): 2x2x2 bricks of 8 consecutive
// 16-byte entries (one 128-byte line), the bricks in (x, y, z) row-major order. Per line the same
// neighbourhood as Morton order, at a few integer operations instead of three bit spreads per step.
__host__ __device__ __forceinline__ unsigned leafBricks(int N) { return (unsigned)((N + 1) >> 1); }
__host__ __device__ __forceinline__ unsigned leafIndex(int N, unsigned x, unsigned y, unsigned z) {
    const unsigned nb = leafBricks(N);
    return ((((x >> 1) * nb + (y >> 1)) * nb + (z >> 1)) << 3) | ((x & 1u) << 2) | ((y & 1u) << 1) | (z & 1u);
}
__host__ __device__ __forceinline__ unsigned long long leafMapSize(int N) {
    const unsigned long long nb = leafBricks(N);
    return 8ull * nb * nb * nb;
}

// NR::interpolate_loglog (Fundamentals/NR.hpp:321-345): logarithmic in x, and in f when both f > 0
__device__ __forceinline__ double interpolateLogLog(double x, double x1, double x2, double f1, double f2) {
    x = log10(x);
    x1 = log10(x1);
    x2 = log10(x2);
    const bool logf = f1 > 0 && f2 > 0;
    if (logf) {
        f1 = log10(f1);
        f2 = log10(f2);
    }
    double fx = f1 + ((x - x1) / (x2 - x1)) * (f2 - f1);
    if (logf) fx = pow(10.0, fx);
    return fx;
}

__device__ __forceinline__ void atomicAddF64(double* p, double v) {
    // explicit global address space: global_atomic_add_f64 instead of a flat atomic
    __hip_atomic_fetch_add((__attribute__((address_space(1))) double*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The trace kernel's Labs drain as buffer atomics (buffer_atomic_add_f64 through a raw buffer descriptor of
// the Labs table): every lane of the drain instruction issues, the lanes without an add at an offset past
// the table, which the buffer range check drops (tools/buffer_atomic_oob.hip). A global atomic under
// `if (lane has an add)` is a branch the compiler's waitcnt pass cannot see through: the next load of the
// walk then waited with vmcnt(0), i.e. for the drain's atomics too, which stay counted for thousands of
// cycles under load (MI355X_MICROARCH.md, float atomic add row). With a fixed count of vector-memory
// operations per step the load that the previous step requested is waited for alone.
}  // namespace (the intrinsic's declaration has external linkage)
__device__ double bufferAtomicAddF64(double v, __amdgpu_buffer_rsrc_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.ptr.buffer.atomic.fadd.f64");
namespace {

// the small tables staged in LDS
struct Shared {
    const double* mesh;   // Cartesian: mesh borders | octree with leaf map: split coordinates
    const double* kext;   // [ncomp][nlambda]
    const double* ksca;
    const double* alb;
    const double* g;
    const DevInstr* instr;
    double* sed;
};

enum StageParts : int { STAGE_MESH = 1, STAGE_TREE = 2, STAGE_OPTICS = 4, STAGE_INSTR = 8 };

__device__ __forceinline__ Shared stageTables(const Args& a, double* lds, int parts) {
    Shared sh;
    double* m = lds + a.ldsMeshOff;
    double* opt = lds + a.ldsOptOff;
    double* idst = lds + a.ldsInstrOff;
    sh.mesh = m;
    sh.kext = opt;
    sh.ksca = opt + a.ncomp * a.nlambda;
    sh.alb = opt + 2 * a.ncomp * a.nlambda;
    sh.g = opt + 3 * a.ncomp * a.nlambda;
    sh.instr = reinterpret_cast<const DevInstr*>(idst);
    sh.sed = lds + a.ldsSedOff;
    const int nmesh = (parts & STAGE_MESH) ? (a.nx + a.ny + a.nz + 3) : 0;
    for (int q = threadIdx.x; q < nmesh; q += blockDim.x) m[q] = a.mesh[q];
    const int ntree = (parts & STAGE_TREE) ? 3 * (a.mapN + 1) : 0;
    for (int q = threadIdx.x; q < ntree; q += blockDim.x) m[q] = a.treeT[q];
    const int nopt = (parts & STAGE_OPTICS) ? 4 * a.ncomp * a.nlambda : 0;
    for (int q = threadIdx.x; q < nopt; q += blockDim.x) opt[q] = a.optics[q];
    const int ninw = (parts & STAGE_INSTR) ? a.ninstr * (int)(sizeof(DevInstr) / sizeof(double)) : 0;
    const double* isrc = reinterpret_cast<const double*>(a.instr);
    for (int q = threadIdx.x; q < ninw; q += blockDim.x) idst[q] = isrc[q];
    __syncthreads();
    return sh;
}

template <int GRID>
__device__ __forceinline__ constexpr int gridParts() {
    return GRID == SKIRT_GRID_CARTESIAN ? STAGE_MESH : ((GRID == SKIRT_GRID_OCTREE || GRID == kBinTreeMap) ? STAGE_TREE : 0);
}

// The counters live in kStatCopies copies of one 64-byte line each (summed by the host): the waves of a
// launch end together, and same-line atomics from all of them would queue on one L2 channel.
constexpr int kStatCopies = 64;
constexpr int kCrossedCopies = 64;
__device__ __forceinline__ void crossedAdd(const Args& a, unsigned n) {
    const unsigned wave = (blockIdx.x * (kBlock / 64) + threadIdx.x / 64) & (kCrossedCopies - 1);
    atomicAdd(a.crossed + (size_t)wave * a.crossedBins + min(n, (unsigned)a.crossedBins - 1u), 1ull);
}
__device__ __forceinline__ void flushStats(const Args& a, const unsigned long long (&vals)[8]) {
    const int lane = threadIdx.x & 63;
    unsigned long long* dst = a.stats + 8 * ((blockIdx.x * (kBlock / 64) + threadIdx.x / 64) & (kStatCopies - 1));
#pragma unroll
    for (int q = 0; q < 8; q++) {
        unsigned long long v = vals[q];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0 && v) atomicAdd(dst + q, v);
    }
}

// ------------------------------------------------------------------ the ray (trace kernel registers)
struct Ray {
    double x, y, z;        // current position along the ray
    double dx, dy, dz;     // direction
    double ix, iy, iz;     // 1/direction (0 where |k| <= 1e-15: that axis is never crossed)
    double tau, s;         // optical depth and path length covered so far
    double kext;           // kappa_ext at the ray's wavelength (one dust component)
    double param;          // see RayRec::param
    double f1, f2;         // FILL: exp(-tau), Lsca | WALK: tau and s at the previous segment end
    double bx0, by0, bz0, bx1, by1, bz1;  // octree walked through the node arrays: box of the node
    double rho0;           // density (component 0) of the current cell
    int ci, cj, ck;        // Cartesian cell indices | octree: node, cell number, leaf size in finest cells
    int jx, jy, jz;        // octree leaf map: finest-level index of the current leaf's lower corner
    int4 pre;              // octree leaf map: the next step's leaf-map entry, requested at the end of this step
    int pfx, pfy, pfz;     //   and the finest-level cell it was requested for (LeafMapGrid::prefetch)
    double ex, ey, ez, eds;  // octree leaf map: the current leaf's exit point and distance, and its wall,
    int ewall;               //   computed once by prefetch for the next step
    int idx, ell;
    unsigned flags, mode;
    unsigned id;           // queue index of the ray (a PEEL ray writes its optical depth back there)
};

// ------------------------------------------------------------------ grids
template <int GRID>
struct Grid;

// Cartesian grid: CartesianDustGrid.cpp:136-283 (mesh borders staged in LDS)
template <>
struct Grid<SKIRT_GRID_CARTESIAN> {
    __device__ static __forceinline__ int locateClip(const double* v, int n, double q) {  // NR::locate_clip
        if (q < v[0]) return 0;
        int jl = -1, ju = n - 1;
        while (ju - jl > 1) {
            const int jm = (ju + jl) >> 1;
            if (q < v[jm]) ju = jm;
            else jl = jm;
        }
        return jl;
    }
    __device__ static __forceinline__ int locateFail(const double* v, int n, double q) {  // NR::locate_fail
        if (q > v[n - 1]) return -1;
        int jl = -1, ju = n - 1;
        while (ju - jl > 1) {
            const int jm = (ju + jl) >> 1;
            if (q < v[jm]) ju = jm;
            else jl = jm;
        }
        return jl;
    }

    // the entry part of the path: up to three segments outside the grid (m = -1), then the first cell;
    // false for an empty path
    template <class SegFn>
    __device__ static __forceinline__ bool begin(const Args& a, const Shared& sh, Ray& r, SegFn seg) {
        const double* xv = sh.mesh;
        const double* yv = xv + a.nx + 1;
        const double* zv = yv + a.ny + 1;
        const double kx = r.dx, ky = r.dy, kz = r.dz;
        double x = r.x, y = r.y, z = r.z, d0 = 0, d1 = 0, d2 = 0;
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
        if (d0 > 0) seg(-1, 0.0, d0);
        if (d1 > 0) seg(-1, 0.0, d1);
        if (d2 > 0) seg(-1, 0.0, d2);
        r.x = x; r.y = y; r.z = z;
        r.ci = locateClip(xv, a.nx + 1, x);
        r.cj = locateClip(yv, a.ny + 1, y);
        r.ck = locateClip(zv, a.nz + 1, z);
        r.rho0 = a.rho[(size_t)dev(a, r.ci, r.cj, r.ck) * a.ncomp];
        return true;
    }

    // device number of cell (i, j, k). Bricked: the 8 cells of each 2x2x2 brick are consecutive and
    // start on a 64-byte line of every Labs row (a ray crosses about 2.5 cells of a brick it enters,
    // whose Labs adds then share one atomic request); bricks in the reference's (i, j, k) order.
    // Unbricked: the reference's index k + Nz j + Nz Ny i (CartesianDustGrid.cpp:305-308).
    __device__ static __forceinline__ int dev(const Args& a, int i, int j, int k) {
        if (!a.brick) return k + a.nz * j + a.nz * a.ny * i;
        const int by = (a.ny + 1) >> 1, bz = (a.nz + 1) >> 1;
        return ((((i >> 1) * by + (j >> 1)) * bz + (k >> 1)) << 3) | ((i & 1) << 2) | ((j & 1) << 1) | (k & 1);
    }

    // one grid step: emits (m, ds); false when the ray ends (left the grid or stopped by seg)
    template <class SegFn>
    __device__ static __forceinline__ bool step(const Args& a, const Shared& sh, Ray& r, SegFn seg) {
        const double* xv = sh.mesh;
        const double* yv = xv + a.nx + 1;
        const double* zv = yv + a.ny + 1;
        const int i = r.ci, j = r.cj, k = r.ck;
        const int m = dev(a, i, j, k);
        const double rho0 = r.rho0;  // loaded by the previous step (or begin), off this step's chain
        const double xE = (r.dx < 0.0) ? xv[i] : xv[i + 1];
        const double yE = (r.dy < 0.0) ? yv[j] : yv[j + 1];
        const double zE = (r.dz < 0.0) ? zv[k] : zv[k + 1];
        const double dsx = (r.ix != 0.0) ? (xE - r.x) * r.ix : kDblMax;
        const double dsy = (r.iy != 0.0) ? (yE - r.y) * r.iy : kDblMax;
        const double dsz = (r.iz != 0.0) ? (zE - r.z) * r.iz : kDblMax;
        // the exit wall (the reference's order of comparisons), then one segment: lanes leaving through
        // different walls share the segment code instead of running it once per wall
        const bool ex = dsx <= dsy && dsx <= dsz;
        const bool ey = !ex && dsy < dsx && dsy <= dsz;
        const bool ez = !ex && !ey && dsz < dsx && dsz < dsy;
        if (!(ex || ey || ez)) return false;  // NaN direction; the reference would loop forever
        const double ds = ex ? dsx : ey ? dsy : dsz;
        if (!seg(m, rho0, ds)) return false;
        const int ni = i + (ex ? ((r.dx < 0.0) ? -1 : 1) : 0);
        const int nj = j + (ey ? ((r.dy < 0.0) ? -1 : 1) : 0);
        const int nk = k + (ez ? ((r.dz < 0.0) ? -1 : 1) : 0);
        if (ni >= a.nx || ni < 0 || nj >= a.ny || nj < 0 || nk >= a.nz || nk < 0) return false;
        r.ci = ni; r.cj = nj; r.ck = nk;
        r.rho0 = a.rho[(size_t)dev(a, ni, nj, nk) * a.ncomp];  // the next step's density, requested now
        r.x = ex ? xE : r.x + r.dx * ds;
        r.y = ey ? yE : r.y + r.dy * ds;
        r.z = ez ? zE : r.z + r.dz * ds;
        return true;
    }

    __device__ static __forceinline__ int whichcell(const Args& a, const Shared& sh, double x, double y, double z) {
        const double* xv = sh.mesh;
        const double* yv = xv + a.nx + 1;
        const double* zv = yv + a.ny + 1;
        const int i = locateFail(xv, a.nx + 1, x), j = locateFail(yv, a.ny + 1, y), k = locateFail(zv, a.nz + 1, z);
        if (i < 0 || j < 0 || k < 0) return -1;
        return dev(a, i, j, k);
    }
};

// Octree grid walked through the node arrays: TreeDustGrid.cpp:390-521 (TopDown and Neighbor
// search), DustGridPath::moveInside. Used for trees the leaf map cannot hold, and by the leaf-map
// walk below for the rare steps whose exit point lies on a cell face.
template <>
struct Grid<kOctreeNodes> {
    __device__ static __forceinline__ void loadBox(const Args& a, int l, double& x0, double& y0, double& z0,
                                                   double& x1, double& y1, double& z1) {
        const double2* b = reinterpret_cast<const double2*>(a.box + 6 * (size_t)l);
        const double2 p = b[0], q = b[1], w = b[2];
        x0 = p.x; y0 = p.y; z0 = q.x; x1 = q.y; y1 = w.x; z1 = w.y;
    }

    // TreeNode::whichnode from the root + OctTreeNode::child(r) / BinTreeNode::child(r)
    // (BinTreeNode.cpp:322-331): the leaf containing (x,y,z) or -1
    __device__ static __forceinline__ int descend(const Args& a, double x, double y, double z) {
        if (!(x >= a.gx0 && x <= a.gx1 && y >= a.gy0 && y <= a.gy1 && z >= a.gz0 && z <= a.gz1)) return -1;
        int l = 0;
        int c0 = a.firstChild[0];
        while (c0 >= 0) {
            const double* cb = a.box + 6 * (size_t)c0 + 3;  // split point = rmax of child 0
            if (a.splitDir) {
                const int d = a.splitDir[l];
                l = c0 + ((d == 0 ? x : d == 1 ? y : z) < cb[d] ? 0 : 1);
            } else {
                l = c0 + (x < cb[0] ? 0 : 1) + (y < cb[1] ? 0 : 2) + (z < cb[2] ? 0 : 4);
            }
            c0 = a.firstChild[l];
        }
        return l;
    }

    // the part of the path before the grid (TreeDustGrid.cpp:404-440): up to three segments outside the
    // grid; on return (x,y,z) is the entry point. False for an empty path.
    __device__ static __forceinline__ bool enterGrid(const Args& a, double& rx, double& ry, double& rz, double kx,
                                                     double ky, double kz, double (&d)[3]) {
        const double eps = a.eps;
        d[0] = d[1] = d[2] = 0;
        if (rx <= a.gx0) {
            if (kx <= 0.0) return false;
            d[0] = (a.gx0 - rx) / kx; rx = a.gx0 + eps; ry += ky * d[0]; rz += kz * d[0];
        } else if (rx >= a.gx1) {
            if (kx >= 0.0) return false;
            d[0] = (a.gx1 - rx) / kx; rx = a.gx1 - eps; ry += ky * d[0]; rz += kz * d[0];
        }
        if (ry <= a.gy0) {
            if (ky <= 0.0) return false;
            d[1] = (a.gy0 - ry) / ky; rx += kx * d[1]; ry = a.gy0 + eps; rz += kz * d[1];
        } else if (ry >= a.gy1) {
            if (ky >= 0.0) return false;
            d[1] = (a.gy1 - ry) / ky; rx += kx * d[1]; ry = a.gy1 - eps; rz += kz * d[1];
        }
        if (rz <= a.gz0) {
            if (kz <= 0.0) return false;
            d[2] = (a.gz0 - rz) / kz; rx += kx * d[2]; ry += ky * d[2]; rz = a.gz0 + eps;
        } else if (rz >= a.gz1) {
            if (kz >= 0.0) return false;
            d[2] = (a.gz1 - rz) / kz; rx += kx * d[2]; ry += ky * d[2]; rz = a.gz1 - eps;
        }
        return true;
    }

    template <class SegFn>
    __device__ static __forceinline__ bool begin(const Args& a, const Shared&, Ray& r, SegFn seg) {
        double rx = r.x, ry = r.y, rz = r.z, d[3];
        if (!enterGrid(a, rx, ry, rz, r.dx, r.dy, r.dz, d)) return false;
        const int node = descend(a, rx, ry, rz);
        if (node < 0) return false;
        for (int q = 0; q < 3; q++)
            if (d[q] > 0) seg(-1, 0.0, d[q]);
        r.x = rx; r.y = ry; r.z = rz;
        r.ci = node;
        r.cj = a.cellnumber[node];
        loadBox(a, node, r.bx0, r.by0, r.bz0, r.bx1, r.by1, r.bz1);
        return true;
    }

    // the node after `node` for a ray leaving it through `wall` at (x,y,z) (already advanced by
    // ds + eps): TreeNode::whichnode(wall, r) over the sorted neighbour list, else the descent from the
    // root, with the reference's nextafter escape when the point has not left the node. May move
    // (x,y,z). Returns -1 when the path leaves the grid.
    __device__ static __forceinline__ int nextNode(const Args& a, int node, int wall, double& x, double& y, double& z,
                                                   double kx, double ky, double kz) {
        if (a.search == SKIRT_TREE_NEIGHBOR) {
            const int q = 6 * node + wall;
            const int nb = a.nbrOffset[q], ne = a.nbrOffset[q + 1];
            for (int n = nb; n < ne; n++) {
                const int c = a.nbrList[n];
                double x0, y0, z0, x1, y1, z1;
                loadBox(a, c, x0, y0, z0, x1, y1, z1);
                if (x >= x0 && x <= x1 && y >= y0 && y <= y1 && z >= z0 && z <= z1) return c;
            }
        }
        int next = descend(a, x, y, z);
        if (next == node) {
            // stuck: advance to the next representable coordinates (TreeDustGrid.cpp:502-519)
            x = nextafter(x, (kx < 0.0) ? -kDblMax : kDblMax);
            y = nextafter(y, (ky < 0.0) ? -kDblMax : kDblMax);
            z = nextafter(z, (kz < 0.0) ? -kDblMax : kDblMax);
            next = descend(a, x, y, z);
            if (next == node) return -1;
        }
        return next;
    }

    template <class SegFn>
    __device__ static __forceinline__ bool step(const Args& a, const Shared&, Ray& r, SegFn seg) {
        const int node = r.ci;
        const double xnext = (r.dx < 0.0) ? r.bx0 : r.bx1;
        const double ynext = (r.dy < 0.0) ? r.by0 : r.by1;
        const double znext = (r.dz < 0.0) ? r.bz0 : r.bz1;
        const double dsx = (r.ix != 0.0) ? (xnext - r.x) * r.ix : kDblMax;
        const double dsy = (r.iy != 0.0) ? (ynext - r.y) * r.iy : kDblMax;
        const double dsz = (r.iz != 0.0) ? (znext - r.z) * r.iz : kDblMax;
        double ds;
        int wall;
        if (dsx <= dsy && dsx <= dsz) { ds = dsx; wall = (r.dx < 0.0) ? 0 : 1; }
        else if (dsy <= dsx && dsy <= dsz) { ds = dsy; wall = (r.dy < 0.0) ? 2 : 3; }
        else { ds = dsz; wall = (r.dz < 0.0) ? 4 : 5; }
        if (!seg(r.cj, a.rho[(size_t)r.cj * a.ncomp], ds)) return false;
        double x = r.x + (ds + a.eps) * r.dx;
        double y = r.y + (ds + a.eps) * r.dy;
        double z = r.z + (ds + a.eps) * r.dz;
        const int next = nextNode(a, node, wall, x, y, z, r.dx, r.dy, r.dz);
        if (next < 0) return false;
        loadBox(a, next, r.bx0, r.by0, r.bz0, r.bx1, r.by1, r.bz1);
        r.x = x; r.y = y; r.z = z;
        r.ci = next;
        r.cj = a.cellnumber[next];
        return true;
    }


    __device__ static __forceinline__ int whichcell(const Args& a, const Shared&, double x, double y, double z) {
        const int l = descend(a, x, y, z);
        return l < 0 ? -1 : a.cellnumber[l];
    }
};

// Octree grid, Bookkeeping search (TreeDustGrid.cpp:523-659): the next node follows from the breadth-first
// numbering (the 8 children of a node are consecutive ids in octant order, so (l-1) % 8 is the octant of
// node l): climb while the node lies on the far side of its father, step to the sibling across the wall,
// descend with "<=" to the leaf holding the exit point. The position is put on the crossed wall exactly
// (no eps). Entry into the grid as for the other searches.
template <>
struct Grid<kOctreeBookkeeping> {
    using Nodes = Grid<kOctreeNodes>;

    template <class SegFn>
    __device__ static __forceinline__ bool begin(const Args& a, const Shared& sh, Ray& r, SegFn seg) {
        return Nodes::begin(a, sh, r, seg);
    }
    __device__ static __forceinline__ int whichcell(const Args& a, const Shared& sh, double x, double y, double z) {
        return Nodes::whichcell(a, sh, x, y, z);
    }

    __device__ static __forceinline__ const double* childBox(const Args& a, int l) {
        return a.box + 6 * (size_t)a.firstChild[l];
    }

    template <class SegFn>
    __device__ static __forceinline__ bool step(const Args& a, const Shared&, Ray& r, SegFn seg) {
        const double xnext = (r.dx < 0.0) ? r.bx0 : r.bx1;
        const double ynext = (r.dy < 0.0) ? r.by0 : r.by1;
        const double znext = (r.dz < 0.0) ? r.bz0 : r.bz1;
        const double dsx = (r.ix != 0.0) ? (xnext - r.x) * r.ix : kDblMax;
        const double dsy = (r.iy != 0.0) ? (ynext - r.y) * r.iy : kDblMax;
        const double dsz = (r.iz != 0.0) ? (znext - r.z) * r.iz : kDblMax;
        int l = r.ci;
        if (dsx <= dsy && dsx <= dsz) {
            if (!seg(r.cj, a.rho[(size_t)r.cj * a.ncomp], dsx)) return false;
            r.x = xnext; r.y += r.dy * dsx; r.z += r.dz * dsx;
            while ((r.dx < 0.0) ? (((l - 1) & 1) == 0) : (((l - 1) & 1) == 1)) {
                l = a.father[l];
                if (l == 0) return false;
            }
            l += (r.dx < 0.0) ? -1 : 1;
            while (a.cellnumber[l] < 0) {
                const double* cb = childBox(a, l);
                const int k = (r.dx < 0.0 ? 1 : 0) + (r.y <= cb[4] ? 0 : 2) + (r.z <= cb[5] ? 0 : 4);
                l = a.firstChild[l] + k;
            }
        } else if (dsy < dsx && dsy <= dsz) {
            if (!seg(r.cj, a.rho[(size_t)r.cj * a.ncomp], dsy)) return false;
            r.x += r.dx * dsy; r.y = ynext; r.z += r.dz * dsy;
            while ((r.dy < 0.0) ? (((l - 1) & 2) == 0) : (((l - 1) & 2) != 0)) {
                l = a.father[l];
                if (l == 0) return false;
            }
            l += (r.dy < 0.0) ? -2 : 2;
            while (a.cellnumber[l] < 0) {
                const double* cb = childBox(a, l);
                const int k = (r.x <= cb[3] ? 0 : 1) + (r.dy < 0.0 ? 2 : 0) + (r.z <= cb[5] ? 0 : 4);
                l = a.firstChild[l] + k;
            }
        } else if (dsz < dsx && dsz < dsy) {
            if (!seg(r.cj, a.rho[(size_t)r.cj * a.ncomp], dsz)) return false;
            r.x += r.dx * dsz; r.y += r.dy * dsz; r.z = znext;
            while ((r.dz < 0.0) ? (((l - 1) & 4) == 0) : (((l - 1) & 4) != 0)) {
                l = a.father[l];
                if (l == 0) return false;
            }
            l += (r.dz < 0.0) ? -4 : 4;
            while (a.cellnumber[l] < 0) {
                const double* cb = childBox(a, l);
                const int k = (r.x <= cb[3] ? 0 : 1) + (r.y <= cb[4] ? 0 : 2) + (r.dz < 0.0 ? 4 : 0);
                l = a.firstChild[l] + k;
            }
        } else {
            return false;  // NaN distances
        }
        r.ci = l;
        r.cj = a.cellnumber[l];
        Nodes::loadBox(a, l, r.bx0, r.by0, r.bz0, r.bx1, r.by1, r.bz1);
        return true;
    }
};

// Octree grid through the leaf map. An octree split at box centres (OctTreeNode::createchildren,
// OctTreeNode.cpp:53-56, Box::center) has, per axis, one table of 2^L + 1 split coordinates T (L the
// deepest level) such that a level-l node with integer coordinate i spans [T[i << (L-l)],
// T[(i+1) << (L-l)]] -- bit for bit, since every split is 0.5*(lo+hi) of two table entries. So:
//   - the box faces come from the T tables in LDS (no box gather);
//   - the leaf containing a point is the leaf map entry of the finest-level cell holding it: one
//     16-byte load instead of the neighbour-list walk. Locating by "T[j] <= x < T[j+1]" is exactly
//     the reference's root descent (x < split -> lower child), so the only steps where it can differ
//     from the inclusive-box neighbour search (TreeNode::whichnode(wall, r)) are those whose exit point
//     lies exactly on a lower face of the leaf found, or that have not left the current leaf; those
//     take the node-array search above. The walk is therefore the reference's, step for step.
// The host builds the map only after checking every node box against the T tables.
// A k-d tree (BinTreeNode::createchildren_splitdir also halves at the centre, one axis at a time) maps
// the same way with per-axis leaf extents (BIN): its entries carry the three shifts instead of a level.
template <bool BIN>
struct LeafMapGrid {
    using Nodes = Grid<kOctreeNodes>;

    // a leaf's extent along x, y, z in finest cells, as shifts
    __device__ static __forceinline__ void shifts(const Args& a, unsigned cl, int& sx, int& sy, int& sz) {
        if (BIN) {
            const unsigned s = cl >> kBinCellBits;
            sx = (int)(s & 7u); sy = (int)((s >> 3) & 7u); sz = (int)((s >> 6) & 7u);
        } else {
            sx = sy = sz = a.mapL - (int)(cl >> kLeafLevelShift);
        }
    }
    __device__ static __forceinline__ int cellOf(unsigned cl) { return (int)(cl & (BIN ? kBinCellMask : kLeafCellMask)); }

    // finest-level index j with T[j] <= v < T[j+1] (the last cell also holds v == T[N]); v in [T[0], T[N]].
    // The split coordinates are uniform to rounding, so the estimate is off by one at most near a
    // split; the loops only run for that rare lane.
    __device__ static __forceinline__ int estimate(int N, double t0, double inv, double v) {
        return max(0, min(N - 1, (int)((v - t0) * inv)));
    }
    __device__ static __forceinline__ int correct(const double* T, int N, int j, double v) {
        const double lo = T[j], hi = T[j + 1];
        if (v < lo) {
            do j--; while (j > 0 && v < T[j]);
            j = max(j, 0);  // v below T[0]: a point outside the grid, whose entry is fetched but not used
        } else if (v >= hi && j < N - 1) {
            do j++; while (j < N - 1 && v >= T[j + 1]);
        }
        return j;
    }

    __device__ static __forceinline__ bool inside(const Args& a, double x, double y, double z) {
        return x >= a.gx0 && x <= a.gx1 && y >= a.gy0 && y <= a.gy1 && z >= a.gz0 && z <= a.gz1;
    }

    // issues the load of the leaf map entry of the point (clamped into the grid, so any point -- even
    // NaN -- reads a valid entry); fx, fy, fz its finest-level indices. The entry of the estimated cell
    // is requested before the estimate is checked against the T tables in LDS; the rare lane whose
    // estimate was off by one requests the right entry again.
    __device__ static __forceinline__ int4 fetch(const Args& a, const Shared& sh, double x, double y, double z,
                                                 int& fx, int& fy, int& fz) {
        const int N = a.mapN;
        const double* tx = sh.mesh;
        const int ex = estimate(N, a.mapX0, a.mapInvX, x);
        const int ey = estimate(N, a.mapY0, a.mapInvY, y);
        const int ez = estimate(N, a.mapZ0, a.mapInvZ, z);
        int4 v = *reinterpret_cast<const int4*>(a.leafMap + leafIndex(N, ex, ey, ez));
        fx = correct(tx, N, ex, x);
        fy = correct(tx + (N + 1), N, ey, y);
        fz = correct(tx + 2 * (N + 1), N, ez, z);
        if (fx != ex || fy != ey || fz != ez) v = *reinterpret_cast<const int4*>(a.leafMap + leafIndex(N, fx, fy, fz));
        return v;
    }

    __device__ static __forceinline__ LeafEntry decode(int4 v) {
        // one 16-byte load: keep the compiler from splitting off the density into a later second load
        asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
        LeafEntry e;
        e.node = v.x;
        e.cl = (unsigned)v.y;
        const long long bits = ((long long)(unsigned)v.w << 32) | (unsigned)v.z;
        e.rho0 = __longlong_as_double(bits);
        return e;
    }

    // leaf map entry of the point (inside the grid); fx, fy, fz its finest-level indices
    __device__ static __forceinline__ LeafEntry lookup(const Args& a, const Shared& sh, double x, double y, double z,
                                                       int& fx, int& fy, int& fz) {
        return decode(fetch(a, sh, x, y, z, fx, fy, fz));
    }

    // r.ck: the leaf's size in finest cells (octree) or its packed shifts (k-d tree); r.bx0, r.by0,
    // r.bz0: the leaf's faces the ray leaves through along x, y, z (read from the T tables once, when
    // the leaf is entered, so the next step starts without an LDS round trip)
    __device__ static __forceinline__ void enterPlanes(Ray& r, int jx, int jy, int jz, const LeafEntry& e,
                                                       double lox, double loy, double loz,
                                                       double hix, double hiy, double hiz) {
        r.ci = e.node;
        r.cj = cellOf(e.cl);
        if (BIN) r.ck = (int)(e.cl >> kBinCellBits);
        r.jx = jx; r.jy = jy; r.jz = jz;
        r.rho0 = e.rho0;
        r.bx0 = (r.dx < 0.0) ? lox : hix;
        r.by0 = (r.dy < 0.0) ? loy : hiy;
        r.bz0 = (r.dz < 0.0) ? loz : hiz;
    }
    __device__ static __forceinline__ void enter(const Args& a, const Shared& sh, Ray& r, int fx, int fy, int fz,
                                                 const LeafEntry& e) {
        const int N1 = a.mapN + 1;
        const double* tx = sh.mesh;
        int sx, sy, sz;
        shifts(a, e.cl, sx, sy, sz);
        const int jx = (fx >> sx) << sx, jy = (fy >> sy) << sy, jz = (fz >> sz) << sz;
        enterPlanes(r, jx, jy, jz, e, tx[jx], tx[N1 + jy], tx[2 * N1 + jz], tx[jx + (1 << sx)],
                    tx[N1 + jy + (1 << sy)], tx[2 * N1 + jz + (1 << sz)]);
        if (!BIN) r.ck = 1 << sx;
    }

    template <class SegFn>
    __device__ static __forceinline__ bool begin(const Args& a, const Shared& sh, Ray& r, SegFn seg) {
        double rx = r.x, ry = r.y, rz = r.z, d[3];
        if (!Nodes::enterGrid(a, rx, ry, rz, r.dx, r.dy, r.dz, d)) return false;
        if (!inside(a, rx, ry, rz)) return false;  // the root descent finds no node
        for (int q = 0; q < 3; q++)
            if (d[q] > 0) seg(-1, 0.0, d[q]);
        int fx, fy, fz;
        const LeafEntry e = lookup(a, sh, rx, ry, rz, fx, fy, fz);
        r.x = rx; r.y = ry; r.z = rz;
        enter(a, sh, r, fx, fy, fz, e);
        prefetch(a, r);
        return true;
    }

    // the exit of the current leaf: the distance to the nearest of its three faces ahead of the ray, the wall
    // (the reference's order of comparisons) and the exit point nudged by eps
    __device__ static __forceinline__ void exitPoint(const Args& a, const Ray& r, double& ds, int& wall, double& x,
                                                     double& y, double& z) {
        const double xnext = r.bx0, ynext = r.by0, znext = r.bz0;
        const double dsx = (r.ix != 0.0) ? (xnext - r.x) * r.ix : kDblMax;
        const double dsy = (r.iy != 0.0) ? (ynext - r.y) * r.iy : kDblMax;
        const double dsz = (r.iz != 0.0) ? (znext - r.z) * r.iz : kDblMax;
        if (dsx <= dsy && dsx <= dsz) { ds = dsx; wall = (r.dx < 0.0) ? 0 : 1; }
        else if (dsy <= dsx && dsy <= dsz) { ds = dsy; wall = (r.dy < 0.0) ? 2 : 3; }
        else { ds = dsz; wall = (r.dz < 0.0) ? 4 : 5; }
        x = r.x + (ds + a.eps) * r.dx;
        y = r.y + (ds + a.eps) * r.dy;
        z = r.z + (ds + a.eps) * r.dz;
    }

    // requests the leaf-map entry of the estimated finest cell of the next exit point: issued at the end of a
    // step, before the wave's Labs drain, it is in flight during the drain and the next step's segment. A load
    // waits for every older vector-memory operation of its wave (vmcnt counts in issue order, atomics
    // included, and a no-return f64 atomic stays counted for thousands of cycles under load): requested
    // after the drain, each step's entry would wait for the previous step's Labs atomic too.
    __device__ static __forceinline__ void prefetch(const Args& a, Ray& r) {
        exitPoint(a, r, r.eds, r.ewall, r.ex, r.ey, r.ez);  // (kept for the step: the ray does not move before it)
        const int N = a.mapN;
        r.pfx = estimate(N, a.mapX0, a.mapInvX, r.ex);
        r.pfy = estimate(N, a.mapY0, a.mapInvY, r.ey);
        r.pfz = estimate(N, a.mapZ0, a.mapInvZ, r.ez);
        r.pre = *reinterpret_cast<const int4*>(a.leafMap + leafIndex(N, r.pfx, r.pfy, r.pfz));
    }

    template <class SegFn>
    __device__ static __forceinline__ bool step(const Args& a, const Shared& sh, Ray& r, SegFn seg) {
        const int N1 = a.mapN + 1;
        const double* tx = sh.mesh;
        const double* ty = tx + N1;
        const double* tz = ty + N1;
        // the exit point prefetch computed at the end of the last step (or at the grid entry): 139 -> 129 VGPRs,
        // C3 within the spread, C5 +0.5 % (profiles/r05_exit_reuse_ab.txt)
        const double ds = r.eds;
        double x = r.ex, y = r.ey, z = r.ez;
        const int wall = r.ewall;
        // the next leaf's entry is requested first; the segment's own work (optical depth, absorption)
        // runs while the load is in flight
        // the entry of the estimated finest cell; its leaf is the right one when the leaf's own faces
        // (read anyway) contain the point, since T is monotone: then the exact finest cell lies in it too
        const int N = a.mapN;
        // requested by the previous step (prefetch), for the same exit point computed the same way
        int fx = r.pfx, fy = r.pfy, fz = r.pfz;
        const int4 raw = r.pre;
        if (!seg(r.cj, r.rho0, ds)) return false;
        if (!inside(a, x, y, z)) return false;  // no neighbour and no root descent contains it
        LeafEntry e = decode(raw);
        int lx, ly, lz;
        shifts(a, e.cl, lx, ly, lz);
        int jx = (fx >> lx) << lx, jy = (fy >> ly) << ly, jz = (fz >> lz) << lz;
        // the new leaf's six faces in one LDS round trip: the lower ones decide whether the exit point
        // lies on a face, the ones ahead of the ray are the next step's exit planes
        double lox = tx[jx], loy = ty[jy], loz = tz[jz];
        double hix = tx[jx + (1 << lx)], hiy = ty[jy + (1 << ly)], hiz = tz[jz + (1 << lz)];
        if (!(x >= lox && x < hix && y >= loy && y < hiy && z >= loz && z < hiz)) {
            // the estimate fell into a neighbouring leaf (or the point is on the grid's far faces): the
            // exact finest cell, its entry and its leaf's faces
            fx = correct(tx, N, fx, x);
            fy = correct(ty, N, fy, y);
            fz = correct(tz, N, fz, z);
            e = decode(*reinterpret_cast<const int4*>(a.leafMap + leafIndex(N, fx, fy, fz)));
            shifts(a, e.cl, lx, ly, lz);
            jx = (fx >> lx) << lx; jy = (fy >> ly) << ly; jz = (fz >> lz) << lz;
            lox = tx[jx]; loy = ty[jy]; loz = tz[jz];
            hix = tx[jx + (1 << lx)]; hiy = ty[jy + (1 << ly)]; hiz = tz[jz + (1 << lz)];
        }
        r.x = x; r.y = y; r.z = z;
        if (e.node == r.ci || x == lox || y == loy || z == loz) {
            // on a face, or not out of the current leaf: the reference's own search decides
            const int next = Nodes::nextNode(a, r.ci, wall, x, y, z, r.dx, r.dy, r.dz);
            if (next < 0) return false;
            const double* b = a.box + 6 * (size_t)next;  // its lower corner is a finest cell of it
            e = lookup(a, sh, b[0], b[1], b[2], fx, fy, fz);
            enter(a, sh, r, fx, fy, fz, e);
            prefetch(a, r);
            return true;
        }
        enterPlanes(r, jx, jy, jz, e, lox, loy, loz, hix, hiy, hiz);
        if (!BIN) r.ck = 1 << lx;
        prefetch(a, r);
        return true;
    }

    __device__ static __forceinline__ int whichcell(const Args& a, const Shared& sh, double x, double y, double z) {
        if (!inside(a, x, y, z)) return -1;
        int fx, fy, fz;
        return cellOf(lookup(a, sh, x, y, z, fx, fy, fz).cl);
    }
};

template <>
struct Grid<SKIRT_GRID_OCTREE> : LeafMapGrid<false> {};
template <>
struct Grid<kBinTreeMap> : LeafMapGrid<true> {};

// Voronoi grid: VoronoiMesh::path (VoronoiMesh.cpp:749-844), cellIndex (:512-541), with the
// reference's arithmetic order (bisector plane through the midpoint, Vec::dot left to right)
template <>
struct Grid<SKIRT_GRID_VORONOI> {
    __device__ static __forceinline__ bool inside(const Args& a, double x, double y, double z) {
        return x >= a.gx0 && x <= a.gx1 && y >= a.gy0 && y <= a.gy1 && z >= a.gz0 && z <= a.gz1;
    }

    // the cell whose site is nearest, over the cells listed for the point's block (Box::cellindices)
    __device__ static __forceinline__ int cellIndex(const Args& a, double x, double y, double z) {
        if (!inside(a, x, y, z)) return -1;
        const int nb = a.vnb;
        const int i = max(0, min(nb - 1, static_cast<int>(nb * (x - a.gx0) / (a.gx1 - a.gx0))));
        const int j = max(0, min(nb - 1, static_cast<int>(nb * (y - a.gy0) / (a.gy1 - a.gy0))));
        const int k = max(0, min(nb - 1, static_cast<int>(nb * (z - a.gz0) / (a.gz1 - a.gz0))));
        const int b = i * nb * nb + j * nb + k;
        int m = -1;
        double best = kDblMax;
        // the list in groups of kCellIndexGroup candidates, each {site, cell} in one 32-byte record, a group's
        // records loaded together (one round trip per group); the candidates are then taken in list order, so
        // the first of equal distances wins as in the reference's loop
        constexpr int G = kCellIndexGroup;
        const int qe = a.blockOffset[b + 1];
        for (int q0 = a.blockOffset[b]; q0 < qe; q0 += G) {
            int c[G];
            double sx[G], sy[G], sz[G];
#pragma unroll
            for (int u = 0; u < G; u++) {
                c[u] = -1;
                sx[u] = sy[u] = sz[u] = 0.0;
                if (q0 + u < qe) {
                    const double2* rec = reinterpret_cast<const double2*>(a.blockSites + q0 + u);
                    const double2 r0 = rec[0], r1 = rec[1];
                    sx[u] = r0.x; sy[u] = r0.y; sz[u] = r1.x;
                    c[u] = (int)(unsigned)__double_as_longlong(r1.y);  // the id, in the low word
                }
            }
#pragma unroll
            for (int u = 0; u < G; u++) {
                const double dx = x - sx[u], dy = y - sy[u], dz = z - sz[u];
                const double d = dx * dx + dy * dy + dz * dz;
                if (c[u] >= 0 && d < best) { best = d; m = c[u]; }
            }
        }
        return m;
    }

    template <class SegFn>
    __device__ static __forceinline__ bool begin(const Args& a, const Shared&, Ray& r, SegFn seg) {
        int none = kNoCell;
        return beginAt(a, r, none, seg);
    }

    // begin() with the cell of the ray's origin cached in `cell` (kNoCell: not known yet). A point strictly
    // inside the grid enters where it is, whatever the direction (enterGrid moves nothing), so its cellIndex
    // serves every ray from that position: the peel-offs and the FILL ray of one event, and the WALK ray
    // that retraces the FILL ray's path in the next one. A point on or outside the grid's faces enters
    // where its direction takes it, so it is located per ray and not cached.
    template <class SegFn>
    __device__ static __forceinline__ bool beginAt(const Args& a, Ray& r, int& cell, SegFn seg) {
        double rx = r.x, ry = r.y, rz = r.z, d[3];
        const bool strict = rx > a.gx0 && rx < a.gx1 && ry > a.gy0 && ry < a.gy1 && rz > a.gz0 && rz < a.gz1;
        if (!Grid<kOctreeNodes>::enterGrid(a, rx, ry, rz, r.dx, r.dy, r.dz, d)) return false;
        int m;
        if (strict && cell != kNoCell) m = cell;
        else {
            m = cellIndex(a, rx, ry, rz);
            if (strict) cell = m;
        }
        if (m < 0) return false;
        for (int q = 0; q < 3; q++)
            if (d[q] > 0) seg(-1, 0.0, d[q]);
        r.x = rx; r.y = ry; r.z = rz;
        r.ci = m;
        r.cj = a.vorStart[m];
        r.ck = 0;
        return true;
    }

    __device__ static __forceinline__ double wallDist(const Args& a, const Ray& r, int w) {
        switch (w) {
        case -1: return (a.gx0 - r.x) / r.dx;
        case -2: return (a.gx1 - r.x) / r.dx;
        case -3: return (a.gy0 - r.y) / r.dy;
        case -4: return (a.gy1 - r.y) / r.dy;
        case -5: return (a.gz0 - r.z) / r.dz;
        default: return (a.gz1 - r.z) / r.dz;
        }
    }

    // the reference's distance along the ray to the bisector plane of sites pr (the current cell) and pi
    // (a neighbour), 0 when the ray moves away from it -- VoronoiMesh.cpp:790-806, same operation order
    __device__ static __forceinline__ double planeDist(const Ray& r, double prx, double pry, double prz, double pix,
                                                       double piy, double piz) {
        const double nx = pix - prx, ny = piy - pry, nz = piz - prz;
        const double ndotk = nx * r.dx + ny * r.dy + nz * r.dz;
        if (!(ndotk > 0)) return 0;
        const double px = 0.5 * (pix + prx), py = 0.5 * (piy + pry), pz = 0.5 * (piz + prz);
        return (nx * (px - r.x) + ny * (py - r.y) + nz * (pz - r.z)) / ndotk;
    }

    __device__ static __forceinline__ void siteAt(const Args& a, int start, double& x, double& y, double& z) {
        const double2 h0 = *reinterpret_cast<const double2*>(a.vorSlots + start);
        const double2 h1 = *reinterpret_cast<const double2*>(a.vorSlots + start + 1);
        x = h0.x; y = h0.y; z = h1.x;
    }

    // the operands of a step: the cell's header (exact site, density, id, neighbour count) and, for the
    // bounds, the float offset D of the site from the ray's position and the direction in float
    struct StepIn {
        const VorEntry* B;
        double pwx, pwy, pwz, rhow;
        int idw, cnt;
        float Dx, Dy, Dz, fkx, fky, fkz;
        float eA, eA2, eB2;  // the cell's error terms: eA, 2 eA, 2 (eA |D|_1 + kVorEpsF max |n|^2)
    };
    // U: the least upper bound of the certain exits; L1 <= L2: the two least lower bounds of the possible
    // exits, w1: the first one's `next`
    struct Best {
        float U, L1, L2;
        int w1;
    };

    // the bounds [lo, hi] of one neighbour's plane distance, in single precision on coordinates scaled by
    // a.vorScale (the entries' offsets are stored scaled): each float operation adds a few 2^-24 of the sum
    // of absolute terms, which kVorEpsF covers with margin; an approximate reciprocal (1 ulp) is covered by
    // the |s| term. Walls are stored as the bisector plane with the site's mirror image (the same plane),
    // so every entry takes the same branch-free arithmetic; lo = hi = FLT_MAX: certainly no exit.
    __device__ static __forceinline__ void bounds(const StepIn& s, const VorEntry& en, bool valid, float& lo,
                                                  float& ucand) {
        // the plane distance s = (n.D + |n|^2/2) / (n.k) = (m.D + 1/2) / (m.k) with m = n / |n|^2, the stored
        // entry, and Cauchy-Schwarz error terms: |d(m.k)| <= eA and |d(m.D + 1/2)| <= eB = eA |D|_1 + kVorEpsF/2,
        // at the cell's largest |m|_1 (vor_terms.hpp; several times the float roundings of the entries, D, k
        // and the fused operations). 29 operations per entry (with n stored: 33; per-entry terms: 38; round
        // 2's sums of the absolute terms of each product: 55); tools/vor_compact_check.cpp, mode r, checks
        // the resulting steps against the reference's.
        const float mx = en.ox, my = en.oy, mz = en.oz;  // m = n / |n|^2 (vor_terms.hpp)
        const float den = fmaf(mz, s.fkz, fmaf(my, s.fky, mx * s.fkx));
        const float num = fmaf(mz, s.Dz, fmaf(my, s.Dy, fmaf(mx, s.Dx, 0.5f)));
        const float inv = __builtin_amdgcn_rcpf(den);
        const float sa = num * inv;
        const float err = fmaf(fmaf(fabsf(sa), s.eA2, s.eB2), inv, fabsf(sa) * kVorEpsF);
        // den > 2 eA: the sign of n.k and the interval [sa - err, sa + err] are certain; den <= -eA: moving away for certain; otherwise (den = 0 included: m = 0 is a
        // degenerate wall) the sign is uncertain: lo = -FLT_MAX. Entries past the count (`valid`), and the
        // NaN padding after a cell's list (den NaN, so neither sure nor maybe): no exit. ucand: the upper
        // bound of a certain exit (lo > 0), else FLT_MAX. Selected as floats, no bool temporaries.
        const float lov = sa - err, hiv = sa + err;
        const bool sure = valid && den > s.eA2;
        const bool maybe = valid && den > -s.eA;
        // (a sure interval wholly behind the ray, hiv <= 0, stays a possible exit, which the exact evaluation
        // would drop: inside the cell no plane the ray moves towards lies behind it, so this happens at
        // rounding level only -- tools/vor_compact_check.cpp, mode r: the same 297 exact re-evaluations in
        // 1,004,001 steps with and without the check; C4 +0.7 %, profiles/r05_vor_behind_ab.txt)
        lo = sure ? lov : (maybe ? -FLT_MAX : FLT_MAX);
        ucand = (sure && lov > 0.f) ? hiv : FLT_MAX;
    }

    // one entry's bounds into the running Best, in list order
    __device__ static __forceinline__ void take(Best& b, float lo, float ucand, int next) {
        b.U = fminf(b.U, ucand);
        b.w1 = lo < b.L1 ? next : b.w1;
        b.L2 = __builtin_amdgcn_fmed3f(b.L1, b.L2, lo);
        b.L1 = fminf(b.L1, lo);
    }

    // The start of a step: the cell's header h0..h2 (loaded with the first entries in the same round), the
    // pending segment (r.ck = 1: the previous cell's segment, cell r.ci, density r.rho0, site r.bx0..bz0,
    // ends on the bisector plane with this cell, whose exact site arrives with this load), and the bounds'
    // operands. False: the ray ended.
    template <class SegFn>
    __device__ static __forceinline__ bool headFrom(const Args& a, Ray& r, StepIn& s, const double2& h0, const double2& h1,
                                                    const int4& h2, SegFn seg) {
        s.pwx = h0.x; s.pwy = h0.y; s.pwz = h1.x; s.rhow = h1.y;
        s.idw = h2.x; s.cnt = h2.y;
        const float eA = __int_as_float(h2.z), eBn = __int_as_float(h2.w);  // the cell's terms (upload)
        if (r.ck) {
            const double sq = planeDist(r, r.bx0, r.by0, r.bz0, s.pwx, s.pwy, s.pwz);
            if (!seg(r.ci, r.rho0, sq)) return false;
            r.x += (sq + a.eps) * r.dx; r.y += (sq + a.eps) * r.dy; r.z += (sq + a.eps) * r.dz;
            r.ck = 0;
        }
        const float sc = a.vorScale;
        s.Dx = (float)((s.pwx - r.x) * sc); s.Dy = (float)((s.pwy - r.y) * sc); s.Dz = (float)((s.pwz - r.z) * sc);
        const float Dn = fabsf(s.Dx) + fabsf(s.Dy) + fabsf(s.Dz);  // |D|_1
        s.fkx = (float)r.dx; s.fky = (float)r.dy; s.fkz = (float)r.dz;
        s.eA = eA; s.eA2 = 2.0f * eA; s.eB2 = 2.0f * fmaf(eA, Dn, eBn);
        return true;
    }

    // The end of a step, from the bounds over all entries: a single certain exit is taken (its exact
    // distance follows from the next cell's header, r.ck = 1); otherwise the reference's rule, exactly,
    // over the possible winners.
    template <class SegFn>
    __device__ static __forceinline__ bool decide(const Args& a, Ray& r, const StepIn& s, const Best& b, SegFn seg) {
        const VorEntry* B = s.B;
        const int cnt = s.cnt;
        if (b.L1 != FLT_MAX && b.L2 > b.U) {
            if (b.w1 >= 0) {  // the exit: its exact distance when the next cell's header arrives
                r.ck = 1;
                r.ci = s.idw; r.rho0 = s.rhow;
                r.bx0 = s.pwx; r.by0 = s.pwy; r.bz0 = s.pwz;
                r.cj = b.w1;
                return true;
            }
            seg(s.idw, s.rhow, wallDist(a, r, b.w1));  // leaves the grid through a wall
            return false;
        }
        // no exit, or several possible exits. An entry whose lower bound exceeds U lies beyond a certain
        // exit, so it can neither win nor tie; a second pass over the (cached) entries collects the others
        // in list order (the first of equal distances wins) and their sites arrive in one round trip. More
        // than kVorCand of them: the whole list, in groups.
        const double kx = r.dx, ky = r.dy, kz = r.dz;
        constexpr int NO_INDEX = (int)0x80000000u;
        double sq = kDblMax;
        int mq = NO_INDEX;
        auto consider = [&](int nxt, double pix, double piy, double piz) {
            const double si = nxt < 0 ? wallDist(a, r, nxt) : planeDist(r, s.pwx, s.pwy, s.pwz, pix, piy, piz);
            if (si > 0 && si < sq) { sq = si; mq = nxt; }
        };
        if (b.L1 != FLT_MAX) {
            int c0 = 0, c1 = 0, c2 = 0, c3 = 0, nc = 0;
            VorEntry e[kVorUnroll];
            for (int q0 = 0; q0 < cnt; q0 += kVorUnroll) {
                vorEntries(B, q0, e);
#pragma unroll
                for (int u = 0; u < kVorUnroll; u++) {
                    float lo, uc;
                    bounds(s, e[u], q0 + u < cnt, lo, uc);
                    if (lo < FLT_MAX && lo <= b.U) {
                        const int nx = e[u].next;
                        c0 = nc == 0 ? nx : c0; c1 = nc == 1 ? nx : c1; c2 = nc == 2 ? nx : c2; c3 = nc == 3 ? nx : c3;
                        nc++;
                    }
                }
            }
            if (nc <= kVorCand) {
                const int cs[kVorCand] = {c0, c1, c2, c3};
                double pix[kVorCand], piy[kVorCand], piz[kVorCand];
#pragma unroll
                for (int u = 0; u < kVorCand; u++) {
                    pix[u] = piy[u] = piz[u] = 0.0;
                    if (u < nc && cs[u] >= 0) siteAt(a, cs[u], pix[u], piy[u], piz[u]);
                }
#pragma unroll
                for (int u = 0; u < kVorCand; u++)
                    if (u < nc) consider(cs[u], pix[u], piy[u], piz[u]);
            } else {
                constexpr int G = kVorFallbackGroup;
                for (int q0 = 0; q0 < cnt; q0 += G) {
                    int nxt[G];
                    double pix[G], piy[G], piz[G];
#pragma unroll
                    for (int u = 0; u < G; u++) {
                        nxt[u] = vorEntry(B, q0 + u).next;
                        pix[u] = piy[u] = piz[u] = 0.0;
                        if (q0 + u < cnt && nxt[u] >= 0) siteAt(a, nxt[u], pix[u], piy[u], piz[u]);
                    }
#pragma unroll
                    for (int u = 0; u < G; u++)
                        if (q0 + u < cnt) consider(nxt[u], pix[u], piy[u], piz[u]);
                }
            }
        }
        if (mq == NO_INDEX) {
            // no exit found: advance by eps and locate again (VoronoiMesh.cpp:831-835)
            r.x += kx * a.eps; r.y += ky * a.eps; r.z += kz * a.eps;
            const int m = cellIndex(a, r.x, r.y, r.z);
            if (m < 0) return false;
            r.ci = m;
            r.cj = a.vorStart[m];
            return true;
        }
        if (!seg(s.idw, s.rhow, sq)) return false;
        r.x += (sq + a.eps) * kx; r.y += (sq + a.eps) * ky; r.z += (sq + a.eps) * kz;
        r.cj = mq;
        return mq >= 0;
    }

    // One step (VoronoiMesh::path, VoronoiMesh.cpp:749-844), lane-serial over the cell's entries. r.cj:
    // the block of the cell the ray is in. A step issues one round of loads (this cell's header and first
    // entries) in the common case. It adds at most two segments (the pending one, and one more when the
    // bounds leave several possible winners), see kSegsPerStep.
    // the loads a step starts with: the cell's header and its first kVorGroups groups of entries (one round)
    struct Load {
        double2 h0, h1;
        int4 h2;
        VorEntry g[kVorGroups][kVorUnroll];
    };
    __device__ static __forceinline__ void stepLoad(const Args& a, const Ray& r, Load& L, bool act = true) {
        // lanes without a ray load block 0: an unconditional load needs no merge of old and new register
        // values (moves, which would wait for the loads right after their issue)
        const VorEntry* B = a.vorSlots + (act ? r.cj : 0);
        L.h0 = *reinterpret_cast<const double2*>(B);
        L.h1 = *reinterpret_cast<const double2*>(B + 1);
        L.h2 = *reinterpret_cast<const int4*>(B + 2);
#pragma unroll
        for (int gi = 0; gi < kVorGroups; gi++) vorEntries(B, gi * kVorUnroll, L.g[gi]);
    }

    template <class SegFn>
    __device__ static __forceinline__ bool step(const Args& a, const Shared& sh, Ray& r, SegFn seg) {
        Load L;
        stepLoad(a, r, L);
        return stepRest(a, sh, r, L, seg);
    }

    // the step from its loads (stepLoad): the trace kernel issues the Labs drain between the two, so the
    // header's wait does not include the drain's atomics (vmcnt counts in issue order)
    template <class SegFn>
    __device__ static __forceinline__ bool stepRest(const Args& a, const Shared&, Ray& r, Load& L, SegFn seg) {
        StepIn s;
        s.B = a.vorSlots + r.cj;
        Best b{FLT_MAX, FLT_MAX, FLT_MAX, 0};
        // kVorGroups groups of entries in flight: they load with the header, and each group's next load is
        // issued as soon as the group is consumed, so a cell with more than kVorUnroll neighbours does not
        // wait for a second round trip
        if (!headFrom(a, r, s, L.h0, L.h1, L.h2, seg)) return false;
        // (the next groups are loaded only while the list lasts: loading them unconditionally -- past the list
        // into the next block -- let the compiler drop the register moves at the join, but made C4 24 % slower,
        // 9.53e7 -> 7.37e7 pkt/s, profiles/r04_ab_c4_vor_uncond_loads_c3c5_prefetch.txt; a lane past its list
        // reading one line that all such lanes share instead: 208 -> 170 register moves, still 5 % slower,
        // profiles/r05_vor_uncond_shared_ab.txt; round 0 peeled and round 1 loaded into registers of its
        // own: 208 -> 146 moves, 245 VGPRs, C4 -0.4 %, the same file)
        constexpr int NG = kVorGroups;
        for (int q0 = 0; q0 < s.cnt; q0 += NG * kVorUnroll) {
#pragma unroll
            for (int gi = 0; gi < NG; gi++) {
                const int qb = q0 + gi * kVorUnroll;
                if (gi > 0 && qb >= s.cnt) break;
#pragma unroll
                for (int u = 0; u < kVorUnroll; u++) {
                    float lo, uc;
                    // (a cell's list is padded to whole groups with NaN entries: no count check per entry)
                    bounds(s, L.g[gi][u], true, lo, uc);
                    take(b, lo, uc, L.g[gi][u].next);
                }
                if (qb + NG * kVorUnroll < s.cnt) vorEntries(s.B, qb + NG * kVorUnroll, L.g[gi]);
            }
        }
        return decide(a, r, s, b, seg);
    }

    __device__ static __forceinline__ int whichcell(const Args& a, const Shared&, double x, double y, double z) {
        return cellIndex(a, x, y, z);
    }

    // VoronoiMesh::isPointClosestTo, over the exact sites of the cell's neighbours (their headers)
    __device__ static __forceinline__ bool closestTo(const Args& a, double x, double y, double z, int m) {
        auto d2 = [&](double sx, double sy, double sz) {
            const double dx = x - sx, dy = y - sy, dz = z - sz;
            return dx * dx + dy * dy + dz * dz;
        };
        const int start = a.vorStart[m];
        double sx, sy, sz;
        siteAt(a, start, sx, sy, sz);
        const double target = d2(sx, sy, sz);
        const int cnt = reinterpret_cast<const int4*>(a.vorSlots + start + 2)->y;
        for (int q = 0; q < cnt; q++) {
            const int nxt = vorEntry(a.vorSlots + start, q).next;
            if (nxt < 0) continue;
            siteAt(a, nxt, sx, sy, sz);
            if (d2(sx, sy, sz) < target) return false;
        }
        return true;
    }
};

// ================================================================== trace kernel
// GLOBAL: the Labs adds as global atomics (a table of 4 GiB or more, Args::labsGlobal), a kernel of its own:
// a run-time choice between the buffer atomic every lane issues and a global atomic only lanes with an add
// issue leaves the waitcnt pass a path with no vector-memory operation in the drain, and the next step's
// leaf-map entry then waited with vmcnt(0), i.e. for the drain's atomic as well. Now vmcnt(1): C3 +0.3 %,
// C2 +0.4 %, C4 and C5 within the spread (the atomic had mostly finished by then; profiles/r06_decode_wait_ab.txt)
template <int GRID, bool ONECOMP, bool CONT, bool STORE, bool GLOBAL = false>
struct Tracer {
    const Args& a;
    const Shared& sh;
    // statistics, kept out of the walk's registers: the lane's segments of its current ray (added per ray
    // to the wave's FILL / WALK / PEEL totals in LDS when the ray ends), and wave-uniform counts of the
    // Labs adds, lane-steps and 64-byte atomic requests (lane 0's values are the wave's)
    unsigned int nseg = 0;
    unsigned int absorbs = 0, laneSlots = 0, requests = 0;
    unsigned* waveSegs;  // LDS, [kBlock / 64][3]: FILL, WALK, PEEL segments of the wave's finished rays
    // Labs adds of this lane not yet issued. f64 atomics execute memory-side at a fixed chip-wide rate
    // of 64-byte requests; lanes of one wave instruction that hit the same 64-byte line share a
    // request. A lane's consecutive adds are consecutive cells of one ray -- spatial neighbours, and
    // with Morton-ordered device cell numbers mostly in the same or the next line -- so the adds wait
    // in LDS (kLabsBuf per lane, [slot][thread]) and are issued transposed: each wave instruction
    // carries the kLabsBuf consecutive adds of 64 / kLabsBuf lanes. A wave also waits for one
    // atomic round trip per burst instead of one per step.
    double* pendVal;    // LDS, [kLabsBuf][kBlock]
    unsigned* pendIdx;  // LDS, [kLabsBuf][kBlock]
    unsigned char* pendHi;  // LDS, [kLabsBuf][kBlock]: bits 32-39 of the element index (Args::labsHi only)
    __amdgpu_buffer_rsrc_t labsRsrc;  // the Labs table as a raw buffer of labsBytes (unless Args::labsGlobal)
    unsigned copyOff = 0;             // this wave's replica (Args::labsCopies), in bytes
    unsigned labsOob = 0;             // a byte offset past every replica: the empty lanes' adds are dropped
    int npend = 0;
    unsigned gstep = 0;  // grid steps of the wave (drainStep's round robin)

    __device__ __forceinline__ void drain() {
        static_assert(kLabsBuf >= 2 && kLabsBuf <= 64 && (kLabsBuf & (kLabsBuf - 1)) == 0, "kLabsBuf: power of 2");
        constexpr int G = 64 / kLabsBuf;  // lanes per wave instruction
        const int lane = threadIdx.x & 63;
        const int wbase = threadIdx.x - lane;
        const int j = lane & (kLabsBuf - 1);
#pragma unroll
        for (int i = 0; i < kLabsBuf; i++) issue(i);
        npend = 0;
    }

    // wave instruction i of a drain: the buffered adds of lanes G i .. G i + G - 1 (G = 64 / kLabsBuf),
    // kLabsBuf consecutive adds of each, transposed onto the wave's lanes
    __device__ __forceinline__ void issue(int i) {
        constexpr int G = 64 / kLabsBuf;
        const int lane = threadIdx.x & 63;
        const int wbase = threadIdx.x - lane;
        const int j = lane & (kLabsBuf - 1);
        const int src = G * i + lane / kLabsBuf;
        const int n = __shfl(npend, src);
        const int q = j * kBlock + wbase + src;
        const unsigned idx = pendIdx[q];
        // the element index: 32 bits, or 40 with the high byte of a table of 2^32 elements or more
        const size_t eidx = a.labsHi ? ((size_t)pendHi[q] << 32 | idx) : (size_t)idx;
        // the requests of this instruction: a lane starts one unless the lane before it (the same
        // ray's previous add) hit the same 64-byte line (these statistics cost nothing measurable: C3 +0.05 %,
        // C2 +0.6 % without them, timing only; profiles/r06_ab.txt)
        const unsigned line = (unsigned)(reinterpret_cast<size_t>(a.labs + eidx) >> 6);
        const unsigned prev = __shfl(line, lane - 1);
        const unsigned long long starts = __ballot(j < n && (j == 0 || prev != line));
        absorbs += (unsigned)__popcll(__ballot(j < n));
        requests += (unsigned)__popcll(starts);
        if constexpr (GLOBAL) {  // a table of 4 GiB or more: global atomics
            if (j < n) atomicAddF64(a.labs + eidx, pendVal[q]);
        } else {
            // every lane issues; a lane without an add adds 0 at the first byte past the table (dropped)
            const double v = j < n ? pendVal[q] : 0.0;
            bufferAtomicAddF64(v, labsRsrc, (int)(j < n ? idx * 8u + copyOff : labsOob), 0, 0);
        }
    }

    // One drain instruction per grid step, round robin over the lane groups: every lane's buffer is
    // emptied every kLabsBuf steps, which holds its at most kLabsBuf adds (one per step), and the adds
    // leave as a steady stream instead of a burst of kLabsBuf instructions (which stalls the issuing
    // wave behind its outstanding atomics and reaches the memory-side atomic units in clumps).
    __device__ __forceinline__ void drainStep() {
        constexpr int G = 64 / kLabsBuf;
        const int i = (int)(gstep++ & (kLabsBuf - 1));
        issue(i);
        if (((threadIdx.x & 63) / G) == i) npend = 0;
    }
    // The same for steps of up to two adds (the Voronoi walk, kSegsPerStep 2): two drain instructions every
    // step, so every lane's buffer is emptied every kLabsBuf / 2 steps. It replaces a full drain whenever a
    // buffer might overflow: the same instructions on average, but that drain sat behind a branch, and after it
    // the waitcnt pass could count no atomics with certainty, so the walk's next load waits (vmcnt(0)) covered
    // the 16 atomics of any drain before them. C4 +0.3 %, 230 -> 211 VGPRs (profiles/r06_vor_drain_ab.txt)
    __device__ __forceinline__ void drainStep2() {
        constexpr int G = 64 / kLabsBuf;
        const int i = (int)(gstep++ & (kLabsBuf / 2 - 1)) * 2;
        issue(i);
        issue(i + 1);
        const int grp = (threadIdx.x & 63) / G;
        if (grp == i || grp == i + 1) npend = 0;
    }

    __device__ __forceinline__ double rho(int m, int h) const { return a.rho[(size_t)m * a.ncomp + h]; }

    // per-segment work; false stops the ray (a WALK reached its optical depth)
    __device__ __forceinline__ bool segment(Ray& r, int m, double rho0, double ds) {
        if (!(ds > 0)) return true;  // DustGridPath::addSegment skips ds <= 0
        double kr = 0.0;  // KappaRho functor (DustSystem.cpp:465-491)
        if (m >= 0) {
            if (ONECOMP) kr = r.kext * rho0;
            else for (int h = 0; h < a.ncomp; h++) kr += sh.kext[h * a.nlambda + r.ell] * rho(m, h);
        }
        const double dtau = kr * ds;
        if (CONT && r.mode == RAY_FILL && m >= 0) {
            // the segment as the path holds it, before s and tau advance; the slot's count lives in
            // pathCnt (no register of the walk carries it)
            const int n = a.pathCnt[r.idx];
            if (n < kPathCap) {
                a.pathBuf[(size_t)r.idx * kPathCap + n] = PathRec{r.s, ds, r.tau, dtau, m, 0};
                a.pathCnt[r.idx] = n + 1;
            } else {
                atomicOr(a.error, ERR_PATH_CAP);
            }
        }
        r.s += ds;
        r.tau += dtau;
        nseg++;
        if (r.mode == RAY_FILL) {
            if (m >= 0 && (!ONECOMP || (STORE && a.store))) {
                // L_abs = (1-albedo) L exp(-tau_{n-1}) (1 - exp(-dtau_n)) (MonteCarloSimulation.cpp:458-462).
                // exp(-tau) is carried in f1 as the running product of exp(-dtau) = 1 - ef, which is exact to
                // about an ulp per segment while ef <= 1 - exp(-kCarryTau); behind a thicker segment (where
                // 1 - ef loses digits: rounds 1-3 carried it unconditionally and the thick pan_oct_sa models'
                // deep cells drifted) it is evaluated anew. One f64 exp less per segment: C2 +0.6 %, C5 +0.5 %,
                // C3 within the spread (profiles/r05_exp_carry_ab.txt)
                double ef;
                if (SKIRT_POLY_EXPM1 && dtau < kCarryTau) ef = oneMinusExpNeg(dtau);
                else ef = -expm1(-dtau);
                const double Lintm = r.param * r.f1 * ef;
                if (dtau < kCarryTau) r.f1 -= r.f1 * ef;
                else r.f1 = exp(-r.tau);
                double albedo;
                if (ONECOMP) albedo = sh.alb[r.ell];
                else {
                    double ksca = 0.0, kext = 0.0;
                    for (int h = 0; h < a.ncomp; h++) {
                        ksca += rho(m, h) * sh.ksca[h * a.nlambda + r.ell];
                        kext += rho(m, h) * sh.kext[h * a.nlambda + r.ell];
                    }
                    albedo = (kext > 0.0) ? ksca / kext : 0.0;
                    r.f2 += albedo * Lintm;
                }
#ifdef SKIRT_DEBUG_FILL  // diagnostic builds only (tools/parity_trace.py): the FILL segments, one packet per run
                printf("E S %d %.17g %.17g %.17g\n", m, ds, dtau, (1.0 - albedo) * Lintm);
#endif
                if (STORE && a.store) {
                    pendVal[npend * kBlock + threadIdx.x] = (1.0 - albedo) * Lintm;
                    if (a.labsHi) {  // (wave-uniform) a table of 2^32 elements or more
                        const unsigned long long e = (unsigned long long)r.ell * (unsigned)a.labsStride + (unsigned)m;
                        pendIdx[npend * kBlock + threadIdx.x] = (unsigned)e;
                        pendHi[npend * kBlock + threadIdx.x] = (unsigned char)(e >> 32);
                    } else {
                        pendIdx[npend * kBlock + threadIdx.x] = (unsigned)r.ell * (unsigned)a.labsStride + (unsigned)m;
                    }
                    npend++;
                }
            }
        } else if (r.mode == RAY_WALK) {
            if (r.tau > r.param) return false;  // the interaction point lies in this segment
            r.f1 = r.tau;
            r.f2 = r.s;
        }
        return true;
    }

    // load queued ray `id` and enter the grid: the part of the path before the grid (segments outside
    // it, m = -1) and the first cell (DustGrid::path); an empty path finishes the ray at once
    __device__ __forceinline__ void load(Ray& r, unsigned id) {
        const double2* c = reinterpret_cast<const double2*>(a.rays + id);
        const double2 c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3];
        const int4 c6 = reinterpret_cast<const int4*>(c)[4];
        r.id = id;
        r.x = c0.x; r.y = c0.y; r.z = c1.x;
        r.dx = c1.y; r.dy = c2.x; r.dz = c2.y;
        // 1/direction, 0 where |k| <= 1e-15 (that axis is never crossed), as the event kernel computed it
        r.ix = (fabs(r.dx) > 1e-15) ? 1.0 / r.dx : 0.0;
        r.iy = (fabs(r.dy) > 1e-15) ? 1.0 / r.dy : 0.0;
        r.iz = (fabs(r.dz) > 1e-15) ? 1.0 / r.dz : 0.0;
        r.param = c3.y;
        r.idx = c6.x;
        r.flags = (unsigned)c6.y;
        r.mode = rayMode(r.flags);
        r.ell = rayEll(r.flags);
        r.tau = 0;
        if (CONT && r.mode == RAY_FILL) a.pathCnt[r.idx] = 0;
#ifdef SKIRT_DEBUG_FILL
        if (r.mode == RAY_FILL)
            printf("E L %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", r.ell, r.x, r.y, r.z, r.dx, r.dy, r.dz, r.param);
#endif
        r.s = c3.x;
        r.kext = sh.kext[r.ell];
        // FILL: f1 = exp(-tau) = 1, f2 = scattered luminosity; WALK: tau and s at the last segment end
        r.f1 = (r.mode == RAY_FILL) ? 1.0 : 0.0;
        r.f2 = (r.mode == RAY_WALK) ? c3.x : 0.0;
        // the segments before the grid of a ray the event kernel entered travel in the first cell's top bits
        // (a ray the event kernel entered brings its segments before the grid in the first cell's top bits)
        nseg = kEnterInEvent<GRID> ? ((unsigned)c6.z >> kOutsideShift) : 0u;
        if (kEnterInEvent<GRID>) {  // entered by the event kernel: the cell and its neighbour list
            r.ci = c6.z & kCellMaskOut;
            r.cj = c6.w;
            r.ck = 0;
        } else if (r.mode != RAY_NONE &&
            !Grid<GRID>::begin(a, sh, r, [&](int m, double rho0, double ds) { return segment(r, m, rho0, ds); })) {
            finish(r);  // FILL: tau = 0, no scattered luminosity; WALK: s = 0; PEEL: tau = 0
            r.mode = RAY_NONE;
        }
    }

    // the ray ended (grid edge or WALK target reached): deliver its result
    __device__ __forceinline__ void finish(const Ray& r) {
        atomicAdd(&waveSegs[(threadIdx.x >> 6) * 3 + (r.mode == RAY_FILL ? 0 : r.mode == RAY_WALK ? 1 : 2)], nseg);
        if (a.crossed && r.mode != RAY_WALK) crossedAdd(a, nseg);
        if (r.mode == RAY_PEEL) {
            a.det[r.idx].tau = r.tau;  // detectKernel turns it into a detection
        } else if (r.mode == RAY_FILL) {
            a.resA[r.idx] = r.tau;
            if (!ONECOMP) a.resB[r.idx] = r.f2;
        } else {
            // DustGridPath::pathlength: interpolate inside the crossing segment; if the path ended first
            // (target >= tau of the path), the end of the last segment
            const double tauint = r.param;
            double s = 0;
            if (tauint > 0) {
                if (r.tau > tauint) s = r.f2 + ((tauint - r.f1) / (r.tau - r.f1)) * (r.s - r.f2);
                else s = r.f2;
            }
            a.resA[r.idx] = s;
        }
    }
};

// Instrument::detect of one peel-off ray (FullInstrument.cpp:107-174 and the Simple/SED/Frame
// variants): what it adds to instrument slot `slot` (FullInstrument: 0 transparent, 1 direct stellar,
// 2 scattered stellar, 3 direct dust, 4 scattered dust, 5.. per scattering level); false if nothing.
// Lextf = L e^{-tau}.
__device__ __forceinline__ bool detectSlot(const DevInstr& ins, unsigned flags, int slot, double Lp, double Lextf,
                                           double& v) {
    v = Lextf;
    if (ins.kind != SKIRT_INSTR_FULL) return slot == 0;
    switch (rayCat(flags)) {
    case CAT_STAR_DIRECT:
        if (slot == 0) v = Lp;
        return slot <= 1;
    case CAT_STAR_SCATTERED: {
        const int lev = rayLevel(flags);
        return slot == 2 || (lev >= 1 && lev <= ins.levels && slot == 5 + lev - 1);
    }
    case CAT_DUST_DIRECT: return slot == 3;
    default: return slot == 4;
    }
}

// frame tally of an instrument: [lambda][pixel][slot] with the slots padded to slotStride (8 for a
// FullInstrument with up to 3 scattering levels), so that one detection's adds fall in one 64-byte line
__device__ __forceinline__ double* frameAt(const Args& a, const DevInstr& ins, int ell, int l, int slot) {
    return a.tally + ins.frameBase + ((long long)ell * ins.nx * ins.ny + l) * ins.slotStride + slot;
}

// Instrument::detect of one peel-off ray with optical depth tau by one lane: SEDs into `sed` (LDS sums
// of the workgroup) or, when null, the global tally; frames with f64 atomics
__device__ __forceinline__ void detectPeel(const Args& a, const DevInstr& ins, unsigned flags, int l, double Lp,
                                           double tau, double* sed) {
    const double Lextf = Lp * exp(-tau);
    const int nl = a.nlambda;
    const int ell = rayEll(flags);
    for (int slot = 0; slot < ins.nslots; slot++) {
        double v;
        if (!detectSlot(ins, flags, slot, Lp, Lextf, v)) continue;
        if (ins.kind != SKIRT_INSTR_FRAME) {
            if (sed) atomicAdd(&sed[ins.sedOff + slot * nl + ell], v);
            else atomicAddF64(a.tally + ins.sedBase + slot * nl + ell, v);
        }
        if (l >= 0 && ins.kind != SKIRT_INSTR_SED) atomicAddF64(frameAt(a, ins, ell, l, slot), v);
    }
}

// DustSystem::writeconvergence (DustSystem.cpp:195-250): the column density of the grid along a ray, as
// DustGridPath::opticalDepth (DustGridPath.hpp:97-108) sums it with DustSystem::density (the cell's
// densities summed over the components, DustSystem.cpp:925-931), over the same walk as the photon paths.
// One lane per ray; rays[6 i .. 6 i + 5] = origin, direction.
template <int GRID>
__global__ void __launch_bounds__(kBlock) columnKernel(const Args a, const double* rays, int n, double* out) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    Shared sh = stageTables(a, lds, gridParts<GRID>());
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r{};
    r.x = rays[6 * i]; r.y = rays[6 * i + 1]; r.z = rays[6 * i + 2];
    r.dx = rays[6 * i + 3]; r.dy = rays[6 * i + 4]; r.dz = rays[6 * i + 5];
    r.ix = (fabs(r.dx) > 1e-15) ? 1.0 / r.dx : 0.0;
    r.iy = (fabs(r.dy) > 1e-15) ? 1.0 / r.dy : 0.0;
    r.iz = (fabs(r.dz) > 1e-15) ? 1.0 / r.dz : 0.0;
    double tau = 0;
    auto seg = [&](int m, double, double ds) {
        if (ds > 0 && m >= 0) {  // (addSegment skips ds <= 0; a segment outside the grid adds 0 x ds)
            double rho = 0;
            for (int h = 0; h < a.ncomp; h++) rho += a.rho[(size_t)m * a.ncomp + h];
            tau += rho * ds;
        }
        return true;
    };
    if (Grid<GRID>::begin(a, sh, r, seg))
        while (Grid<GRID>::step(a, sh, r, seg)) {}
    out[i] = tau;
}

// ================================================================== dust emission sources on the device
// The grey-body emission spectrum of every cell and the per-wavelength cell distribution of the dust
// phases (DustLib::calculate with AllCellsDustLib + GreyBodyDustEmissivity, DustLib.cpp:60-185,
// GreyBodyDustEmissivity.cpp:19-43, DustMix::equilibrium DustMix.cpp:689-712; cell luminosities and
// NR::cdf of PanMonteCarloSimulation.cpp:193-205, 273-294), computed from the device tallies so the
// self-absorption cycles never leave the GPU. Reference cell order, like the host restatement
// (host/dustemission.cpp), which the tests compare against.
struct EmisArgs {
    int ncells, nlambda, ncomp, ntemp;
    const int* devCell;          // reference cell -> device cell (null: identity)
    const double* labs;          // [nlambda][device cell]
    const double* labsDust;      // same, or null
    const double* rho;           // [device cell][ncomp]
    const double* volume;        // [reference cell]
    const double* kabs;          // [ncomp][nlambda]
    const double* sigmaabs;      // [ncomp][nlambda]
    const double* mu;            // [ncomp]
    const double* Tv;            // [ntemp]
    const double* planckabs;     // [ncomp][ntemp]
    const double* lambda;        // [nlambda]
    const double* dlambda;       // [nlambda]
    int labsStride;              // Labs row length
    double* lv;                  // out [nlambda][ncells]
    double* cdf;                 // out [nlambda][ncells + 1]
    double* ltot;                // out [nlambda]
    double* blockSums;           // scratch [nlambda][nblocks]
    int nblocks;
};

__device__ __forceinline__ double planckB(double T, double lambda) {  // PlanckFunction
    const double h = 6.62606957e-34, c = 2.99792458e8, k = 1.3806488e-23;
    const double x = h * c / (lambda * k * T);
    return 2.0 * h * c * c / pow(lambda, 5) / (exp(x) - 1.0);
}

__global__ void __launch_bounds__(kBlock) cellSpectraKernel(const EmisArgs e) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= e.ncells) return;
    const int Nl = e.nlambda;
    const size_t S = e.labsStride;
    const int dm = e.devCell ? e.devCell[m] : m;
    // PanDustSystem::Labs(m): stellar sum, continued by the dust sum
    double Labsbol = 0;
    for (int ell = 0; ell < Nl; ell++) Labsbol += e.labs[ell * S + dm];
    if (e.labsDust)
        for (int ell = 0; ell < Nl; ell++) Labsbol += e.labsDust[ell * S + dm];
    // J_lambda is needed only for the absorbed power of each component, and the emission spectrum Lv is
    // accumulated in the cell's own column of the output (the arithmetic of the host restatement, one
    // operation at a time), so any number of wavelengths fits
    const double fac = 4.0 * M_PI * e.volume[m];
    auto meanIntensity = [&](int ell) {  // DustSystem::meanintensityv
        double L = 0;
        L += e.labs[ell * S + dm];
        if (e.labsDust) L += e.labsDust[ell * S + dm];
        double kr = 0.0;
        for (int h = 0; h < e.ncomp; h++) kr += e.kabs[h * Nl + ell] * e.rho[(size_t)dm * e.ncomp + h];
        const double J = L / (kr * fac) / e.dlambda[ell];
        return isfinite(J) ? J : 0.0;
    };
    double* Lv = e.lv + m;  // Lv[ell] at Lv[ell * ncells]
    const size_t N = e.ncells;
    for (int ell = 0; ell < Nl; ell++) Lv[ell * N] = 0.0;
    for (int h = 0; h < e.ncomp; h++) {
        // DustMix::equilibrium -> invplanckabs (NR::locate_clip + linear interpolation)
        const double* sa = e.sigmaabs + h * Nl;
        double pa = 0.0;
        for (int ell = 0; ell < Nl; ell++) pa += sa[ell] * meanIntensity(ell) * e.dlambda[ell];
        const double* tab = e.planckabs + (size_t)h * e.ntemp;
        int p;
        if (pa < tab[0]) p = 0;
        else {
            int jl = -1, ju = e.ntemp - 1;
            while (ju - jl > 1) { const int jm = (ju + jl) >> 1; if (pa < tab[jm]) ju = jm; else jl = jm; }
            p = jl;
        }
        const double T = e.Tv[p] + ((pa - tab[p]) / (tab[p + 1] - tab[p])) * (e.Tv[p + 1] - e.Tv[p]);
        const double w = e.ncomp > 1 ? e.rho[(size_t)dm * e.ncomp + h] : 1.0;
        for (int ell = 0; ell < Nl; ell++) {
            double ev = 0.0;
            ev += sa[ell] * planckB(T, e.lambda[ell]);
            ev /= e.mu[h];
            if (e.ncomp > 1) Lv[ell * N] += ev * w;
            else Lv[ell * N] = ev;
        }
    }
    double total = 0.0;
    for (int ell = 0; ell < Nl; ell++) {
        const double v = Lv[ell * N] * e.dlambda[ell];
        Lv[ell * N] = v;
        total += v;
    }
    for (int ell = 0; ell < Nl; ell++) {
        const double lum = total > 0 ? Lv[ell * N] / total : Lv[ell * N];
        Lv[ell * N] = Labsbol > 0.0 ? Labsbol * lum : 0.0;
    }
}

// per wavelength: sums of kBlock consecutive cells
__global__ void __launch_bounds__(kBlock) cellBlockSumKernel(const EmisArgs e) {
    __shared__ double red[kBlock];
    const int ell = blockIdx.y, b = blockIdx.x, m = b * kBlock + threadIdx.x;
    red[threadIdx.x] = m < e.ncells ? e.lv[(size_t)ell * e.ncells + m] : 0.0;
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) e.blockSums[(size_t)ell * e.nblocks + b] = red[0];
}

// per wavelength (one block each): exclusive scan of the block sums and the total. Each thread sums a
// contiguous chunk of the block sums, the chunk sums are scanned in LDS, and each thread then writes its
// chunk's exclusive prefixes (a single thread walking all block sums took 3 ms per call on C5).
__global__ void __launch_bounds__(kBlock) cellScanBlocksKernel(const EmisArgs e) {
    __shared__ double part[kBlock];
    const int ell = blockIdx.x;
    double* bs = e.blockSums + (size_t)ell * e.nblocks;
    const int per = (e.nblocks + kBlock - 1) / kBlock;
    const int b0 = min(e.nblocks, (int)threadIdx.x * per), b1 = min(e.nblocks, b0 + per);
    double sum = 0;
    for (int b = b0; b < b1; b++) sum += bs[b];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < kBlock; off <<= 1) {  // inclusive Hillis-Steele scan of the chunk sums
        const double v = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0.0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    double run = threadIdx.x ? part[threadIdx.x - 1] : 0.0;
    for (int b = b0; b < b1; b++) {
        const double v = bs[b];
        bs[b] = run;
        run += v;
    }
    if (threadIdx.x == kBlock - 1) e.ltot[ell] = part[kBlock - 1];
}

// the normalized cumulative distribution: X[0] = 0, X[m+1] = (sum of Lv[0..m]) / Ltot
__global__ void __launch_bounds__(kBlock) cellCdfKernel(const EmisArgs e) {
    __shared__ double sc[kBlock];
    const int ell = blockIdx.y, b = blockIdx.x, m = b * kBlock + threadIdx.x;
    const int N = e.ncells;
    sc[threadIdx.x] = m < N ? e.lv[(size_t)ell * N + m] : 0.0;
    __syncthreads();
    for (int off = 1; off < kBlock; off <<= 1) {  // inclusive Hillis-Steele scan
        const double v = threadIdx.x >= off ? sc[threadIdx.x - off] : 0.0;
        __syncthreads();
        sc[threadIdx.x] += v;
        __syncthreads();
    }
    const double total = e.ltot[ell];
    double* X = e.cdf + (size_t)ell * (N + 1);
    if (m < N) X[m + 1] = total > 0 ? (e.blockSums[(size_t)ell * e.nblocks + b] + sc[threadIdx.x]) / total : 0.0;
    if (m == 0) X[0] = 0.0;
}

// NR::locate_clip over a table in global memory (n entries): the largest j <= n - 2 with v[j] <= q, 0 below v[0]
__device__ __forceinline__ int locateClipTable(const double* v, int n, double q) {
    if (q < v[0]) return 0;
    int jl = -1, ju = n - 1;
    while (ju - jl > 1) {
        const int jm = (ju + jl) >> 1;
        if (q < v[jm]) ju = jm;
        else jl = jm;
    }
    return jl;
}

// A guide table over a CDF of N + 1 entries: G[k] = locate_clip(v, k / N), k = 0 .. N. A draw q then only
// bisects [G[k], G[k + 1]] with k = floor(q N) -- two or three dependent loads instead of log2(N) ~ 20 (the
// dust-phase launch draws a cell from 622,490 per packet in C5).
__global__ void __launch_bounds__(kBlock) cellGuideKernel(const double* cdf, int* guide, int N) {
    const int ell = blockIdx.y, k = blockIdx.x * kBlock + threadIdx.x;
    if (k > N) return;
    const double* v = cdf + (size_t)ell * (N + 1);
    guide[(size_t)ell * (N + 1) + k] = locateClipTable(v, N + 1, (double)k / (double)N);
}

// locate_clip(v, N + 1, q) through the guide table: the bracket [G[k], G[k + 1] + 1) holds the answer when
// v[G[k]] <= q and q < v[G[k + 1] + 1] (or the bracket ends at the table's last index) -- checked, since
// floor(q N) may round across a bucket edge; otherwise the whole table is bisected. Within a valid bracket
// the bisection finds the same largest j with v[j] <= q as the full one.
__device__ __forceinline__ int locateGuided(const double* v, const int* G, int N, double q) {
    const int k = max(0, min(N - 1, static_cast<int>(q * (double)N)));
    const int lo = G[k], hi = G[k + 1] + 1;
    if (!(v[lo] <= q) || (hi < N && !(q < v[hi]))) return locateClipTable(v, N + 1, q);
    int jl = lo, ju = hi;
    while (ju - jl > 1) {
        const int jm = (ju + jl) >> 1;
        if (q < v[jm]) ju = jm;
        else jl = jm;
    }
    return jl;
}

// fills the leaf map: one thread per finest-level cell descends the (checked) tree by its index bits
// (a k-d tree by the bit of its split axis at that axis' depth)
__global__ void __launch_bounds__(kBlock) buildLeafMapKernel(LeafEntry* map, const int* firstChild, const signed char* splitDir,
                                                             const int* cellnumber, const double* rho, int ncomp, int L) {
    const int N = 1 << L;
    const unsigned long long n = leafMapSize(N);
    for (unsigned long long q = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; q < n;
         q += (unsigned long long)gridDim.x * blockDim.x) {
        unsigned fx = 0, fy = 0, fz = 0;
        {  // inverse of leafIndex
            const unsigned long long nb = leafBricks(N), br = q >> 3;
            fx = (unsigned)(2 * (br / (nb * nb)) + ((q >> 2) & 1u));
            fy = (unsigned)(2 * ((br / nb) % nb) + ((q >> 1) & 1u));
            fz = (unsigned)(2 * (br % nb) + (q & 1u));
            fx = min(fx, (unsigned)N - 1u); fy = min(fy, (unsigned)N - 1u); fz = min(fz, (unsigned)N - 1u);
        }
        int node = 0, level = 0;
        LeafEntry e;
        if (splitDir) {
            int lv[3] = {0, 0, 0};
            const unsigned f[3] = {fx, fy, fz};
            while (firstChild[node] >= 0) {
                const int d = splitDir[node];
                const int bit = L - 1 - lv[d];
                lv[d]++;
                node = firstChild[node] + (int)((f[d] >> bit) & 1u);
            }
            e.cl = (unsigned)cellnumber[node] |
                   ((unsigned)(L - lv[0]) | (unsigned)(L - lv[1]) << 3 | (unsigned)(L - lv[2]) << 6) << kBinCellBits;
        } else {
            while (firstChild[node] >= 0) {
                const int bit = L - 1 - level;
                node = firstChild[node] + (int)((fx >> bit) & 1u) + 2 * (int)((fy >> bit) & 1u) + 4 * (int)((fz >> bit) & 1u);
                level++;
            }
            e.cl = (unsigned)cellnumber[node] | ((unsigned)level << kLeafLevelShift);
        }
        const int cell = cellnumber[node];
        e.node = node;
        e.rho0 = rho[(size_t)cell * ncomp];
        map[q] = e;
    }
}

// CONT: continuous scattering (the FILL rays record their dust segments); its own instantiations keep
// the recording out of the other kernels' registers
// STORE false: a phase that stores no absorption (a.store = 0), one dust component, no continuous
// scattering: no Labs buffers and no drain (its own instantiation, traceKernelNoStore)
template <int GRID, bool ONECOMP, bool CONT, bool STORE, bool GLOBAL = false>
__device__ __forceinline__ void traceBody(const Args& a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // reset the counters the next event iteration appends to (nobody else uses them now)
        CTR(a.ctr, 1 - a.parity) = 0;  // ray count of the next iteration
        CTR(a.ctr, 2 + a.parity) = 0;  // active list just consumed by the event kernel
        CTR(a.ctr, 8 + (1 - a.parity)) = 0;  // the next iteration's WALK rays
    }
    // the iteration's rays: ctr[q] from the bottom of the queue, then the WALK rays ctr[8 + q] from its top
    // (Args::walkBack), pulled last: the short WALK paths fill the lanes that the long FILL and peel-off
    // paths free at the end of a launch, instead of idling until the launch's longest path ends
    const unsigned int nfront = CTR(a.ctr, a.parity);
    if (nfront + CTR(a.ctr, 8 + a.parity) == 0) return;  // an iteration after the end of the phase
    // the front rays (growing up from 0) and the WALK rays (growing down from rayCap - 1) must not meet:
    // the event and continuous peel-off kernels reserved them independently, so this is the first point
    // where both totals are final; an overflow fails the phase instead of tracing overwritten records
    if ((unsigned long long)nfront + CTR(a.ctr, 8 + a.parity) > (unsigned long long)a.rayCap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.error, ERR_QUEUE);
        return;
    }
    Shared sh = stageTables(a, lds, gridParts<GRID>() | STAGE_OPTICS);

    Tracer<GRID, ONECOMP, CONT, STORE, GLOBAL> T{a, sh};
    T.labsOob = a.labsCopies > 1 ? (unsigned)a.labsCopies * a.labsCopyStride : a.labsBytes;
    T.labsRsrc = __builtin_amdgcn_make_buffer_rsrc(a.labs, 0, (int)T.labsOob, 0x00020000);
    if (a.labsCopies > 1)
        T.copyOff = (unsigned)((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) % (unsigned)a.labsCopies) * a.labsCopyStride;
    // after the grid and optics tables: the segment counts, then the Labs buffers (STORE only)
    T.waveSegs = reinterpret_cast<unsigned*>(lds + a.ldsInstrOff);
    T.pendVal = lds + a.ldsInstrOff + kSegWords;
    T.pendIdx = reinterpret_cast<unsigned*>(T.pendVal + kLabsBuf * kBlock);
    T.pendHi = reinterpret_cast<unsigned char*>(T.pendIdx + kLabsBuf * kBlock);  // (allocated when a.labsHi)
    if (threadIdx.x < 3 * (kBlock / 64)) T.waveSegs[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const unsigned int nrays = nfront + CTR(a.ctr, 8 + a.parity);
    Ray r;
    r.mode = RAY_NONE;
    bool done = false;
    // the wave reserves queue ids kPullChunk at a time and hands them to its idle lanes; the next
    // reservation is requested while the current one still lasts, so a pull rarely waits for the atomic
    // (128 on the tree and Cartesian grids: C3 +0.5 %, C2 +1.2 %; 64 on Voronoi grids, C4 -0.2 % at 128;
    // 256 is slower on all, profiles/r05_pull_chunk_ab.txt)
    constexpr unsigned kPullChunk = GRID == SKIRT_GRID_VORONOI ? 64 : 128;
    unsigned cur = 0, curEnd = 0, nxt = 0;
    bool haveNext = false;
    auto reserve = [&]() {
        unsigned int base = 0;
        if (lane == 0) base = atomicAdd(CTRP(a.ctr, 4), kPullChunk);
        return __shfl(base, 0);
    };
    while (true) {
        const bool idle = (r.mode == RAY_NONE) && !done;
        const unsigned long long imask = __ballot(idle);
        const unsigned long long amask = __ballot(r.mode != RAY_NONE);
        if (imask == 0 && amask == 0) break;
        if (imask != 0 && (amask == 0 || __popcll(imask) >= a.threshold)) {
            const unsigned int rank = (unsigned int)__popcll(imask & ((1ull << lane) - 1ull));
            const unsigned int k = (unsigned int)__popcll(imask);
            const unsigned int avail = curEnd - cur;
            if (avail < k && !haveNext) { nxt = reserve(); haveNext = true; }
            const unsigned int id = rank < avail ? cur + rank : nxt + (rank - avail);
            if (avail >= k) cur += k;
            else { cur = nxt + (k - avail); curEnd = nxt + kPullChunk; haveNext = false; }
            if (!haveNext && curEnd - cur < kPullChunk / 2 && cur < nrays) { nxt = reserve(); haveNext = true; }
            if (idle) {
                if (id >= nrays) done = true;
                else T.load(r, id < nfront ? id : (unsigned)a.rayCap - 1u - (id - nfront));  // a RAY_NONE record (empty path) leaves the lane idle
            }
            // vmcnt(0) here, on the pull's path: without it the waitcnt pass put one at the join with the steps,
            // where a while-iteration without a pull then also waited for the last step's Labs atomic (C2 +1-2 %,
            // C3, C4, C5 within the spread; profiles/r06_pull_wait_ab.txt)
            __builtin_amdgcn_s_waitcnt(0x0F70);
        }
#pragma unroll 1
        for (int it = 0; it < kStepsPerPull; it++) {
            const unsigned long long live = __ballot(r.mode != RAY_NONE);
            if (live == 0) break;
            T.laneSlots += 64;
            auto seg = [&](int m, double rho0, double ds) { return T.segment(r, m, rho0, ds); };
            if (r.mode != RAY_NONE) {
                if (!Grid<GRID>::step(a, sh, r, seg)) {
                    T.finish(r);
                    r.mode = RAY_NONE;
                }
            }
            if constexpr (!STORE) {
            } else if constexpr (kSegsPerStep<GRID> == 1) {
                T.drainStep();  // one drain instruction per step
            } else if (SKIRT_VOR_DRAIN2) {
                static_assert(kSegsPerStep<GRID> == 2, "two drains per step hold two adds per step");
                T.drainStep2();
            } else {
                // a buffer without room for another step's adds: issue the wave's adds
                if (__ballot(T.npend > kLabsBuf - kSegsPerStep<GRID>)) T.drain();
            }
        }
    }
    if constexpr (STORE) T.drain();
    // (wave totals: lane 0 contributes them)
    const unsigned* ws = T.waveSegs + (threadIdx.x >> 6) * 3;
    const bool l0 = lane == 0;
    const unsigned long long vals[8] = {0, l0 ? ws[0] : 0u, l0 ? ws[1] : 0u, l0 ? ws[2] : 0u, 0,
                                        l0 ? T.absorbs : 0u, l0 ? T.laneSlots : 0u, l0 ? T.requests : 0u};
    flushStats(a, vals);
}

template <int GRID, bool ONECOMP, bool CONT, bool GLOBAL = false>
__global__ void __launch_bounds__(kBlock) SKIRT_TRACE_ATTR traceKernel(const Args a) {
    traceBody<GRID, ONECOMP, CONT, true, GLOBAL>(a);
}

// a phase that stores no absorption (the dust emission phase), one component, no continuous scattering:
// without the Labs buffers' LDS and registers, at 4 waves per SIMD
template <int GRID>
__global__ void __launch_bounds__(kBlock) SKIRT_NOSTORE_TRACE_ATTR traceKernelNoStore(const Args a) {
    traceBody<GRID, true, false, false>(a);
}

// the Voronoi walk at its own occupancy (SKIRT_VOR_TRACE_ATTR)
template <bool ONECOMP, bool CONT, bool GLOBAL = false>
__global__ void __launch_bounds__(kBlock) SKIRT_VOR_TRACE_ATTR traceKernelVor(const Args a) {
    traceBody<SKIRT_GRID_VORONOI, ONECOMP, CONT, true, GLOBAL>(a);
}

// the detections of this iteration's peel-off rays (their optical depths are in the queue now)
__global__ void __launch_bounds__(kBlock) detectKernel(const Args a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const unsigned int nrays = CTR(a.ctr, 5 + a.parity);  // this iteration's detection records
    if (nrays == 0) return;
    Shared sh = stageTables(a, lds, STAGE_INSTR);
    const int copies = a.detCopies;
    for (int q = threadIdx.x; q < copies * a.nsed; q += blockDim.x) sh.sed[q] = 0.0;
    __syncthreads();
    unsigned int detects = 0;
    // eight lanes per ray, one per instrument slot (mod 8): the frame adds of one detection fall in one
    // 64-byte line (frameAt) and leave in one wave instruction, so they share one atomic request. Each
    // group of 8 lanes sums SEDs into its own LDS copy (up to 8 copies, as many as the LDS holds): the 8
    // rays of an instruction mostly hit the same few (slot, wavelength) sums, which one copy would
    // serialize. Without room for one copy (very many wavelengths x slots) the SED adds go to the tally.
    const int lane = threadIdx.x & 63, sub = lane & 7;
    double* sed = copies ? sh.sed + ((lane >> 3) & (copies - 1)) * a.nsed : nullptr;
    const unsigned int waves = gridDim.x * (blockDim.x / 64);
    const unsigned int wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    for (unsigned int base = wave * 8; base < nrays; base += waves * 8) {
        const unsigned int id = base + (lane >> 3);
        if (id >= nrays) continue;
        const DetRec d = a.det[id];
        const unsigned flags = d.flags;
        const DevInstr& ins = sh.instr[rayInstr(flags)];
        const int l = d.l, ell = rayEll(flags);
        const double Lp = d.Lp, Lextf = Lp * exp(-d.tau);
        for (int slot = sub; slot < ins.nslots; slot += 8) {
            double v;
            if (!detectSlot(ins, flags, slot, Lp, Lextf, v)) continue;
            if (ins.kind != SKIRT_INSTR_FRAME) {
                if (sed) atomicAdd(&sed[ins.sedOff + slot * a.nlambda + ell], v);
                else atomicAddF64(a.tally + ins.sedBase + slot * a.nlambda + ell, v);
            }
            if (l >= 0 && ins.kind != SKIRT_INSTR_SED) atomicAddF64(frameAt(a, ins, ell, l, slot), v);
        }
        if (sub == 0) detects++;
    }
    // flush the per-workgroup SED sums
    __syncthreads();
    for (int q = threadIdx.x; copies && q < a.nsed; q += blockDim.x) {
        double v = 0.0;
        for (int g = 0; g < copies; g++) v += sh.sed[g * a.nsed + q];
        if (v != 0.0) {
            int ii = 0;
            while (ii + 1 < a.ninstr && sh.instr[ii + 1].sedOff <= q) ii++;
            atomicAddF64(a.tally + sh.instr[ii].sedBase + (q - sh.instr[ii].sedOff), v);
        }
    }
    const unsigned long long vals[8] = {0, 0, 0, 0, detects, 0, 0, 0};
    flushStats(a, vals);
}

// ================================================================== event kernel
struct Packet {
    double rx, ry, rz, kx, ky, kz, L, Lth;
    int ell, nscatt, stellar, state;
    PacketRng rng;
};

template <int GRID, bool ONECOMP>
struct Events {
    const Args& a;
    const Shared& sh;
    unsigned int packets = 0, detects = 0, segFill = 0, segWalk = 0, segPeel = 0;

    __device__ __forceinline__ double rho(int m, int h) const { return a.rho[(size_t)m * a.ncomp + h]; }

    // queues ray `pos`. The trace kernel enters the grid, except for Voronoi grids (kEnterInEvent): their
    // cellIndex loops over a block's site list, which costs the trace kernel more than it costs here. A
    // path found empty here (no dust system, or a Voronoi ray missing the grid) is finished here.
    __device__ __forceinline__ void emitRay(unsigned pos, const Packet& p, double dx, double dy, double dz, double prm,
                                            int idx, unsigned flags, int& vcell) {
        Ray r;
        r.x = p.rx; r.y = p.ry; r.z = p.rz;
        r.dx = dx; r.dy = dy; r.dz = dz;
        r.ix = (fabs(dx) > 1e-15) ? 1.0 / dx : 0.0;
        r.iy = (fabs(dy) > 1e-15) ? 1.0 / dy : 0.0;
        r.iz = (fabs(dz) > 1e-15) ? 1.0 / dz : 0.0;
        r.s = 0;
        r.ci = r.cj = 0;
        const unsigned mode = rayMode(flags);
        int4* dst = reinterpret_cast<int4*>(a.rays + pos);
        bool entered = a.hasDust;
        unsigned nseg = 0;
        if constexpr (kEnterInEvent<GRID>) {
            if (entered) entered = Grid<GRID>::beginAt(a, r, vcell, [&](int, double, double ds) {
                if (ds > 0) { r.s += ds; nseg++; }  // outside the grid: no optical depth
                return true;
            });
            // (the trace kernel counts them with the ray's other segments: they travel in the record)
        }
        if (kEnterInEvent<GRID> && a.crossed && mode != RAY_WALK && a.hasDust) {
            if (!entered) crossedAdd(a, 0);  // (a path that misses the grid has no segments)
        }
        if (!entered) {
            if (mode != RAY_PEEL) {  // a peel-off's detection record already holds tau = 0
                a.resA[idx] = 0.0;  // FILL: tau = 0 (and no scattered luminosity); WALK: s = 0
                if (!ONECOMP) a.resB[idx] = 0.0;
                if (mode == RAY_FILL && a.continuous) a.pathCnt[idx] = 0;  // an empty path: no dust segments
            }
            dst[4] = make_int4(idx, (int)RAY_NONE, 0, 0);
            return;
        }
        double2* d2 = reinterpret_cast<double2*>(dst);
        d2[0] = make_double2(r.x, r.y);
        d2[1] = make_double2(r.z, dx);
        d2[2] = make_double2(dy, dz);
        d2[3] = make_double2(r.s, prm);
        // (the segments before the grid, for the cells-crossed histogram, in the first cell's top bits)
        dst[4] = make_int4(idx, (int)flags, r.ci | (int)(min(nseg, 7u) << kOutsideShift), r.cj);
    }

    __device__ __forceinline__ void load(int s, Packet& p) const {
        p.rx = a.srx[s]; p.ry = a.sry[s]; p.rz = a.srz[s];
        p.kx = a.skx[s]; p.ky = a.sky[s]; p.kz = a.skz[s];
        p.L = a.sL[s]; p.Lth = a.sLth[s];
        p.ell = a.sell[s]; p.nscatt = a.snscatt[s]; p.stellar = a.sstellar[s]; p.state = a.sstate[s];
        p.rng.k0 = (uint32_t)a.seed; p.rng.k1 = (uint32_t)(a.seed >> 32); p.rng.tag = a.tag;
        p.rng.plo = a.splo[s]; p.rng.phi = a.sphi[s]; p.rng.block = a.sblock[s];
        p.rng.w2 = a.sw2[s]; p.rng.w3 = a.sw3[s]; p.rng.have = a.shave[s];
    }
    __device__ __forceinline__ void store(int s, const Packet& p) const {
        a.srx[s] = p.rx; a.sry[s] = p.ry; a.srz[s] = p.rz;
        a.skx[s] = p.kx; a.sky[s] = p.ky; a.skz[s] = p.kz;
        a.sL[s] = p.L; a.sLth[s] = p.Lth;
        a.sell[s] = p.ell; a.snscatt[s] = p.nscatt; a.sstellar[s] = p.stellar; a.sstate[s] = p.state;
        a.splo[s] = p.rng.plo; a.sphi[s] = p.rng.phi; a.sblock[s] = p.rng.block;
        a.sw2[s] = p.rng.w2; a.sw3[s] = p.rng.w3; a.shave[s] = p.rng.have;
    }

    __device__ __forceinline__ int pixel(const DevInstr& ins, const Packet& p) const {
        // SingleFrameInstrument::pixelondetector (SingleFrameInstrument.cpp:130-147)
        const double xpp = -ins.sinphi * p.rx + ins.cosphi * p.ry;
        const double ypp = -ins.cosphi * ins.costheta * p.rx - ins.sinphi * ins.costheta * p.ry + ins.sintheta * p.rz;
        const double xp = ins.cospa * xpp - ins.sinpa * ypp;
        const double yp = ins.sinpa * xpp + ins.cospa * ypp;
        const int i = static_cast<int>(floor((xp - ins.xpmin) / ins.xpsiz));
        const int j = static_cast<int>(floor((yp - ins.ypmin) / ins.ypsiz));
        return (i < 0 || i >= ins.nx || j < 0 || j >= ins.ny) ? -1 : i + ins.nx * j;
    }

    // weight of the scattering peel-off towards instrument `ins` (MonteCarloSimulation.cpp:319-363,
    // unpolarized; Henyey-Greenstein value DustMix.cpp:665-669); false aborts the peel-off
    __device__ __forceinline__ bool peelWeight(const DevInstr& ins, const Packet& p, double kx, double ky, double kz,
                                               double& I) const {
        const double cosalpha = kx * ins.kobs[0] + ky * ins.kobs[1] + kz * ins.kobs[2];
        if (ONECOMP) {
            const double g = sh.g[p.ell];
            const double t = 1.0 + g * g - 2 * g * cosalpha;
            I = 0.0 + (1.0 * ((1.0 - g) * (1.0 + g) / sqrt(t * t * t))) * 1.0;
            return true;
        }
        const int m = Grid<GRID>::whichcell(a, sh, p.rx, p.ry, p.rz);
        if (m == -1) return false;
        double sum = 0;
        for (int h = 0; h < a.ncomp; h++) sum += sh.ksca[h * a.nlambda + p.ell] * rho(m, h);
        if (sum <= 0) return false;
        I = 0;
        for (int h = 0; h < a.ncomp; h++) {
            const double wv = sh.ksca[h * a.nlambda + p.ell] * rho(m, h) / sum;
            const double g = sh.g[h * a.nlambda + p.ell];
            const double t = 1.0 + g * g - 2 * g * cosalpha;
            I += (wv * ((1.0 - g) * (1.0 + g) / sqrt(t * t * t))) * 1.0;
        }
        return true;
    }

    // Instrument::detect without a dust system (tau = 0): FullInstrument then holds only the
    // transparent arrays (FullInstrument.cpp:58-60, 115-120)
    __device__ __forceinline__ void detectNow(const DevInstr& ins, const Packet& p, double Lp, int l) {
        detects++;
        if (ins.kind != SKIRT_INSTR_FRAME) atomicAddF64(a.tally + ins.sedBase + p.ell, Lp);
        if (l >= 0 && ins.kind != SKIRT_INSTR_SED) atomicAddF64(frameAt(a, ins, p.ell, l, 0), Lp);
    }

    // SpecialFunctions::LambertW1 (SpecialFunctions.cpp:579-626), the W_{-1} branch; as the host's
    // lambertW1 (host/build.cpp), whose argument checks the callers here never fail
    __device__ static double lambertW1(double z) {
        const double eps = 1.0e-12;
        const double em1 = 0.3678794411714423215955237701614608;
        if (z == 0.0) return -kDblMax;
        const double q = z + em1;
        const double r = -sqrt(q);
        const double t8 = -8.401032217523977370984161688514 +
                          r * (12.250753501314460424 + r * (-18.100697012472442755 + r * 27.029044799010561650));
        const double t5 = 3.066858901050631912893148922704 +
                          r * (-4.175335600258177138854984177460 + r * (5.858023729874774148815053846119 + r * t8));
        const double t1 = 2.331643981597124203363536062168 +
                          r * (-1.812187885639363490240191647568 +
                               r * (1.936631114492359755363277457668 + r * (-2.353551201881614516821543561516 + r * t5)));
        const double w0 = -1.0 + r * t1;
        if (q < 3.0e-3) return w0;
        double w;
        if (z < -1e-6) {
            w = w0;
        } else {
            const double l1 = log(-z);
            const double l2 = log(-l1);
            w = l1 - l2 + l2 / l1;
        }
        for (int i = 0; i < 10; i++) {  // Halley iteration
            const double e = exp(w);
            double t = w * e - z;
            const double p = w + 1.0;
            t /= e * p - 0.5 * (p + 1.0) * t / p;
            w -= t;
            if (fabs(t) < eps * (1.0 + fabs(w))) break;
        }
        return w;
    }

    // ExpDiskGeometry::randomR / randomz and SepAxGeometry::generatePosition (R, phi = 2 pi u, z;
    // Position(R, phi, z, CYLINDRICAL)); gp = {hR, hz, Rmax, zmax, Rmin, rho0, 0, kind}
    __device__ __forceinline__ void expDiskPosition(PacketRng& rng, const double* gp, double& x, double& y,
                                                    double& z) const {
        const double hR = gp[0], hz = gp[1], Rmax = gp[2], zmax = gp[3], Rmin = gp[4];
        double R, X;
        do {
            X = rng.uniform();
            R = hR * (-1.0 - lambertW1((X - 1.0) / M_E));
        } while ((Rmax > 0.0 && R >= Rmax) || R <= Rmin);
        const double phi = 2.0 * M_PI * rng.uniform();
        double zz;
        do {
            X = rng.uniform();
            zz = (X <= 0.5) ? hz * log(2.0 * X) : -hz * log(2.0 * (1.0 - X));
        } while (zmax > 0.0 && fabs(zz) >= zmax);
        x = R * cos(phi);
        y = R * sin(phi);
        z = zz;
    }

    // Random::direction() (Random.cpp:179-184): theta = acos(2u-1), phi = 2 pi u', evaluated as
    // cos(theta) = 2u-1, sin(theta) = sqrt(1-cos^2) and sin/cos(2 pi u') = sinpi/cospi(2u') -- the
    // same values to rounding, without acos or a large-argument reduction. The reference's 1e-8
    // pole cut-offs in Direction(theta, phi) are never reached by a deviate in (0,1).
    __device__ __forceinline__ void isotropic(PacketRng& rng, double& x, double& y, double& z) const {
        const double ct = 2.0 * rng.uniform() - 1.0;
        const double u = rng.uniform();
        const double st = sqrt((1.0 - ct) * (1.0 + ct));
        double sp, cp;
        sincospi(2.0 * u, &sp, &cp);
        x = st * cp; y = st * sp; z = ct;
    }

    // simulatescattering: DustSystem::randomMixForPosition + DustMix::scatteringDirectionAndPolarization
    // (HG, DustMix.cpp:609-613) + Random::direction(k, costheta) (Random.cpp:188-222)
    __device__ __forceinline__ void scatter(Packet& p) const {
        int hmix = 0;
        if (!ONECOMP) {
            const int m = Grid<GRID>::whichcell(a, sh, p.rx, p.ry, p.rz);
            if (m >= 0) {
                double Xv[9];
                Xv[0] = 0.0;
                for (int h = 0; h < a.ncomp; h++) Xv[h + 1] = Xv[h] + sh.ksca[h * a.nlambda + p.ell] * rho(m, h);
                const double norm = Xv[a.ncomp];
                const double X = p.rng.uniform();
                for (int h = 1; h < a.ncomp; h++)
                    if (Xv[h] / norm <= X) hmix = h;
            }
        }
        const double g = sh.g[hmix * a.nlambda + p.ell];
        double nx, ny, nz;
        if (fabs(g) < 1e-6) {
            isotropic(p.rng, nx, ny, nz);
        } else {
            const double f = ((1.0 - g) * (1.0 + g)) / (1.0 - g + 2.0 * g * p.rng.uniform());
            const double costheta = (1.0 + g * g - f * f) / (2.0 * g);
            double sinphi, cosphi;  // phi = 2 pi u (Random.cpp:190), as sinpi/cospi(2u)
            sincospi(2.0 * p.rng.uniform(), &sinphi, &cosphi);
            const double sintheta = sqrt(fabs((1.0 - costheta) * (1.0 + costheta)));
            const double kx = p.kx, ky = p.ky, kz = p.kz;
            if (kz > 0.99999) { nx = cosphi * sintheta; ny = sinphi * sintheta; nz = costheta; }
            else if (kz < -0.99999) { nx = cosphi * sintheta; ny = sinphi * sintheta; nz = -costheta; }
            else {
                const double root = sqrt((1.0 - kz) * (1.0 + kz));
                nx = sintheta / root * (-kx * kz * cosphi + ky * sinphi) + kx * costheta;
                ny = -sintheta / root * (ky * kz * cosphi + kx * sinphi) + ky * costheta;
                nz = root * sintheta * cosphi + kz * costheta;
            }
        }
        p.nscatt++;
        p.kx = nx; p.ky = ny; p.kz = nz;
    }

    // false when no packet results (wavelength without luminosity, or a selected component without
    // luminosity)
    __device__ __forceinline__ bool launch(Packet& p, unsigned long long idx) {
        return a.phase == SKIRT_PHASE_STELLAR ? launchStellar(p, idx) : launchCell(p, idx);
    }

    // the launch of dodustemissionchunk (biased cell choice, PanMonteCarloSimulation.cpp:296-325) and of
    // dodustselfabsorptionchunk (natural choice, :207-216): a cell, a uniform position in its box
    // (Random::position, Random.cpp:226-234), an isotropic direction; a dust packet (stellar = -1)
    __device__ __forceinline__ bool launchCell(Packet& p, unsigned long long idx) {
        const int ell = (int)(idx / a.npp);
        const double Ltot = a.cellLtot[ell];
        if (!(Ltot > 0)) return false;  // the chunk emits nothing at this wavelength
        packets++;
        const double L0 = Ltot / (double)a.npp;
        p.Lth = L0 / a.minWeightReduction;
        p.rng.start(a.seed, a.tag, idx);
        p.ell = ell;
        const int N = a.ncells;
        const double* cdf = a.cellCdf + (size_t)ell * (N + 1);
        const int* guide = a.cellGuide + (size_t)ell * (N + 1);
        const double X = p.rng.uniform();
        int m;
        double L = L0;
        if (a.phase == SKIRT_PHASE_DUST_EMISSION) {
            const double xi = a.cellBias;
            if (X < xi) m = max(0, min(N - 1, static_cast<int>(N * X / xi)));
            else m = locateGuided(cdf, guide, N, (X - xi) / (1 - xi));
            const double Lmean = Ltot / N;
            const double weight = 1.0 / (1 - xi + xi * Lmean / a.cellLv[(size_t)ell * N + m]);
            L = L0 * weight;
        } else {
            m = locateGuided(cdf, guide, N, X);
        }
        if (GRID == SKIRT_GRID_VORONOI) m = a.devCell[m];  // the Voronoi arrays are in device order
        double b[6];
        cellBox(m, b);
        // VoronoiMesh::randomPosition: points in the enclosing box until one lies in the cell
        for (int trial = 0; trial < (GRID == SKIRT_GRID_VORONOI ? 10000 : 1); trial++) {
            const double x = p.rng.uniform();
            const double y = p.rng.uniform();
            const double z = p.rng.uniform();
            p.rx = b[0] + x * (b[3] - b[0]);
            p.ry = b[1] + y * (b[4] - b[1]);
            p.rz = b[2] + z * (b[5] - b[2]);
            if (GRID != SKIRT_GRID_VORONOI || Grid<SKIRT_GRID_VORONOI>::closestTo(a, p.rx, p.ry, p.rz, m)) break;
        }
        isotropic(p.rng, p.kx, p.ky, p.kz);
        p.L = L;
        p.nscatt = 0;
        p.stellar = -1;
        return true;
    }

    // NR::locate_clip over a table in global memory
    __device__ static __forceinline__ int locateClipGlobal(const double* v, int n, double q) {
        if (q < v[0]) return 0;
        int jl = -1, ju = n - 1;
        while (ju - jl > 1) {
            const int jm = (ju + jl) >> 1;
            if (q < v[jm]) ju = jm;
            else jl = jm;
        }
        return jl;
    }

    // the box of cell m (CartesianDustGrid::box, TreeDustGrid::getnode(m)->extent()): reference cell
    // numbers, except the Voronoi grid's device numbers
    __device__ __forceinline__ void cellBox(int m, double (&b)[6]) const {
        if (GRID == SKIRT_GRID_CARTESIAN) {
            const double* xv = sh.mesh;
            const double* yv = xv + a.nx + 1;
            const double* zv = yv + a.ny + 1;
            const int i = m / (a.nz * a.ny), j = (m / a.nz) % a.ny, k = m % a.nz;
            b[0] = xv[i]; b[1] = yv[j]; b[2] = zv[k]; b[3] = xv[i + 1]; b[4] = yv[j + 1]; b[5] = zv[k + 1];
        } else if (GRID == SKIRT_GRID_VORONOI) {
            for (int q = 0; q < 6; q++) b[q] = a.cellBbox[6 * (size_t)m + q];
        } else {
            const double* bx = a.box + 6 * (size_t)a.cellNode[m];
            for (int q = 0; q < 6; q++) b[q] = bx[q];
        }
    }

    // StellarSystem::launch + GeometricStellarComp::launch + PlummerGeometry sampling (see below)
    __device__ __forceinline__ bool launchStellar(Packet& p, unsigned long long idx) {
        const int ell = (int)(idx / a.npp);
        const double L0 = a.lumtot[ell] / (double)a.npp;
        if (!(L0 > 0)) return false;  // dostellaremissionchunk skips such wavelengths
        packets++;
        p.Lth = L0 / a.minWeightReduction;
        p.rng.start(a.seed, a.tag, idx);
        p.ell = ell;
        int h = 0;
        double L = L0;
        const int N = a.nstar;
        if (N > 1) {
            const double X = p.rng.uniform();
            const double xi = a.emissionBias;
            if (X < xi) h = max(0, min(N - 1, static_cast<int>(N * X / xi)));
            else {
                const double* Xv = a.cdf + (size_t)ell * (N + 1);
                const double q = (X - xi) / (1.0 - xi);
                if (!(q < Xv[0])) {
                    int lo = -1, hi = N;
                    while (hi - lo > 1) { const int jm = (hi + lo) >> 1; if (q < Xv[jm]) hi = jm; else lo = jm; }
                    h = lo;
                }
            }
            const double Lh = a.lum[(size_t)h * a.nlambda + ell];
            if (!(Lh > 0)) return false;
            const double Lmean = a.lumtot[ell] / N;
            L = L0 * (1.0 / (1.0 - xi + xi * Lmean / Lh));
        }
        const double* gp = a.geomParam + 8 * h;
        if ((int)gp[7] == SKIRT_GEOM_POINT) {
            p.rx = 0.0; p.ry = 0.0; p.rz = 0.0;  // PointGeometry::generatePosition: no draws
        } else if ((int)gp[7] == SKIRT_GEOM_EXPDISK) {
            expDiskPosition(p.rng, gp, p.rx, p.ry, p.rz);
        } else if ((int)gp[7] == SKIRT_GEOM_SERSIC) {
            // SersicGeometry::randomradius (SersicFunction::inversemass: locate_clip + log-log
            // interpolation of the cumulative mass table) and SpheGeometry::generatePosition
            const double* sv = a.geomTable + (size_t)kSersicTable * h;
            const double* Mv = sv + kSersicTable / 2;
            constexpr int Ns = kSersicTable / 2;
            const double M = p.rng.uniform();
            double sr;
            if (M <= Mv[0]) sr = sv[0];
            else if (M >= Mv[Ns - 1]) sr = sv[Ns - 1];
            else {
                int jl = -1, ju = Ns - 1;  // NR::locate_clip
                while (ju - jl > 1) { const int jm = (ju + jl) >> 1; if (M < Mv[jm]) ju = jm; else jl = jm; }
                sr = interpolateLogLog(M, Mv[jl], Mv[jl + 1], sv[jl], sv[jl + 1]);
            }
            const double rr = gp[0] * sr;
            double ux, uy, uz;
            isotropic(p.rng, ux, uy, uz);
            p.rx = rr * ux; p.ry = rr * uy; p.rz = rr * uz;
        } else {
            // PlummerGeometry::randomradius (t = u^(1/3)) and SpheGeometry::generatePosition
            const double c = gp[0];
            const double t = cbrt(p.rng.uniform());
            const double rr = c * t / sqrt((1.0 - t) * (1.0 + t));
            double ux, uy, uz;
            isotropic(p.rng, ux, uy, uz);
            p.rx = rr * ux; p.ry = rr * uy; p.rz = rr * uz;
        }
        // the emission direction Random::direction()
        isotropic(p.rng, p.kx, p.ky, p.kz);
        p.L = L;
        p.nscatt = 0;
        p.stellar = h;
        return true;
    }

    // simulatepropagation part 1: the optical depth of the interaction (Random::exponcutoff and the
    // composite biasing with weight p/q, MonteCarloSimulation.cpp:519-534)
    __device__ __forceinline__ double sampleTau(Packet& p, double taupath) const {
        double tauint = -1.0;
        if (a.xi != 0.0) {
            const double X = p.rng.uniform();
            if (X < a.xi) tauint = p.rng.uniform() * taupath;
        }
        if (tauint < 0.0) {
            if (taupath < 1e-10) tauint = p.rng.uniform() * taupath;
            else {
                const double norm = 1.0 - exp(-taupath);
                double x = -log(1.0 - p.rng.uniform() * norm);
                while (x > taupath) x = -log(1.0 - p.rng.uniform() * norm);
                tauint = x;
            }
        }
        if (a.xi != 0.0) {
            const double pr = -exp(-tauint) / expm1(-taupath);
            const double q = (1.0 - a.xi) * pr + a.xi / taupath;
            p.L = p.L * (pr / q);
        }
        return tauint;
    }
};

// peel-off set queued by a slot in this iteration
enum PeelKind : int { PEEL_NONE = 0, PEEL_EMISSION = 1, PEEL_SCATTER = 2 };

// Block-wide reservation on shared counters: every thread of the block calls it with its counts c0, c1
// (either may be 0); one atomic per counter per block (a device-wide counter serializes its
// atomics, so one per block instead of one per wave) returns each thread's first index in r0, r1.
// wave totals and the block's bases go through `scratch` (static LDS, 2 * (kBlock / 64) + 2 words).
template <class T0, class T1>
__device__ __forceinline__ void blockReserve(T0* ctr0, T0 c0, T0& r0, T1* ctr1, T1 c1, T1& r1, unsigned long long* scratch) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int W = kBlock / 64;
    T0 i0 = c0;
    T1 i1 = c1;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T0 v0 = __shfl_up(i0, off);
        const T1 v1 = __shfl_up(i1, off);
        if (lane >= off) { i0 += v0; i1 += v1; }
    }
    if (lane == 63) { scratch[wave] = (unsigned long long)i0; scratch[W + wave] = (unsigned long long)i1; }
    __syncthreads();
    T0 w0 = 0, t0 = 0;
    T1 w1 = 0, t1 = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
        const T0 s0 = (T0)scratch[w];
        const T1 s1 = (T1)scratch[W + w];
        if (w < wave) { w0 += s0; w1 += s1; }
        t0 += s0; t1 += s1;
    }
    if (threadIdx.x == 0) scratch[2 * W] = (ctr0 && t0) ? (unsigned long long)atomicAdd(ctr0, t0) : 0ull;
    if (threadIdx.x == 64) scratch[2 * W + 1] = (ctr1 && t1) ? (unsigned long long)atomicAdd(ctr1, t1) : 0ull;
    __syncthreads();
    r0 = (T0)scratch[2 * W] + w0 + i0 - c0;
    r1 = (T1)scratch[2 * W + 1] + w1 + i1 - c1;
    __syncthreads();  // the scratch words are reused by the next call
}

// three counters at once (scratch: 3 * (kBlock / 64) + 3 words)
__device__ __forceinline__ void blockReserve3(unsigned* ctr0, unsigned c0, unsigned& r0, unsigned* ctr1, unsigned c1,
                                              unsigned& r1, unsigned* ctr2, unsigned c2, unsigned& r2,
                                              unsigned long long* scratch) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int W = kBlock / 64;
    unsigned i0 = c0, i1 = c1, i2 = c2;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned v0 = __shfl_up(i0, off), v1 = __shfl_up(i1, off), v2 = __shfl_up(i2, off);
        if (lane >= off) { i0 += v0; i1 += v1; i2 += v2; }
    }
    if (lane == 63) { scratch[wave] = i0; scratch[W + wave] = i1; scratch[2 * W + wave] = i2; }
    __syncthreads();
    unsigned w0 = 0, w1 = 0, w2 = 0, t0 = 0, t1 = 0, t2 = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
        const unsigned s0 = (unsigned)scratch[w], s1 = (unsigned)scratch[W + w], s2 = (unsigned)scratch[2 * W + w];
        if (w < wave) { w0 += s0; w1 += s1; w2 += s2; }
        t0 += s0; t1 += s1; t2 += s2;
    }
    if (threadIdx.x == 0) scratch[3 * W] = t0 ? atomicAdd(ctr0, t0) : 0u;
    if (threadIdx.x == 64) scratch[3 * W + 1] = t1 ? atomicAdd(ctr1, t1) : 0u;
    if (threadIdx.x == 128) scratch[3 * W + 2] = t2 ? atomicAdd(ctr2, t2) : 0u;
    __syncthreads();
    r0 = (unsigned)scratch[3 * W] + w0 + i0 - c0;
    r1 = (unsigned)scratch[3 * W + 1] + w1 + i1 - c1;
    r2 = (unsigned)scratch[3 * W + 2] + w2 + i2 - c2;
    __syncthreads();  // the scratch words are reused by the next call
}

// four counters at once (scratch: 4 * (kBlock / 64) + 4 words); the first lane of wave q issues counter q's atomic
static_assert(kBlock >= 256, "blockReserve4 needs four waves per block");
__device__ __forceinline__ void blockReserve4(unsigned* const (&ctr)[4], const unsigned (&c)[4], unsigned (&r)[4],
                                              unsigned long long* scratch) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int W = kBlock / 64;
    unsigned in[4];
#pragma unroll
    for (int q = 0; q < 4; q++) in[q] = c[q];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        unsigned v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) v[q] = __shfl_up(in[q], off);
        if (lane >= off) {
#pragma unroll
            for (int q = 0; q < 4; q++) in[q] += v[q];
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int q = 0; q < 4; q++) scratch[q * W + wave] = in[q];
    }
    __syncthreads();
    unsigned w[4] = {0, 0, 0, 0}, t[4] = {0, 0, 0, 0};
#pragma unroll
    for (int ww = 0; ww < W; ww++) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const unsigned sv = (unsigned)scratch[q * W + ww];
            if (ww < wave) w[q] += sv;
            t[q] += sv;
        }
    }
#pragma unroll
    for (int q = 0; q < 4; q++)
        if (threadIdx.x == 64 * q) scratch[4 * W + q] = t[q] ? atomicAdd(ctr[q], t[q]) : 0u;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; q++) r[q] = (unsigned)scratch[4 * W + q] + w[q] + in[q] - c[q];
    __syncthreads();  // the scratch words are reused by the next call
}

// Global packet index of the j-th packet of this call. A sharded call (IdenticalAssigner,
// IdenticalAssigner.cpp:37-58: every process runs its block of chunks at every wavelength) shoots
// packets [sliceLo, sliceLo + sliceCnt) of each wavelength; the Philox stream is keyed on the global
// index, so the packets are the same whatever the number of ranks.
__device__ __forceinline__ unsigned long long globalPacket(const Args& a, unsigned long long j) {
    if (a.sliceCnt == a.npp) return j;
    const unsigned long long ell = j / a.sliceCnt;
    return ell * a.npp + a.sliceLo + (j - ell * a.sliceCnt);
}

template <int GRID, bool ONECOMP>
__global__ void __launch_bounds__(kBlock) SKIRT_EVENT_ATTR eventKernel(const Args a) {
    __shared__ unsigned long long resv[4 * (kBlock / 64) + 4];
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (blockIdx.x == 0 && threadIdx.x == 0) CTR(a.ctr, 4) = 0;  // the trace kernel's pull counter
    if (!a.init && CTR(a.ctr, 2 + a.parity) == 0) return;  // an iteration after the end of the phase
    Shared sh = stageTables(a, lds, gridParts<GRID>() | STAGE_OPTICS | STAGE_INSTR);
    Events<GRID, ONECOMP> E{a, sh};
    const int lane = threadIdx.x & 63;
    const unsigned long long total = a.end - a.first;
    const unsigned int nwork = a.init ? (unsigned)a.nslots : CTR(a.ctr, 2 + a.parity);
    const int* actIn = a.act[a.parity];
    int* actOut = a.act[1 - a.parity];
    const unsigned int stride = gridDim.x * blockDim.x;
    // every lane of a wave runs the same number of rounds (wave-collective claims and appends below)
    const unsigned int rounds = (nwork + stride - 1) / stride;
    // the active-list entry of the lane's next round is loaded a round ahead, so a round's first round trip
    // is its slot's state (and the trace result, loaded with it)
    const unsigned int w0 = blockIdx.x * blockDim.x + threadIdx.x;
    int slotNext = (w0 < nwork) ? (a.init ? (int)w0 : actIn[w0]) : 0;
    for (unsigned int round = 0; round < rounds; round++) {
        const unsigned int w = round * stride + w0;
        const bool valid = w < nwork;
        const int slot = slotNext;
        const unsigned int wn = w + stride;
        if (round + 1 < rounds) slotNext = (wn < nwork) ? (a.init ? (int)wn : actIn[wn]) : 0;
        Packet p;
        p.state = S_NEW;
        double resA = 0.0, resB = 0.0;
        int vcell = kNoCell;  // Voronoi: the cell of the packet's position, while it stays there
        if (valid && !a.init) {
            E.load(slot, p);
            resA = a.resA[slot];
            if (!ONECOMP) resB = a.resB[slot];
            if (kEnterInEvent<GRID>) vcell = a.svcell[slot];
        }
        int peel = PEEL_NONE;
        unsigned mainMode = RAY_NONE;
        double mainParam = 0;
        double ox = 0, oy = 0, oz = 0;  // direction before scattering (peel-off weights)
        if (valid && !a.init) {
            if (p.state == S_FILL) {
                // end of fillOpticalDepth + simulateescapeandabsorption; termination; simulatepropagation
                const double taupath = resA;
                if (taupath < 0.0 || isnan(taupath) || isinf(taupath)) {
                    atomicOr(a.error, ERR_TAU);
                    p.state = S_NEW;
                } else {
                    if (ONECOMP) p.L = p.L * sh.alb[p.ell] * (-expm1(-taupath));
                    else p.L = resB;
                    if (p.L <= 0 || (p.L <= p.Lth && p.nscatt >= a.minScatt)) {
                        p.state = S_NEW;
                    } else {
                        p.state = S_WALK;
                        double tauint = 0.0;  // taupath == 0: no propagation (MonteCarloSimulation.cpp:522)
                        if (taupath != 0.0) tauint = E.sampleTau(p, taupath);
                        if (tauint > 0) { mainMode = RAY_WALK; mainParam = tauint; }
                        else resA = 0.0;  // no walk: the interaction point is where the packet is
                    }
                }
            }
            if (p.state == S_WALK && mainMode == RAY_NONE) {
                // propagate to the interaction point; peel-off round; scatter; next FILL
                const double s = resA;
                vcell = kNoCell;  // the packet moves
                p.rx = p.rx + s * p.kx;
                p.ry = p.ry + s * p.ky;
                p.rz = p.rz + s * p.kz;
                // peeloffscattering, unless the continuous peel-off replaces it (MonteCarloSimulation.cpp:291)
                bool ok = a.ninstr > 0 && a.peel && !a.continuous;
                if (ok && !ONECOMP) { double I; ok = E.peelWeight(sh.instr[0], p, p.kx, p.ky, p.kz, I); }
                if (ok) { peel = PEEL_SCATTER; ox = p.kx; oy = p.ky; oz = p.kz; }
                E.scatter(p);
                mainMode = RAY_FILL;
                mainParam = p.L;
                p.state = S_FILL;
            }
        }
        // slots without a packet claim the next global packet indices (one atomic per block)
        bool need = valid && p.state == S_NEW && mainMode == RAY_NONE;
        while (__syncthreads_or(need)) {
            unsigned long long idx = 0;
            unsigned int unused = 0;
            blockReserve<unsigned long long, unsigned int>(a.claim, need ? 1ull : 0ull, idx, nullptr, 0u, unused, resv);
            if (need) {
                if (idx >= total) need = false;  // exhausted: the slot retires
                else if (E.launch(p, globalPacket(a, a.first + idx))) {
                    vcell = kNoCell;  // a new position
                    if (!(p.L > 0) && !a.crossed) {
                        // a zero-weight dust packet (a cell without emission drawn uniformly): every
                        // tally it would touch receives 0, so it ends here -- unless the cells-crossed
                        // statistics are on: the reference still traces its paths (dodustemissionchunk,
                        // PanMonteCarloSimulation.cpp:316-329), which count in ds_crossed
                    } else if (a.hasDust) {
                        peel = (a.ninstr > 0 && a.peel) ? PEEL_EMISSION : PEEL_NONE;
                        mainMode = RAY_FILL;
                        mainParam = p.L;
                        p.state = S_FILL;
                        need = false;
                    } else {
                        // no dust system: tau = 0 for every peel-off and the packet ends here
                        for (int i = 0; i < a.ninstr; i++) {
                            const DevInstr& ins = sh.instr[i];
                            const int l = ins.kind == SKIRT_INSTR_SED ? -1 : E.pixel(ins, p);
                            if (ins.kind == SKIRT_INSTR_FRAME && l < 0) continue;
                            E.detectNow(ins, p, p.L, l);
                        }
                    }
                }
            }
        }
        // rays this lane queues: its peel-offs and its next FILL/WALK ray
        int nray = 0;
        if (peel != PEEL_NONE) {
            for (int i = 0; i < a.ninstr; i++) {
                const DevInstr& ins = sh.instr[i];
                if (ins.kind == SKIRT_INSTR_FRAME && E.pixel(ins, p) < 0) continue;
                nray++;
            }
        }
        if (mainMode != RAY_NONE) nray++;
        // the queue space of the block's rays, the slots staying active and the detection records of
        // the peel-offs: one atomic each per block
        const bool active = mainMode != RAY_NONE;
        const int npeel = nray - (mainMode != RAY_NONE ? 1 : 0);
        // a WALK ray goes to the top of the queue (Args::walkBack)
        const bool back = a.walkBack && mainMode == RAY_WALK;
        unsigned int pos, apos, dpos, wpos;
        {
            unsigned* const ctrs[4] = {CTRP(a.ctr, a.parity), CTRP(a.ctr, 2 + (1 - a.parity)), CTRP(a.ctr, 5 + a.parity),
                                       CTRP(a.ctr, 8 + a.parity)};
            const unsigned cnt[4] = {(unsigned)nray - (back ? 1u : 0u), active ? 1u : 0u, (unsigned)npeel, back ? 1u : 0u};
            unsigned res[4];
            blockReserve4(ctrs, cnt, res, resv);
            pos = res[0]; apos = res[1]; dpos = res[2]; wpos = res[3];
        }
        // the queue holds rayCap records (ensurePool sizes it for the slots' most rays per iteration): a
        // lane whose records would fall outside it writes none and fails the phase (ERR_QUEUE); the trace
        // kernel checks that the front and the WALK region do not meet
        if ((unsigned long long)pos + (unsigned)(nray - (back ? 1 : 0)) > (unsigned long long)a.rayCap ||
            (back && wpos >= (unsigned)a.rayCap) ||
            (unsigned long long)dpos + (unsigned)npeel > (unsigned long long)(a.rayCap - a.nslots)) {
            atomicOr(a.error, ERR_QUEUE);
            nray = 0;
        }
        int inext = 0;  // next instrument to consider for a peel-off
        for (int k = 0; k < nray; k++) {
            double dx, dy, dz, prm;
            int idx;
            unsigned flags, at;
            if (k < npeel) {
                int i = inext, l;
                while (true) {  // the next instrument that receives this peel-off
                    const DevInstr& ins = sh.instr[i];
                    l = ins.kind == SKIRT_INSTR_SED ? -1 : E.pixel(ins, p);
                    if (ins.kind == SKIRT_INSTR_FRAME && l < 0) { i++; continue; }
                    break;
                }
                inext = i + 1;
                const DevInstr& ins = sh.instr[i];
                double Lp = p.L;
                unsigned cat, level = 0;
                if (peel == PEEL_EMISSION) {
                    cat = p.stellar >= 0 ? CAT_STAR_DIRECT : CAT_DUST_DIRECT;
                } else {
                    double I = 0;
                    E.peelWeight(ins, p, ox, oy, oz, I);  // the direction before scattering
                    Lp = p.L * I;
                    cat = p.stellar >= 0 ? CAT_STAR_SCATTERED : CAT_DUST_SCATTERED;
                    level = (unsigned)min(p.nscatt, 255);  // nscatt already counts this scattering
                }
                dx = ins.kobs[0]; dy = ins.kobs[1]; dz = ins.kobs[2];
                prm = Lp;
                flags = RAY_PEEL | (cat << 2) | ((unsigned)i << 4) | (level << 10) | ((unsigned)p.ell << 18);
                // its detection record (the trace kernel adds the optical depth; a path that misses the
                // grid leaves tau = 0)
                idx = (int)(dpos + k);
                a.det[idx] = DetRec{Lp, 0.0, l, flags};
                at = pos++;
            } else {
                dx = p.kx; dy = p.ky; dz = p.kz;
                prm = mainParam;
                idx = slot;
                flags = mainMode | ((unsigned)p.ell << 18);
                at = back ? (unsigned)a.rayCap - 1u - wpos : pos++;
            }
            E.emitRay(at, p, dx, dy, dz, prm, idx, flags, vcell);  // (one call site: one inlined grid entry)
        }
        // the slot stays active while it has a FILL/WALK ray in flight
        if (active) actOut[apos] = slot;
        if (valid) E.store(slot, p);
        if (kEnterInEvent<GRID> && valid) a.svcell[slot] = vcell;
    }
    const unsigned long long vals[8] = {E.packets, E.segFill, E.segWalk, E.segPeel, E.detects, 0, 0, 0};
    flushStats(a, vals);
}

// MonteCarloSimulation::continuouspeeloffscattering (MonteCarloSimulation.cpp:367-434), unpolarized. Runs
// before the event kernel of an iteration: every slot whose FILL ray just returned peels off, from a
// uniformly drawn point of every recorded path segment with scattering dust, toward every instrument,
// with the luminosity the segment scatters (albedo e^-tau0 (1 - e^-dtau)) times the phase function. The
// draws are the first of the packet's stream after the FILL, as in the reference (fillOpticalDepth,
// continuouspeeloffscattering, simulateescapeandabsorption, ...); the event kernel continues the stream.
// Two passes over the segments with the same draws: one counts the rays (a frame instrument skips a point
// outside its field), one writes them into the space reserved for the block.
template <int GRID, bool ONECOMP>
__global__ void __launch_bounds__(kBlock) contKernel(const Args a) {
    __shared__ unsigned long long resv[3 * (kBlock / 64) + 3];
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const unsigned int nwork = CTR(a.ctr, 2 + a.parity);
    if (nwork == 0) return;
    Shared sh = stageTables(a, lds, gridParts<GRID>() | STAGE_OPTICS | STAGE_INSTR);
    Events<GRID, ONECOMP> E{a, sh};
    const int* actIn = a.act[a.parity];
    const unsigned int stride = gridDim.x * blockDim.x;
    const unsigned int rounds = (nwork + stride - 1) / stride;  // every lane runs every round (block reserves)
    const int Nl = a.nlambda;
    for (unsigned int round = 0; round < rounds; round++) {
        const unsigned int w = round * stride + blockIdx.x * blockDim.x + threadIdx.x;
        const int slot = w < nwork ? actIn[w] : 0;
        Packet p;
        p.state = S_NEW;
        if (w < nwork) E.load(slot, p);
        const bool fill = w < nwork && p.state == S_FILL;
        const int nrec = fill ? a.pathCnt[slot] : 0;
        const PathRec* rec = a.pathBuf + (size_t)slot * kPathCap;
        // the weights of one segment (rho(m,h) kappa_sca(h) / ksca) and its albedo; false: no scattering dust
        auto weights = [&](int m, double* wv, double& albedo) {
            double ksca = 0.0, kext = 0.0;
            for (int h = 0; h < a.ncomp; h++) {
                const double rho = a.rho[(size_t)m * a.ncomp + h];
                wv[h] = rho * sh.ksca[h * Nl + p.ell];
                ksca += rho * sh.ksca[h * Nl + p.ell];
                kext += rho * sh.kext[h * Nl + p.ell];
            }
            if (!(ksca > 0.0)) return false;
            for (int h = 0; h < a.ncomp; h++) wv[h] /= ksca;
            albedo = ksca / kext;
            return true;
        };
        // pass 1: the rays this slot emits
        const PacketRng rng0 = p.rng;
        unsigned int nray = 0;
        for (int n = 0; n < nrec; n++) {
            double wv[8], albedo;
            if (!weights(rec[n].m, wv, albedo)) continue;
            const double s = rec[n].s0 + p.rng.uniform() * rec[n].ds;
            Packet q = p;
            q.rx = p.rx + s * p.kx; q.ry = p.ry + s * p.ky; q.rz = p.rz + s * p.kz;
            for (int i = 0; i < a.ninstr; i++)
                if (!(sh.instr[i].kind == SKIRT_INSTR_FRAME && E.pixel(sh.instr[i], q) < 0)) nray++;
        }
        unsigned int pos = 0, dpos = 0, unused = 0;
        blockReserve3(CTRP(a.ctr, a.parity), nray, pos, CTRP(a.ctr, 7), 0u, unused, CTRP(a.ctr, 5 + a.parity), nray, dpos,
                      resv);
        // (the WALK rays of the event kernel that follows are reserved from the queue's top later: the trace
        // kernel checks that the two regions do not meet)
        if (nray && (pos + nray > (unsigned)a.rayCap || dpos + nray > (unsigned)(a.rayCap - a.nslots))) {
            atomicOr(a.error, ERR_QUEUE);  // cannot happen with the pool sized for kPathCap (ensurePool)
            nray = 0;
        }
        // pass 2: the same draws again, now writing the rays and their detection records
        if (nray) {
            PacketRng rng = rng0;
            for (int n = 0; n < nrec; n++) {
                double wv[8], albedo;
                if (!weights(rec[n].m, wv, albedo)) continue;
                const double factorm = albedo * exp(-rec[n].tau0) * (-expm1(-rec[n].dtau));
                const double s = rec[n].s0 + rng.uniform() * rec[n].ds;
                Packet q = p;
                q.rx = p.rx + s * p.kx; q.ry = p.ry + s * p.ky; q.rz = p.rz + s * p.kz;
                int qcell = kNoCell;  // the point's cell (Voronoi), located once for all instruments
                for (int i = 0; i < a.ninstr; i++) {
                    const DevInstr& ins = sh.instr[i];
                    const int l = ins.kind == SKIRT_INSTR_SED ? -1 : E.pixel(ins, q);
                    if (ins.kind == SKIRT_INSTR_FRAME && l < 0) continue;
                    const double cosalpha = p.kx * ins.kobs[0] + p.ky * ins.kobs[1] + p.kz * ins.kobs[2];
                    double I = 0;
                    for (int h = 0; h < a.ncomp; h++) {
                        const double g = sh.g[h * Nl + p.ell];
                        const double t = 1.0 + g * g - 2 * g * cosalpha;
                        const double wgt = wv[h] * ((1.0 - g) * (1.0 + g) / sqrt(t * t * t));
                        I += wgt * 1.0;
                    }
                    // PhotonPackage::launchScatteringPeelOff(pp, bfrnew, bfkobs, factorm * I)
                    const double Lp = p.L * (factorm * I);
                    const unsigned cat = p.stellar >= 0 ? CAT_STAR_SCATTERED : CAT_DUST_SCATTERED;
                    const unsigned level = (unsigned)min(p.nscatt + 1, 255);
                    const unsigned flags = RAY_PEEL | (cat << 2) | ((unsigned)i << 4) | (level << 10) | ((unsigned)p.ell << 18);
                    a.det[dpos] = DetRec{Lp, 0.0, l, flags};
                    E.emitRay(pos++, q, ins.kobs[0], ins.kobs[1], ins.kobs[2], Lp, (int)dpos, flags, qcell);
                    dpos++;
                }
            }
        }
        if (fill) {  // the stream continues after the continuous draws
            a.sblock[slot] = p.rng.block; a.sw2[slot] = p.rng.w2; a.sw3[slot] = p.rng.w3; a.shave[slot] = p.rng.have;
        }
    }
    const unsigned long long vals[8] = {0, E.segFill, E.segWalk, E.segPeel, 0, 0, 0, 0};
    flushStats(a, vals);
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
    // device cell space: ndev >= ncells device cell numbers (octrees leave unused numbers so that every
    // group of 8 sibling leaves starts on a 64-byte line), Labs rows of labsStride (ndev rounded up to 8)
    int ndev = 0;
    int labsStride = 0;
    bool brick = false;  // Cartesian cells numbered in 2x2x2 bricks
    double eps = 0, gx0 = 0, gx1 = 0, gy0 = 0, gy1 = 0, gz0 = 0, gz1 = 0;
    double* dMesh = nullptr;
    double* dBox = nullptr;
    int *dFirstChild = nullptr, *dCellnumber = nullptr, *dNbrOffset = nullptr, *dNbrList = nullptr;
    signed char* dSplitDir = nullptr;  // k-d tree split axes (null for octrees)
    int* dFather = nullptr;            // octree fathers (Bookkeeping search)
    bool binTree = false;
    // Voronoi grid
    double *dSite = nullptr, *dCellBbox = nullptr;
    VorEntry* dVorSlots = nullptr;
    int *dVorStart = nullptr, *dBlockOffset = nullptr;
    BlockSite* dBlockSites = nullptr;
    std::vector<VorEntry> vorSlotsHost;  // host copy: upload_media writes the densities into the headers
    std::vector<int> vorStartHost;
    double vorScale = 1.0;
    int vnb = 0;
    // octree leaf map (mapL < 0: walk the node arrays)
    int mapL = -1, mapN = 0;
    double mapInv[3] = {0, 0, 0};
    double mapOrigin[3] = {0, 0, 0};
    double* dTreeT = nullptr;
    LeafEntry* dLeafMap = nullptr;
    bool mapReady = false;
    int lastWalk = -1;  // SKIRT_WALK_* of the last run
    // device cell numbering: devCell[reference cell] (empty = identity). Octree cells are renumbered in
    // Morton (depth-first, children in octant order) order so that neighbouring cells share Labs lines;
    // rho is uploaded and Labs downloaded through it.
    std::vector<int> devCell;
    // media
    int ncomp = 0, nlambda = 0;
    double *dRho = nullptr, *dOptics = nullptr;
    // sources
    int nstar = 0;
    double *dGeomParam = nullptr, *dLum = nullptr, *dLumtot = nullptr, *dCdf = nullptr;
    // the first and last wavelength with stellar luminosity: a stellar phase shoots only the packet indices of
    // [lumLo, lumHi] (the others launch nothing, MonteCarloSimulation.cpp:272-273; each packet's stream is
    // keyed by its own index, so skipping them changes no other packet)
    int lumLo = 0, lumHi = -1;
    double* dGeomTable = nullptr;  // SersicGeometry tables, kSersicTable per component
    double emissionBias = 0.5;
    // dust-phase cell sources and the dust Labs tally
    double *dCellLv = nullptr, *dCellCdf = nullptr, *dCellLtot = nullptr;
    int* dCellGuide = nullptr;  // guide tables of the cell CDFs (cellGuideKernel)
    size_t cellGuideCount = 0;
    double cellBias = 0.5;
    int* dCellNode = nullptr;
    double* dLabsDust = nullptr;
    bool ownLabsDust = true;
    // Labs replicas (SKIRT_AMD_LABS_COPIES > 1): the absorbing phases add into them, folded at the phase end
    double* dLabsRep = nullptr;
    size_t labsRepBytes = 0;
    // trace launches have added into the replicas since their last fold: a phase that ended early (an error
    // return after its first trace launch) left partial adds there, which the next storing phase clears
    bool labsRepDirty = false;
    // grey-body emissivity tables for the device-side dust emission sources
    int emisNtemp = 0;
    double *dEmisVolume = nullptr, *dEmisKabs = nullptr, *dEmisSigma = nullptr, *dEmisMu = nullptr, *dEmisTv = nullptr,
           *dEmisPlanck = nullptr, *dEmisLambda = nullptr, *dEmisDlambda = nullptr, *dEmisScratch = nullptr;
    int* dDevCell = nullptr;
    // instruments
    std::vector<DevInstr> instr;
    DevInstr* dInstr = nullptr;
    size_t nInstrTally = 0;
    int nsed = 0;
    // tallies
    double *dLabs = nullptr, *dTally = nullptr;
    bool ownLabs = true, ownTally = true;
    unsigned long long *dClaim = nullptr, *dStats = nullptr;
    unsigned long long* dCrossed = nullptr;  // kCrossedCopies x crossedBins (skirt_mcrt_set_crossed)
    int crossedBins = 0;
    unsigned int *dError = nullptr, *dCtr = nullptr, *hCtr = nullptr;  // kMaxHalves x 8 counters; hCtr: poll ring
    // the pipeline's streams: sE runs the event, continuous peel-off and detect kernels, sT[h] the trace
    // kernels of half h; with CU masks (cusT, cusE) they run on disjoint sets of CUs. One half without
    // masks runs everything on the caller's stream.
    int halves = 1, cusT = 0, cusE = 0;  // requested (SKIRT_AMD_HALVES, SKIRT_AMD_TRACE_CUS, SKIRT_AMD_EVENT_CUS)
    hipStream_t sE = nullptr, sT[kMaxHalves] = {};
    int streamCusT = -1, streamCusE = -1;  // the masks the owned streams were created with
    int nCusT = 0, nCusE = 0;              // CUs behind each stream (grid sizes)
    hipEvent_t evFork = nullptr, evJoin[1 + kMaxHalves] = {}, evE[kMaxHalves] = {}, evT[kMaxHalves] = {};
    // one half without masks: the detect kernel of iteration k runs on sD, beside the event and trace kernels
    // of iteration k + 1 on the caller's stream (the detection records alternate between two regions by
    // iteration parity, Args::det); evDet[q]: the detect kernel of the last parity-q iteration is done
    hipStream_t sD = nullptr;
    hipEvent_t evDetT = nullptr, evDet[2] = {}, evDetJoin = nullptr;
    std::vector<hipEvent_t> pollEv;      // kMaxHalves x kPollRing events behind the counter copies
    // slot pool
    int nslots = 0, rayCap = 0, poolHalves = 0;
    bool poolPath = false;  // the pool holds the continuous-scattering path records
    bool poolDetPair = false;  // the pool holds two detection-record regions (one per iteration parity)
    void* dPool = nullptr;               // one pool of nslots slots per half
    size_t poolBytes = 0;
    // config
    // threshold 0: 16 idle lanes before a trace wave pulls rays, 8 on Voronoi grids (C3 +0.6 %, C2 +0.5 %, C5
    // +0.5 % against 8; C4 -0.1 %; profiles/r06_pull_threshold.txt)
    int traceGrid = 0, threshold = 0, slotsWanted = 0;
    // WALK rays at the end of the pull order: SKIRT_AMD_WALK_BACK=1 / 0, default (-1) on Voronoi grids only.
    // It shortens every grid's launch tail, but on the tree and Cartesian grids the launch's main part then
    // runs without the atomic-free WALK paths between the absorbing FILL paths: C3 2.16e8 -> 2.08e8, C2
    // 2.9e8 -> 2.8e8; C4 9.30e7 -> 9.38e7 (profiles/r03_walk_back_ab.txt)
    int walkBack = getenv("SKIRT_AMD_WALK_BACK") ? atoi(getenv("SKIRT_AMD_WALK_BACK")) : -1;
    int traceBlocksPerCU = 0;  // the occupancy the last trace launch was sized for
    int lastDetCopies = 0;  // SED copies of the last run's detect kernel
    double lastMs = 0;
    bool phaseTimed = false;  // ev0/ev1 recorded by the last phase (an empty slice records nothing)
    std::vector<hipEvent_t> traceEv;  // pairs around the trace launches not yet timed
    int traceLaunches = 0;
    uint64_t packagesTotal = 0;       // packet indices of the phases run since the last zero_tallies (SkirtStats::packages)
    double traceMs = 0;               // all timed trace launches since the context was created
    uint64_t traceLaunchesTotal = 0;
    int numCUs = 0;
    size_t ldsMax = 64 * 1024;  // LDS one workgroup may allocate (hipDeviceProp_t::sharedMemPerBlock; 160 KiB on gfx950)
    int lastIterations = 0;
    // multi-process reduction of the tallies (skirt_mcrt_set_reducer)
    SkirtReduceTallyFn reduce = nullptr;
    void* reduceUser = nullptr;
    bool instrReduced = false;
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

// slot pool: one pool per pipeline half, each with its ray queue, SoA packet state, per-slot
// results and two active lists; nslots counts the slots of one half
// With continuous scattering every slot may also queue one peel-off per instrument and recorded path
// segment in one iteration, and keeps the dust segments of its last path (kPathCap each).
int ensurePool(SkirtMcrt* c, int nslots, bool continuous, int halves, bool detPair) {
    const int ninstr = (int)c->instr.size();
    const size_t rays = (size_t)nslots * (1 + ninstr) + (continuous ? (size_t)nslots * kPathCap * ninstr : 0);
    if (rays >= (size_t)INT32_MAX) return fail(c, SKIRT_ERR_UNSUPPORTED, "ray queue too large");
    const int rayCap = (int)rays;
    const size_t path = continuous ? (size_t)nslots * (kPathCap * sizeof(PathRec) + sizeof(int)) : 0;
    const size_t half = (size_t)rayCap * sizeof(RayRec) + (detPair ? 2 : 1) * (size_t)(rayCap - nslots) * sizeof(DetRec) +
                        (size_t)nslots * (10 * 8 + 5 * 4 + 6 * 4 + 2 * 4) + path + 4096;
    if (c->dPool && c->nslots == nslots && c->rayCap == rayCap && c->poolPath == (path > 0) && c->poolHalves == halves &&
        c->poolDetPair == detPair)
        return SKIRT_OK;
    c->poolPath = path > 0;
    c->poolDetPair = detPair;
    if (c->dPool) { (void)hipFree(c->dPool); c->dPool = nullptr; }
    HIPCHECK(c, hipMalloc(&c->dPool, halves * half));
    c->poolBytes = half;
    c->nslots = nslots;
    c->rayCap = rayCap;
    c->poolHalves = halves;
    return SKIRT_OK;
}

// A stream restricted to `want` CUs (0: all), spread evenly over the XCDs: CU k of the mask is taken when
// k mod 32 < want / 8 (or, for the complementary set, k mod 32 >= 32 - want / 8), so that each XCD
// contributes the same share whether the runtime numbers CUs XCD by XCD or round-robin.
int makeStream(SkirtMcrt* c, hipStream_t* s, int want, bool high, int* got) {
    if (want <= 0 || want >= c->numCUs) {
        *got = c->numCUs;
        HIPCHECK(c, hipStreamCreateWithFlags(s, hipStreamNonBlocking));
        return SKIRT_OK;
    }
    const int words = (c->numCUs + 31) / 32;
    std::vector<uint32_t> mask(words, 0u);
    const int per = std::max(1, want * 32 / std::max(32, c->numCUs));
    int n = 0;
    for (int k = 0; k < c->numCUs; k++) {
        const int r = k % 32;
        if (high ? r >= 32 - per : r < per) { mask[k / 32] |= 1u << (k % 32); n++; }
    }
    *got = n;
    HIPCHECK(c, hipExtStreamCreateWithCUMask(s, (uint32_t)words, mask.data()));
    return SKIRT_OK;
}

// the pipeline streams for the requested halves and CU masks (created once per mask configuration)
int ensureStreams(SkirtMcrt* c) {
    if (c->halves == 1 && c->cusT == 0 && c->cusE == 0) {
        c->nCusT = c->nCusE = c->numCUs;
        return SKIRT_OK;  // everything on the caller's stream
    }
    if (c->sE && c->streamCusT == c->cusT && c->streamCusE == c->cusE) return SKIRT_OK;
    (void)hipStreamSynchronize(c->stream);
    if (c->sE) { (void)hipStreamDestroy(c->sE); c->sE = nullptr; }
    for (auto& s : c->sT)
        if (s) { (void)hipStreamDestroy(s); s = nullptr; }
    int rc = makeStream(c, &c->sE, c->cusE, true, &c->nCusE);
    for (int h = 0; h < kMaxHalves && !rc; h++) rc = makeStream(c, &c->sT[h], c->cusT, false, &c->nCusT);
    if (rc) return rc;
    c->streamCusT = c->cusT;
    c->streamCusE = c->cusE;
    return SKIRT_OK;
}

void carvePool(SkirtMcrt* c, Args& a, int h) {
    char* p = static_cast<char*>(c->dPool) + (size_t)h * c->poolBytes;
    const size_t n = (size_t)c->nslots;
    auto takeD = [&](double*& d) { d = reinterpret_cast<double*>(p); p += n * 8; };
    auto takeI = [&](int*& d) { d = reinterpret_cast<int*>(p); p += n * 4; };
    auto takeU = [&](uint32_t*& d) { d = reinterpret_cast<uint32_t*>(p); p += n * 4; };
    a.rays = reinterpret_cast<RayRec*>(p);
    p += (size_t)c->rayCap * sizeof(RayRec);
    a.det = reinterpret_cast<DetRec*>(p);  // at most one peel-off per instrument and slot per iteration
    p += (c->poolDetPair ? 2 : 1) * (size_t)(c->rayCap - c->nslots) * sizeof(DetRec);
    takeD(a.srx); takeD(a.sry); takeD(a.srz); takeD(a.skx); takeD(a.sky); takeD(a.skz); takeD(a.sL); takeD(a.sLth);
    takeD(a.resA); takeD(a.resB);
    takeI(a.sell); takeI(a.snscatt); takeI(a.sstellar); takeI(a.sstate); takeI(a.svcell);
    takeU(a.splo); takeU(a.sphi); takeU(a.sblock); takeU(a.sw2); takeU(a.sw3); takeU(a.shave);
    takeI(a.act[0]); takeI(a.act[1]);
    a.pathBuf = nullptr;
    a.pathCnt = nullptr;
    if (c->poolPath) {
        p = reinterpret_cast<char*>(((uintptr_t)p + 15) & ~(uintptr_t)15);
        a.pathBuf = reinterpret_cast<PathRec*>(p);
        p += n * kPathCap * sizeof(PathRec);
        takeI(a.pathCnt);
    }
    a.nslots = c->nslots;
    a.rayCap = c->rayCap;
    a.ctr = c->dCtr + kCtrWords * h;
}

// Decides whether the octree can be walked through a leaf map (Grid<SKIRT_GRID_OCTREE>): every node
// box must equal the box its level and integer coordinates give in the per-axis split tables, and the
// tree must be at most kMaxMapLevel deep. Uploads the tables; the map itself is built at the first
// phase (it caches the densities). SKIRT_AMD_LEAFMAP=0 forces the node-array walk.
int planLeafMap(SkirtMcrt* c, const SkirtGridDesc* g) {
    c->mapL = -1;
    c->mapReady = false;
    if (c->dLeafMap) { (void)hipFree(c->dLeafMap); c->dLeafMap = nullptr; }
    const char* env = getenv("SKIRT_AMD_LEAFMAP");
    if (env && env[0] == '0') return SKIRT_OK;
    const bool bin = g->split_dir != nullptr;
    if (c->ndev >= (int)(1u << (bin ? kBinCellBits : kLeafLevelShift))) return SKIRT_OK;
    const int maxL = bin ? kMaxBinMapLevel : kMaxMapLevel;
    struct Item { int node, lv[3], idx[3]; };  // per-axis depth and integer coordinate
    std::vector<Item> stack{{0, {0, 0, 0}, {0, 0, 0}}};
    std::vector<Item> nodes;
    nodes.reserve(g->nnodes);
    int L = 0;
    while (!stack.empty()) {
        const Item it = stack.back();
        stack.pop_back();
        nodes.push_back(it);
        L = std::max(L, std::max(it.lv[0], std::max(it.lv[1], it.lv[2])));
        if (L > maxL) return SKIRT_OK;
        const int fc = g->first_child[it.node];
        if (fc < 0) continue;
        if (bin) {
            const int d = g->split_dir[it.node];
            for (int k = 0; k < 2; k++) {
                Item ch = it;
                ch.node = fc + k;
                ch.lv[d]++;
                ch.idx[d] = 2 * it.idx[d] + k;
                stack.push_back(ch);
            }
        } else {
            for (int k = 0; k < 8; k++) {
                Item ch;
                ch.node = fc + k;
                for (int ax = 0; ax < 3; ax++) {
                    ch.lv[ax] = it.lv[ax] + 1;
                    ch.idx[ax] = 2 * it.idx[ax] + ((k >> ax) & 1);
                }
                stack.push_back(ch);
            }
        }
    }
    if ((int)nodes.size() != g->nnodes) return SKIRT_OK;  // not a tree reachable from node 0
    const int N = 1 << L;
    std::vector<double> T(3 * (size_t)(N + 1));
    for (int ax = 0; ax < 3; ax++) {
        double* t = T.data() + ax * (N + 1);
        t[0] = g->box[ax];
        t[N] = g->box[3 + ax];
        for (int w = N; w > 1; w >>= 1)  // Box::center of every node, coarse to fine
            for (int lo = 0; lo < N; lo += w) t[lo + w / 2] = 0.5 * (t[lo] + t[lo + w]);
        for (int j = 0; j < N; j++)
            if (!(t[j] < t[j + 1])) return SKIRT_OK;
    }
    for (const Item& it : nodes) {
        const double* b = g->box + 6 * (size_t)it.node;
        for (int ax = 0; ax < 3; ax++) {
            const int sh = L - it.lv[ax];
            const double* t = T.data() + ax * (N + 1);
            if (b[ax] != t[it.idx[ax] << sh] || b[3 + ax] != t[(it.idx[ax] + 1) << sh]) return SKIRT_OK;
        }
    }
    int rc = upload(c, c->dTreeT, T.data(), T.size());
    if (rc) return rc;
    c->mapL = L;
    c->mapN = N;
    for (int ax = 0; ax < 3; ax++) c->mapInv[ax] = N / (g->box[3 + ax] - g->box[ax]);
    for (int ax = 0; ax < 3; ax++) c->mapOrigin[ax] = T[ax * (N + 1)];
    return SKIRT_OK;
}

// the grid and density fields of the kernel arguments (every kernel that walks the grid)
void gridArgs(const SkirtMcrt* c, Args& a) {
    a.ncells = c->ncells;
    a.labsStride = c->labsStride;
    a.nx = c->nx; a.ny = c->ny; a.nz = c->nz;
    a.brick = c->brick ? 1 : 0;
    a.mesh = c->dMesh;
    a.gx0 = c->gx0; a.gx1 = c->gx1; a.gy0 = c->gy0; a.gy1 = c->gy1; a.gz0 = c->gz0; a.gz1 = c->gz1;
    a.box = c->dBox; a.firstChild = c->dFirstChild; a.cellnumber = c->dCellnumber;
    a.splitDir = c->binTree ? c->dSplitDir : nullptr;
    a.father = c->dFather;
    a.nbrOffset = c->dNbrOffset; a.nbrList = c->dNbrList; a.eps = c->eps; a.search = c->search;
    a.site = c->dSite; a.vorStart = c->dVorStart; a.vorSlots = c->dVorSlots; a.vorScale = (float)c->vorScale; a.cellBbox = c->dCellBbox;
    a.devCell = c->dDevCell;
    a.vnb = c->vnb; a.blockOffset = c->dBlockOffset; a.blockSites = c->dBlockSites;
    a.ncomp = std::max(1, c->ncomp); a.nlambda = c->nlambda;
    a.rho = c->dRho;
}

int ensureLeafMap(SkirtMcrt* c) {
    if (c->mapL < 0 || c->mapReady) return SKIRT_OK;
    const size_t n = (size_t)leafMapSize(1 << c->mapL);
    if (!c->dLeafMap) HIPCHECK(c, hipMalloc(&c->dLeafMap, n * sizeof(LeafEntry)));
    const int blocks = (int)std::min<size_t>((n + kBlock - 1) / kBlock, 65536);
    hipLaunchKernelGGL(buildLeafMapKernel, dim3(blocks), dim3(kBlock), 0, c->stream, c->dLeafMap, c->dFirstChild,
                       c->binTree ? c->dSplitDir : nullptr, c->dCellnumber, c->dRho, std::max(1, c->ncomp), c->mapL);
    HIPCHECK(c, hipGetLastError());
    c->mapReady = true;
    return SKIRT_OK;
}

// ================================================================== setup: density sampling
// The setup's hot loop (skirt_mcrt_sample_density): one thread per item (a cell or a tree node), its
// samples in order, so that every sum is accumulated as the host loop accumulates it (build.cpp cell
// densities and tree subdivision). The geometry densities follow the host's Geometry::density operation
// for operation (PlummerGeometry.cpp:49-54, ExpDiskGeometry::density, SersicGeometry::density with the
// SersicFunction log-log interpolation, PointGeometry).
struct DensArgs {
    int ncomp, ntab, nsample, mode;
    const int* kind;
    const double* param;  // ncomp x 8
    const double* norm;   // ncomp
    const double* table;  // ncomp x 2 ntab
    const double* boxes;  // n x 6
    const uint32_t* words;
    double* out;
    size_t n;
};

__device__ double geomDensity(const DensArgs& d, int h, double x, double y, double z) {
    const double* p = d.param + 8 * h;
    switch (d.kind[h]) {
    case SKIRT_GEOM_PLUMMER: {
        const double r = sqrt(x * x + y * y + z * z);
        const double s = r / p[0];
        return p[1] * pow(1.0 + s * s, -2.5);
    }
    case SKIRT_GEOM_EXPDISK: {
        const double R = sqrt(x * x + y * y);
        const double absz = fabs(z);
        const double hR = p[0], hz = p[1], Rmax = p[2], zmax = p[3], Rmin = p[4], rho0 = p[5];
        if (Rmax > 0.0 && R > Rmax) return 0.0;
        if (zmax > 0.0 && absz > zmax) return 0.0;
        if (R < Rmin) return 0.0;
        return rho0 * exp(-R / hR) * exp(-absz / hz);
    }
    case SKIRT_GEOM_SERSIC: {
        const double r = sqrt(x * x + y * y + z * z);
        const double s = r / p[0];
        const double* sv = d.table + (size_t)2 * d.ntab * h;
        const double* Sv = sv + d.ntab;
        const int Ns = d.ntab;
        if (s <= sv[0]) return p[2] * Sv[0];
        if (s >= sv[Ns - 1]) return p[2] * Sv[Ns - 1];
        int jl = -1, ju = Ns - 1;  // NR::locate_clip (s >= sv[0] here)
        while (ju - jl > 1) {
            const int jm = (ju + jl) >> 1;
            if (s < sv[jm]) ju = jm;
            else jl = jm;
        }
        // NR::interpolate_loglog
        const double lx = log10(s), x1 = log10(sv[jl]), x2 = log10(sv[jl + 1]);
        double f1 = Sv[jl], f2 = Sv[jl + 1];
        const bool logf = f1 > 0 && f2 > 0;
        if (logf) { f1 = log10(f1); f2 = log10(f2); }
        double fx = f1 + ((lx - x1) / (x2 - x1)) * (f2 - f1);
        if (logf) fx = pow(10.0, fx);
        return p[2] * fx;
    }
    default:  // SKIRT_GEOM_POINT
        return (x * x + y * y + z * z) == 0 ? INFINITY : 0.0;
    }
}

__global__ void __launch_bounds__(kBlock) densitySampleKernel(const DensArgs d) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= d.n) return;
    const double* b = d.boxes + 6 * q;
    const uint32_t* w = d.words + (size_t)3 * d.nsample * q;
    constexpr double kWordMax = 4294967295.0;  // MTRandom::deviate
    if (d.mode == SKIRT_DENS_COMPONENTS) {
        double* o = d.out + (size_t)d.ncomp * q;
        for (int h = 0; h < d.ncomp; h++) o[h] = 0.0;
        for (int k = 0; k < d.nsample; k++) {
            const double fx = (double)w[3 * k] / kWordMax, fy = (double)w[3 * k + 1] / kWordMax,
                         fz = (double)w[3 * k + 2] / kWordMax;
            const double x = b[0] + fx * (b[3] - b[0]), y = b[1] + fy * (b[4] - b[1]), z = b[2] + fz * (b[5] - b[2]);
            for (int h = 0; h < d.ncomp; h++) o[h] += d.norm[h] * geomDensity(d, h, x, y, z);
        }
    } else {
        double sum = 0, sx = 0, sy = 0, sz = 0, mn = 0, mx = 0;
        for (int k = 0; k < d.nsample; k++) {
            const double fx = (double)w[3 * k] / kWordMax, fy = (double)w[3 * k + 1] / kWordMax,
                         fz = (double)w[3 * k + 2] / kWordMax;
            const double x = b[0] + fx * (b[3] - b[0]), y = b[1] + fy * (b[4] - b[1]), z = b[2] + fz * (b[5] - b[2]);
            double rho = 0;
            for (int h = 0; h < d.ncomp; h++) rho += d.norm[h] * geomDensity(d, h, x, y, z);
            sum += rho;
            sx += rho * x;
            sy += rho * y;
            sz += rho * z;
            if (k == 0 || rho < mn) mn = rho;  // std::min_element / max_element: the first extreme
            if (k == 0 || mx < rho) mx = rho;
        }
        double* o = d.out + 6 * q;
        o[0] = sum; o[1] = sx; o[2] = sy; o[3] = sz; o[4] = mn; o[5] = mx;
    }
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
        hipMalloc(&c->dClaim, sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->dStats, 8 * kStatCopies * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->dError, sizeof(unsigned int)) != hipSuccess ||
        hipMalloc(&c->dCtr, kMaxHalves * kCtrWords * sizeof(unsigned int)) != hipSuccess ||
        hipHostMalloc(&c->hCtr, kMaxHalves * kPollRing * kCtrWords * sizeof(unsigned int)) != hipSuccess ||
        hipEventCreateWithFlags(&c->evFork, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return SKIRT_ERR_HIP;
    }
    for (int h = 0; h < kMaxHalves; h++)
        if (hipEventCreateWithFlags(&c->evE[h], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->evT[h], hipEventDisableTiming) != hipSuccess) {
            delete c;
            return SKIRT_ERR_HIP;
        }
    for (auto& e : c->evJoin)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            delete c;
            return SKIRT_ERR_HIP;
        }
    // pipeline layout (tuning knobs; see runPhase)
    if (const char* s = getenv("SKIRT_AMD_HALVES")) c->halves = std::max(1, std::min(kMaxHalves, atoi(s)));
    if (const char* s = getenv("SKIRT_AMD_TRACE_CUS")) c->cusT = std::max(0, atoi(s));
    if (const char* s = getenv("SKIRT_AMD_EVENT_CUS")) c->cusE = std::max(0, atoi(s));
    c->stream = c->own;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
        c->numCUs = prop.multiProcessorCount;
        if (prop.sharedMemPerBlock > 0) c->ldsMax = prop.sharedMemPerBlock;
    }
    (void)hipMemset(c->dStats, 0, 8 * kStatCopies * sizeof(unsigned long long));
    (void)hipMemset(c->dError, 0, sizeof(unsigned int));
    *out = c;
    return SKIRT_OK;
}

int skirt_mcrt_set_stream(SkirtMcrt* c, void* s) {
    if (!c) return SKIRT_ERR_ARG;
    c->stream = s ? (hipStream_t)s : c->own;
    return SKIRT_OK;
}

int skirt_mcrt_configure(SkirtMcrt* c, int slots, int grid, int threshold) {
    if (!c) return SKIRT_ERR_ARG;
    if (slots < 0 || grid < 0 || threshold < 0) return fail(c, SKIRT_ERR_ARG, "negative configuration value");
    c->slotsWanted = slots;
    c->traceGrid = grid;
    if (threshold) c->threshold = std::max(1, std::min(64, threshold));
    return SKIRT_OK;
}

int skirt_mcrt_upload_grid(SkirtMcrt* c, const SkirtGridDesc* g) {
    if (!c || !g) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    c->ncells = g->ncells;
    c->ndev = g->ncells;
    c->brick = false;
    c->devCell.clear();
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
        // device numbers in 2x2x2 bricks (Grid<SKIRT_GRID_CARTESIAN>::dev); SKIRT_AMD_CELL_ALIGN=0: the
        // reference's numbering
        const char* alignEnv = getenv("SKIRT_AMD_CELL_ALIGN");
        c->brick = !(alignEnv && alignEnv[0] == '0');
        if (c->brick) {
            const long long bx = (g->nx + 1) / 2, by = (g->ny + 1) / 2, bz = (g->nz + 1) / 2;
            if (8 * bx * by * bz >= (1ll << 31)) return fail(c, SKIRT_ERR_UNSUPPORTED, "Cartesian grid too large");
            c->devCell.assign(g->ncells, 0);
            for (int i = 0; i < g->nx; i++)
                for (int j = 0; j < g->ny; j++)
                    for (int k = 0; k < g->nz; k++)
                        c->devCell[k + g->nz * j + g->nz * g->ny * i] =
                            (int)((((i >> 1) * by + (j >> 1)) * bz + (k >> 1)) << 3) | ((i & 1) << 2) | ((j & 1) << 1) | (k & 1);
            c->ndev = (int)(8 * bx * by * bz);
        }
        c->gx0 = g->xv[0]; c->gx1 = g->xv[g->nx];
        c->gy0 = g->yv[0]; c->gy1 = g->yv[g->ny];
        c->gz0 = g->zv[0]; c->gz1 = g->zv[g->nz];
        int rc = upload(c, c->dMesh, mesh.data(), mesh.size());
        if (rc) return rc;
    } else if (g->kind == SKIRT_GRID_OCTREE) {
        if (g->nnodes < 1 || !g->box || !g->first_child || !g->cellnumber || !g->nbr_offset)
            return fail(c, SKIRT_ERR_ARG, "bad octree grid");
        // validate the index arrays so that the kernels never read out of bounds
        const bool bin = g->split_dir != nullptr;
        const int arity = bin ? 2 : 8;
        int nleaf = 0;
        for (int l = 0; l < g->nnodes; l++) {
            const int fc = g->first_child[l];
            if (fc >= 0 && (fc + arity > g->nnodes || fc <= l)) return fail(c, SKIRT_ERR_ARG, "octree child index out of range");
            if (fc >= 0 && bin && (g->split_dir[l] < 0 || g->split_dir[l] > 2)) return fail(c, SKIRT_ERR_ARG, "bad k-d tree split axis");
            if (fc < 0) {
                if (g->cellnumber[l] < 0 || g->cellnumber[l] >= g->ncells) return fail(c, SKIRT_ERR_ARG, "octree cell number out of range");
                nleaf++;
            }
        }
        if (nleaf != g->ncells) return fail(c, SKIRT_ERR_ARG, "octree leaf count != ncells");
        const int nnbr = g->nbr_offset[6 * (size_t)g->nnodes];
        for (size_t q = 0; q < 6 * (size_t)g->nnodes; q++)
            if (g->nbr_offset[q] < 0 || g->nbr_offset[q] > g->nbr_offset[q + 1]) return fail(c, SKIRT_ERR_ARG, "bad neighbor offsets");
        for (int q = 0; q < nnbr; q++)
            if (g->nbr_list[q] < 0 || g->nbr_list[q] >= g->nnodes) return fail(c, SKIRT_ERR_ARG, "neighbor index out of range");
        if (g->search < SKIRT_TREE_TOPDOWN || g->search > SKIRT_TREE_BOOKKEEPING) return fail(c, SKIRT_ERR_ARG, "bad tree search method");
        std::vector<int> father;
        if (g->search == SKIRT_TREE_BOOKKEEPING) {
            // the Bookkeeping search reads octants off the breadth-first numbering: every group of
            // children must start at an id = 1 (mod 8) (TreeDustGrid.cpp:525)
            if (bin) return fail(c, SKIRT_ERR_ARG, "Bookkeeping method is not compatible with binary tree");
            father.assign(g->nnodes, -1);
            for (int l = 0; l < g->nnodes; l++) {
                const int fc = g->first_child[l];
                if (fc < 0) continue;
                if ((fc - 1) % 8 != 0) return fail(c, SKIRT_ERR_ARG, "octree not numbered breadth-first for the Bookkeeping search");
                for (int k = 0; k < 8; k++) father[fc + k] = l;
            }
        }
        c->nnodes = g->nnodes;
        c->eps = g->eps;
        c->search = g->search;
        c->gx0 = g->box[0]; c->gy0 = g->box[1]; c->gz0 = g->box[2];
        c->gx1 = g->box[3]; c->gy1 = g->box[4]; c->gz1 = g->box[5];
        int rc;
        if ((rc = upload(c, c->dBox, g->box, 6 * (size_t)g->nnodes))) return rc;
        if ((rc = upload(c, c->dFirstChild, g->first_child, (size_t)g->nnodes))) return rc;
        c->binTree = bin;
        if (!father.empty() && (rc = upload(c, c->dFather, father.data(), father.size()))) return rc;
        if (bin) {
            std::vector<signed char> dirs(g->split_dir, g->split_dir + g->nnodes);
            for (int l = 0; l < g->nnodes; l++)
                if (g->first_child[l] < 0) dirs[l] = 0;
            if ((rc = upload(c, c->dSplitDir, dirs.data(), dirs.size()))) return rc;
        }
        // Morton order of the leaves: depth-first, children in octant order (x, y, z bits). A ray crosses
        // about 2.5 of the 8 children of a node it enters, so 8 sibling leaves are numbered from a
        // multiple of 8 (one 64-byte line of every Labs row), leaving unused device cells before them:
        // the ray's Labs adds into them then share one atomic request (SKIRT_AMD_CELL_ALIGN=0: no gaps).
        c->devCell.assign(g->ncells, -1);
        {
            const char* alignEnv = getenv("SKIRT_AMD_CELL_ALIGN");
            const bool align = arity == 8 && !(alignEnv && alignEnv[0] == '0');
            std::vector<int> stack{0};
            int next = 0, used = 0;
            auto number = [&](int l) -> bool {
                if (c->devCell[g->cellnumber[l]] >= 0) return false;
                c->devCell[g->cellnumber[l]] = next++;
                used++;
                return true;
            };
            while (!stack.empty()) {
                const int l = stack.back();
                stack.pop_back();
                const int fc = g->first_child[l];
                if (fc < 0) {
                    if (!number(l)) return fail(c, SKIRT_ERR_ARG, "octree cell number used twice");
                    continue;
                }
                bool leaves = align;
                for (int k = 0; k < arity && leaves; k++) leaves = g->first_child[fc + k] < 0;
                if (leaves) {  // the sibling leaves, aligned: the same depth-first order
                    next = (next + 7) & ~7;
                    for (int k = 0; k < arity; k++)
                        if (!number(fc + k)) return fail(c, SKIRT_ERR_ARG, "octree cell number used twice");
                } else {
                    for (int k = arity - 1; k >= 0; k--) stack.push_back(fc + k);
                }
            }
            if (used != g->ncells) return fail(c, SKIRT_ERR_ARG, "octree leaves do not cover the cells");
            c->ndev = next;
        }
        std::vector<int> cellNode(g->ncells, 0);
        for (int l = 0; l < g->nnodes; l++)
            if (g->first_child[l] < 0) cellNode[g->cellnumber[l]] = l;
        if ((rc = upload(c, c->dCellNode, cellNode.data(), cellNode.size()))) return rc;
        std::vector<int> cn(g->cellnumber, g->cellnumber + g->nnodes);
        for (int l = 0; l < g->nnodes; l++)
            if (cn[l] >= 0) cn[l] = c->devCell[cn[l]];
        if ((rc = upload(c, c->dCellnumber, cn.data(), (size_t)g->nnodes))) return rc;
        if ((rc = upload(c, c->dNbrOffset, g->nbr_offset, 6 * (size_t)g->nnodes + 1))) return rc;
        std::vector<int> dummy(1, 0);
        if ((rc = upload(c, c->dNbrList, nnbr ? g->nbr_list : dummy.data(), nnbr ? (size_t)nnbr : 1))) return rc;
        if ((rc = planLeafMap(c, g))) return rc;
    } else if (g->kind == SKIRT_GRID_VORONOI) {
        const int N = g->ncells;
        if (N < 1 || !g->site || !g->cell_nbr_offset || !g->cell_nbr_list || !g->cell_bbox || g->nblocks < 1 ||
            !g->block_offset || !g->block_list)
            return fail(c, SKIRT_ERR_ARG, "bad Voronoi grid");
        if (N > kCellMaskOut) return fail(c, SKIRT_ERR_UNSUPPORTED, "more than 2^28 Voronoi cells");
        const int nnbr = g->cell_nbr_offset[N];
        for (int m = 0; m < N; m++)
            if (g->cell_nbr_offset[m] < 0 || g->cell_nbr_offset[m] > g->cell_nbr_offset[m + 1])
                return fail(c, SKIRT_ERR_ARG, "bad Voronoi neighbour offsets");
        for (int q = 0; q < nnbr; q++)
            if (g->cell_nbr_list[q] < -6 || g->cell_nbr_list[q] >= N) return fail(c, SKIRT_ERR_ARG, "Voronoi neighbour out of range");
        const size_t nb3 = (size_t)g->nblocks * g->nblocks * g->nblocks;
        const int nbl = g->block_offset[nb3];
        for (int q = 0; q < nbl; q++)
            if (g->block_list[q] < 0 || g->block_list[q] >= N) return fail(c, SKIRT_ERR_ARG, "Voronoi block list out of range");
        c->eps = g->eps;
        c->gx0 = g->extent[0]; c->gy0 = g->extent[1]; c->gz0 = g->extent[2];
        c->gx1 = g->extent[3]; c->gy1 = g->extent[4]; c->gz1 = g->extent[5];
        c->vnb = g->nblocks;
        // device cell numbers in Morton order of the sites (21 bits per axis, ties by reference number):
        // cells adjacent in space are adjacent in memory, for the neighbour lists, the densities and the
        // Labs tallies alike. Every list keeps its reference order (first-minimum choices depend on it).
        c->devCell.assign(N, 0);
        {
            std::vector<std::pair<uint64_t, int>> key(N);
            const double ext[3] = {c->gx1 - c->gx0, c->gy1 - c->gy0, c->gz1 - c->gz0};
            const double lo[3] = {c->gx0, c->gy0, c->gz0};
            for (int m = 0; m < N; m++) {
                uint64_t code = 0;
                for (int d = 0; d < 3; d++) {
                    const double f = (g->site[3 * (size_t)m + d] - lo[d]) / ext[d];
                    const uint64_t u = (uint64_t)std::max(0.0, std::min(2097151.0, f * 2097152.0));
                    for (int bit = 0; bit < 21; bit++) code |= ((u >> bit) & 1ull) << (3 * bit + (2 - d));
                }
                key[m] = {code, m};
            }
            std::sort(key.begin(), key.end());
            for (int q = 0; q < N; q++) c->devCell[key[q].second] = q;
        }
        std::vector<int> refOf(N);
        for (int m = 0; m < N; m++) refOf[c->devCell[m]] = m;
        std::vector<double> site(3 * (size_t)N), bbox(6 * (size_t)N);
        // each device cell's block: kVorHead header slots + one slot per neighbour, in pairs (see VorEntry);
        // the array is padded by kVorPad slots, since a step loads whole groups of entries
        std::vector<int> start(N + 1, 0);
        for (int d = 0; d < N; d++) {
            const int m = refOf[d];
            const int cnt = g->cell_nbr_offset[m + 1] - g->cell_nbr_offset[m];
            if (cnt < 1) return fail(c, SKIRT_ERR_ARG, "Voronoi cell without neighbours");
            // whole groups of kVorUnroll entries (even)
            const int per = kVorUnroll;
            start[d + 1] = start[d] + kVorHead + (cnt + per - 1) / per * per;
        }
        if ((size_t)start[N] + kVorPad >= (size_t)INT32_MAX) return fail(c, SKIRT_ERR_UNSUPPORTED, "Voronoi mesh too large");
        std::vector<VorEntry> slots((size_t)start[N] + kVorPad, VorEntry{0.f, 0.f, 0.f, -1});
        // offsets in units of the domain's largest half-width: single-precision squares stay in range
        c->vorScale = 2.0 / std::max({c->gx1 - c->gx0, c->gy1 - c->gy0, c->gz1 - c->gz0});
        for (int d = 0; d < N; d++) {
            const int m = refOf[d];
            const double* sm = g->site + 3 * (size_t)m;
            for (int q = 0; q < 3; q++) site[3 * (size_t)d + q] = sm[q];
            for (int q = 0; q < 6; q++) bbox[6 * (size_t)d + q] = g->cell_bbox[6 * (size_t)m + q];
            VorEntry* blk = slots.data() + start[d];
            const double head[4] = {sm[0], sm[1], sm[2], 0.0};  // rho of component 0: set by upload_media
            std::memcpy(blk, head, sizeof head);
            const int cnt = g->cell_nbr_offset[m + 1] - g->cell_nbr_offset[m];
            std::vector<float> off(3 * (size_t)cnt);
            int o = 0;
            for (int q = g->cell_nbr_offset[m]; q < g->cell_nbr_offset[m + 1]; q++, o++) {
                const int id = g->cell_nbr_list[q];
                VorEntry e;
                if (id < 0) {
                    // a wall (-1 xmin, -2 xmax, ... -6 zmax) is the bisector plane of the site and its mirror
                    // image: the offset to the mirror site along the wall's axis (NaN when the site lies on
                    // the wall: the step then evaluates the list exactly)
                    const int axis = (-id - 1) / 2;
                    const double lim[6] = {c->gx0, c->gx1, c->gy0, c->gy1, c->gz0, c->gz1};
                    const double w = lim[-id - 1] - sm[axis];
                    double n[3] = {0.0, 0.0, 0.0};
                    n[axis] = w != 0.0 ? 2.0 * w * c->vorScale : NAN;
                    float o[3];
                    vorRecipOffset(n[0], n[1], n[2], o);  // m = n / |n|^2 (vor_terms.hpp)
                    e = VorEntry{o[0], o[1], o[2], id};
                } else {
                    const double* si = g->site + 3 * (size_t)id;
                    float o[3];
                    vorRecipOffset((si[0] - sm[0]) * c->vorScale, (si[1] - sm[1]) * c->vorScale,
                                   (si[2] - sm[2]) * c->vorScale, o);
                    e = VorEntry{o[0], o[1], o[2], start[c->devCell[id]]};
                }
                // entry o in its pair (see VorEntry): {ox0, ox1, oy0, oy1} {oz0, oz1, next0, next1}
                float* P = reinterpret_cast<float*>(blk + kVorHead + (o & ~1));
                const int h = o & 1;
                P[h] = e.ox; P[2 + h] = e.oy; P[4 + h] = e.oz;
                std::memcpy(P + 6 + h, &e.next, 4);
                off[3 * (size_t)o] = e.ox; off[3 * (size_t)o + 1] = e.oy; off[3 * (size_t)o + 2] = e.oz;
            }
            // the padding up to the next block: NaN entries, no exit for any direction (bounds())
            for (int q = cnt; q < start[d + 1] - start[d] - kVorHead; q++) {
                float* P = reinterpret_cast<float*>(blk + kVorHead + (q & ~1));
                const int h = q & 1;
                P[h] = P[2 + h] = P[4 + h] = NAN;
                const int none = -1;
                std::memcpy(P + 6 + h, &none, 4);
            }
            // the header's last words: id, count and the cell's error terms of the bounds (vor_terms.hpp)
            float eA, eB;
            vorRecipErrorTerms(off.data(), cnt, 3, &eA, &eB);
            int ids[4] = {d, cnt, 0, 0};
            std::memcpy(&ids[2], &eA, 4);
            std::memcpy(&ids[3], &eB, 4);
            std::memcpy(blk + 2, ids, sizeof ids);
        }
        c->vorSlotsHost = std::move(slots);
        std::vector<BlockSite> blocks(std::max(nbl, 1), BlockSite{0.0, 0.0, 0.0, -1, 0});
        for (int q = 0; q < nbl; q++) {
            const int m = g->block_list[q];
            blocks[q] = BlockSite{g->site[3 * (size_t)m], g->site[3 * (size_t)m + 1], g->site[3 * (size_t)m + 2], c->devCell[m], 0};
        }
        int rc;
        if ((rc = upload(c, c->dSite, site.data(), site.size()))) return rc;
        if ((rc = upload(c, c->dCellBbox, bbox.data(), bbox.size()))) return rc;
        if ((rc = upload(c, c->dVorStart, start.data(), start.size()))) return rc;
        if ((rc = upload(c, c->dVorSlots, c->vorSlotsHost.data(), c->vorSlotsHost.size()))) return rc;
        c->vorStartHost = std::move(start);
        if ((rc = upload(c, c->dBlockOffset, g->block_offset, nb3 + 1))) return rc;
        if ((rc = upload(c, c->dBlockSites, blocks.data(), blocks.size()))) return rc;
        if ((rc = upload(c, c->dDevCell, c->devCell.data(), c->devCell.size()))) return rc;
    } else {
        return fail(c, SKIRT_ERR_UNSUPPORTED, "unsupported grid kind");
    }
    c->labsStride = (c->ndev + 7) & ~7;
    c->gridKind = g->kind;
    return SKIRT_OK;
}

int skirt_mcrt_upload_media(SkirtMcrt* c, const SkirtMediaDesc* m) {
    if (!c || !m) return SKIRT_ERR_ARG;
    if (c->gridKind < 0) return fail(c, SKIRT_ERR_STATE, "upload the grid before the media");
    if (m->ncells != c->ncells || m->ncomp < 1 || m->ncomp > 8 || m->nlambda < 1)
        return fail(c, SKIRT_ERR_ARG, "media sizes do not match the grid (1 <= ncomp <= 8)");
    if (m->nlambda >= (1 << 14)) return fail(c, SKIRT_ERR_ARG, "at most 16383 wavelengths");
    HIPCHECK(c, hipSetDevice(c->device));
    c->mapReady = false;  // the leaf map caches the densities
    c->ncomp = m->ncomp;
    c->nlambda = m->nlambda;
    const size_t nt = (size_t)m->ncomp * m->nlambda;
    std::vector<double> opt(4 * nt);
    std::memcpy(opt.data(), m->kext, nt * sizeof(double));
    std::memcpy(opt.data() + nt, m->ksca, nt * sizeof(double));
    std::memcpy(opt.data() + 2 * nt, m->albedo, nt * sizeof(double));
    std::memcpy(opt.data() + 3 * nt, m->g, nt * sizeof(double));
    int rc;
    if (c->devCell.empty()) {
        if ((rc = upload(c, c->dRho, m->rho, (size_t)m->ncells * m->ncomp))) return rc;
    } else {
        std::vector<double> rho((size_t)c->ndev * m->ncomp, 0.0);  // unused device cells: no dust
        for (int q = 0; q < m->ncells; q++)
            for (int h = 0; h < m->ncomp; h++) rho[(size_t)c->devCell[q] * m->ncomp + h] = m->rho[(size_t)q * m->ncomp + h];
        if ((rc = upload(c, c->dRho, rho.data(), rho.size()))) return rc;
    }
    if ((rc = upload(c, c->dOptics, opt.data(), opt.size()))) return rc;
    if (c->gridKind == SKIRT_GRID_VORONOI && !c->vorSlotsHost.empty()) {
        // the density of component 0 in every cell's header, next to its site
        for (int q = 0; q < m->ncells; q++) {
            const double v = m->rho[(size_t)q * m->ncomp];
            std::memcpy(reinterpret_cast<char*>(c->vorSlotsHost.data() + c->vorStartHost[c->devCell[q]]) + 3 * sizeof(double),
                        &v, sizeof v);
        }
        if ((rc = upload(c, c->dVorSlots, c->vorSlotsHost.data(), c->vorSlotsHost.size()))) return rc;
    }
    return SKIRT_OK;
}

int skirt_mcrt_upload_sources(SkirtMcrt* c, const SkirtSourceDesc* s) {
    if (!c || !s) return SKIRT_ERR_ARG;
    if (s->ncomp < 1 || s->nlambda < 1) return fail(c, SKIRT_ERR_ARG, "bad source sizes");
    // device geometry table: the 8 parameters of each component with its kind in the last word
    std::vector<double> gp(8 * (size_t)s->ncomp);
    bool tables = false;
    for (int h = 0; h < s->ncomp; h++) {
        if (s->geom_kind[h] != SKIRT_GEOM_PLUMMER && s->geom_kind[h] != SKIRT_GEOM_EXPDISK &&
            s->geom_kind[h] != SKIRT_GEOM_SERSIC && s->geom_kind[h] != SKIRT_GEOM_POINT)
            return fail(c, SKIRT_ERR_UNSUPPORTED, "unsupported source geometry");
        if (s->geom_kind[h] == SKIRT_GEOM_SERSIC) {
            if (!s->geom_table) return fail(c, SKIRT_ERR_ARG, "SersicGeometry without its tables");
            tables = true;
        }
        for (int q = 0; q < 7; q++) gp[8 * h + q] = s->geom_param[8 * h + q];
        gp[8 * h + 7] = (double)s->geom_kind[h];
    }
    HIPCHECK(c, hipSetDevice(c->device));
    if (c->nlambda && c->nlambda != s->nlambda) return fail(c, SKIRT_ERR_ARG, "sources and media disagree on nlambda");
    if (s->nlambda >= (1 << 14)) return fail(c, SKIRT_ERR_ARG, "at most 16383 wavelengths");
    c->nstar = s->ncomp;
    c->emissionBias = s->emission_bias;
    c->nlambda = s->nlambda;
    int rc;
    if ((rc = upload(c, c->dGeomParam, gp.data(), gp.size()))) return rc;
    if (tables) {
        if ((rc = upload(c, c->dGeomTable, s->geom_table, (size_t)kSersicTable * s->ncomp))) return rc;
    } else if (c->dGeomTable) {
        (void)hipFree(c->dGeomTable);
        c->dGeomTable = nullptr;
    }
    if ((rc = upload(c, c->dLum, s->lum, (size_t)s->ncomp * s->nlambda))) return rc;
    if ((rc = upload(c, c->dLumtot, s->lumtot, (size_t)s->nlambda))) return rc;
    c->lumLo = 0;
    c->lumHi = -1;
    for (int ell = 0; ell < s->nlambda; ell++)
        if (s->lumtot[ell] > 0) {
            if (c->lumHi < 0) c->lumLo = ell;
            c->lumHi = ell;
        }
    if ((rc = upload(c, c->dCdf, s->cdf, (size_t)s->nlambda * (s->ncomp + 1)))) return rc;
    return SKIRT_OK;
}

int skirt_mcrt_set_instruments(SkirtMcrt* c, const SkirtInstrDesc* in, int n) {
    if (!c || n < 0 || (n > 0 && !in)) return SKIRT_ERR_ARG;
    if (n > 63) return fail(c, SKIRT_ERR_ARG, "at most 63 instruments");
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
        if (d.levels < 0 || d.levels > 250) return fail(c, SKIRT_ERR_ARG, "scattering levels out of range");
        d.nslots = d.kind == SKIRT_INSTR_FULL ? 5 + d.levels : 1;
        for (int q = 0; q < 3; q++) d.kobs[q] = in[i].kobs[q];
        d.sinphi = in[i].sinphi; d.cosphi = in[i].cosphi; d.sintheta = in[i].sintheta; d.costheta = in[i].costheta;
        d.sinpa = in[i].sinpa; d.cospa = in[i].cospa;
        d.xpmin = in[i].xpmin; d.xpsiz = in[i].xpsiz; d.ypmin = in[i].ypmin; d.ypsiz = in[i].ypsiz;
        d.slotStride = d.nslots == 1 ? 1 : (d.nslots + 7) / 8 * 8;
        // every frame starts on a 64-byte line (the tally itself is at least 256-byte aligned), so that a
        // detection's slots (slotStride 8) share one line and one atomic request also after another
        // instrument's SEDs
        off = (off + 7) & ~7LL;
        d.frameBase = off;
        const long long nframes = (d.kind == SKIRT_INSTR_SED) ? 0 : (long long)d.slotStride * c->nlambda * d.nx * d.ny;
        off += nframes;
        d.sedBase = off;
        const long long nseds = (d.kind == SKIRT_INSTR_FRAME) ? 0 : (long long)d.nslots * c->nlambda;
        off += nseds;
        d.sedOff = sedOff;
        sedOff += (int)nseds;
        c->instr.push_back(d);
    }
    c->nInstrTally = (size_t)off;
    c->nsed = sedOff;
    int rc = upload(c, c->dInstr, c->instr.data(), c->instr.size());
    if (rc) return rc;
    if (c->ownTally && c->dTally) { (void)hipFree(c->dTally); c->dTally = nullptr; }
    if (c->dPool) { (void)hipFree(c->dPool); c->dPool = nullptr; c->nslots = 0; }
    return SKIRT_OK;
}

int skirt_mcrt_tally_sizes(SkirtMcrt* c, size_t* nl, size_t* ni) {
    if (!c) return SKIRT_ERR_ARG;
    if (nl) *nl = (size_t)c->labsStride * c->nlambda;
    if (ni) *ni = c->nInstrTally;
    return SKIRT_OK;
}

static int ensureTallies(SkirtMcrt* c) {
    const size_t nl = (size_t)c->labsStride * c->nlambda;
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
    const size_t nl = (size_t)c->labsStride * c->nlambda;
    if (c->dLabs && nl) HIPCHECK(c, hipMemsetAsync(c->dLabs, 0, nl * sizeof(double), c->stream));
    if (c->dTally && c->nInstrTally) HIPCHECK(c, hipMemsetAsync(c->dTally, 0, c->nInstrTally * sizeof(double), c->stream));
    HIPCHECK(c, hipMemsetAsync(c->dStats, 0, 8 * kStatCopies * sizeof(unsigned long long), c->stream));
    HIPCHECK(c, hipMemsetAsync(c->dError, 0, sizeof(unsigned int), c->stream));
    if (c->dCrossed)
        HIPCHECK(c, hipMemsetAsync(c->dCrossed, 0, (size_t)kCrossedCopies * c->crossedBins * sizeof(unsigned long long), c->stream));
    c->instrReduced = false;
    c->packagesTotal = 0;
    return SKIRT_OK;
}

int skirt_mcrt_run_stellar(SkirtMcrt* c, uint64_t npp, uint64_t first, uint64_t count, uint64_t seed,
                           const SkirtPhaseParams* p) {
    return skirt_mcrt_run_phase(c, SKIRT_PHASE_STELLAR, 0, npp, first, count, seed, p);
}

// the guide tables of the cell CDFs (dCellCdf must hold them), on the engine's stream
static int buildCellGuide(SkirtMcrt* c) {
    const int N = c->ncells, Nl = c->nlambda;
    const size_t n = (size_t)Nl * (N + 1);
    if (c->dCellGuide && c->cellGuideCount != n) { (void)hipFree(c->dCellGuide); c->dCellGuide = nullptr; }
    if (!c->dCellGuide) HIPCHECK(c, hipMalloc(&c->dCellGuide, n * sizeof(int)));
    c->cellGuideCount = n;
    hipLaunchKernelGGL(cellGuideKernel, dim3((N + 1 + kBlock - 1) / kBlock, Nl), dim3(kBlock), 0, c->stream,
                       (const double*)c->dCellCdf, c->dCellGuide, N);
    HIPCHECK(c, hipGetLastError());
    return SKIRT_OK;
}

int skirt_mcrt_upload_cell_sources(SkirtMcrt* c, const SkirtCellSourceDesc* src) {
    if (!c || !src) return SKIRT_ERR_ARG;
    if (c->gridKind < 0) return fail(c, SKIRT_ERR_STATE, "upload the grid before cell sources");
    if (src->ncells != c->ncells || src->nlambda != c->nlambda || !src->lv || !src->cdf || !src->ltot)
        return fail(c, SKIRT_ERR_ARG, "cell sources do not match the grid and wavelengths");
    if (!(src->emission_bias >= 0 && src->emission_bias < 1)) return fail(c, SKIRT_ERR_ARG, "emission bias outside [0,1)");
    HIPCHECK(c, hipSetDevice(c->device));
    const size_t nl = (size_t)c->nlambda, nc = (size_t)c->ncells;
    int rc;
    if ((rc = upload(c, c->dCellLv, src->lv, nl * nc))) return rc;
    if ((rc = upload(c, c->dCellCdf, src->cdf, nl * (nc + 1)))) return rc;
    if ((rc = upload(c, c->dCellLtot, src->ltot, nl))) return rc;
    c->cellBias = src->emission_bias;
    return buildCellGuide(c);
}

static int ensureDustLabs(SkirtMcrt* c);

// scratch of the cell-source scans and the dust Labs sum: block sums of every wavelength (or of the
// whole dust table) plus two result slots
static int ensureEmisScratch(SkirtMcrt* c) {
    if (c->dEmisScratch) return SKIRT_OK;
    const size_t nb = (size_t)c->nlambda * (((size_t)c->ncells + kBlock - 1) / kBlock);
    const size_t nbAll = ((size_t)c->labsStride * c->nlambda + kBlock - 1) / kBlock;
    HIPCHECK(c, hipMalloc(&c->dEmisScratch, (std::max(nb, nbAll) + 2) * sizeof(double)));
    return SKIRT_OK;
}

int skirt_mcrt_upload_emissivity(SkirtMcrt* c, const SkirtEmissivityDesc* d) {
    if (!c || !d) return SKIRT_ERR_ARG;
    if (c->gridKind < 0 || !c->dRho) return fail(c, SKIRT_ERR_STATE, "upload the grid and media before the emissivity");
    if (d->ncells != c->ncells || d->nlambda != c->nlambda || d->ncomp != c->ncomp || d->ntemp < 2)
        return fail(c, SKIRT_ERR_ARG, "emissivity tables do not match the grid, wavelengths and media");
    HIPCHECK(c, hipSetDevice(c->device));
    const size_t nl = (size_t)d->nlambda, nh = (size_t)d->ncomp;
    int rc;
    if ((rc = upload(c, c->dEmisVolume, d->volume, (size_t)d->ncells))) return rc;
    if ((rc = upload(c, c->dEmisKabs, d->kabs, nh * nl))) return rc;
    if ((rc = upload(c, c->dEmisSigma, d->sigmaabs, nh * nl))) return rc;
    if ((rc = upload(c, c->dEmisMu, d->mu, nh))) return rc;
    if ((rc = upload(c, c->dEmisTv, d->tv, (size_t)d->ntemp))) return rc;
    if ((rc = upload(c, c->dEmisPlanck, d->planckabs, nh * d->ntemp))) return rc;
    if ((rc = upload(c, c->dEmisLambda, d->lambda, nl))) return rc;
    if ((rc = upload(c, c->dEmisDlambda, d->dlambda, nl))) return rc;
    if (!c->devCell.empty() && (rc = upload(c, c->dDevCell, c->devCell.data(), c->devCell.size()))) return rc;
    c->emisNtemp = d->ntemp;
    c->cellBias = d->emission_bias;
    return SKIRT_OK;
}

int skirt_mcrt_compute_cell_sources(SkirtMcrt* c, int include_dust) {
    if (!c) return SKIRT_ERR_ARG;
    if (!c->emisNtemp) return fail(c, SKIRT_ERR_STATE, "no emissivity uploaded");
    if (!c->dLabs) return fail(c, SKIRT_ERR_STATE, "no Labs tally");
    HIPCHECK(c, hipSetDevice(c->device));
    if (include_dust) {
        int rc = ensureDustLabs(c);
        if (rc) return rc;
    }
    const int N = c->ncells, Nl = c->nlambda;
    const int nblocks = (N + kBlock - 1) / kBlock;
    auto alloc = [&](double*& p, size_t n) -> int {
        if (!p) HIPCHECK(c, hipMalloc(&p, n * sizeof(double)));
        return SKIRT_OK;
    };
    int rc;
    if ((rc = alloc(c->dCellLv, (size_t)Nl * N)) || (rc = alloc(c->dCellCdf, (size_t)Nl * (N + 1))) ||
        (rc = alloc(c->dCellLtot, (size_t)Nl)) || (rc = ensureEmisScratch(c)))
        return rc;
    EmisArgs e{};
    e.ncells = N; e.nlambda = Nl; e.ncomp = c->ncomp; e.ntemp = c->emisNtemp; e.labsStride = c->labsStride;
    e.devCell = c->devCell.empty() ? nullptr : c->dDevCell;
    e.labs = c->dLabs; e.labsDust = include_dust ? c->dLabsDust : nullptr;
    e.rho = c->dRho; e.volume = c->dEmisVolume; e.kabs = c->dEmisKabs; e.sigmaabs = c->dEmisSigma; e.mu = c->dEmisMu;
    e.Tv = c->dEmisTv; e.planckabs = c->dEmisPlanck; e.lambda = c->dEmisLambda; e.dlambda = c->dEmisDlambda;
    e.lv = c->dCellLv; e.cdf = c->dCellCdf; e.ltot = c->dCellLtot; e.blockSums = c->dEmisScratch; e.nblocks = nblocks;
    hipLaunchKernelGGL(cellSpectraKernel, dim3(nblocks), dim3(kBlock), 0, c->stream, e);
    hipLaunchKernelGGL(cellBlockSumKernel, dim3(nblocks, Nl), dim3(kBlock), 0, c->stream, e);
    hipLaunchKernelGGL(cellScanBlocksKernel, dim3(Nl), dim3(kBlock), 0, c->stream, e);
    hipLaunchKernelGGL(cellCdfKernel, dim3(nblocks, Nl), dim3(kBlock), 0, c->stream, e);
    HIPCHECK(c, hipGetLastError());
    return buildCellGuide(c);
}

int skirt_mcrt_dust_labs_total(SkirtMcrt* c, double* total) {
    if (!c || !total) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    int rc = ensureDustLabs(c);
    if (rc) return rc;
    const size_t n = (size_t)c->labsStride * c->nlambda;  // unused device cells hold zeros
    if ((rc = ensureEmisScratch(c))) return rc;
    // reuse the cell-sum kernels on the dust table viewed as one "wavelength" of n cells
    EmisArgs e{};
    e.ncells = (int)n; e.nlambda = 1; e.lv = c->dLabsDust; e.blockSums = c->dEmisScratch;
    e.nblocks = (int)((n + kBlock - 1) / kBlock);
    e.ltot = c->dEmisScratch + e.nblocks;  // one slot past the block sums
    hipLaunchKernelGGL(cellBlockSumKernel, dim3(e.nblocks, 1), dim3(kBlock), 0, c->stream, e);
    hipLaunchKernelGGL(cellScanBlocksKernel, dim3(1), dim3(kBlock), 0, c->stream, e);
    HIPCHECK(c, hipGetLastError());
    HIPCHECK(c, hipMemcpyAsync(total, e.ltot, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    return SKIRT_OK;
}

static int ensureDustLabs(SkirtMcrt* c) {
    const size_t nl = (size_t)c->labsStride * c->nlambda;
    if (!c->dLabsDust && nl) {
        HIPCHECK(c, hipMalloc(&c->dLabsDust, nl * sizeof(double)));
        HIPCHECK(c, hipMemsetAsync(c->dLabsDust, 0, nl * sizeof(double), c->stream));
        c->ownLabsDust = true;
    }
    return SKIRT_OK;
}

int skirt_mcrt_bind_dust_labs(SkirtMcrt* c, double* d) {
    if (!c || !d) return SKIRT_ERR_ARG;
    if (c->ownLabsDust && c->dLabsDust) (void)hipFree(c->dLabsDust);
    // the Labs replicas (dLabsRep) stay: they depend on the table's size only, not on where it lives
    c->dLabsDust = d;
    c->ownLabsDust = false;
    return SKIRT_OK;
}

int skirt_mcrt_zero_dust_labs(SkirtMcrt* c) {
    if (!c) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    int rc = ensureDustLabs(c);
    if (rc) return rc;
    const size_t nl = (size_t)c->labsStride * c->nlambda;
    if (nl) HIPCHECK(c, hipMemsetAsync(c->dLabsDust, 0, nl * sizeof(double), c->stream));
    return SKIRT_OK;
}

int skirt_mcrt_download_dust_labs(SkirtMcrt* c, double* labs) {
    if (!c || !labs) return SKIRT_ERR_ARG;
    int rc = skirt_mcrt_synchronize(c);
    if (rc) return rc;
    const size_t nl = (size_t)c->labsStride * c->nlambda;
    if (!c->dLabsDust) { std::fill(labs, labs + nl, 0.0); return SKIRT_OK; }
    std::vector<double> t(nl);
    HIPCHECK(c, hipMemcpy(t.data(), c->dLabsDust, nl * sizeof(double), hipMemcpyDeviceToHost));
    const bool perm = !c->devCell.empty();
    for (int ell = 0; ell < c->nlambda; ell++)
        for (int m = 0; m < c->ncells; m++)
            labs[(size_t)m * c->nlambda + ell] = t[(size_t)ell * c->labsStride + (perm ? c->devCell[m] : m)];
    return SKIRT_OK;
}

static const char* const kSummedTwice =
    "the instrument tallies were already summed over the processes: zero the tallies before another phase";
static int runPhase(SkirtMcrt* c, int phase, uint32_t cycle, uint64_t npp, uint64_t first, uint64_t count,
                    uint64_t sliceLo, uint64_t sliceCnt, uint64_t seed, const SkirtPhaseParams* p);
static int phaseEndReduce(SkirtMcrt* c, int phase, const SkirtPhaseParams* p);

int skirt_mcrt_run_phase(SkirtMcrt* c, int phase, uint32_t cycle, uint64_t npp, uint64_t first, uint64_t count,
                         uint64_t seed, const SkirtPhaseParams* p) {
    if (!c || !p) return SKIRT_ERR_ARG;
    if (first + count > npp * (uint64_t)c->nlambda) return fail(c, SKIRT_ERR_ARG, "packet range exceeds npp*nlambda");
    if (c->instrReduced) return fail(c, SKIRT_ERR_STATE, kSummedTwice);
    int rc = runPhase(c, phase, cycle, npp, first, count, 0, npp, seed, p);
    return rc ? rc : phaseEndReduce(c, phase, p);
}

int skirt_mcrt_run_phase_shard(SkirtMcrt* c, int phase, uint32_t cycle, uint64_t npp, int rank, int world,
                               uint64_t seed, const SkirtPhaseParams* p) {
    if (!c || !p) return SKIRT_ERR_ARG;
    if (world < 1 || rank < 0 || rank >= world) return fail(c, SKIRT_ERR_ARG, "bad shard (rank, world)");
    if (world > 1 && !c->reduce) return fail(c, SKIRT_ERR_STATE, "a sharded phase needs a reducer (skirt_mcrt_set_reducer)");
    if (c->instrReduced) return fail(c, SKIRT_ERR_STATE, kSummedTwice);
    // SequentialAssigner over the packets of one wavelength (SequentialAssigner.cpp:37-59), the same
    // block at every wavelength (IdenticalAssigner.cpp:37-58)
    uint64_t lo = 0, cnt = 0;
    skirt_mcrt_shard_slice(npp, rank, world, &lo, &cnt);
    int rc = runPhase(c, phase, cycle, npp, 0, cnt * (uint64_t)c->nlambda, lo, cnt, seed, p);
    return rc ? rc : phaseEndReduce(c, phase, p);
}

void skirt_mcrt_shard_slice(uint64_t npp, int rank, int world, uint64_t* lo, uint64_t* count) {
    const unsigned __int128 n = npp;
    const uint64_t a = (uint64_t)(n * (unsigned)rank / (unsigned)world);
    const uint64_t b = (uint64_t)(n * (unsigned)(rank + 1) / (unsigned)world);
    if (lo) *lo = a;
    if (count) *count = b - a;
}

int skirt_mcrt_set_reducer(SkirtMcrt* c, SkirtReduceTallyFn fn, void* user) {
    if (!c) return SKIRT_ERR_ARG;
    c->reduce = fn;
    c->reduceUser = user;
    return SKIRT_OK;
}

int skirt_mcrt_reduce_instruments(SkirtMcrt* c) {
    if (!c) return SKIRT_ERR_ARG;
    if (!c->reduce || c->instrReduced || !c->dTally || !c->nInstrTally) return SKIRT_OK;
    HIPCHECK(c, hipSetDevice(c->device));
    // marked summed only once the reducer succeeded: a failed reduction can be retried
    if (c->reduce(c->reduceUser, SKIRT_TALLY_INSTRUMENTS, c->dTally, c->nInstrTally, (void*)c->stream))
        return fail(c, SKIRT_ERR_STATE, "the instrument reduction failed");
    c->instrReduced = true;
    return SKIRT_OK;
}

// the Labs replicas of an absorbing phase (Args::labsCopies) added into the table, in replica order, and
// zeroed for the next phase
__global__ void labsFoldKernel(double* dst, double* rep, size_t n, int copies, size_t strideElems) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        double sum = 0.0;
        for (int k = 0; k < copies; k++) {
            sum += rep[k * strideElems + i];
            rep[k * strideElems + i] = 0.0;
        }
        dst[i] += sum;
    }
}

// PanDustSystem::sumResults at the end of a phase (PanDustSystem.cpp:394-403): the stellar Labs after the
// stellar phase, the dust Labs after a self-absorption cycle, summed over the processes by the caller's
// reducer, enqueued behind the phase on the engine stream. Instrument::sumResults (Instrument.cpp:57)
// comes once, before the tallies are read (skirt_mcrt_reduce_instruments / download).
static int phaseEndReduce(SkirtMcrt* c, int phase, const SkirtPhaseParams* p) {
    if (!c->reduce) return SKIRT_OK;
    const size_t n = (size_t)c->labsStride * c->nlambda;
    int r = 0;
    if (phase == SKIRT_PHASE_STELLAR && p->store_absorption && c->dLabs && n)
        r = c->reduce(c->reduceUser, SKIRT_TALLY_LABS, c->dLabs, n, (void*)c->stream);
    else if (phase == SKIRT_PHASE_DUST_SELFABS && c->dLabsDust && n)
        r = c->reduce(c->reduceUser, SKIRT_TALLY_DUST_LABS, c->dLabsDust, n, (void*)c->stream);
    return r ? fail(c, SKIRT_ERR_STATE, "the absorption reduction failed") : SKIRT_OK;
}

static int runPhase(SkirtMcrt* c, int phase, uint32_t cycle, uint64_t npp, uint64_t first, uint64_t count,
                    uint64_t sliceLo, uint64_t sliceCnt, uint64_t seed, const SkirtPhaseParams* p) {
    if (phase < SKIRT_PHASE_STELLAR || phase > SKIRT_PHASE_DUST_SELFABS) return fail(c, SKIRT_ERR_ARG, "unknown phase");
    if (cycle >= (1u << 30)) return fail(c, SKIRT_ERR_ARG, "cycle number too large");
    const bool cellPhase = phase != SKIRT_PHASE_STELLAR;
    if (cellPhase && (!c->dCellLtot || !p->has_dust)) return fail(c, SKIRT_ERR_STATE, "a dust phase needs a dust system and uploaded cell sources");
    if (c->gridKind < 0 && p->has_dust) return fail(c, SKIRT_ERR_STATE, "no grid uploaded");
    if (!cellPhase && !c->dLumtot) return fail(c, SKIRT_ERR_STATE, "no sources uploaded");
    if (p->has_dust && !c->dRho) return fail(c, SKIRT_ERR_STATE, "no media uploaded");
    if (first + count > npp * (uint64_t)c->nlambda) return fail(c, SKIRT_ERR_ARG, "packet range exceeds npp*nlambda");
    if (p->min_weight_reduction <= 0 || p->scatt_bias < 0 || p->scatt_bias > 1) return fail(c, SKIRT_ERR_ARG, "bad phase parameters");
    HIPCHECK(c, hipSetDevice(c->device));
    int rc = ensureTallies(c);
    if (rc) return rc;
    if (phase == SKIRT_PHASE_DUST_SELFABS && (rc = ensureDustLabs(c))) return rc;
    c->lastMs = 0;
    c->phaseTimed = false;
    c->lastIterations = 0;
    if (c->traceLaunches) {  // time the previous call's launches before their events are reused
        HIPCHECK(c, hipStreamSynchronize(c->stream));
        float ms = 0;
        for (int k = 0; k < c->traceLaunches; k++)
            if (hipEventElapsedTime(&ms, c->traceEv[2 * k], c->traceEv[2 * k + 1]) == hipSuccess) c->traceMs += ms;
        c->traceLaunchesTotal += (uint64_t)c->traceLaunches;
        c->traceLaunches = 0;
    }
    c->packagesTotal += count;
    if (!cellPhase) {
        // the wavelengths outside [lumLo, lumHi] launch nothing: their packet indices (per wavelength sliceCnt
        // of them, wavelength-slowest) are left out of the phase instead of being claimed and skipped one by one
        const uint64_t lo = c->lumHi < 0 ? 0 : (uint64_t)c->lumLo * sliceCnt;
        const uint64_t hi = c->lumHi < 0 ? 0 : (uint64_t)(c->lumHi + 1) * sliceCnt;
        const uint64_t b = std::max(first, lo), e = std::min(first + count, hi);
        first = b;
        count = e > b ? e - b : 0;
    }
    if (count == 0) return SKIRT_OK;
    if (!c->dOptics) {  // a dust-free simulation still stages (zero) optical tables
        std::vector<double> z(4 * (size_t)c->nlambda, 0.0);
        if ((rc = upload(c, c->dOptics, z.data(), z.size()))) return rc;
    }
    // slot pool: enough packets in flight to fill the chip many times over, bounded by the phase size.
    // 2^24 slots (6.6 GB of packet state and ray queues with one instrument) make each iteration's trace
    // launch long enough that its drain tail and the event kernel amortise (round 1, C3: 2^21 slots 1.87e8
    // pkt/s, 2^22 1.98e8, 2^23 2.04e8, 2^24 2.05e8; round 4 at the configurations' sizes, 2^24 against
    // 2^23: C3 +1.5 %, C2 +0.7 %, C4 +0.7 %, C5 +0.3 %, profiles/r04_slots_2e24.txt)
    int slots = c->slotsWanted > 0 ? c->slotsWanted : (1 << 24);
    // continuous scattering (MonteCarloSimulation::continuousScattering): peel-offs from every dust segment
    // of every path replace the ones at the interaction points; fewer slots, each with a longer queue
    const bool continuous = p->continuous_scattering && phase != SKIRT_PHASE_DUST_SELFABS && p->has_dust &&
                            !c->instr.empty();
    // (the queue holds kPathCap peel-offs per instrument and slot: the slots shrink with the instruments)
    if (continuous) slots = std::min(slots, std::max(64, kContSlots / std::max(1, (int)c->instr.size())));
    if ((uint64_t)slots > count) slots = (int)count;
    // (a phase that fits the pool runs its packets in lockstep; admitting them in 2 or 4 waves instead changes
    // neither the C5 step nor its 164 trace launches: the tail iterations are the few long-lived packets either
    // way, profiles/r06_ab.txt)
    const int halves = (continuous || !p->has_dust || slots < 2 * 64 * kMaxHalves) ? 1 : c->halves;
    slots = std::max(slots, 64 * halves) / halves;  // per half
    const bool forked = c->halves > 1 || c->cusT || c->cusE;  // the pipeline runs on the owned streams
    // the detect kernel of an iteration beside the next iteration's event kernel (one pipeline on the
    // caller's stream, peel-offs at the interaction points): C3 +1.9 %, C2 within the spread; beside the
    // next trace kernel as well, C3 +1.6 %, C2 -1.5 %. Not for Voronoi grids: C4 -2.2 %, and -2.6 % again
    // after the counter-line and event-grid changes (profiles/r05_detect_aside_ab.txt)
    const bool detAside = !forked && !continuous && !c->instr.empty() && p->has_dust &&
                          c->gridKind != SKIRT_GRID_VORONOI;
    if ((rc = ensurePool(c, slots, continuous, halves, detAside))) return rc;
    if ((rc = ensureStreams(c))) return rc;
    if (detAside && !c->sD) {
        HIPCHECK(c, hipStreamCreateWithFlags(&c->sD, hipStreamNonBlocking));
        HIPCHECK(c, hipEventCreateWithFlags(&c->evDetT, hipEventDisableTiming));
        HIPCHECK(c, hipEventCreateWithFlags(&c->evDet[0], hipEventDisableTiming));
        HIPCHECK(c, hipEventCreateWithFlags(&c->evDet[1], hipEventDisableTiming));
        HIPCHECK(c, hipEventCreateWithFlags(&c->evDetJoin, hipEventDisableTiming));
    }
    hipStream_t sE = forked ? c->sE : c->stream;
    hipStream_t sT[kMaxHalves];
    for (int h = 0; h < kMaxHalves; h++) sT[h] = forked ? c->sT[h] : c->stream;

    Args a{};
    gridArgs(c, a);
    const bool bookkeeping = c->gridKind == SKIRT_GRID_OCTREE && c->search == SKIRT_TREE_BOOKKEEPING;
    const bool leafMap = c->gridKind == SKIRT_GRID_OCTREE && c->mapL >= 0 && p->has_dust && !bookkeeping;
    if (leafMap) {
        if ((rc = ensureLeafMap(c))) return rc;
        a.leafMap = c->dLeafMap; a.treeT = c->dTreeT; a.mapL = c->mapL; a.mapN = c->mapN;
        a.mapInvX = c->mapInv[0]; a.mapInvY = c->mapInv[1]; a.mapInvZ = c->mapInv[2];
        a.mapX0 = c->mapOrigin[0]; a.mapY0 = c->mapOrigin[1]; a.mapZ0 = c->mapOrigin[2];
    }
    a.optics = c->dOptics;
    a.nstar = c->nstar; a.geomParam = c->dGeomParam; a.geomTable = c->dGeomTable; a.lum = c->dLum;
    a.lumtot = c->dLumtot; a.cdf = c->dCdf; a.emissionBias = c->emissionBias;
    a.ninstr = (int)c->instr.size(); a.instr = c->dInstr; a.nsed = c->nsed;
    a.npp = npp; a.first = first; a.end = first + count; a.seed = seed;
    a.sliceLo = sliceLo; a.sliceCnt = sliceCnt;
    a.tag = (unsigned)phase | (cycle << 2);  // Philox counter word 1: streams differ per phase and cycle
    a.phase = phase;
    a.peel = phase != SKIRT_PHASE_DUST_SELFABS;
    a.continuous = continuous ? 1 : 0;
    a.cellLv = c->dCellLv; a.cellCdf = c->dCellCdf; a.cellGuide = c->dCellGuide; a.cellLtot = c->dCellLtot; a.cellBias = c->cellBias;
    a.cellNode = c->dCellNode;
    a.minWeightReduction = p->min_weight_reduction; a.minScatt = p->min_scatt_events; a.xi = p->scatt_bias;
    // absorption: the stellar phase as its parameters say (into Labs), self-absorption always (into the
    // dust Labs), dust emission never (MonteCarloSimulation.cpp:287, PanMonteCarloSimulation.cpp:223, 331)
    a.store = phase == SKIRT_PHASE_STELLAR ? (p->store_absorption ? 1 : 0) : (phase == SKIRT_PHASE_DUST_SELFABS ? 1 : 0);
    a.hasDust = p->has_dust ? 1 : 0;
    if (a.store && !c->dLabs) return fail(c, SKIRT_ERR_STATE, "no Labs buffer");
    // the trace kernel adds to Labs through a buffer descriptor (32-bit byte offsets, one byte past the end
    // for the drain's empty lanes) while the table holds at most 4 GiB - 8 (e.g. 2^21 cells x 255
    // wavelengths), with global atomics beyond (SKIRT_AMD_LABS_GLOBAL=1 forces them: tests)
    const uint64_t labsElems = (uint64_t)c->labsStride * (uint64_t)c->nlambda;
    // 2^32 elements or more (32 GiB): the buffered adds carry 40-bit element indices (SKIRT_AMD_LABS_HI=1 forces
    // that path: tests); 2^40 elements at most
    if (a.store && labsElems >= (1ull << 40)) return fail(c, SKIRT_ERR_UNSUPPORTED, "Labs table of 2^40 elements or more");
    const bool forceHi = getenv("SKIRT_AMD_LABS_HI") && atoi(getenv("SKIRT_AMD_LABS_HI")) != 0;
    a.labsHi = (a.store && (forceHi || labsElems > 0xffffffffull)) ? 1 : 0;
    const bool forceGlobal = getenv("SKIRT_AMD_LABS_GLOBAL") && atoi(getenv("SKIRT_AMD_LABS_GLOBAL")) != 0;
    a.labsGlobal = (forceGlobal || a.labsHi || labsElems * sizeof(double) > 0xfffffff8ull) ? 1 : 0;
    a.labs = phase == SKIRT_PHASE_DUST_SELFABS ? c->dLabsDust : c->dLabs;
    a.labsBytes = a.labsGlobal ? 0u : (unsigned)(labsElems * sizeof(double));
    // The trace waves add into K replicas of the table (wave w into w % K), folded into it at the phase end:
    // the adds to one cell spread over K lines, which the memory-side atomic unit works on side by side.
    // In the stellar phase the replicas pay while they stay near the MALL (256 MB): C3 (a 129 MB table) 2:
    // +1.1 %, 3: +1.2 %, 4: +0.8 %, 6: -1 %, 8: -3.4 %; C2 (21 MB) 4: +2 %, 8: +3.3 %. The self-absorption
    // cycles' adds crowd onto fewer lines and gain up to 6: C5 with 3 in the stellar phase and 6 in the
    // cycles +9.0 % against none, +3.6 % against 2 everywhere; C3 +1.2 % (profiles/r05_labs_copies_ab.txt).
    // K = 400 MiB (self-absorption: 800 MiB) / the table, at most 8; SKIRT_AMD_LABS_COPIES sets it (1: none)
    double* const labsTarget = a.labs;
    a.labsCopies = 1;
    a.labsCopyStride = 0;
    {
        const uint64_t tableBytes = (uint64_t)a.labsBytes > 0 ? (uint64_t)a.labsBytes : 1;
        const uint64_t budget = phase == SKIRT_PHASE_DUST_SELFABS ? (800ull << 20) : (400ull << 20);
        const int Kauto = (int)std::min<uint64_t>(8, std::max<uint64_t>(1, budget / tableBytes));
        const int K = getenv("SKIRT_AMD_LABS_COPIES") ? atoi(getenv("SKIRT_AMD_LABS_COPIES")) : Kauto;
        const uint64_t stride = ((uint64_t)a.labsBytes + 255) & ~255ull;
        if (a.store && !a.labsGlobal && K > 1 && K <= 64 && stride * (uint64_t)K <= 0xfffffff0ull) {
            const size_t need = (size_t)stride * K;
            if (c->labsRepBytes < need) {
                if (c->dLabsRep) HIPCHECK(c, hipFree(c->dLabsRep));
                c->dLabsRep = nullptr;
                c->labsRepBytes = 0;
                HIPCHECK(c, hipMalloc(&c->dLabsRep, need));
                HIPCHECK(c, hipMemsetAsync(c->dLabsRep, 0, need, c->stream));
                c->labsRepBytes = need;
            }
            if (c->labsRepDirty) {  // (the failed phase's trace launches may still run on the pipeline streams)
                HIPCHECK(c, hipDeviceSynchronize());
                HIPCHECK(c, hipMemsetAsync(c->dLabsRep, 0, c->labsRepBytes, c->stream));
            }
            c->labsRepDirty = true;  // until the fold at this phase's end
            a.labs = c->dLabsRep;
            a.labsCopies = K;
            a.labsCopyStride = (unsigned)stride;
        }
    }
    a.tally = c->dTally;
    a.error = c->dError; a.stats = c->dStats;
    a.crossed = c->dCrossed; a.crossedBins = c->crossedBins;
    a.claim = c->dClaim;
    a.threshold = c->threshold > 0 ? c->threshold : (c->gridKind == SKIRT_GRID_VORONOI ? 8 : 16);
    a.walkBack = c->walkBack >= 0 ? c->walkBack : (c->gridKind == SKIRT_GRID_VORONOI ? 1 : 0);
    // LDS layout (doubles): mesh | optics | instruments | SED sums
    int off = 0;
    a.ldsMeshOff = off;
    off += (c->gridKind == SKIRT_GRID_CARTESIAN && a.hasDust) ? (c->nx + c->ny + c->nz + 3) : 0;
    off += leafMap ? 3 * (c->mapN + 1) : 0;
    off = (off + 1) & ~1;
    a.ldsOptOff = off;
    off += 4 * a.ncomp * a.nlambda;
    off = (off + 1) & ~1;
    a.ldsInstrOff = off;
    off += a.ninstr * (int)(sizeof(DevInstr) / sizeof(double));
    a.ldsSedOff = off;
    off += c->nsed;
    // a phase storing no absorption with one component runs traceKernelNoStore (no Labs buffers)
    const bool noStore = !a.store && a.ncomp == 1 && !continuous && c->gridKind != SKIRT_GRID_VORONOI &&
                         !getenv("SKIRT_AMD_NO_NOSTORE");
    const size_t ldsTrace = (size_t)a.ldsInstrOff * sizeof(double)          // grid tables + optics
                            + (size_t)kSegWords * sizeof(double)                          // + segment counts
                            + (noStore ? 0 : (size_t)kLabsBuf * kBlock * (sizeof(double) + sizeof(unsigned)))  // + Labs buffers
                            + (a.labsHi ? (size_t)kLabsBuf * kBlock : 0);  // + their high index bytes
    const size_t ldsEvent = (size_t)a.ldsSedOff * sizeof(double);           // + instruments
    // budget: what one workgroup may allocate (160 KiB on gfx950). The trace and event kernels need their
    // tables; the detect kernel keeps as many SED copies as fit (8, 4, 2, 1), or none (SEDs to the tally)
    const size_t budget = c->ldsMax;
    if (ldsTrace > budget || ldsEvent > budget)
        return fail(c, SKIRT_ERR_UNSUPPORTED, "grid and optical tables do not fit in LDS (" +
                                                  std::to_string(std::max(ldsTrace, ldsEvent)) + " of " +
                                                  std::to_string(budget) + " bytes)");
    // SKIRT_AMD_DET_COPIES caps the copies (tests of the fallbacks)
    const int capCopies = getenv("SKIRT_AMD_DET_COPIES") ? atoi(getenv("SKIRT_AMD_DET_COPIES")) : kDetectCopies;
    a.detCopies = kDetectCopies;
    while (a.detCopies > 0 && a.detCopies > capCopies) a.detCopies >>= 1;
    while (a.detCopies > 0 && ldsEvent + (size_t)a.detCopies * c->nsed * sizeof(double) > budget) a.detCopies >>= 1;
    const size_t ldsDetect = ldsEvent + (size_t)a.detCopies * c->nsed * sizeof(double);
    c->lastDetCopies = a.detCopies;
    // launches above 64 KiB of dynamic LDS declare it first
    if (ldsDetect > 64 * 1024)
        HIPCHECK(c, hipFuncSetAttribute((const void*)detectKernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)ldsDetect));
    const int kind = c->gridKind == SKIRT_GRID_CARTESIAN ? SKIRT_GRID_CARTESIAN
                     : c->gridKind == SKIRT_GRID_VORONOI ? SKIRT_GRID_VORONOI
                     : bookkeeping ? kOctreeBookkeeping
                     : (leafMap ? (c->binTree ? kBinTreeMap : SKIRT_GRID_OCTREE) : kOctreeNodes);
    c->lastWalk = kind == SKIRT_GRID_CARTESIAN ? SKIRT_WALK_CARTESIAN
                  : kind == SKIRT_GRID_OCTREE  ? SKIRT_WALK_OCTREE_MAP
                  : kind == kBinTreeMap        ? SKIRT_WALK_KDTREE_MAP
                  : kind == kOctreeBookkeeping ? SKIRT_WALK_OCTREE_BOOKKEEPING
                  : kind == SKIRT_GRID_VORONOI ? SKIRT_WALK_VORONOI
                                               : SKIRT_WALK_TREE_NODES;
    const bool one = a.ncomp == 1;
    const void* traceFn = nullptr;
    auto pick = [&](auto fn1, auto fnN, auto fn1c, auto fnNc, const void* fnNoStore) {
        traceFn = continuous ? (one ? (const void*)fn1c : (const void*)fnNc) : (one ? (const void*)fn1 : (const void*)fnN);
        if (noStore) traceFn = fnNoStore;
    };
#define SKIRT_PICK4(G, L) pick(traceKernel<G, true, false, L>, traceKernel<G, false, false, L>, traceKernel<G, true, true, L>, \
                              traceKernel<G, false, true, L>, (const void*)traceKernelNoStore<G>)
#define SKIRT_PICK(G) (a.labsGlobal ? SKIRT_PICK4(G, true) : SKIRT_PICK4(G, false))
    if (kind == SKIRT_GRID_CARTESIAN) SKIRT_PICK(SKIRT_GRID_CARTESIAN);
    else if (kind == SKIRT_GRID_OCTREE) SKIRT_PICK(SKIRT_GRID_OCTREE);
    else if (kind == kBinTreeMap) SKIRT_PICK(kBinTreeMap);
    else if (kind == kOctreeBookkeeping) SKIRT_PICK(kOctreeBookkeeping);
    else if (kind == SKIRT_GRID_VORONOI) {
        if (a.labsGlobal)
            pick(traceKernelVor<true, false, true>, traceKernelVor<false, false, true>, traceKernelVor<true, true, true>,
                 traceKernelVor<false, true, true>, nullptr);
        else
            pick(traceKernelVor<true, false>, traceKernelVor<false, false>, traceKernelVor<true, true>,
                 traceKernelVor<false, true>, nullptr);
    }
    else SKIRT_PICK(kOctreeNodes);
#undef SKIRT_PICK
#undef SKIRT_PICK4
    if (ldsTrace > 64 * 1024)
        HIPCHECK(c, hipFuncSetAttribute(traceFn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsTrace));
    int tgrid = c->traceGrid;
    if (tgrid <= 0) {
        int per = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, traceFn, kBlock, ldsTrace) != hipSuccess || per < 1) per = 2;
        tgrid = std::max(1, c->nCusT) * per;
        c->traceBlocksPerCU = per;
    }
    // event kernel blocks per CU: 3 (3 waves/SIMD, the registers allow it). Voronoi: C4 +0.6 % against 2
    // (profiles/r04_event_bpc_sweep.txt); the other grids, once the block reservations no longer serialize on
    // one counter line: C3 +0.7 %, C2 +2.3 % against 2, 4 the same as 3 (profiles/r05_event_bpc_ab.txt)
#ifndef SKIRT_EVENT_BPC
#define SKIRT_EVENT_BPC 3
#endif
    const int ebpc = SKIRT_EVENT_BPC;
    const int egrid = std::max(1, std::min((slots + kBlock - 1) / kBlock, std::max(1, c->nCusE) * ebpc));
    const int dgrid = std::max(1, std::max(1, c->nCusE) * 4);

    HIPCHECK(c, hipMemsetAsync(c->dClaim, 0, sizeof(unsigned long long), c->stream));
    HIPCHECK(c, hipMemsetAsync(c->dCtr, 0, kMaxHalves * kCtrWords * sizeof(unsigned int), c->stream));
    HIPCHECK(c, hipEventRecord(c->ev0, c->stream));
    if (forked) {  // the pipeline streams start after the caller's stream
        HIPCHECK(c, hipEventRecord(c->evFork, c->stream));
        HIPCHECK(c, hipStreamWaitEvent(sE, c->evFork, 0));
        for (int h = 0; h < halves; h++) HIPCHECK(c, hipStreamWaitEvent(sT[h], c->evFork, 0));
    }
    auto launchEvent = [&](const Args& aa, hipStream_t st) {
#define SKIRT_EVENT(G, O) hipLaunchKernelGGL((eventKernel<G, O>), dim3(egrid), dim3(kBlock), ldsEvent, st, aa)
        if (kind == SKIRT_GRID_CARTESIAN) { if (one) SKIRT_EVENT(SKIRT_GRID_CARTESIAN, true); else SKIRT_EVENT(SKIRT_GRID_CARTESIAN, false); }
        else if (kind == SKIRT_GRID_OCTREE) { if (one) SKIRT_EVENT(SKIRT_GRID_OCTREE, true); else SKIRT_EVENT(SKIRT_GRID_OCTREE, false); }
        else if (kind == kBinTreeMap) { if (one) SKIRT_EVENT(kBinTreeMap, true); else SKIRT_EVENT(kBinTreeMap, false); }
        else if (kind == kOctreeBookkeeping) { if (one) SKIRT_EVENT(kOctreeBookkeeping, true); else SKIRT_EVENT(kOctreeBookkeeping, false); }
        else if (kind == SKIRT_GRID_VORONOI) { if (one) SKIRT_EVENT(SKIRT_GRID_VORONOI, true); else SKIRT_EVENT(SKIRT_GRID_VORONOI, false); }
        else { if (one) SKIRT_EVENT(kOctreeNodes, true); else SKIRT_EVENT(kOctreeNodes, false); }
#undef SKIRT_EVENT
    };
    auto launchCont = [&](const Args& aa, hipStream_t st) {
#define SKIRT_CONT(G, O) hipLaunchKernelGGL((contKernel<G, O>), dim3(egrid), dim3(kBlock), ldsEvent, st, aa)
        if (kind == SKIRT_GRID_CARTESIAN) { if (one) SKIRT_CONT(SKIRT_GRID_CARTESIAN, true); else SKIRT_CONT(SKIRT_GRID_CARTESIAN, false); }
        else if (kind == SKIRT_GRID_OCTREE) { if (one) SKIRT_CONT(SKIRT_GRID_OCTREE, true); else SKIRT_CONT(SKIRT_GRID_OCTREE, false); }
        else if (kind == kBinTreeMap) { if (one) SKIRT_CONT(kBinTreeMap, true); else SKIRT_CONT(kBinTreeMap, false); }
        else if (kind == kOctreeBookkeeping) { if (one) SKIRT_CONT(kOctreeBookkeeping, true); else SKIRT_CONT(kOctreeBookkeeping, false); }
        else if (kind == SKIRT_GRID_VORONOI) { if (one) SKIRT_CONT(SKIRT_GRID_VORONOI, true); else SKIRT_CONT(SKIRT_GRID_VORONOI, false); }
        else { if (one) SKIRT_CONT(kOctreeNodes, true); else SKIRT_CONT(kOctreeNodes, false); }
#undef SKIRT_CONT
    };
    auto launchTrace = [&](const Args& aa, hipStream_t st) {
        // the kernel picked above (traceFn), launched through its generic entry
        void* args[] = {const_cast<Args*>(&aa)};
        return hipLaunchKernel(traceFn, dim3(tgrid), dim3(kBlock), args, ldsTrace, st);
    };
    if ((int)c->pollEv.size() < kMaxHalves * kPollRing) {
        while ((int)c->pollEv.size() < kMaxHalves * kPollRing) {
            hipEvent_t e;
            HIPCHECK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->pollEv.push_back(e);
        }
    }
    // Per half, iteration it (parity q = it & 1): the event kernel consumes active list ctr[2+q] and
    // queues rays into ctr[q] and the next active list into ctr[2+1-q]; the trace kernel walks the
    // ctr[q] rays and resets ctr[1-q] and ctr[2+q] for the next iteration; the detect kernel turns the
    // finished peel-off rays into detections. After every detect kernel the half's counters are copied
    // to pinned memory behind an event; the host reads each copy kPollRing copies later (by then long
    // complete), so it never drains a stream. A half whose active count was 0 is finished; the few
    // iterations launched after that point find no work and exit at once.
    // Stream order: sE runs, per half in turn, the detect kernel of the half's last iteration and the
    // event kernel of its next one; sT[h] runs the half's trace kernels. With two halves, one half's
    // detect + event kernels thus run while the other half's trace kernel runs (on CUs of their own when
    // the streams are CU-masked): sE = ev0(0) ev1(0) det0(0) ev0(1) det1(0) ev1(1) ...; sT[0] = tr0(0)
    // tr0(1) ...; each kernel waits only for its own half's previous kernel on the other stream.
    Args ah[kMaxHalves], prev[kMaxHalves];
    int its[kMaxHalves] = {0}, polls[kMaxHalves] = {0};
    int pollIt[kMaxHalves][kPollRing] = {};  // the iteration count each copy was taken at
    bool done[kMaxHalves] = {false}, pendingDet[kMaxHalves] = {false};
    DetRec* detBase[kMaxHalves] = {};
    for (int h = 0; h < halves; h++) {
        ah[h] = a;
        carvePool(c, ah[h], h);
        detBase[h] = ah[h].det;
    }
    // the detect kernel of half h's last trace launch (on sE, after that launch), then the counter copy
    // With detAside it runs on sD after the trace launch; the next iteration of the same parity, which
    // writes that region of detection records again, waits for it (evDet). Its record count is then
    // zeroed for that iteration's event kernel to append to.
    bool detUsed[2] = {false, false};
    auto detect = [&](int h) -> int {
        pendingDet[h] = false;
        const Args& d = prev[h];
        hipStream_t sd = detAside ? c->sD : sE;
        if (detAside) {
            HIPCHECK(c, hipEventRecord(c->evDetT, sT[h]));
            HIPCHECK(c, hipStreamWaitEvent(sd, c->evDetT, 0));
        } else if (sE != sT[h]) {
            HIPCHECK(c, hipStreamWaitEvent(sE, c->evT[h], 0));
        }
        hipLaunchKernelGGL(detectKernel, dim3(dgrid), dim3(kBlock), ldsDetect, sd, d);
        HIPCHECK(c, hipGetLastError());
        HIPCHECK(c, hipMemsetAsync(CTRP(d.ctr, 5 + d.parity), 0, sizeof(unsigned int), sd));
        if (detAside) {
            HIPCHECK(c, hipEventRecord(c->evDet[d.parity], sd));
            detUsed[d.parity] = true;
        }
        return SKIRT_OK;
    };
    // iterations per pipeline half before the phase is declared stuck; SKIRT_AMD_MAX_ITERATIONS lowers the cap
    // (tests of the error exits)
    const int maxIts = getenv("SKIRT_AMD_MAX_ITERATIONS") ? atoi(getenv("SKIRT_AMD_MAX_ITERATIONS")) : 10000000;
    int total = 0;
    while (true) {
        bool all = true;
        for (int h = 0; h < halves; h++) {
            if (done[h]) continue;
            all = false;
            Args& aa = ah[h];
            if (pendingDet[h] && (rc = detect(h))) return rc;
            if (its[h] > 0 && its[h] % kPollEvery == 0) {
                const int slot = polls[h] % kPollRing;
                unsigned int* hc = c->hCtr + (h * kPollRing + slot) * kCtrWords;
                hipEvent_t pe = c->pollEv[h * kPollRing + slot];
                if (polls[h] >= kPollRing) {
                    // the copy made kPollRing polls ago: is the half finished?
                    HIPCHECK(c, hipEventSynchronize(pe));
                    if (CTR(hc, 2 + (pollIt[h][slot] & 1)) == 0) { done[h] = true; continue; }
                }
                HIPCHECK(c, hipMemcpyAsync(hc, aa.ctr, 8 * kCtrStride * sizeof(unsigned int), hipMemcpyDeviceToHost, sE));
                HIPCHECK(c, hipEventRecord(pe, sE));
                pollIt[h][slot] = its[h];
                polls[h]++;
            }
            if (its[h] > maxIts) return fail(c, SKIRT_ERR_STATE, "photon phase did not terminate");
            aa.parity = its[h] & 1;
            aa.init = (its[h] == 0) ? 1 : 0;
            if (detAside) {
                // this iteration's detection records: the region of its parity, free once the detect kernel of
                // the last iteration of that parity is done
                aa.det = detBase[h] + (size_t)aa.parity * (size_t)(c->rayCap - c->nslots);
                if (detUsed[aa.parity]) HIPCHECK(c, hipStreamWaitEvent(sE, c->evDet[aa.parity], 0));
            }
            if (aa.continuous && !aa.init) {  // the continuous peel-offs of the FILL rays that just returned
                launchCont(aa, sE);
                HIPCHECK(c, hipGetLastError());
            }
            launchEvent(aa, sE);
            HIPCHECK(c, hipGetLastError());
            if (!a.hasDust) { done[h] = true; its[h]++; continue; }  // every packet completes in the event kernel
            if (sE != sT[h]) {
                HIPCHECK(c, hipEventRecord(c->evE[h], sE));
                HIPCHECK(c, hipStreamWaitEvent(sT[h], c->evE[h], 0));
            }
            if ((int)c->traceEv.size() < 2 * (c->traceLaunches + 1)) {
                hipEvent_t e0, e1;
                HIPCHECK(c, hipEventCreate(&e0));
                HIPCHECK(c, hipEventCreate(&e1));
                c->traceEv.push_back(e0);
                c->traceEv.push_back(e1);
            }
            // the detect kernel of the last iteration runs beside this iteration's event kernel only
            if (detAside && detUsed[1 - aa.parity])
                HIPCHECK(c, hipStreamWaitEvent(sT[h], c->evDet[1 - aa.parity], 0));
            HIPCHECK(c, hipEventRecord(c->traceEv[2 * c->traceLaunches], sT[h]));
            HIPCHECK(c, launchTrace(aa, sT[h]));
            HIPCHECK(c, hipGetLastError());
            HIPCHECK(c, hipEventRecord(c->traceEv[2 * c->traceLaunches + 1], sT[h]));
            c->traceLaunches++;
            if (sE != sT[h]) HIPCHECK(c, hipEventRecord(c->evT[h], sT[h]));
            if (a.ninstr > 0) { prev[h] = aa; pendingDet[h] = true; }
            its[h]++;
            total++;
        }
        if (all) break;
    }
    for (int h = 0; h < halves; h++)
        if (pendingDet[h] && (rc = detect(h))) return rc;
    int it = total;
    c->lastIterations = it;
    if (detAside && (detUsed[0] || detUsed[1])) {  // the caller's stream continues after the last detect kernel
        HIPCHECK(c, hipEventRecord(c->evDetJoin, c->sD));
        HIPCHECK(c, hipStreamWaitEvent(c->stream, c->evDetJoin, 0));
    }
    if (forked) {  // the caller's stream continues after the pipeline streams
        HIPCHECK(c, hipEventRecord(c->evJoin[0], sE));
        HIPCHECK(c, hipStreamWaitEvent(c->stream, c->evJoin[0], 0));
        for (int h = 0; h < halves; h++) {
            HIPCHECK(c, hipEventRecord(c->evJoin[1 + h], sT[h]));
            HIPCHECK(c, hipStreamWaitEvent(c->stream, c->evJoin[1 + h], 0));
        }
    }
    if (a.labsCopies > 1) {
        hipLaunchKernelGGL(labsFoldKernel, dim3(2048), dim3(kBlock), 0, c->stream, labsTarget, c->dLabsRep,
                           (size_t)labsElems, a.labsCopies, (size_t)a.labsCopyStride / sizeof(double));
        HIPCHECK(c, hipGetLastError());
        c->labsRepDirty = false;  // the fold zeroes the replicas
    }
    HIPCHECK(c, hipEventRecord(c->ev1, c->stream));
    c->phaseTimed = true;
    return SKIRT_OK;
}

int skirt_mcrt_synchronize(SkirtMcrt* c) {
    if (!c) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    float ms = 0;
    // only events this phase recorded: an elapsed time over unrecorded ones fails, and the failure would stay
    // behind as the thread's last error for the next launch check of any engine on this thread
    if (c->phaseTimed && hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) c->lastMs = ms;
    for (int k = 0; k < c->traceLaunches; k++)
        if (hipEventElapsedTime(&ms, c->traceEv[2 * k], c->traceEv[2 * k + 1]) == hipSuccess) c->traceMs += ms;
    c->traceLaunchesTotal += (uint64_t)c->traceLaunches;
    c->traceLaunches = 0;  // timed: the event pairs can be reused
    unsigned int e = 0;
    HIPCHECK(c, hipMemcpy(&e, c->dError, sizeof e, hipMemcpyDeviceToHost));
    if (e & ERR_TAU) return fail(c, SKIRT_ERR_NUMERIC, "the optical depth along the path is not a positive number");
    if (e & ERR_PATH_CAP)
        return fail(c, SKIRT_ERR_UNSUPPORTED, "continuous scattering: a path crosses more than " +
                                                  std::to_string(kPathCap) + " dust cells");
    if (e) return fail(c, SKIRT_ERR_STATE, "ray queue overflow");
    return SKIRT_OK;
}

int skirt_mcrt_download(SkirtMcrt* c, double* labs, double* instr) {
    if (!c) return SKIRT_ERR_ARG;
    int rc = instr ? skirt_mcrt_reduce_instruments(c) : SKIRT_OK;
    if (rc) return rc;
    rc = skirt_mcrt_synchronize(c);
    if (rc) return rc;
    const size_t nl = (size_t)c->labsStride * c->nlambda;
    if (labs && nl) {
        if (!c->dLabs) return fail(c, SKIRT_ERR_STATE, "no Labs buffer");
        std::vector<double> t(nl);
        HIPCHECK(c, hipMemcpy(t.data(), c->dLabs, nl * sizeof(double), hipMemcpyDeviceToHost));
        const bool perm = !c->devCell.empty();
        for (int ell = 0; ell < c->nlambda; ell++)
            for (int m = 0; m < c->ncells; m++)
                labs[(size_t)m * c->nlambda + ell] = t[(size_t)ell * c->labsStride + (perm ? c->devCell[m] : m)];
    }
    if (instr && c->nInstrTally) {
        if (!c->dTally) return fail(c, SKIRT_ERR_STATE, "no instrument buffer");
        std::vector<double> t(c->nInstrTally);
        HIPCHECK(c, hipMemcpy(t.data(), c->dTally, c->nInstrTally * sizeof(double), hipMemcpyDeviceToHost));
        // per instrument, the reference's order: frames [slot][lambda][pixel], then SEDs [slot][lambda]
        size_t o = 0;
        const size_t nl = (size_t)c->nlambda;
        for (const DevInstr& d : c->instr) {
            const size_t npix = (size_t)d.nx * d.ny;
            if (d.kind != SKIRT_INSTR_SED)
                for (int slot = 0; slot < d.nslots; slot++)
                    for (size_t ell = 0; ell < nl; ell++)
                        for (size_t l = 0; l < npix; l++)
                            instr[o++] = t[d.frameBase + (ell * npix + l) * d.slotStride + slot];
            if (d.kind != SKIRT_INSTR_FRAME)
                for (size_t q = 0; q < (size_t)d.nslots * nl; q++) instr[o++] = t[d.sedBase + q];
        }
    }
    return SKIRT_OK;
}

int skirt_mcrt_set_crossed(SkirtMcrt* c, int bins) {
    if (!c || bins < 0 || bins > (1 << 20)) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    if (c->dCrossed) {
        HIPCHECK(c, hipStreamSynchronize(c->stream));
        (void)hipFree(c->dCrossed);
        c->dCrossed = nullptr;
    }
    c->crossedBins = bins;
    if (!bins) return SKIRT_OK;
    const size_t n = (size_t)kCrossedCopies * bins;
    HIPCHECK(c, hipMalloc(&c->dCrossed, n * sizeof(unsigned long long)));
    HIPCHECK(c, hipMemsetAsync(c->dCrossed, 0, n * sizeof(unsigned long long), c->stream));
    return SKIRT_OK;
}

int skirt_mcrt_download_crossed(SkirtMcrt* c, uint64_t* hist, int bins) {
    if (!c || !hist || bins < 0) return SKIRT_ERR_ARG;
    if (!c->dCrossed) return fail(c, SKIRT_ERR_STATE, "the cells-crossed histogram is off (skirt_mcrt_set_crossed)");
    HIPCHECK(c, hipSetDevice(c->device));
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    std::vector<unsigned long long> h((size_t)kCrossedCopies * c->crossedBins);
    HIPCHECK(c, hipMemcpy(h.data(), c->dCrossed, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (int b = 0; b < bins; b++) {
        uint64_t v = 0;
        if (b < c->crossedBins)
            for (int k = 0; k < kCrossedCopies; k++) v += h[(size_t)k * c->crossedBins + b];
        hist[b] = v;
    }
    return SKIRT_OK;
}

int skirt_mcrt_column_densities(SkirtMcrt* c, const double* rays, int n, double* out) {
    if (!c || n < 0 || (n > 0 && (!rays || !out))) return SKIRT_ERR_ARG;
    if (n == 0) return SKIRT_OK;
    if (!c->dRho) return fail(c, SKIRT_ERR_STATE, "no grid and media uploaded");
    HIPCHECK(c, hipSetDevice(c->device));
    Args a{};
    gridArgs(c, a);
    a.ldsMeshOff = a.ldsOptOff = a.ldsInstrOff = a.ldsSedOff = 0;
    double* d = nullptr;
    HIPCHECK(c, hipMalloc(&d, (size_t)n * 7 * sizeof(double)));
    int rc = SKIRT_OK;
    hipError_t e = hipMemcpyAsync(d, rays, (size_t)n * 6 * sizeof(double), hipMemcpyHostToDevice, c->stream);
    const dim3 grid((n + kBlock - 1) / kBlock);
    // the walks of the photon paths, through the node arrays for trees (equal to the leaf-map walk,
    // tests/test_gpu_parity.py::test_leaf_map_walk_equals_node_walk)
    if (e == hipSuccess) {
        if (c->gridKind == SKIRT_GRID_CARTESIAN)
            hipLaunchKernelGGL(columnKernel<SKIRT_GRID_CARTESIAN>, grid, dim3(kBlock),
                               (size_t)(c->nx + c->ny + c->nz + 3) * sizeof(double), c->stream, a, d, n, d + 6 * (size_t)n);
        else if (c->gridKind == SKIRT_GRID_VORONOI)
            hipLaunchKernelGGL(columnKernel<SKIRT_GRID_VORONOI>, grid, dim3(kBlock), 0, c->stream, a, d, n, d + 6 * (size_t)n);
        else if (c->search == SKIRT_TREE_BOOKKEEPING)
            hipLaunchKernelGGL(columnKernel<kOctreeBookkeeping>, grid, dim3(kBlock), 0, c->stream, a, d, n, d + 6 * (size_t)n);
        else
            hipLaunchKernelGGL(columnKernel<kOctreeNodes>, grid, dim3(kBlock), 0, c->stream, a, d, n, d + 6 * (size_t)n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out, d + 6 * (size_t)n, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) rc = fail(c, SKIRT_ERR_HIP, hipGetErrorString(e));
    (void)hipFree(d);
    return rc;
}

int skirt_mcrt_stats(SkirtMcrt* c, SkirtStats* out) {
    if (!c || !out) return SKIRT_ERR_ARG;
    HIPCHECK(c, hipSetDevice(c->device));
    HIPCHECK(c, hipStreamSynchronize(c->stream));
    std::vector<unsigned long long> copies(8 * kStatCopies);
    HIPCHECK(c, hipMemcpy(copies.data(), c->dStats, copies.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < kStatCopies; k++)
        for (int q = 0; q < 8; q++) v[q] += copies[8 * k + q];
    out->packets = v[0];
    out->segments_fill = v[1];
    out->segments_walk = v[2];
    out->segments_peel = v[3];
    out->detects = v[4];
    out->absorb_adds = v[5];
    out->lane_slots = v[6];
    out->iterations = (uint64_t)c->lastIterations;
    out->kernel_ms = c->lastMs;
    out->trace_ms = c->traceMs;
    out->trace_launches = c->traceLaunchesTotal;
    out->grid_walk = c->lastWalk;
    out->map_level = c->mapL;
    out->labs_requests = v[7];
    out->device_cells = c->ndev;
    out->trace_blocks_per_cu = (uint64_t)c->traceBlocksPerCU;
    out->packages = c->packagesTotal;
    return SKIRT_OK;
}

const char* skirt_mcrt_last_error(SkirtMcrt* c) { return c ? c->err.c_str() : "null context"; }

void skirt_mcrt_destroy(SkirtMcrt* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->dMesh, c->dBox, c->dFirstChild, c->dSplitDir, c->dFather, c->dCellnumber, c->dNbrOffset, c->dNbrList, c->dTreeT,
                    c->dLeafMap, c->dCellLv, c->dCellCdf, c->dCellGuide, c->dCellLtot, c->dCellNode, c->dEmisVolume, c->dEmisKabs,
                    c->dEmisSigma, c->dEmisMu, c->dEmisTv, c->dEmisPlanck, c->dEmisLambda, c->dEmisDlambda,
                    c->dEmisScratch, c->dDevCell, c->dSite, c->dCellBbox, c->dVorStart, c->dVorSlots,
                    c->dBlockOffset, c->dBlockSites, c->dRho,
                    c->dOptics, c->dGeomParam, c->dGeomTable, c->dLum, c->dLumtot, c->dCdf, c->dInstr,
                    c->dClaim, c->dStats, c->dError, c->dCtr, c->dPool, c->dCrossed};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (c->hCtr) (void)hipHostFree(c->hCtr);
    if (c->ownLabs && c->dLabs) (void)hipFree(c->dLabs);
    if (c->ownTally && c->dTally) (void)hipFree(c->dTally);
    if (c->ownLabsDust && c->dLabsDust) (void)hipFree(c->dLabsDust);
    if (c->dLabsRep) (void)hipFree(c->dLabsRep);
    for (hipEvent_t e : c->traceEv) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->pollEv) (void)hipEventDestroy(e);
    if (c->evFork) (void)hipEventDestroy(c->evFork);
    for (hipEvent_t e : c->evJoin)
        if (e) (void)hipEventDestroy(e);
    for (int h = 0; h < kMaxHalves; h++) {
        if (c->evE[h]) (void)hipEventDestroy(c->evE[h]);
        if (c->evT[h]) (void)hipEventDestroy(c->evT[h]);
        if (c->sT[h]) (void)hipStreamDestroy(c->sT[h]);
    }
    if (c->sE) (void)hipStreamDestroy(c->sE);
    if (c->sD) (void)hipStreamDestroy(c->sD);
    for (hipEvent_t e : {c->evDetT, c->evDet[0], c->evDet[1], c->evDetJoin})
        if (e) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

int skirt_mcrt_sample_density(int device, const SkirtDensityDesc* dens, const double* boxes, size_t n,
                              const uint32_t* words, int nsample, int mode, double* out) {
    if (!dens || dens->ncomp < 1 || !dens->geom_kind || !dens->geom_param || !dens->norm || nsample < 1 ||
        (mode != SKIRT_DENS_COMPONENTS && mode != SKIRT_DENS_NODE) || (n && (!boxes || !words || !out)))
        return SKIRT_ERR_ARG;
    for (int h = 0; h < dens->ncomp; h++) {
        const int k = dens->geom_kind[h];
        if (k < SKIRT_GEOM_PLUMMER || k > SKIRT_GEOM_POINT) return SKIRT_ERR_ARG;
        if (k == SKIRT_GEOM_SERSIC && (!dens->dens_table || dens->ntab < 2)) return SKIRT_ERR_ARG;
    }
    if (n == 0) return SKIRT_OK;
    const size_t nout = n * (mode == SKIRT_DENS_NODE ? 6 : (size_t)dens->ncomp);
    const size_t nw = n * 3 * (size_t)nsample;
    const size_t ntable = dens->dens_table ? (size_t)2 * dens->ntab * dens->ncomp : 0;
    if (hipSetDevice(device) != hipSuccess) return SKIRT_ERR_HIP;
    hipStream_t st = nullptr;
    char* buf = nullptr;
    // one allocation: parameters, boxes, words, output
    const size_t offParam = 0, offNorm = offParam + 8 * (size_t)dens->ncomp * sizeof(double);
    const size_t offKind = offNorm + (size_t)dens->ncomp * sizeof(double);
    const size_t offTable = (offKind + (size_t)dens->ncomp * sizeof(int) + 15) & ~(size_t)15;
    const size_t offBoxes = (offTable + ntable * sizeof(double) + 15) & ~(size_t)15;
    const size_t offOut = (offBoxes + 6 * n * sizeof(double) + 15) & ~(size_t)15;
    const size_t offWords = (offOut + nout * sizeof(double) + 15) & ~(size_t)15;
    const size_t total = offWords + nw * sizeof(uint32_t);
    int rc = SKIRT_OK;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return SKIRT_ERR_HIP;
    if (hipMalloc(&buf, total) != hipSuccess) {
        (void)hipStreamDestroy(st);
        return SKIRT_ERR_HIP;
    }
    DensArgs d{};
    d.ncomp = dens->ncomp;
    d.ntab = dens->ntab;
    d.nsample = nsample;
    d.mode = mode;
    d.param = reinterpret_cast<const double*>(buf + offParam);
    d.norm = reinterpret_cast<const double*>(buf + offNorm);
    d.kind = reinterpret_cast<const int*>(buf + offKind);
    d.table = ntable ? reinterpret_cast<const double*>(buf + offTable) : nullptr;
    d.boxes = reinterpret_cast<const double*>(buf + offBoxes);
    d.out = reinterpret_cast<double*>(buf + offOut);
    d.words = reinterpret_cast<const uint32_t*>(buf + offWords);
    d.n = n;
    const size_t nblocks = (n + kBlock - 1) / kBlock;
    if (hipMemcpyAsync(buf + offParam, dens->geom_param, 8 * (size_t)dens->ncomp * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(buf + offNorm, dens->norm, (size_t)dens->ncomp * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(buf + offKind, dens->geom_kind, (size_t)dens->ncomp * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
        (ntable && hipMemcpyAsync(buf + offTable, dens->dens_table, ntable * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipMemcpyAsync(buf + offBoxes, boxes, 6 * n * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(buf + offWords, words, nw * sizeof(uint32_t), hipMemcpyHostToDevice, st) != hipSuccess ||
        nblocks > 0x7fffffffu) {
        rc = SKIRT_ERR_HIP;
    } else {
        hipLaunchKernelGGL(densitySampleKernel, dim3((unsigned)nblocks), dim3(kBlock), 0, st, d);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(out, buf + offOut, nout * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = SKIRT_ERR_HIP;
    }
    (void)hipStreamSynchronize(st);
    (void)hipFree(buf);
    (void)hipStreamDestroy(st);
    return rc;
}

}  // extern "C"
