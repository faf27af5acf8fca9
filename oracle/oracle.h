/* CPU ORACLE for the SKIRT photon-shooting hot path -- TEST INFRASTRUCTURE ONLY.
 *
 * This library is the checker, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. It restates, in plain single-threaded C++ that follows the
 * reference line by line, the per-packet life cycle of SKIRT v7.3:
 *   MonteCarloSimulation::dostellaremissionchunk   SKIRTcore/MonteCarloSimulation.cpp:265-301
 *   peeloffemission / peeloffscattering           MonteCarloSimulation.cpp:305-363
 *   simulateescapeandabsorption                   MonteCarloSimulation.cpp:438-515
 *   simulatepropagation / simulatescattering      MonteCarloSimulation.cpp:519-549
 *   PanMonteCarloSimulation dust phases           PanMonteCarloSimulation.cpp:187-344
 *   CartesianDustGrid::path                       CartesianDustGrid.cpp:136-283
 *   TreeDustGrid::path (TopDown, Neighbor)        TreeDustGrid.cpp:390-521, DustGridPath.cpp:46-173
 *   FullInstrument/Simple/SED/Frame ::detect      FullInstrument.cpp:107-174 etc.
 *   Random uniform/exponcutoff/direction          Random.cpp:89-222
 *
 * Two random-number modes:
 *   ORACLE_RNG_MT     one MT19937 stream continuing from model setup, packets in the reference's
 *                     order -- bit-for-bit the output of `skirt -t 1`. Parity PINNED: the reference
 *                     binary is rebuilt from its own sources by oracle/ref.mk (oracle/_ref/skirt, never
 *                     shipped), tests/test_reference_rebuild.py regenerates every tests/golden/ref file
 *                     with it byte for byte, and tests/test_oracle_golden.py holds this mode to all 34
 *                     fixtures (SEDs, FITS frames, ds_isrf, ds_cellprops, ds_crossed, ds_convergence).
 *   ORACLE_RNG_PHILOX one Philox4x32-10 stream per packet, keyed exactly like the GPU engine
 *                     (see DESIGN.md "Random numbers"), so GPU and oracle agree packet by packet.
 * Model setup (ski parsing, grids, densities, tables) is shared with the product host library.
 */
#ifndef SKIRT_ORACLE_H
#define SKIRT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_RNG_MT = 0, ORACLE_RNG_PHILOX = 1 };
/* photon phases (the engine's SKIRT_PHASE_* values; Philox tag = phase | cycle << 2) */
enum { ORACLE_PHASE_STELLAR = 0, ORACLE_PHASE_DUST_EMISSION = 1, ORACLE_PHASE_DUST_SELFABS = 2 };
/* `phases` argument of oracle_run: which of the simulation's phases run (0 = all it has) */
enum { ORACLE_PHASES_STELLAR = 1, ORACLE_PHASES_DUST = 2, ORACLE_PHASES_ALL = 3 };

typedef struct OracleRun OracleRun;

/* Builds the model from `ski` and runs it on the CPU.
 *  rng          ORACLE_RNG_MT or ORACLE_RNG_PHILOX
 *  nthreads     worker threads (Philox mode only; MT mode is single-threaded by definition)
 *  packages     if > 0, overrides the ski's packages (photon packets per wavelength)
 *  seed         if nonzero, overrides the ski's random seed
 *  packet_begin/packet_end  restrict the stellar phase to this global packet range (end == 0: all)
 *  phases       ORACLE_PHASES_* mask; 0 runs every phase of the simulation: stellar emission, then for
 *               a Pan dust system with dust emission the self-absorption cycles (if enabled) and the
 *               dust emission phase (PanMonteCarloSimulation::runSelf)
 *  outprefix    if non-NULL, writes SKIRT-format outputs (<prefix>_<instr>_sed.dat, FITS frames, ds_isrf)
 * Returns NULL on failure (see oracle_last_error()). */
OracleRun* oracle_run(const char* ski, const char* datadir, int rng, int nthreads, double packages,
                      uint64_t seed, uint64_t packet_begin, uint64_t packet_end, int phases,
                      const char* outprefix);
/* The same on rank `rank` of `world` processes (Philox mode only): every phase shoots the rank's slice
 * [npp*rank/world, npp*(rank+1)/world) of every wavelength, the reference's IdenticalAssigner
 * (IdenticalAssigner.cpp:37-58), like skirt_mcrt_run_phase_shard. reduce(user, tally, data, n) must sum a
 * host array over the processes in place: the stellar Labs after the stellar phase, the dust Labs after
 * every self-absorption cycle (ORACLE_TALLY_*); it may be NULL when only the stellar phase runs. The caller
 * sums the instrument tallies at the end. */
enum { ORACLE_TALLY_LABS = 0, ORACLE_TALLY_DUST_LABS = 1 };
typedef int (*OracleReduceFn)(void* user, int tally, double* data, size_t n);
OracleRun* oracle_run_shard(const char* ski, const char* datadir, int rng, int nthreads, double packages,
                            uint64_t seed, uint64_t packet_begin, uint64_t packet_end, int phases,
                            const char* outprefix, int rank, int world, OracleReduceFn reduce, void* user);
const char* oracle_last_error(void);

/* stellar Labs(m, ell) row-major, Ncells x Nlambda (PanDustSystem::_Labsstelvv) */
const double* oracle_labs(OracleRun* r, int* ncells, int* nlambda);
/* dust Labs of the last self-absorption cycle (PanDustSystem::_Labsdustvv), or NULL */
const double* oracle_labs_dust(OracleRun* r);
/* Labsdusttot after every self-absorption cycle; returns the number of cycles */
int oracle_selfabs_cycles(OracleRun* r, const double** totals);
/* instrument accumulators before calibration: frames [nslots][nlambda][nframe], seds [nslots][nlambda] */
int oracle_instrument(OracleRun* r, int i, const double** frames, const double** seds, int* nslots,
                      int* nframe, int* nlambda);
int oracle_num_instruments(OracleRun* r);
/* DustGrid::path of the ski's dust grid (built with the ski's seed) for n rays of 6 doubles each
 * (position, unit direction). Per ray at most maxseg segments are written to out, 7 doubles each: the
 * cell's box {xmin ymin zmin xmax ymax zmax} (NaN for the segments before the grid) and ds; nseg[i] is
 * the ray's segment count (capped at maxseg), *ncells the grid's cell count. Returns 0, -1 on failure. */
int oracle_grid_paths(const char* ski, const char* datadir, int n, const double* rays, int maxseg, double* out,
                      int* nseg, int* ncells);
/* dust component `comp` of the model: its normalization factor (the dust mass of a normalized geometry)
 * and the mix's kappa_ext and the wavelengths (nlambda each, either may be NULL) */
int oracle_dust_component(const char* ski, const char* datadir, int comp, double* nf, double* kext, double* lambda,
                          int* nlambda);
/* n random positions of stellar component `comp` (its geometry's generatePosition on an MT19937 stream
 * seeded with `seed`), 3 doubles each, and the geometry's density there (density may be NULL) */
int oracle_star_positions(const char* ski, const char* datadir, int comp, int n, uint64_t seed, double* out,
                          double* density);
/* statistics: number of packets launched, path segments traversed, wall seconds of the photon phases */
double oracle_seconds(OracleRun* r);
uint64_t oracle_packets(OracleRun* r);
uint64_t oracle_segments(OracleRun* r);
/* out = {segments of the FILL paths (fillOpticalDepth), segments of the peel-off paths (opticaldepth),
 * absorption adds into Labs}: the counts behind the engine's statistics (SkirtStats) */
void oracle_counts(OracleRun* r, uint64_t out[3]);
/* DustSystem's _crossed histogram (DustSystem.cpp:959-1000): hist[n] = paths (FILL and peel-off) of n
 * segments; returns the number of bins up to the last nonzero one (the last of 65536 bins counts longer
 * paths) */
int oracle_crossed(OracleRun* r, const uint64_t** hist);
void oracle_free(OracleRun* r);

/* test switch: how the absorption sums evaluate exp(-tau_{n-1}). 0: the reference's exp(-taustart) per segment
 * (default); 1: the running product of 1 - (-expm1(-dtau)) along the path, as the GPU engine did until round 3;
 * 2: the engine's carry since round 5, f - f * (-expm1(-dtau)) while dtau < 0.5, exp(-tau) anew behind a
 * thicker segment */
void oracle_set_engine_attenuation(int mode);

/* study hook (tools/labs_locality.cpp): called, from the worker threads, for every FILL path that stores
 * absorption, with the packet's wavelength, start position and direction, and the reference cell numbers
 * of the path's dust segments in path order (the cells its Labs adds go to). NULL turns it off. */
typedef void (*OracleFillHook)(void* user, int ell, const double r[3], const double k[3], const int* cells, int n);
void oracle_set_fill_hook(OracleFillHook hook, void* user);

/* Philox4x32-10 known-answer access for tests: out[4] = philox(ctr[4], key[2]) */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
