/* skirt_mcrt.h -- C ABI of the MI355X photon-packet engine (the drop-in boundary).
 *
 * The reference runs every photon phase as Parallel::call(this, &X::do...chunk, assigner) over
 * std::threads (SKIRTcore/Parallel.cpp:76-111), each chunk calling the plugin surface concurrently:
 *   StellarComp::launch            SKIRTcore/StellarComp.hpp:42, StellarSystem.cpp:116-158
 *   DustGrid::path / whichcell     SKIRTcore/DustGrid.hpp:70-106 (CartesianDustGrid, TreeDustGrid)
 *   DustSystem::fillOpticalDepth / opticaldepth / absorb   SKIRTcore/DustSystem.hpp:352,366,397
 *   Instrument::detect             SKIRTcore/Instrument.hpp:69-87, FullInstrument.cpp:107-174
 * This ABI replaces those call sites (MonteCarloSimulation.cpp:256-257 stellar emission,
 * PanMonteCarloSimulation.cpp:144-145 self-absorption, :260-261 dust emission) with one device launch
 * per phase. The host describes the grid, media, sources and instruments once as flat arrays; each
 * run call shoots a range of global packet indices (run_phase) or one rank's slice of every wavelength
 * (run_phase_shard), so a phase can be sharded over GPUs (one process per GPU) with results independent
 * of the shard count.
 *
 * Conventions: plain C, host owns every host buffer, all functions return 0 on success and a nonzero
 * SKIRT_ERR_* code on failure (message via skirt_mcrt_last_error), no exceptions cross the boundary.
 * Run calls are asynchronous on the engine's HIP stream; skirt_mcrt_synchronize or any download
 * waits for completion. One context per simulation per GPU; a context is not reentrant.
 * Layouts: Labs is row-major (cell, wavelength) like DustSystem::_Labs*vv (Table.hpp:104-105).
 * Instrument tallies (as downloaded) are per instrument [nslots][nlambda][nframe] frames followed by
 * [nslots][nlambda] SEDs, slots as in FullInstrument (trav, strdir, strsca, dusdir, dussca,
 * scattering levels...) or a single "total" slot for Simple/SED/Frame instruments. These are host
 * layouts: the device buffers (skirt_mcrt_tally_sizes, bind_tallies) are wavelength-major with padded
 * rows and are converted by the downloads.
 */
#ifndef SKIRT_MCRT_H
#define SKIRT_MCRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SKIRT_MCRT_ABI_VERSION 14  /* 11: SkirtStats::packages; 12: SkirtStats::labs_cache_sets; 13: without it;
                                     14: skirt_mcrt_voronoi_cells */

enum {
    SKIRT_OK = 0,
    SKIRT_ERR_ARG = 1,       /* invalid argument / inconsistent sizes */
    SKIRT_ERR_HIP = 2,       /* a HIP runtime call failed */
    SKIRT_ERR_STATE = 3,     /* call order violated (e.g. run before upload) */
    SKIRT_ERR_NUMERIC = 4,   /* "optical depth along the path is not a positive number" (DustSystem.cpp:976-979) */
    SKIRT_ERR_UNSUPPORTED = 5  /* a model outside the engine's limits, e.g. a Labs table (cells x wavelengths,
                                  f64) of 2^40 elements or more, a Voronoi mesh above 2^31 slots, tables that do not fit
                                  one workgroup's LDS, or (skirt_sim_write) a path reaching the last
                                  ds_crossed bin; the message names the limit and the sizes */
};

enum { SKIRT_GRID_CARTESIAN = 0, SKIRT_GRID_OCTREE = 1, SKIRT_GRID_VORONOI = 2 };
enum { SKIRT_TREE_TOPDOWN = 0, SKIRT_TREE_NEIGHBOR = 1, SKIRT_TREE_BOOKKEEPING = 2 /* octrees only */ };
enum { SKIRT_GEOM_PLUMMER = 0, SKIRT_GEOM_EXPDISK = 1, SKIRT_GEOM_SERSIC = 2, SKIRT_GEOM_POINT = 3 };
enum { SKIRT_INSTR_FULL = 0, SKIRT_INSTR_SIMPLE = 1, SKIRT_INSTR_SED = 2, SKIRT_INSTR_FRAME = 3 };
enum { SKIRT_PHASE_STELLAR = 0, SKIRT_PHASE_DUST_EMISSION = 1, SKIRT_PHASE_DUST_SELFABS = 2 };

typedef struct SkirtMcrt SkirtMcrt;

/* Dust grid (replaces DustGrid::path/whichcell). Cartesian: border arrays of nx+1, ny+1, nz+1
 * values, cell index m = k + nz*j + nz*ny*i (CartesianDustGrid.cpp:305-308). Octree (and k-d tree, see
 * split_dir): the reference's
 * breadth-first node vector (TreeDustGrid.cpp:50-164): per node a box {xmin,ymin,zmin,xmax,ymax,zmax},
 * the index of its first of 8 consecutive children (-1 for a leaf) and its cell number (-1 for
 * non-leaves); neighbor lists per (node, wall) in CSR form, walls BACK FRONT LEFT RIGHT BOTTOM TOP,
 * each list sorted by decreasing overlap (TreeNode::sortneighbors). */
typedef struct {
    int kind;
    int ncells;
    int nx, ny, nz;
    const double *xv, *yv, *zv;
    int nnodes;
    const double* box;          /* 6 * nnodes */
    const int* first_child;     /* nnodes */
    const int* cellnumber;      /* nnodes */
    const int* nbr_offset;      /* 6 * nnodes + 1 */
    const int* nbr_list;        /* nbr_offset[6*nnodes] entries */
    double eps;                 /* TreeDustGrid::_eps / VoronoiMesh::_eps = 1e-12 * |extent widths| */
    int search;                 /* SKIRT_TREE_* */
    /* Voronoi (VoronoiMesh.cpp:250-306, 512-541, 749-844): per cell its site and neighbour list (CSR;
     * walls -1 xmin, -2 xmax, -3 ymin, -4 ymax, -5 zmin, -6 zmax), its enclosing box; the domain; the
     * nb^3 block lists of cells whose box overlaps each block (for the nearest-site cell index) */
    const double* site;         /* 3 * ncells */
    const int* cell_nbr_offset; /* ncells + 1 */
    const int* cell_nbr_list;
    const double* cell_bbox;    /* 6 * ncells */
    double extent[6];           /* xmin ymin zmin xmax ymax zmax */
    int nblocks;                /* nb blocks per axis */
    const int* block_offset;    /* nb^3 + 1 */
    const int* block_list;
    /* binary trees (BinTreeDustGrid, the k-d tree; BinTreeNode.cpp): per node the axis its two children
     * split (0 x, 1 y, 2 z; ignored for leaves). NULL for octrees. first_child then points at the first
     * of 2 consecutive children. */
    const signed char* split_dir;
} SkirtGridDesc;

/* Dust media (replaces DustSystem::density and the KappaRho functor, DustSystem.cpp:465-491).
 * rho is ncells x ncomp row-major; the optical tables are ncomp x nlambda row-major. */
typedef struct {
    int ncells, ncomp, nlambda;
    const double* rho;
    const double* kext;
    const double* ksca;
    const double* albedo;
    const double* g;            /* Henyey-Greenstein asymmetry parameter */
} SkirtMediaDesc;

/* Stellar sources (replaces StellarSystem::launch, StellarSystem.cpp:116-158). */
typedef struct {
    int ncomp, nlambda;
    const int* geom_kind;       /* ncomp, SKIRT_GEOM_* */
    const double* geom_param;   /* ncomp x 8: PlummerGeometry {c, rho0, 0...};
                                   ExpDiskGeometry {hR, hz, Rmax, zmax, Rmin, rho0, 0, 0};
                                   SersicGeometry {reff, n, rho0, 0...} (tables in geom_table) */
    const double* lum;          /* ncomp x nlambda, W */
    const double* lumtot;       /* nlambda, sum over components */
    const double* cdf;          /* nlambda x (ncomp+1) normalized cumulative luminosity */
    double emission_bias;
    const double* geom_table;   /* ncomp x 202 (NULL if no component needs it): SersicGeometry's
                                   SersicFunction tables {s_0..s_100, M_0..M_100} */
} SkirtSourceDesc;

/* Distant instruments (DistantInstrument.cpp:27-50, SingleFrameInstrument.cpp:24-38, 130-147). */
typedef struct {
    int kind;                   /* SKIRT_INSTR_* */
    int nx, ny;
    int scattering_levels;      /* FullInstrument only */
    double kobs[3];
    double sinphi, cosphi, sintheta, costheta, sinpa, cospa;
    double xpmin, xpsiz, ypmin, ypsiz;
} SkirtInstrDesc;

/* Cell sources of a dust phase (the per-chunk cell distribution of PanMonteCarloSimulation.cpp:193-205
 * and 273-294): per wavelength the luminosity Labsbol(m) * dustluminosity(m, ell) of every dust cell
 * (reference cell order), its normalized cumulative distribution NR::cdf over the cells, and the total.
 * emission_bias is PanDustSystem::emissionBias (used by the dust emission phase). */
typedef struct {
    int ncells, nlambda;
    const double* lv;           /* nlambda x ncells */
    const double* cdf;          /* nlambda x (ncells + 1) */
    const double* ltot;         /* nlambda */
    double emission_bias;
} SkirtCellSourceDesc;

/* Grey-body dust emissivity for the device-side dust emission sources (GreyBodyDustEmissivity with
 * AllCellsDustLib): cell volumes (reference order), per component kappa_abs and the population's
 * sigma_abs per wavelength, mu, the DustMix temperature grid and Planck-integrated absorption table
 * (DustMix.cpp:238-263), the wavelength grid. */
typedef struct {
    int ncells, nlambda, ncomp, ntemp;
    const double* volume;       /* ncells */
    const double* kabs;         /* ncomp x nlambda */
    const double* sigmaabs;     /* ncomp x nlambda */
    const double* mu;           /* ncomp */
    const double* tv;           /* ntemp */
    const double* planckabs;    /* ncomp x ntemp */
    const double* lambda;       /* nlambda */
    const double* dlambda;      /* nlambda */
    double emission_bias;       /* PanDustSystem::emissionBias */
} SkirtEmissivityDesc;

/* MonteCarloSimulation properties used by the photon loop (MonteCarloSimulation.cpp:31-35). */
typedef struct {
    double min_weight_reduction;
    int min_scatt_events;
    double scatt_bias;
    int store_absorption;       /* DustSystem::storeabsorptionrates() */
    int has_dust;
    int continuous_scattering;  /* MonteCarloSimulation::continuousScattering: peel-offs from every dust
                                   segment of each path (continuouspeeloffscattering, MonteCarloSimulation.cpp:
                                   367-434) instead of at the interaction points */
} SkirtPhaseParams;

typedef struct {
    uint64_t packets;           /* packets launched (primary, excluding peel-offs) */
    uint64_t segments_fill;     /* grid segments walked by fillOpticalDepth-equivalent passes */
    uint64_t segments_walk;     /* segments walked to locate interaction points */
    uint64_t segments_peel;     /* segments walked by peel-off optical depth passes */
    uint64_t detects;           /* peel-off detections */
    uint64_t absorb_adds;       /* Labs atomic updates */
    uint64_t lane_slots;        /* trace kernel: 64 x wave steps (segments / lane_slots = SIMD lane use) */
    uint64_t iterations;        /* event/trace iterations of the last run call */
    double kernel_ms;           /* device time of the last run call (HIP events on the engine stream) */
    double trace_ms;            /* trace-kernel time (HIP events around each launch), cumulative */
    uint64_t trace_launches;    /* trace-kernel launches timed so far, cumulative */
    int32_t grid_walk;          /* walk of the last run: SKIRT_WALK_* */
    int32_t map_level;          /* tree leaf-map depth (finest cells per axis = 2^map_level), -1 without */
    uint64_t labs_requests;     /* 64-byte atomic requests carrying the Labs adds (adds sharing a line in
                                   one wave instruction share a request) */
    uint64_t device_cells;      /* device cell numbers, >= ncells (octree sibling groups start on a line) */
    uint64_t trace_blocks_per_cu; /* trace-kernel workgroups per CU the last phase ran (register and LDS bound) */
    uint64_t packages;          /* packet indices shot, launched or not (per phase: the slice's packages x
                                   wavelengths; wavelengths or cells without luminosity launch none):
                                   SURVEY 8(d)'s throughput unit, summed over the phases since the last
                                   skirt_mcrt_zero_tallies */
} SkirtStats;

/* grid walks of the trace kernel (SkirtStats::grid_walk) */
enum { SKIRT_WALK_CARTESIAN = 0, SKIRT_WALK_OCTREE_MAP = 1, SKIRT_WALK_VORONOI = 2, SKIRT_WALK_TREE_NODES = 3,
       SKIRT_WALK_KDTREE_MAP = 4, SKIRT_WALK_OCTREE_BOOKKEEPING = 5 };

int skirt_mcrt_abi_version(void);
int skirt_mcrt_create(int device, SkirtMcrt** out);
/* use an existing HIP stream (hipStream_t) instead of the engine's own; NULL restores the own stream */
int skirt_mcrt_set_stream(SkirtMcrt* ctx, void* hip_stream);
int skirt_mcrt_upload_grid(SkirtMcrt* ctx, const SkirtGridDesc* grid);
int skirt_mcrt_upload_media(SkirtMcrt* ctx, const SkirtMediaDesc* media);
int skirt_mcrt_upload_sources(SkirtMcrt* ctx, const SkirtSourceDesc* src);
int skirt_mcrt_set_instruments(SkirtMcrt* ctx, const SkirtInstrDesc* instr, int n);
/* device tally buffers: Labs (stored wavelength-major [nlambda][row] on the device, rows of device cells
 * padded to a 64-byte line; n_labs >= ncells*nlambda) and the concatenated instrument tallies. Optionally bind caller-owned device memory of the
 * sizes returned by skirt_mcrt_tally_sizes (e.g. torch tensors, so they can be all-reduced in place).
 * Any 8-byte alignment is correct; 64-byte aligned buffers (hipMalloc, torch) let the adds of one line
 * share an atomic request (sibling cells of Labs, the slots of one frame pixel). */
int skirt_mcrt_tally_sizes(SkirtMcrt* ctx, size_t* n_labs, size_t* n_instr);
int skirt_mcrt_bind_tallies(SkirtMcrt* ctx, double* d_labs, double* d_instr);
int skirt_mcrt_zero_tallies(SkirtMcrt* ctx);
/* Stellar emission phase over global packet indices [first, first+count) of a phase with npp packets
 * per wavelength (packet p has wavelength index p / npp). Asynchronous. */
int skirt_mcrt_run_stellar(SkirtMcrt* ctx, uint64_t npp, uint64_t first, uint64_t count, uint64_t seed,
                           const SkirtPhaseParams* params);
/* One photon phase over global packets [first, first+count) of npp*nlambda (packet p has wavelength
 * p / npp and its own random stream, selected by phase and cycle):
 *   SKIRT_PHASE_STELLAR       as skirt_mcrt_run_stellar (cycle ignored)
 *   SKIRT_PHASE_DUST_EMISSION dodustemissionchunk (PanMonteCarloSimulation.cpp:269-344): packets from the
 *                             uploaded cell sources with the emission bias, peel-off on, no absorption stored
 *   SKIRT_PHASE_DUST_SELFABS  dodustselfabsorptionchunk (:187-240): natural cell choice, no peel-off,
 *                             absorption into the dust Labs tally; `cycle` numbers the self-absorption
 *                             cycles of the simulation (0, 1, ...)
 * npp = 0 (a simulation of zero packages, which the reference runs: no chunks, zero tallies) is an empty
 * phase; its phase-end sums still run, so every rank of a sharded run makes the same collective calls. */
int skirt_mcrt_run_phase(SkirtMcrt* ctx, int phase, uint32_t cycle, uint64_t npp, uint64_t first, uint64_t count,
                         uint64_t seed, const SkirtPhaseParams* params);
/* Multi-GPU (one process per GPU): rank `rank` of `world` shoots packets [lo, lo + count) of EVERY
 * wavelength, lo and count from skirt_mcrt_shard_slice. This is the reference's IdenticalAssigner
 * (IdenticalAssigner.cpp:37-58), which gives each process a block of chunks at every wavelength through a
 * SequentialAssigner (SequentialAssigner.cpp:37-59), with chunks of one packet. Philox streams are keyed
 * on the global packet index (wavelength * npp + packet), so the union of the ranks' packets equals one
 * unsharded run. world > 1 requires a reducer (below), which run_phase_shard calls at the phase end. */
int skirt_mcrt_run_phase_shard(SkirtMcrt* ctx, int phase, uint32_t cycle, uint64_t npp, int rank, int world,
                               uint64_t seed, const SkirtPhaseParams* params);
void skirt_mcrt_shard_slice(uint64_t npp, int rank, int world, uint64_t* lo, uint64_t* count);
/* The cross-process sum of the tallies (PanDustSystem::sumResults, PanDustSystem.cpp:394-403;
 * Instrument::sumResults, Instrument.cpp:57-66). The engine calls fn(user, tally, d_buf, n, hip_stream)
 * with a device buffer of n doubles that the callback must sum over all processes IN PLACE, ordered
 * after the work already enqueued on hip_stream (e.g. ncclAllReduce(d_buf, d_buf, n, ncclDouble, ncclSum,
 * comm, stream), an MPI_Allreduce after a stream synchronize, or torch.distributed over RCCL):
 *   SKIRT_TALLY_LABS         at the end of every stellar run that stores absorption
 *   SKIRT_TALLY_DUST_LABS    at the end of every self-absorption run (before Labsdusttot is read)
 *   SKIRT_TALLY_INSTRUMENTS  once before the instrument tallies are read (skirt_mcrt_download, or
 *                            skirt_mcrt_reduce_instruments); again only after a further run or zeroing
 * A nonzero return fails the calling function. fn NULL disables the reduction (single process). Every
 * run of a phase must start from tallies that are zero on all ranks but one, or zero everywhere (as in
 * the reference, where each phase runs once per simulation). */
enum { SKIRT_TALLY_LABS = 0, SKIRT_TALLY_DUST_LABS = 1, SKIRT_TALLY_INSTRUMENTS = 2 };
typedef int (*SkirtReduceTallyFn)(void* user, int tally, double* d_buf, size_t n, void* hip_stream);
int skirt_mcrt_set_reducer(SkirtMcrt* ctx, SkirtReduceTallyFn fn, void* user);
int skirt_mcrt_reduce_instruments(SkirtMcrt* ctx);
int skirt_mcrt_upload_cell_sources(SkirtMcrt* ctx, const SkirtCellSourceDesc* src);
/* The same cell sources computed on the device from the current Labs tally (plus the dust Labs when
 * include_dust): grey-body spectra at the cells' equilibrium temperatures, cell luminosities and their
 * per-wavelength cumulative distribution. Asynchronous on the engine stream. */
int skirt_mcrt_upload_emissivity(SkirtMcrt* ctx, const SkirtEmissivityDesc* emis);
int skirt_mcrt_compute_cell_sources(SkirtMcrt* ctx, int include_dust);
/* PanDustSystem::Labsdusttot of the device dust Labs (waits for the engine stream) */
int skirt_mcrt_dust_labs_total(SkirtMcrt* ctx, double* total);
/* the dust Labs tally (PanDustSystem::_Labsdustvv; device layout as Labs): bind caller memory (e.g. a torch
 * tensor to all-reduce), zero it (rebootLabsdust) and copy it to host row-major (cell, wavelength) */
int skirt_mcrt_bind_dust_labs(SkirtMcrt* ctx, double* d_labs_dust);
int skirt_mcrt_zero_dust_labs(SkirtMcrt* ctx);
int skirt_mcrt_download_dust_labs(SkirtMcrt* ctx, double* labs_dust);
int skirt_mcrt_synchronize(SkirtMcrt* ctx);

/* Setup: density sampling on a device (no engine context needed). The host keeps the reference's random
 * stream (it draws the Mersenne-twister words in the reference's order) and the decisions; the device
 * evaluates the dust density at `nsample` positions per item, box_min + u * (box_max - box_min) with
 * u = word / (2^32 - 1) (MTRandom, Random::position(Box)), three words per position, and reduces them in
 * sample order:
 *   SKIRT_DENS_COMPONENTS  out[n x ncomp]: per component the sum of its density over the samples (the cell
 *                          densities, DustSystem::setupSelfAfter, DustSystem.cpp:152-178)
 *   SKIRT_DENS_NODE        out[n x 6]: {sum rho, sum rho x, sum rho y, sum rho z, min rho, max rho} of the
 *                          total density (TreeNodeSampleDensityCalculator: mass, barycentre and density
 *                          dispersion of a tree node, TreeDustGrid.cpp:174-222)
 * The density of component h is norm[h] times its geometry's (PlummerGeometry / ExpDiskGeometry /
 * SersicGeometry / PointGeometry::density), in the host's operation order; the device's exp, pow and log10
 * may differ from the host's by an ulp. Synchronous. */
enum { SKIRT_DENS_COMPONENTS = 0, SKIRT_DENS_NODE = 1 };
typedef struct {
    int ncomp;
    const int* geom_kind;       /* ncomp, SKIRT_GEOM_* */
    const double* geom_param;   /* ncomp x 8, laid out as SkirtSourceDesc::geom_param */
    const double* norm;         /* ncomp: the component's normalization (its dust mass) */
    const double* dens_table;   /* ncomp x 2*ntab (NULL if no SersicGeometry): SersicFunction s_i, then S(s_i) */
    int ntab;
} SkirtDensityDesc;
int skirt_mcrt_sample_density(int device, const SkirtDensityDesc* dens, const double* boxes, size_t n,
                              const uint32_t* words, int nsample, int mode, double* out);

/* The cells of a Voronoi tessellation on HIP device `device` (setup, §8(f)2; the reference computes them with
 * Voro++, VoronoiMesh.cpp:310-376): the host construction of skirt_host_voronoi_build (the domain box clipped
 * by the bisector planes of the nearest sites, nearest first, until no farther site can cut it), one cell per
 * thread in the same f64 operations, so every output equals the host's bit for bit. `extent` = {xmin, ymin,
 * zmin, xmax, ymax, zmax}; `nodes`/`perm`: the k-d tree over the sites whose nearest-site queries the cells
 * use (leaves hold perm[lo..hi), children after their parent). Outputs per site i: its sorted distinct
 * neighbour ids (walls -1..-6) at ids[i * max_ids], their count nids[i] (-1: the cell outgrew the device's
 * fixed capacities; the caller builds it), bbox[6 i ..] (min xyz, max xyz of its vertices), volume[i],
 * centroid[3 i ..]. Synchronous. */
typedef struct {
    int lo, hi, left, right, dim; /* left < 0: a leaf */
    double split, bmin[3], bmax[3];
} SkirtKdNode;
int skirt_mcrt_voronoi_cells(int device, const double* sites, int nsites, const double extent[6],
                             const SkirtKdNode* nodes, int nnodes, const int* perm, int max_ids, int* ids, int* nids,
                             double* bbox, double* volume, double* centroid);

/* Copies tallies to host (Labs converted to row-major cell x wavelength); either pointer may be NULL.
 * With a reducer set, the instrument tallies are summed over the processes first. */
int skirt_mcrt_download(SkirtMcrt* ctx, double* labs, double* instr);
int skirt_mcrt_stats(SkirtMcrt* ctx, SkirtStats* out);
/* DustSystem's cells-crossed statistics (writeCellsCrossed; the _crossed histogram of
 * DustSystem::fillOpticalDepth / opticaldepth, DustSystem.cpp:959-1000): with bins > 0 every FILL path and
 * every peel-off path of the following phases counts one in bin min(segments, bins - 1), its number of
 * segments including those before the grid; zeroed by skirt_mcrt_zero_tallies; bins = 0 turns it off. */
int skirt_mcrt_set_crossed(SkirtMcrt* ctx, int bins);
/* the histogram summed over the device copies: hist[b] for b < bins (waits for the engine's stream).
 * Per process, as in the reference: DustSystem::write (DustSystem.cpp:1004-1024) writes the root process's
 * own _crossed through TextOutFile (root only, TextOutFile.cpp:24-25) and no sumResults covers it, so in a
 * sharded run each rank's histogram counts the paths of its own slice (the ranks' histograms sum to the
 * unsharded run's). */
int skirt_mcrt_download_crossed(SkirtMcrt* ctx, uint64_t* hist, int bins);

/* DustSystem::writeconvergence (DustSystem.cpp:195-250): the column density of the uploaded grid along n
 * rays (rays[6 i .. 6 i + 5] = origin, direction), summed as DustGridPath::opticalDepth with the cell
 * densities of all components, over the photon paths' walk; out[i] in kg/m2. Blocks until done. */
int skirt_mcrt_column_densities(SkirtMcrt* ctx, const double* rays, int n, double* out);
/* engine knobs (0 = default): packet slots in flight, trace-kernel workgroups, and the number of idle
 * lanes at which a trace wave pulls new rays (1..64) */
int skirt_mcrt_configure(SkirtMcrt* ctx, int slots, int grid, int pull_threshold);
const char* skirt_mcrt_last_error(SkirtMcrt* ctx);
void skirt_mcrt_destroy(SkirtMcrt* ctx);

#ifdef __cplusplus
}
#endif
#endif
