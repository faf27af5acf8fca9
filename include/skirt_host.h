/* skirt_host.h -- C API of the host side: .ski file -> model -> MI355X engine -> SKIRT-format outputs.
 *
 * This is the native replacement of the reference's simulation driver for the photon-shooting phases
 * (Simulation::setupAndRun, SKIRTcore/Simulation.cpp:65-75; MonteCarloSimulation::runstellaremission,
 * MonteCarloSimulation.cpp:251-261; MonteCarloSimulation::write, :553-558). Setup (ski parsing, grid
 * construction, cell density sampling, optical tables, instrument geometry) runs on the host exactly as
 * in the reference; the photon loop runs on the GPU through include/skirt_mcrt.h.
 *
 * Multi-GPU: one process per GPU. Each process loads the same ski, attaches its device, sets the
 * engine's reducer (e.g. an RCCL all-reduce) and runs its shard of every phase
 * (skirt_sim_run_stellar_shard, skirt_sim_run_dust_shard); skirt_sim_fetch then returns the whole
 * simulation's tallies on every rank, and one rank calls skirt_sim_write.
 */
#ifndef SKIRT_HOST_H
#define SKIRT_HOST_H

#include <stdint.h>

#include "skirt_mcrt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct SkirtSim SkirtSim;

typedef struct {
    int pan;                    /* PanMonteCarloSimulation (1) or Oligo (0) */
    int ncells, nlambda, ncomp, ninstruments, grid_kind;
    int nnodes;                 /* octree nodes (0 for Cartesian) */
    uint64_t npp;               /* photon packets per wavelength (ceil(packages)) */
    uint64_t total_packets;     /* npp * nlambda for the stellar phase */
    uint64_t seed;
    int store_absorption, has_dust;
    double setup_seconds;
} SkirtSimInfo;

/* Parses the ski file and performs the host setup. packages > 0 overrides the ski's packages,
 * seed != 0 overrides its random seed. datadir NULL = the packaged skirt_amd/data. Returns NULL on
 * failure (skirt_sim_error). */
SkirtSim* skirt_sim_load(const char* ski, const char* datadir, double packages, uint64_t seed);
/* As skirt_sim_load; setup_device >= 0 runs the setup's density sampling (tree subdivision and cell
 * densities, the setup's hot loop) on that HIP device through skirt_mcrt_sample_density. The host still
 * draws the reference's random numbers and takes the subdivision decisions; densities may differ from the
 * host's by an ulp (the device's exp/pow/log10). -1: on the host, bit-identical to the reference. */
SkirtSim* skirt_sim_load_ex(const char* ski, const char* datadir, double packages, uint64_t seed, int setup_device);
int skirt_sim_info(SkirtSim* sim, SkirtSimInfo* info);
/* The seed of the photon phases' Philox streams (default: the setup seed). The grid, densities and every
 * other setup draw stay those of the setup seed, so runs that differ only in this seed are independent
 * Monte Carlo realisations on one and the same grid (per-cell statistics against a reference run). */
int skirt_sim_set_photon_seed(SkirtSim* sim, uint64_t seed);
/* creates the engine on HIP device `device` and uploads grid, media, sources and instruments */
int skirt_sim_attach(SkirtSim* sim, int device);
SkirtMcrt* skirt_sim_engine(SkirtSim* sim);
/* stellar emission over global packets [first, first+count) (count 0 = all); asynchronous */
int skirt_sim_run_stellar(SkirtSim* sim, uint64_t first, uint64_t count);
/* PanMonteCarloSimulation::runSelf after the stellar phase (PanMonteCarloSimulation.cpp:96-105): for a
 * Pan dust system with dust emission, the self-absorption cycles (if enabled; host-side grey-body
 * spectra and cell sources between cycles, convergence as the reference) and the dust emission phase,
 * whose detections add to the instrument tallies. Single process; fetches the stellar Labs first.
 * Returns after launching the dust emission phase (asynchronous, like run_stellar). */
int skirt_sim_run_dust(SkirtSim* sim);
/* Multi-GPU: the same phases on rank `rank` of `world` processes (one per GPU). Every phase shoots this
 * rank's slice of EVERY wavelength (skirt_mcrt_run_phase_shard, the reference's IdenticalAssigner), and
 * the engine's reducer (skirt_mcrt_set_reducer, required for world > 1) sums the stellar Labs after the
 * stellar phase, the dust Labs after every self-absorption cycle and the instruments before they are
 * read, so every rank follows the same self-absorption schedule as one process would. */
int skirt_sim_run_stellar_shard(SkirtSim* sim, int rank, int world);
int skirt_sim_run_dust_shard(SkirtSim* sim, int rank, int world);
/* dust Labs of the last self-absorption cycle (row-major cell x wavelength), or NULL; downloads it
 * (waiting for the device) when skirt_sim_fetch has not done so since the last skirt_sim_run_dust */
const double* skirt_sim_labs_dust(SkirtSim* sim);
/* Labsdusttot after every self-absorption cycle; returns the number of cycles */
int skirt_sim_selfabs_totals(SkirtSim* sim, const double** totals);
/* waits and copies the device tallies into the host accumulators */
int skirt_sim_fetch(SkirtSim* sim);
/* host accumulators after skirt_sim_fetch (same layouts as include/skirt_mcrt.h) */
const double* skirt_sim_labs(SkirtSim* sim);
/* the cell densities of the setup, ncells x ncomp row-major (DustSystem::_rhovv); NULL without dust */
const double* skirt_sim_density(SkirtSim* sim);
const double* skirt_sim_instrument(SkirtSim* sim, int i, int* nslots, int* nframe, int* has_frames, int* has_seds);
/* replaces the host accumulators (e.g. after an all-reduce done by the caller) */
int skirt_sim_set_tallies(SkirtSim* sim, const double* labs, const double* instr);
/* writes <prefix>_<instrument>_sed.dat, FITS frames and ds_isrf / ds_cellprops files */
int skirt_sim_write(SkirtSim* sim, const char* prefix);
const char* skirt_sim_error(void);
void skirt_sim_free(SkirtSim* sim);

/* Voronoi dust grids for a binding inside SKIRT. The reference's VoronoiMesh
 * keeps its cells' neighbour lists in an implementation type private to VoronoiMesh.cpp, so a binding
 * hands over the generating sites (VoronoiMesh::particlePosition, in cell order) and the domain, and this
 * host library tessellates them again (the same tessellation, neighbour order and block lists as the .ski
 * driver, pinned to the reference's Voronoi fixtures). skirt_host_voronoi_describe fills the Voronoi fields
 * of a SkirtGridDesc, valid while the SkirtVoronoi lives. */
typedef struct SkirtVoronoi SkirtVoronoi;
SkirtVoronoi* skirt_host_voronoi_build(const double* sites, int nsites, const double extent[6]);
/* As skirt_host_voronoi_build, with the cells computed on HIP device `device` (skirt_mcrt_voronoi_cells) and
 * the ones outgrowing its capacities on the host (*host_cells of them, if host_cells is not NULL); device < 0:
 * every cell on the host. The tessellation is the host build's, bit for bit, either way. */
SkirtVoronoi* skirt_host_voronoi_build_ex(const double* sites, int nsites, const double extent[6], int device,
                                          int* host_cells);
/* copies the cells' volumes (ncells) and centroids (3 per cell); either pointer may be NULL */
int skirt_host_voronoi_cells(const SkirtVoronoi* v, double* volume, double* centroid);
int skirt_host_voronoi_describe(const SkirtVoronoi* v, SkirtGridDesc* grid);
void skirt_host_voronoi_free(SkirtVoronoi* v);

/* The engine's input descriptors without a device (tests of the maintainer binding's extraction,
 * INTEGRATION.md): skirt_sim_describe writes the SkirtGridDesc, SkirtMediaDesc, SkirtSourceDesc and
 * SkirtInstrDesc that skirt_sim_attach would upload for this model to `path` (truncated first);
 * skirt_host_write_descriptors appends the given descriptors in the same canonical form (NULL pointers
 * and ninstr < 0 are skipped): one record per field, "<name> <type> <count>\n" followed by count raw
 * values (type d double, i int32, b int8), array lengths as skirt_mcrt.h states them. */
int skirt_sim_describe(SkirtSim* sim, const char* path);
int skirt_host_write_descriptors(const char* path, const SkirtGridDesc* grid, const SkirtMediaDesc* media,
                                 const SkirtSourceDesc* sources, const SkirtInstrDesc* instr, int ninstr);

/* The cross-GPU sums in C++: RCCL (NCCL API) all-reduces over xGMI, the MI355X counterpart of the
 * reference's MPI_Allreduce of the absorption tables and instrument arrays (PanDustSystem.cpp:394-404,
 * Instrument.cpp:57-66, MPIsupport/ProcessManager.cpp:133-137).
 * skirt_rccl_create makes one communicator per device of this process (ncclCommInitAll over `devices`);
 * skirt_rccl_reducer is the engine's reducer callback (skirt_mcrt_set_reducer) and skirt_rccl_rank(r, rank)
 * its user pointer for the engine of rank `rank`: the callback sums the tally in place, ncclSum of doubles,
 * on the stream the engine hands it. Each rank's engine must then be driven by its own host thread (the
 * collectives of the ranks meet on the devices). A process that runs one rank of a multi-process job
 * creates its communicator through its own bootstrap (e.g. ncclCommInitRank, or torch.distributed) and can
 * use the same callback through skirt_rccl_wrap. */
typedef struct SkirtRccl SkirtRccl;
int skirt_rccl_create(int ndev, const int* devices, SkirtRccl** out);
/* wraps an existing communicator (an ncclComm_t) of one rank: ndev = 1, rank 0 */
int skirt_rccl_wrap(void* nccl_comm, SkirtRccl** out);
void* skirt_rccl_rank(SkirtRccl* r, int rank);
SkirtReduceTallyFn skirt_rccl_reducer(void);
/* The reference's Parallel::call stops every worker at the first exception and rethrows it in the parent
 * (SKIRTcore/Parallel.cpp:181-193). Across devices: skirt_rccl_abort marks the job failed (`why` is kept as the
 * first failure's message), after which no rank of `r` enqueues another all-reduce (the reducer returns
 * non-zero, also to ranks waiting for the others before one), and aborts owned communicators
 * (ncclCommAbort), which returns ranks already waiting in an all-reduce on the device. Idempotent.
 * The reducer of several ranks in one process waits, before each all-reduce, until every rank has arrived
 * or one has failed, so a rank that fails between two collectives leaves none of its peers waiting. */
int skirt_rccl_abort(SkirtRccl* r, const char* why);
void skirt_rccl_destroy(SkirtRccl* r);
/* The driver of `skirt-mi355x -g N`: loads the ski once per device, runs every phase of the simulation
 * with each device shooting its rank's slice of every wavelength (one host thread per device) and the
 * tallies summed by skirt_rccl at each phase end, then writes the outputs from rank 0. The first device
 * thread that fails stops the others (skirt_rccl_abort) and its error is returned; SKIRT_AMD_FAIL_DEVICE=d
 * makes device d's thread fail before its first phase (tests). packages > 0 and
 * seed != 0 override the ski's. stats (may be NULL) receives rank 0's statistics; seconds (may be NULL)
 * the wall time of the photon phases. */
int skirt_sim_run_devices(const char* ski, const char* datadir, int ndev, double packages, uint64_t seed,
                          const char* outprefix, SkirtStats* stats, double* seconds);

#ifdef __cplusplus
}
#endif
#endif
