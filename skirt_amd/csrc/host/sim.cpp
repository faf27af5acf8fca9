// Host driver: .ski -> Model -> device engine -> outputs (include/skirt_host.h).
#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/skirt_host.h"
#include "dustemission.hpp"
#include "model.hpp"
#include "outputs.hpp"

using namespace skirt;

namespace {

constexpr int kCrossedBins = 16384;  // cells-crossed histogram bins written to ds_crossed (paths of 0 .. 16383 cells);
// the device keeps one more, which counts the longer paths
thread_local std::string g_err;
}

struct SkirtSim {
    Model m;
    double setupSeconds = 0;
    uint64_t npp = 0;
    SkirtMcrt* eng = nullptr;
    std::vector<double> labs;                 // Ncells x Nlambda (stellar)
    std::vector<double> labsDust;             // Ncells x Nlambda (last self-absorption cycle)
    bool dustLabsOnDevice = false;            // labsDust is still to be downloaded (skirt_sim_fetch)
    std::vector<double> dustTotals;           // Labsdusttot after every self-absorption cycle
    std::vector<double> instrAll;             // concatenated, per instrument frames [slot][lambda][pixel] + SEDs
    std::vector<size_t> instrOff;             // per instrument offset into instrAll
    std::vector<std::vector<double>> frames, seds;
    ~SkirtSim() {
        if (eng) skirt_mcrt_destroy(eng);
    }
    size_t instrTotal() const {
        size_t n = 0;
        for (auto& ins : m.instruments) {
            if (ins.hasFrames()) n += (size_t)ins.nslots() * m.wl.n() * ins.nframe();
            if (ins.hasSeds()) n += (size_t)ins.nslots() * m.wl.n();
        }
        return n;
    }
    void splitInstr() {
        frames.assign(m.instruments.size(), {});
        seds.assign(m.instruments.size(), {});
        size_t off = 0;
        for (size_t i = 0; i < m.instruments.size(); i++) {
            const Instrument& ins = m.instruments[i];
            size_t nf = ins.hasFrames() ? (size_t)ins.nslots() * m.wl.n() * ins.nframe() : 0;
            size_t ns = ins.hasSeds() ? (size_t)ins.nslots() * m.wl.n() : 0;
            frames[i].assign(instrAll.begin() + off, instrAll.begin() + off + nf);
            off += nf;
            seds[i].assign(instrAll.begin() + off, instrAll.begin() + off + ns);
            off += ns;
        }
    }
};

namespace {
int check(SkirtSim* s, int rc) {
    if (rc != SKIRT_OK) g_err = s && s->eng ? skirt_mcrt_last_error(s->eng) : "engine error";
    return rc;
}
}  // namespace

namespace skirt {
// the calling thread's skirt_sim_error message (rccl_reducer.cpp: a device thread's failure, reported on
// the caller's thread)
void setSimError(const std::string& msg) { g_err = msg; }
}  // namespace skirt

extern "C" {

const char* skirt_sim_error(void) { return g_err.c_str(); }


namespace {
// SkirtGeometry parameters as SkirtSourceDesc::geom_param lays them out; returns the SKIRT_GEOM_* kind
int packGeometry(const Geometry& g, double* p) {
    for (int q = 0; q < 8; q++) p[q] = 0.0;
    switch (g.kind) {
    case GeometryKind::Point: return SKIRT_GEOM_POINT;
    case GeometryKind::Sersic: p[0] = g.reff; p[1] = g.n; p[2] = g.rho0; return SKIRT_GEOM_SERSIC;
    case GeometryKind::ExpDisk: {
        const double v[6] = {g.hR, g.hz, g.Rmax, g.zmax, g.Rmin, g.rho0};
        for (int q = 0; q < 6; q++) p[q] = v[q];
        return SKIRT_GEOM_EXPDISK;
    }
    default: p[0] = g.c; p[1] = g.rho0; return SKIRT_GEOM_PLUMMER;
    }
}

static_assert((int)kDensComponents == (int)SKIRT_DENS_COMPONENTS && (int)kDensNode == (int)SKIRT_DENS_NODE,
              "density sampling modes");

static_assert(sizeof(KdNode) == sizeof(SkirtKdNode) && offsetof(KdNode, split) == offsetof(SkirtKdNode, split) &&
                  offsetof(KdNode, bmax) == offsetof(SkirtKdNode, bmax),
              "the host k-d tree node is the C ABI's SkirtKdNode");

// a Voronoi tessellation's cells on a HIP device through skirt_mcrt_voronoi_cells
VoronoiCellsFn deviceVoronoiCells(int device) {
    return [device](const std::vector<double>& sites, const double box[6], const std::vector<KdNode>& nodes,
                    const std::vector<int>& perm, int maxIds, int* ids, int* nids, double* bbox, double* volume,
                    double* centroid) {
        const int rc = skirt_mcrt_voronoi_cells(device, sites.data(), (int)(sites.size() / 3), box,
                                                reinterpret_cast<const SkirtKdNode*>(nodes.data()), (int)nodes.size(),
                                                perm.data(), maxIds, ids, nids, bbox, volume, centroid);
        if (rc)
            throw std::runtime_error("Voronoi cells on device " + std::to_string(device) + " failed (error " +
                                     std::to_string(rc) + ")");
    };
}

// the setup's density sampling (and a Voronoi grid's cells) on a HIP device through
// skirt_mcrt_sample_density (skirt_mcrt_voronoi_cells)
struct DeviceDensitySampler final : DensitySampler {
    int device;
    VoronoiCellsFn cells;
    explicit DeviceDensitySampler(int d) : device(d), cells(deviceVoronoiCells(d)) {}
    const VoronoiCellsFn* voronoiCells() const override { return &cells; }
    void sample(const std::vector<DustComp>& dust, const double* boxes, size_t n, const uint32_t* words, int nsample,
                int mode, double* out) override {
        const int nc = (int)dust.size();
        std::vector<int> kind(nc);
        std::vector<double> param(8 * (size_t)nc), norm(nc), table;
        int ntab = 0;
        for (int h = 0; h < nc; h++)
            if (dust[h].geom.kind == GeometryKind::Sersic) ntab = std::max(ntab, (int)dust[h].geom.sv.size());
        if (ntab) table.assign(2 * (size_t)ntab * nc, 0.0);
        for (int h = 0; h < nc; h++) {
            const Geometry& g = dust[h].geom;
            kind[h] = packGeometry(g, &param[8 * (size_t)h]);
            norm[h] = dust[h].nf;
            if (g.kind == GeometryKind::Sersic) {
                if ((int)g.sv.size() != ntab || g.Sv.size() != g.sv.size())
                    throw std::runtime_error("Sersic density tables of unequal lengths");
                std::copy(g.sv.begin(), g.sv.end(), table.begin() + 2 * (size_t)ntab * h);
                std::copy(g.Sv.begin(), g.Sv.end(), table.begin() + 2 * (size_t)ntab * h + ntab);
            }
        }
        const SkirtDensityDesc d{nc, kind.data(), param.data(), norm.data(), ntab ? table.data() : nullptr, ntab};
        const int rc = skirt_mcrt_sample_density(device, &d, boxes, n, words, nsample, mode, out);
        if (rc) throw std::runtime_error("density sampling on device " + std::to_string(device) + " failed (error " +
                                         std::to_string(rc) + ")");
    }
};
}  // namespace

SkirtSim* skirt_sim_load(const char* ski, const char* datadir, double packages, uint64_t seed) {
    return skirt_sim_load_ex(ski, datadir, packages, seed, -1);
}

SkirtSim* skirt_sim_load_ex(const char* ski, const char* datadir, double packages, uint64_t seed, int setup_device) {
    try {
        auto s = std::make_unique<SkirtSim>();
        auto t0 = std::chrono::steady_clock::now();
        unsigned long theSeed = seed ? (unsigned long)seed : readSkiSeed(ski);
        // a seed of 0 (mod 2^32) fills the generator's state with zeros: it emits only zeros, which the
        // deviates reject forever (the reference hangs in its setup); refuse it
        if ((theSeed & 0xffffffffUL) == 0) throw std::runtime_error("random seed 0 (mod 2^32) is not usable");
        MTRandom mt(theSeed);  // setup draws exactly like the reference (density / tree sampling)
        std::unique_ptr<DeviceDensitySampler> sampler;
        if (setup_device >= 0) sampler.reset(new DeviceDensitySampler(setup_device));
        s->m = loadSki(ski, mt, datadir && *datadir ? datadir : defaultDataDir(), sampler.get());
        s->m.seed = theSeed;
        if (packages > 0) s->m.packages = packages;
        s->npp = (uint64_t)std::ceil(s->m.packages);
        s->setupSeconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        s->labs.assign(s->m.hasDust && s->m.storeAbsorption ? (size_t)s->m.ncells() * s->m.wl.n() : 0, 0.0);
        s->instrAll.assign(s->instrTotal(), 0.0);
        s->splitInstr();
        return s.release();
    } catch (std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

int skirt_sim_info(SkirtSim* s, SkirtSimInfo* o) {
    if (!s || !o) return SKIRT_ERR_ARG;
    o->pan = s->m.pan;
    o->ncells = s->m.ncells();
    o->nlambda = s->m.wl.n();
    o->ncomp = s->m.ncomp();
    o->ninstruments = (int)s->m.instruments.size();
    o->grid_kind = s->m.grid.kind == GridKind::Octree ? SKIRT_GRID_OCTREE
                   : s->m.grid.kind == GridKind::Voronoi ? SKIRT_GRID_VORONOI : SKIRT_GRID_CARTESIAN;
    o->nnodes = s->m.grid.kind == GridKind::Octree ? s->m.grid.tree.nnodes() : 0;
    o->npp = s->npp;
    o->total_packets = s->npp * (uint64_t)s->m.wl.n();
    o->seed = s->m.seed;
    o->store_absorption = s->m.hasDust && s->m.storeAbsorption;
    o->has_dust = s->m.hasDust;
    o->setup_seconds = s->setupSeconds;
    return SKIRT_OK;
}

int skirt_sim_set_photon_seed(SkirtSim* s, uint64_t seed) {
    if (!s || !seed) return SKIRT_ERR_ARG;
    s->m.seed = seed;
    return SKIRT_OK;
}

}  // extern "C"

namespace {
// The descriptors skirt_sim_attach uploads (and skirt_sim_describe writes), over the model's arrays
struct Descs {
    bool hasGrid = false;
    SkirtGridDesc g{};
    SkirtMediaDesc md{};
    SkirtSourceDesc sd{};
    std::vector<SkirtInstrDesc> ids;
    std::vector<double> kext, ksca, alb, gg, gp, lum, cdf, gt;
    std::vector<int> gk;
};

void buildDescs(const Model& m, Descs& d) {
    const int Nl = m.wl.n();
    if (m.hasDust) {
        d.hasGrid = true;
        SkirtGridDesc& g = d.g;
        g.ncells = m.ncells();
        if (m.grid.kind == GridKind::Voronoi) {
            const VoronoiGrid& v = m.grid.vor;
            g.kind = SKIRT_GRID_VORONOI;
            g.site = v.site.data();
            g.cell_nbr_offset = v.nbrOffset.data();
            g.cell_nbr_list = v.nbrList.data();
            g.cell_bbox = v.bbox.data();
            g.extent[0] = v.xmin; g.extent[1] = v.ymin; g.extent[2] = v.zmin;
            g.extent[3] = v.xmax; g.extent[4] = v.ymax; g.extent[5] = v.zmax;
            g.eps = v.eps;
            g.nblocks = v.nb;
            g.block_offset = v.blockOffset.data();
            g.block_list = v.blockList.data();
        } else if (m.grid.kind == GridKind::Cartesian) {
            g.kind = SKIRT_GRID_CARTESIAN;
            g.nx = m.grid.cart.Nx; g.ny = m.grid.cart.Ny; g.nz = m.grid.cart.Nz;
            g.xv = m.grid.cart.xv.data(); g.yv = m.grid.cart.yv.data(); g.zv = m.grid.cart.zv.data();
        } else {
            const OctreeGrid& t = m.grid.tree;
            g.kind = SKIRT_GRID_OCTREE;
            g.nnodes = t.nnodes();
            g.box = t.box.data();
            g.first_child = t.firstChild.data();
            g.split_dir = t.binary ? t.dir.data() : nullptr;
            g.cellnumber = t.cellnumber.data();
            g.nbr_offset = t.nbrOffset.data();
            g.nbr_list = t.nbrList.data();
            g.eps = t.eps;
            g.search = t.search == 0 ? SKIRT_TREE_TOPDOWN : t.search == 2 ? SKIRT_TREE_BOOKKEEPING : SKIRT_TREE_NEIGHBOR;
        }
        const int nc = m.ncomp();
        d.kext.resize(nc * Nl); d.ksca.resize(nc * Nl); d.alb.resize(nc * Nl); d.gg.resize(nc * Nl);
        for (int h = 0; h < nc; h++)
            for (int ell = 0; ell < Nl; ell++) {
                d.kext[h * Nl + ell] = m.dust[h].mix.kext[ell];
                d.ksca[h * Nl + ell] = m.dust[h].mix.ksca[ell];
                d.alb[h * Nl + ell] = m.dust[h].mix.albedo[ell];
                d.gg[h * Nl + ell] = m.dust[h].mix.g[ell];
            }
        d.md = SkirtMediaDesc{m.ncells(), nc, Nl, m.rho.data(), d.kext.data(), d.ksca.data(), d.alb.data(), d.gg.data()};
    }
    const int ns = (int)m.starL.size();
    d.gk.assign(ns, SKIRT_GEOM_PLUMMER);
    d.gp.assign(8 * ns, 0.0);
    d.lum.resize(ns * Nl);
    d.cdf.resize(Nl * (ns + 1));
    for (int h = 0; h < ns; h++) {
        const Geometry& g = m.starGeom[h];
        d.gk[h] = packGeometry(g, &d.gp[8 * h]);
        if (g.kind == GeometryKind::Sersic) {
            d.gt.resize(202 * (size_t)ns, 0.0);
            for (int q = 0; q < 101; q++) {
                d.gt[202 * (size_t)h + q] = g.sv[q];
                d.gt[202 * (size_t)h + 101 + q] = g.Mv[q];
            }
        }
        for (int ell = 0; ell < Nl; ell++) d.lum[h * Nl + ell] = m.starL[h][ell];
    }
    for (int ell = 0; ell < Nl; ell++)
        for (int q = 0; q <= ns; q++) d.cdf[ell * (ns + 1) + q] = m.starX[ell][q];
    d.sd = SkirtSourceDesc{ns, Nl, d.gk.data(), d.gp.data(), d.lum.data(), m.starLtot.data(), d.cdf.data(),
                           m.starEmissionBias, d.gt.empty() ? nullptr : d.gt.data()};
    for (const Instrument& ins : m.instruments) {
        SkirtInstrDesc x{};
        x.kind = (int)ins.kind;
        x.nx = ins.Nx; x.ny = ins.Ny;
        x.scattering_levels = ins.scatteringLevels;
        for (int q = 0; q < 3; q++) x.kobs[q] = ins.kobs[q];
        x.sinphi = ins.sinphi; x.cosphi = ins.cosphi; x.sintheta = ins.sintheta; x.costheta = ins.costheta;
        x.sinpa = ins.sinpa; x.cospa = ins.cospa;
        x.xpmin = ins.xpmin; x.xpsiz = ins.xpsiz; x.ypmin = ins.ypmin; x.ypsiz = ins.ypsiz;
        d.ids.push_back(x);
    }
}
}  // namespace

extern "C" {

int skirt_sim_attach(SkirtSim* s, int device) {
    if (!s) return SKIRT_ERR_ARG;
    if (s->eng) { skirt_mcrt_destroy(s->eng); s->eng = nullptr; }
    int rc = skirt_mcrt_create(device, &s->eng);
    if (rc) { g_err = "cannot create the engine on device " + std::to_string(device); return rc; }
    const Model& m = s->m;
    Descs d;
    buildDescs(m, d);
    if (d.hasGrid) {
        if ((rc = check(s, skirt_mcrt_upload_grid(s->eng, &d.g)))) return rc;
        if ((rc = check(s, skirt_mcrt_upload_media(s->eng, &d.md)))) return rc;
    }
    if ((rc = check(s, skirt_mcrt_upload_sources(s->eng, &d.sd)))) return rc;
    if ((rc = check(s, skirt_mcrt_set_instruments(s->eng, d.ids.data(), (int)d.ids.size())))) return rc;
    size_t nl = 0, ni = 0;
    skirt_mcrt_tally_sizes(s->eng, &nl, &ni);
    // the device tally pads each frame pixel's slots to a 64-byte line; downloads restore this layout
    if (ni < s->instrAll.size()) { g_err = "instrument tally size mismatch"; return SKIRT_ERR_STATE; }
    // DustSystem writeCellsCrossed: the engine keeps the cells-crossed histogram for ds_crossed
    if (m.hasDust && m.writeCellsCrossed && (rc = check(s, skirt_mcrt_set_crossed(s->eng, kCrossedBins + 1)))) return rc;
    return check(s, skirt_mcrt_zero_tallies(s->eng));
}

int skirt_sim_describe(SkirtSim* s, const char* path) {
    if (!s || !path) return SKIRT_ERR_ARG;
    Descs d;
    buildDescs(s->m, d);
    if (FILE* f = std::fopen(path, "wb")) std::fclose(f);  // the writer appends
    else { g_err = std::string("cannot write ") + path; return SKIRT_ERR_ARG; }
    int rc = skirt_host_write_descriptors(path, d.hasGrid ? &d.g : nullptr, d.hasGrid ? &d.md : nullptr, &d.sd,
                                          d.ids.data(), (int)d.ids.size());
    if (rc) g_err = std::string("cannot write ") + path;
    return rc;
}

SkirtMcrt* skirt_sim_engine(SkirtSim* s) { return s ? s->eng : nullptr; }

int skirt_sim_run_stellar(SkirtSim* s, uint64_t first, uint64_t count) {
    if (!s || !s->eng) { g_err = "no engine attached"; return SKIRT_ERR_STATE; }
    uint64_t total = s->npp * (uint64_t)s->m.wl.n();
    if (count == 0) count = total - std::min(first, total);
    SkirtPhaseParams p{s->m.minWeightReduction, s->m.minScattEvents, s->m.scattBias,
                       s->m.hasDust && s->m.storeAbsorption ? 1 : 0, s->m.hasDust ? 1 : 0, s->m.continuousScattering ? 1 : 0};
    return check(s, skirt_mcrt_run_stellar(s->eng, s->npp, first, count, s->m.seed, &p));
}

int skirt_sim_run_stellar_shard(SkirtSim* s, int rank, int world) {
    if (!s || !s->eng) { g_err = "no engine attached"; return SKIRT_ERR_STATE; }
    SkirtPhaseParams p{s->m.minWeightReduction, s->m.minScattEvents, s->m.scattBias,
                       s->m.hasDust && s->m.storeAbsorption ? 1 : 0, s->m.hasDust ? 1 : 0, s->m.continuousScattering ? 1 : 0};
    return check(s, skirt_mcrt_run_phase_shard(s->eng, SKIRT_PHASE_STELLAR, 0, s->npp, rank, world, s->m.seed, &p));
}

int skirt_sim_run_dust(SkirtSim* s) { return skirt_sim_run_dust_shard(s, 0, 1); }

int skirt_sim_run_dust_shard(SkirtSim* s, int rank, int world) {
    if (!s || !s->eng) { g_err = "no engine attached"; return SKIRT_ERR_STATE; }
    if (world < 1 || rank < 0 || rank >= world) {
        g_err = "bad shard (rank, world)";
        return SKIRT_ERR_ARG;
    }
    const Model& m = s->m;
    if (!(m.hasDust && m.pan && m.dustEmission)) return SKIRT_OK;  // no dust emission: nothing to do
    try {
        int rc;
        const int Nl = m.wl.n();
        // SKIRT_AMD_PHASE_TIMES: wall time of the host driver's stages (a stage ending in a device
        // synchronization includes the device work queued before it)
        static const bool timing = getenv("SKIRT_AMD_PHASE_TIMES") != nullptr;
        auto t0 = std::chrono::steady_clock::now();
        auto stage = [&](const char* what) {
            if (!timing) return;
            const auto t1 = std::chrono::steady_clock::now();
            fprintf(stderr, "[dust] %-28s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
            t0 = t1;
        };
        const std::vector<PlanckTable> tables = planckTables(m);
        stage("planck tables");
        SkirtPhaseParams p{m.minWeightReduction, m.minScattEvents, m.scattBias, 0, 1, m.continuousScattering ? 1 : 0};
        // The cell sources between phases: on the device from the device tallies (default), or on the
        // host by the restatement the oracle shares (SKIRT_AMD_HOST_SOURCES=1)
        const char* env = getenv("SKIRT_AMD_HOST_SOURCES");
        const bool hostSources = env && env[0] == '1';
        std::vector<double> lum;
        CellSources src;
        if (hostSources) {
            // the stellar phase's Labs on the host (already summed over the processes at its phase end)
            if (!s->labs.empty() && (rc = check(s, skirt_mcrt_download(s->eng, s->labs.data(), nullptr)))) return rc;
        } else {
            std::vector<double> sigma, kabs, mu, planck;
            for (int h = 0; h < m.ncomp(); h++) {
                const DustMix& mx = m.dust[h].mix;
                sigma.insert(sigma.end(), mx.sigmaabs.begin(), mx.sigmaabs.end());
                kabs.insert(kabs.end(), mx.kabs.begin(), mx.kabs.end());
                mu.push_back(mx.mu);
                planck.insert(planck.end(), tables[h].planckabs.begin(), tables[h].planckabs.end());
            }
            SkirtEmissivityDesc ed{m.ncells(), Nl, m.ncomp(), (int)tables[0].Tv.size(), m.volume.data(), kabs.data(),
                                   sigma.data(), mu.data(), tables[0].Tv.data(), planck.data(), m.wl.lambda.data(),
                                   m.wl.dlambda.data(), m.dustEmissionBias};
            if ((rc = check(s, skirt_mcrt_upload_emissivity(s->eng, &ed)))) return rc;
            stage("emissivity upload");
        }
        auto prepare = [&](bool withDust) -> int {
            if (!hostSources) return check(s, skirt_mcrt_compute_cell_sources(s->eng, withDust ? 1 : 0));
            const std::vector<double>* dust = withDust ? &s->labsDust : nullptr;
            dustEmissionSpectra(m, tables, totalLabs(m, s->labs, dust), lum);
            cellSources(m, s->labs, dust, lum, src);
            SkirtCellSourceDesc d{src.ncells, src.nlambda, src.lv.data(), src.cdf.data(), src.ltot.data(),
                                  m.dustEmissionBias};
            return check(s, skirt_mcrt_upload_cell_sources(s->eng, &d));
        };
        s->dustTotals.clear();
        if (m.selfAbsorption) {
            // PanMonteCarloSimulation::rundustselfabsorption (PanMonteCarloSimulation.cpp:109-181). The
            // first cycle's spectra come from the stellar Labs alone: the dust Labs start at zero (also
            // on the device, where an earlier run may have left its last cycle's tally)
            s->labsDust.assign((size_t)m.ncells() * Nl, 0.0);
            if ((rc = check(s, skirt_mcrt_zero_dust_labs(s->eng)))) return rc;
            SelfAbsorptionSchedule sched;
            sched.fixedCycles = m.cycles;
            uint32_t cycle = 0;
            while (sched.next()) {
                if ((rc = prepare(true))) return rc;  // calculatedustemission, Labsbolv = Labs(m)
                if ((rc = check(s, skirt_mcrt_zero_dust_labs(s->eng)))) return rc;  // rebootLabsdust
                uint64_t npp = (uint64_t)std::ceil(m.packages * SelfAbsorptionSchedule::factor(sched.stage));
                // this rank's slice of every wavelength; the engine's reducer sums the dust Labs over the
                // processes at the phase end (PanDustSystem::Labsdusttot sums over processes)
                if ((rc = check(s, skirt_mcrt_run_phase_shard(s->eng, SKIRT_PHASE_DUST_SELFABS, cycle++, npp, rank,
                                                              world, m.seed, &p))))
                    return rc;
                double total = 0;
                if (hostSources) {
                    if ((rc = check(s, skirt_mcrt_download_dust_labs(s->eng, s->labsDust.data())))) return rc;
                    total = tableTotal(s->labsDust);
                } else if ((rc = check(s, skirt_mcrt_dust_labs_total(s->eng, &total)))) {
                    return rc;
                }
                s->dustTotals.push_back(total);
                sched.finishCycle(total);
                stage("self-absorption cycle");
            }
            // the final dust Labs reach the host with the other tallies (skirt_sim_fetch), not here
            s->dustLabsOnDevice = !hostSources;
        }
        // PanMonteCarloSimulation::rundustemission (PanMonteCarloSimulation.cpp:245-264)
        if ((rc = prepare(m.selfAbsorption))) return rc;
        uint64_t npp = (uint64_t)std::ceil(m.packages * m.emissionBoost);
        rc = check(s, skirt_mcrt_run_phase_shard(s->eng, SKIRT_PHASE_DUST_EMISSION, 0, npp, rank, world, m.seed, &p));
        stage("dust emission (launched)");
        return rc;
    } catch (std::exception& e) {
        g_err = e.what();
        return SKIRT_ERR_ARG;
    }
}

const double* skirt_sim_labs_dust(SkirtSim* s) {
    if (!s || s->labsDust.empty()) return nullptr;
    if (s->dustLabsOnDevice) {  // still on the device (skirt_sim_fetch not called yet): download it now
        if (!s->eng || check(s, skirt_mcrt_download_dust_labs(s->eng, s->labsDust.data()))) return nullptr;
        s->dustLabsOnDevice = false;
    }
    return s->labsDust.data();
}

int skirt_sim_selfabs_totals(SkirtSim* s, const double** totals) {
    if (!s || !totals) return -1;
    *totals = s->dustTotals.empty() ? nullptr : s->dustTotals.data();
    return (int)s->dustTotals.size();
}

int skirt_sim_fetch(SkirtSim* s) {
    if (!s || !s->eng) { g_err = "no engine attached"; return SKIRT_ERR_STATE; }
    int rc = check(s, skirt_mcrt_download(s->eng, s->labs.empty() ? nullptr : s->labs.data(),
                                          s->instrAll.empty() ? nullptr : s->instrAll.data()));
    if (rc) return rc;
    if (s->dustLabsOnDevice) {
        if ((rc = check(s, skirt_mcrt_download_dust_labs(s->eng, s->labsDust.data())))) return rc;
        s->dustLabsOnDevice = false;
    }
    s->splitInstr();
    return SKIRT_OK;
}

const double* skirt_sim_labs(SkirtSim* s) { return s && !s->labs.empty() ? s->labs.data() : nullptr; }
const double* skirt_sim_density(SkirtSim* s) { return s && !s->m.rho.empty() ? s->m.rho.data() : nullptr; }

const double* skirt_sim_instrument(SkirtSim* s, int i, int* nslots, int* nframe, int* hasFrames, int* hasSeds) {
    if (!s || i < 0 || i >= (int)s->m.instruments.size()) return nullptr;
    const Instrument& ins = s->m.instruments[i];
    if (nslots) *nslots = ins.nslots();
    if (nframe) *nframe = ins.hasFrames() ? ins.nframe() : 0;
    if (hasFrames) *hasFrames = ins.hasFrames();
    if (hasSeds) *hasSeds = ins.hasSeds();
    size_t off = 0;
    for (int q = 0; q < i; q++) {
        const Instrument& o = s->m.instruments[q];
        if (o.hasFrames()) off += (size_t)o.nslots() * s->m.wl.n() * o.nframe();
        if (o.hasSeds()) off += (size_t)o.nslots() * s->m.wl.n();
    }
    return s->instrAll.data() + off;
}

int skirt_sim_set_tallies(SkirtSim* s, const double* labs, const double* instr) {
    if (!s) return SKIRT_ERR_ARG;
    if (labs && !s->labs.empty()) std::copy(labs, labs + s->labs.size(), s->labs.begin());
    if (instr && !s->instrAll.empty()) std::copy(instr, instr + s->instrAll.size(), s->instrAll.begin());
    s->splitInstr();
    return SKIRT_OK;
}

int skirt_sim_write(SkirtSim* s, const char* prefix) {
    if (!s || !prefix) return SKIRT_ERR_ARG;
    std::string overflow;  // a limit met by ds_crossed, reported after every other output is written
    try {
        writeOutputs(s->m, prefix, s->frames, s->seds,
                     totalLabs(s->m, s->labs, s->labsDust.empty() ? nullptr : &s->labsDust));
        if (s->m.hasDust && s->m.writeCellsCrossed && s->eng) {
            std::vector<uint64_t> hist(kCrossedBins + 1);
            int rc = check(s, skirt_mcrt_download_crossed(s->eng, hist.data(), kCrossedBins + 1));
            if (rc) return rc;
            // the device's extra bin counts every longer path: the reference's _crossed grows without limit
            // (DustSystem.cpp:969), so such a path cannot be written as an exact count
            if (hist[kCrossedBins])
                overflow = "ds_crossed: " + std::to_string(hist[kCrossedBins]) + " paths crossed " +
                           std::to_string(kCrossedBins) + " or more cells, beyond the histogram's bins";
            else {
                hist.resize(kCrossedBins);
                writeCellsCrossed(s->m, prefix, hist);
            }
        }
        if (s->m.hasDust && s->m.writeConvergence && s->eng) {
            // the six half axes from the origin (DustSystem.cpp:213-242), walked by the engine
            const double rays[36] = {0, 0, 0, 1, 0, 0, 0, 0, 0, -1, 0, 0, 0, 0, 0, 0, 1, 0,
                                     0, 0, 0, 0, -1, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, -1};
            double col[6];
            int rc = check(s, skirt_mcrt_column_densities(s->eng, rays, 6, col));
            if (rc) return rc;
            double sigma[3];
            for (int ax = 0; ax < 3; ax++) {
                sigma[ax] = 0.0;
                sigma[ax] += col[2 * ax];
                sigma[ax] += col[2 * ax + 1];
            }
            writeConvergence(s->m, prefix, sigma);
        }
    } catch (std::exception& e) {
        g_err = e.what();
        return SKIRT_ERR_ARG;
    }
    if (!overflow.empty()) {
        g_err = overflow;
        return SKIRT_ERR_UNSUPPORTED;
    }
    return SKIRT_OK;
}

void skirt_sim_free(SkirtSim* s) { delete s; }

struct SkirtVoronoi {
    VoronoiGrid g;
};

SkirtVoronoi* skirt_host_voronoi_build(const double* sites, int nsites, const double extent[6]) {
    return skirt_host_voronoi_build_ex(sites, nsites, extent, -1, nullptr);
}

SkirtVoronoi* skirt_host_voronoi_build_ex(const double* sites, int nsites, const double extent[6], int device,
                                          int* host_cells) {
    if (!sites || nsites < 1 || !extent) {
        g_err = "skirt_host_voronoi_build: no sites or no extent";
        return nullptr;
    }
    try {
        auto v = std::make_unique<SkirtVoronoi>();
        std::vector<double> sv(sites, sites + 3 * (size_t)nsites);
        const VoronoiCellsFn dev = device >= 0 ? deviceVoronoiCells(device) : VoronoiCellsFn();
        buildVoronoi(v->g, sv, extent[0], extent[3], extent[1], extent[4], extent[2], extent[5],
                     device >= 0 ? &dev : nullptr, host_cells);
        return v.release();
    } catch (std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

int skirt_host_voronoi_cells(const SkirtVoronoi* v, double* volume, double* centroid) {
    if (!v) return SKIRT_ERR_ARG;
    if (volume) std::copy(v->g.volume.begin(), v->g.volume.end(), volume);
    if (centroid) std::copy(v->g.centroid.begin(), v->g.centroid.end(), centroid);
    return SKIRT_OK;
}

int skirt_host_voronoi_describe(const SkirtVoronoi* v, SkirtGridDesc* g) {
    if (!v || !g) return SKIRT_ERR_ARG;
    const VoronoiGrid& vg = v->g;
    g->kind = SKIRT_GRID_VORONOI;
    g->ncells = vg.ncells();
    g->site = vg.site.data();
    g->cell_nbr_offset = vg.nbrOffset.data();
    g->cell_nbr_list = vg.nbrList.data();
    g->cell_bbox = vg.bbox.data();
    g->extent[0] = vg.xmin; g->extent[1] = vg.ymin; g->extent[2] = vg.zmin;
    g->extent[3] = vg.xmax; g->extent[4] = vg.ymax; g->extent[5] = vg.zmax;
    g->eps = vg.eps;
    g->nblocks = vg.nb;
    g->block_offset = vg.blockOffset.data();
    g->block_list = vg.blockList.data();
    return SKIRT_OK;
}

void skirt_host_voronoi_free(SkirtVoronoi* v) { delete v; }

}  // extern "C"
