// GpuPhotonEngine.cpp -- maintainer-side binding of the MI355X engine into SKIRT v7.3 (see the header).
// Compiled against the reference's headers by integration/check_binding.sh; never part of the engine build.
#include "GpuPhotonEngine.hpp"

#include <cmath>
#include <vector>

#include "Array.hpp"
#include "ArrayTable.hpp"
#include "Box.hpp"
#include "CartesianDustGrid.hpp"
#include "DistantInstrument.hpp"
#include "DustMix.hpp"
#include "DustSystem.hpp"
#include "ExpDiskGeometry.hpp"
#include "FatalError.hpp"
#include "FrameInstrument.hpp"
#include "FullInstrument.hpp"
#include "GeometricStellarComp.hpp"
#include "InstrumentSystem.hpp"
#include "MoveableMesh.hpp"
#include "NR.hpp"
#include "PanDustSystem.hpp"
#include "PlummerGeometry.hpp"
#include "PointGeometry.hpp"
#include "SEDInstrument.hpp"
#include "SersicFunction.hpp"
#include "SersicGeometry.hpp"
#include "SimpleInstrument.hpp"
#include "StellarSystem.hpp"
#include "TreeDustGrid.hpp"
#include "TreeNode.hpp"
#include "VoronoiDustGrid.hpp"
#include "VoronoiMesh.hpp"
#include "WavelengthGrid.hpp"
#include "skirt_host.h"

namespace
{
    // Every process hands its own share of the tallies to the simulation items (DustSystem::absorb, the
    // detector arrays), and the reference's PanDustSystem::sumResults and Instrument::sumResults add them
    // over the processes (PanDustSystem.cpp:394-403, Instrument.cpp:57-66). The engine's device-side
    // reduction is therefore a no-op here; it is what a binding without MPI would fill with ncclAllReduce.
    int keepLocal(void*, int, double*, size_t, void*)
    {
        return 0;
    }

    // the engine's upload of the descriptors (the default sink)
    class UploadSink : public GpuDescriptorSink
    {
    public:
        explicit UploadSink(SkirtMcrt* ctx) : _ctx(ctx) {}
        void grid(const SkirtGridDesc& g) override { check(skirt_mcrt_upload_grid(_ctx, &g)); }
        void media(const SkirtMediaDesc& m) override { check(skirt_mcrt_upload_media(_ctx, &m)); }
        void sources(const SkirtSourceDesc& s) override { check(skirt_mcrt_upload_sources(_ctx, &s)); }
        void instruments(const SkirtInstrDesc* d, int n) override { check(skirt_mcrt_set_instruments(_ctx, d, n)); }

    private:
        void check(int rc) const
        {
            if (rc != SKIRT_OK) throw FATALERROR(QString("MI355X engine: ") + skirt_mcrt_last_error(_ctx));
        }
        SkirtMcrt* _ctx;
    };

    // adds an engine tally to a detector array; an array the reference left unsized (e.g. the dust slots
    // of a FullInstrument without dust emission, FullInstrument.cpp:61-78) must receive nothing
    void addTally(Array& target, const double* src, size_t n, const char* what)
    {
        if (target.size() == n)
        {
            for (size_t i = 0; i < n; i++) target[i] += src[i];
            return;
        }
        for (size_t i = 0; i < n; i++)
            if (src[i] != 0.) throw FATALERROR(QString("MI355X engine: tally for an unsized ") + what);
    }
}

////////////////////////////////////////////////////////////////////

GpuPhotonEngine::GpuPhotonEngine(WavelengthGrid* lambdagrid, StellarSystem* ss, DustSystem* ds,
                                 InstrumentSystem* is, int device)
    : _lambdagrid(lambdagrid), _ss(ss), _ds(ds), _is(is)
{
    if (skirt_mcrt_abi_version() != SKIRT_MCRT_ABI_VERSION)
        throw FATALERROR("MI355X engine: libskirt_amd.so does not match skirt_mcrt.h");
    if (skirt_mcrt_create(device, &_ctx) != SKIRT_OK)
        throw FATALERROR("MI355X engine: cannot create a context on device " + QString::number(device));
    _Nlambda = _lambdagrid->Nlambda();
    _Ncells = _ds ? _ds->Ncells() : 0;
    UploadSink upload(_ctx);
    _sink = &upload;
    describeAll();
    _sink = nullptr;
    check(skirt_mcrt_set_reducer(_ctx, keepLocal, nullptr));
    check(skirt_mcrt_zero_tallies(_ctx));
    _params.store_absorption = _ds && _ds->storeabsorptionrates() ? 1 : 0;
    _params.has_dust = _ds ? 1 : 0;
}

////////////////////////////////////////////////////////////////////

GpuPhotonEngine::GpuPhotonEngine(WavelengthGrid* lambdagrid, StellarSystem* ss, DustSystem* ds, InstrumentSystem* is,
                                 GpuDescriptorSink* sink)
    : _lambdagrid(lambdagrid), _ss(ss), _ds(ds), _is(is), _sink(sink)
{
    _Nlambda = _lambdagrid->Nlambda();
    _Ncells = _ds ? _ds->Ncells() : 0;
}

void GpuPhotonEngine::describe(WavelengthGrid* lambdagrid, StellarSystem* ss, DustSystem* ds, InstrumentSystem* is,
                               GpuDescriptorSink& sink)
{
    GpuPhotonEngine items(lambdagrid, ss, ds, is, &sink);
    items.describeAll();
}

void GpuPhotonEngine::describeAll()
{
    if (_ds)
    {
        describeGrid();
        describeMedia();
    }
    describeSources();
    describeInstruments();
}

////////////////////////////////////////////////////////////////////

GpuPhotonEngine::~GpuPhotonEngine()
{
    if (_ctx) skirt_mcrt_destroy(_ctx);
    if (_voronoi) skirt_host_voronoi_free(_voronoi);
    if (_rccl) skirt_rccl_destroy(_rccl);  // (a wrapped communicator stays the caller's)
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::sumOnDevices(void* ncclComm, int rank)
{
    if (skirt_rccl_wrap(ncclComm, &_rccl) != SKIRT_OK)
        throw FATALERROR("MI355X engine: cannot wrap the RCCL communicator");
    _sumRank = rank;
    check(skirt_mcrt_set_reducer(_ctx, skirt_rccl_reducer(), skirt_rccl_rank(_rccl, 0)));
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::check(int rc) const
{
    if (rc != SKIRT_OK) throw FATALERROR(QString("MI355X engine: ") + skirt_mcrt_last_error(_ctx));
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::setPhaseParams(double minWeightReduction, int minScattEvents, double scattBias,
                                     bool continuousScattering)
{
    _params.min_weight_reduction = minWeightReduction;
    _params.min_scatt_events = minScattEvents;
    _params.scatt_bias = scattBias;
    _params.continuous_scattering = continuousScattering ? 1 : 0;
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::describeGrid()
{
    DustGrid* grid = _ds->dustGrid();
    SkirtGridDesc g{};
    g.ncells = _Ncells;
    std::vector<double> xv, yv, zv, box;
    std::vector<int> firstChild, cellnumber, nbrOffset, nbrList;
    std::vector<signed char> splitDir;

    if (CartesianDustGrid* cg = dynamic_cast<CartesianDustGrid*>(grid))
    {
        // the borders as CartesianDustGrid::setupSelfAfter computes them (CartesianDustGrid.cpp:31-36)
        auto borders = [](MoveableMesh* mesh, double lo, double hi, std::vector<double>& v)
        {
            Array t = mesh->mesh();
            v.resize(t.size());
            for (size_t i = 0; i < t.size(); i++) v[i] = t[i] * (hi - lo) + lo;
            return mesh->numBins();
        };
        g.kind = SKIRT_GRID_CARTESIAN;
        g.nx = borders(cg->meshX(), cg->minX(), cg->maxX(), xv);
        g.ny = borders(cg->meshY(), cg->minY(), cg->maxY(), yv);
        g.nz = borders(cg->meshZ(), cg->minZ(), cg->maxZ(), zv);
        g.xv = xv.data();
        g.yv = yv.data();
        g.zv = zv.data();
    }
    else if (TreeDustGrid* tg = dynamic_cast<TreeDustGrid*>(grid))
    {
        // the breadth-first node vector (TreeDustGrid.cpp:50-164); children of a node are created with
        // consecutive identifiers (TreeNode::createchildren), so one first-child index describes them
        const std::vector<TreeNode*>& tree = tg->_tree;
        const int Nnodes = static_cast<int>(tree.size());
        bool binary = false;
        box.resize(6 * static_cast<size_t>(Nnodes));
        firstChild.assign(Nnodes, -1);
        cellnumber.assign(Nnodes, -1);
        splitDir.assign(Nnodes, -1);  // (leaves: -1, as the .ski driver stores them)
        nbrOffset.assign(6 * static_cast<size_t>(Nnodes) + 1, 0);
        for (int l = 0; l < Nnodes; l++)
        {
            const TreeNode* node = tree[l];
            const double b[6] = {node->xmin(), node->ymin(), node->zmin(), node->xmax(), node->ymax(), node->zmax()};
            for (int q = 0; q < 6; q++) box[6 * static_cast<size_t>(l) + q] = b[q];
            cellnumber[l] = tg->_cellnumberv[l];
            const std::vector<TreeNode*>& ch = node->children();
            if (!ch.empty())
            {
                firstChild[l] = ch[0]->id();
                if (ch.size() == 2)
                {
                    // a k-d node (BinTreeNode): the axis along which the first child stops short
                    binary = true;
                    splitDir[l] = ch[0]->xmax() < node->xmax() ? 0 : ch[0]->ymax() < node->ymax() ? 1 : 2;
                }
            }
            for (int w = 0; w < 6; w++)
            {
                if (static_cast<int>(node->_neighbors.size()) == 6)
                    for (const TreeNode* nb : node->_neighbors[w]) nbrList.push_back(nb->id());
                nbrOffset[6 * static_cast<size_t>(l) + w + 1] = static_cast<int>(nbrList.size());
            }
        }
        g.kind = SKIRT_GRID_OCTREE;
        g.nnodes = Nnodes;
        g.box = box.data();
        g.first_child = firstChild.data();
        g.cellnumber = cellnumber.data();
        g.nbr_offset = nbrOffset.data();
        g.nbr_list = nbrList.data();
        g.split_dir = binary ? splitDir.data() : nullptr;
        g.eps = tg->_eps;
        switch (tg->searchMethod())
        {
        case TreeDustGrid::TopDown: g.search = SKIRT_TREE_TOPDOWN; break;
        case TreeDustGrid::Bookkeeping: g.search = SKIRT_TREE_BOOKKEEPING; break;
        default: g.search = SKIRT_TREE_NEIGHBOR; break;
        }
    }
    else if (VoronoiDustGrid* vg = dynamic_cast<VoronoiDustGrid*>(grid))
    {
        // the generating sites in cell order, tessellated again by the host library (skirt_host.h)
        const VoronoiMesh* mesh = vg->_mesh;
        std::vector<double> sites(3 * static_cast<size_t>(_Ncells));
        for (int m = 0; m < _Ncells; m++)
        {
            Position p = mesh->particlePosition(m);
            sites[3 * static_cast<size_t>(m)] = p.x();
            sites[3 * static_cast<size_t>(m) + 1] = p.y();
            sites[3 * static_cast<size_t>(m) + 2] = p.z();
        }
        Box e = mesh->extent();
        const double extent[6] = {e.xmin(), e.ymin(), e.zmin(), e.xmax(), e.ymax(), e.zmax()};
        _voronoi = skirt_host_voronoi_build(sites.data(), _Ncells, extent);
        if (!_voronoi) throw FATALERROR(QString("MI355X engine: ") + skirt_sim_error());
        if (skirt_host_voronoi_describe(_voronoi, &g) != SKIRT_OK)
            throw FATALERROR("MI355X engine: cannot describe the Voronoi tessellation");
    }
    else
    {
        throw FATALERROR("MI355X engine: dust grid type " + QString(grid->metaObject()->className()) + " is not supported");
    }
    _sink->grid(g);
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::describeMedia()
{
    // rho(m,h) and the per-component optical properties of the KappaRho functor (DustSystem.cpp:465-491)
    const int Ncomp = _ds->Ncomp();
    std::vector<double> rho(static_cast<size_t>(_Ncells) * Ncomp);
    std::vector<double> kext(Ncomp * _Nlambda), ksca(Ncomp * _Nlambda), alb(Ncomp * _Nlambda), g(Ncomp * _Nlambda);
    for (int m = 0; m < _Ncells; m++)
        for (int h = 0; h < Ncomp; h++) rho[static_cast<size_t>(m) * Ncomp + h] = _ds->density(m, h);
    for (int h = 0; h < Ncomp; h++)
    {
        DustMix* mix = _ds->mix(h);
        if (mix->polarization()) throw FATALERROR("MI355X engine: polarized dust mixes are not supported");
        for (int ell = 0; ell < _Nlambda; ell++)
        {
            kext[h * _Nlambda + ell] = mix->kappaext(ell);
            ksca[h * _Nlambda + ell] = mix->kappasca(ell);
            alb[h * _Nlambda + ell] = mix->albedo(ell);
            g[h * _Nlambda + ell] = mix->_asymmparv[ell];  // no public getter (DustMix.hpp:402)
        }
    }
    SkirtMediaDesc md = {_Ncells, Ncomp, _Nlambda, rho.data(), kext.data(), ksca.data(), alb.data(), g.data()};
    _sink->media(md);
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::describeSources()
{
    // StellarSystem::launch (StellarSystem.cpp:116-158): per component its geometry and luminosities, the
    // per-wavelength cumulative luminosity distribution over the components, the emission bias
    QList<StellarComp*> comps = _ss->components();
    const int Ncomp = comps.size();
    std::vector<int> kind(Ncomp, SKIRT_GEOM_PLUMMER);
    std::vector<double> param(8 * static_cast<size_t>(Ncomp), 0.), lum(Ncomp * _Nlambda), lumtot(_Nlambda);
    std::vector<double> cdf(_Nlambda * (Ncomp + 1)), table;
    for (int h = 0; h < Ncomp; h++)
    {
        GeometricStellarComp* sc = dynamic_cast<GeometricStellarComp*>(comps[h]);
        if (!sc) throw FATALERROR("MI355X engine: stellar component type " + QString(comps[h]->metaObject()->className()) + " is not supported");
        Geometry* geo = sc->geometry();
        double* p = &param[8 * static_cast<size_t>(h)];
        if (PlummerGeometry* pg = dynamic_cast<PlummerGeometry*>(geo))
        {
            p[0] = pg->scale();
            p[1] = pg->_rho0;  // PlummerGeometry.cpp:30 (no public getter)
        }
        else if (ExpDiskGeometry* eg = dynamic_cast<ExpDiskGeometry*>(geo))
        {
            kind[h] = SKIRT_GEOM_EXPDISK;
            p[0] = eg->radialScale();
            p[1] = eg->axialScale();
            p[2] = eg->radialTrunc();
            p[3] = eg->axialTrunc();
            p[4] = eg->innerRadius();
            p[5] = eg->_rho0;  // ExpDiskGeometry.cpp:42
        }
        else if (SersicGeometry* sg = dynamic_cast<SersicGeometry*>(geo))
        {
            kind[h] = SKIRT_GEOM_SERSIC;
            p[0] = sg->radius();
            p[1] = sg->index();
            p[2] = sg->_rho0;  // SersicGeometry.cpp (setupSelfBefore)
            const SersicFunction* sf = sg->_sersicfunction;
            if (sf->_sv.size() != 101 || sf->_Mv.size() != 101)
                throw FATALERROR("MI355X engine: unexpected SersicFunction table size");
            table.resize(202 * static_cast<size_t>(Ncomp), 0.);
            for (int q = 0; q < 101; q++)
            {
                table[202 * static_cast<size_t>(h) + q] = sf->_sv[q];
                table[202 * static_cast<size_t>(h) + 101 + q] = sf->_Mv[q];
            }
        }
        else if (dynamic_cast<PointGeometry*>(geo))
        {
            kind[h] = SKIRT_GEOM_POINT;
        }
        else
        {
            throw FATALERROR("MI355X engine: geometry type " + QString(geo->metaObject()->className()) + " is not supported");
        }
        for (int ell = 0; ell < _Nlambda; ell++) lum[h * _Nlambda + ell] = sc->luminosity(ell);
    }
    for (int ell = 0; ell < _Nlambda; ell++)
    {
        lumtot[ell] = _ss->luminosity(ell);
        Array pv(Ncomp), Xv;
        for (int h = 0; h < Ncomp; h++) pv[h] = lum[h * _Nlambda + ell];
        NR::cdf(Xv, pv);
        for (int q = 0; q <= Ncomp; q++) cdf[ell * (Ncomp + 1) + q] = Xv[q];
    }
    SkirtSourceDesc sd = {Ncomp, _Nlambda, kind.data(), param.data(), lum.data(), lumtot.data(), cdf.data(),
                          _ss->emissionBias(), table.empty() ? nullptr : table.data()};
    _sink->sources(sd);
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::describeInstruments()
{
    // DistantInstrument::setupSelfBefore (DistantInstrument.cpp:27-50) and
    // SingleFrameInstrument::setupSelfBefore (SingleFrameInstrument.cpp:26-42), from the public properties
    std::vector<SkirtInstrDesc> descs;
    for (Instrument* instr : _is->instruments())
    {
        DistantInstrument* di = dynamic_cast<DistantInstrument*>(instr);
        SkirtInstrDesc d{};
        if (dynamic_cast<FullInstrument*>(instr))
        {
            d.kind = SKIRT_INSTR_FULL;
            d.scattering_levels = static_cast<FullInstrument*>(instr)->scatteringLevels();
        }
        else if (dynamic_cast<SimpleInstrument*>(instr)) d.kind = SKIRT_INSTR_SIMPLE;
        else if (dynamic_cast<FrameInstrument*>(instr)) d.kind = SKIRT_INSTR_FRAME;
        else if (dynamic_cast<SEDInstrument*>(instr)) d.kind = SKIRT_INSTR_SED;
        else throw FATALERROR("MI355X engine: instrument type " + QString(instr->metaObject()->className()) + " is not supported");
        Direction k = di->bfkobs(Position());
        d.kobs[0] = k.x();
        d.kobs[1] = k.y();
        d.kobs[2] = k.z();
        d.costheta = cos(di->inclination());
        d.sintheta = sin(di->inclination());
        d.cosphi = cos(di->azimuth());
        d.sinphi = sin(di->azimuth());
        d.cospa = cos(di->positionAngle());
        d.sinpa = sin(di->positionAngle());
        if (SingleFrameInstrument* sf = dynamic_cast<SingleFrameInstrument*>(instr))
        {
            d.nx = sf->pixelsX();
            d.ny = sf->pixelsY();
            d.xpmin = sf->centerX() - 0.5 * sf->fieldOfViewX();
            d.xpsiz = sf->fieldOfViewX() / sf->pixelsX();
            d.ypmin = sf->centerY() - 0.5 * sf->fieldOfViewY();
            d.ypsiz = sf->fieldOfViewY() / sf->pixelsY();
        }
        descs.push_back(d);
    }
    _sink->instruments(descs.data(), static_cast<int>(descs.size()));
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::runPhase(int phase, uint32_t cycle, uint64_t Npp, uint64_t seed, int rank, int size)
{
    check(skirt_mcrt_run_phase_shard(_ctx, phase, cycle, Npp, rank, size, seed, &_params));
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::runStellar(uint64_t Npp, uint64_t seed, int rank, int size)
{
    runPhase(SKIRT_PHASE_STELLAR, 0, Npp, seed, rank, size);
    if (_params.store_absorption && handsTallies())
    {
        // DustSystem::absorb, as simulateescapeandabsorption calls it (MonteCarloSimulation.cpp:438-515)
        std::vector<double> labs(static_cast<size_t>(_Ncells) * _Nlambda);
        check(skirt_mcrt_download(_ctx, labs.data(), nullptr));
        for (int m = 0; m < _Ncells; m++)
            for (int ell = 0; ell < _Nlambda; ell++)
            {
                double L = labs[static_cast<size_t>(m) * _Nlambda + ell];
                if (L != 0.) _ds->absorb(m, ell, L, true);
            }
    }
    else
    {
        check(skirt_mcrt_synchronize(_ctx));
    }
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::uploadCellSources(const Array& Labsbolv)
{
    // the per-wavelength cell luminosities and their distribution of dodustselfabsorptionchunk and
    // dodustemissionchunk (PanMonteCarloSimulation.cpp:190-205, 273-294), for every wavelength at once
    PanDustSystem* pds = dynamic_cast<PanDustSystem*>(_ds);
    if (!pds) throw FATALERROR("MI355X engine: dust phases need a PanDustSystem");
    const size_t Nc = static_cast<size_t>(_Ncells);
    std::vector<double> lv(_Nlambda * Nc, 0.), cdf(_Nlambda * (Nc + 1)), ltot(_Nlambda);
    for (int ell = 0; ell < _Nlambda; ell++)
    {
        Array Lv(Nc), Xv;
        for (size_t m = 0; m < Nc; m++)
        {
            double Labsbol = Labsbolv[m];
            if (Labsbol > 0.0) Lv[m] = Labsbol * pds->dustluminosity(static_cast<int>(m), ell);
            lv[ell * Nc + m] = Lv[m];
        }
        ltot[ell] = Lv.sum();
        if (ltot[ell] > 0) NR::cdf(Xv, Lv);
        for (size_t q = 0; q <= Nc; q++) cdf[ell * (Nc + 1) + q] = ltot[ell] > 0 ? Xv[q] : 0.;
    }
    SkirtCellSourceDesc d = {_Ncells, _Nlambda, lv.data(), cdf.data(), ltot.data(), pds->emissionBias()};
    check(skirt_mcrt_upload_cell_sources(_ctx, &d));
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::runSelfAbsorptionCycle(uint32_t cycle, const Array& Labsbolv, uint64_t Npp, uint64_t seed,
                                             int rank, int size)
{
    uploadCellSources(Labsbolv);
    check(skirt_mcrt_zero_dust_labs(_ctx));
    runPhase(SKIRT_PHASE_DUST_SELFABS, cycle, Npp, seed, rank, size);
    std::vector<double> labs(static_cast<size_t>(_Ncells) * _Nlambda);
    check(skirt_mcrt_download_dust_labs(_ctx, labs.data()));
    if (!handsTallies()) return;  // rank 0 holds the device-summed tallies (sumOnDevices)
    for (int m = 0; m < _Ncells; m++)
        for (int ell = 0; ell < _Nlambda; ell++)
        {
            double L = labs[static_cast<size_t>(m) * _Nlambda + ell];
            if (L != 0.) _ds->absorb(m, ell, L, false);
        }
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::runDustEmission(const Array& Labsbolv, uint64_t Npp, uint64_t seed, int rank, int size)
{
    uploadCellSources(Labsbolv);
    runPhase(SKIRT_PHASE_DUST_EMISSION, 0, Npp, seed, rank, size);
    check(skirt_mcrt_synchronize(_ctx));
}

////////////////////////////////////////////////////////////////////

void GpuPhotonEngine::finish()
{
    size_t Nlabs = 0, Ninstr = 0;
    check(skirt_mcrt_tally_sizes(_ctx, &Nlabs, &Ninstr));
    std::vector<double> tallies(Ninstr);
    check(skirt_mcrt_download(_ctx, nullptr, tallies.data()));
    if (!handsTallies()) return;  // rank 0 holds the device-summed tallies (sumOnDevices)
    // per instrument [slot][ell][pixel] frames, then [slot][ell] SEDs (skirt_mcrt.h); the FullInstrument
    // slots are trav, strdir, strsca, dusdir, dussca and the scattering levels (FullInstrument.cpp:107-174)
    const double* t = tallies.data();
    for (Instrument* instr : _is->instruments())
    {
        const size_t Nl = static_cast<size_t>(_Nlambda);
        if (FullInstrument* fi = dynamic_cast<FullInstrument*>(instr))
        {
            const size_t nf = static_cast<size_t>(fi->pixelsX()) * fi->pixelsY();
            Array* frames[] = {&fi->_ftrav, &fi->_fstrdirv, &fi->_fstrscav, &fi->_fdusdirv, &fi->_fdusscav};
            Array* seds[] = {&fi->_Ftrav, &fi->_Fstrdirv, &fi->_Fstrscav, &fi->_Fdusdirv, &fi->_Fdusscav};
            const int Nslots = 5 + fi->_Nscatt;
            for (int s = 0; s < Nslots; s++, t += Nl * nf)
                addTally(s < 5 ? *frames[s] : fi->_fstrscavv[s - 5], t, Nl * nf, "FullInstrument frame");
            for (int s = 0; s < Nslots; s++, t += Nl)
                addTally(s < 5 ? *seds[s] : fi->_Fstrscavv[s - 5], t, Nl, "FullInstrument SED");
        }
        else if (SimpleInstrument* si = dynamic_cast<SimpleInstrument*>(instr))
        {
            const size_t nf = static_cast<size_t>(si->pixelsX()) * si->pixelsY();
            addTally(si->_ftotv, t, Nl * nf, "SimpleInstrument frame");
            t += Nl * nf;
            addTally(si->_Ftotv, t, Nl, "SimpleInstrument SED");
            t += Nl;
        }
        else if (FrameInstrument* fr = dynamic_cast<FrameInstrument*>(instr))
        {
            const size_t nf = static_cast<size_t>(fr->pixelsX()) * fr->pixelsY();
            addTally(fr->_ftotv, t, Nl * nf, "FrameInstrument frame");
            t += Nl * nf;
        }
        else if (SEDInstrument* se = dynamic_cast<SEDInstrument*>(instr))
        {
            addTally(se->_Ftotv, t, Nl, "SEDInstrument SED");
            t += Nl;
        }
    }
    if (t > tallies.data() + Ninstr) throw FATALERROR("MI355X engine: instrument tally size mismatch");
}

////////////////////////////////////////////////////////////////////
