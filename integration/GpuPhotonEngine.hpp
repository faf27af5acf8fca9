// GpuPhotonEngine.hpp -- the binding a SKIRT v7.3 maintainer adds to SKIRTcore to run the photon phases on
// MI355X GPUs through the engine's C ABI (include/skirt_mcrt.h). INTEGRATION.md section 2 shows where it is
// called from; integration/check_binding.sh compiles it against the reference's headers.
//
// The binding replaces the three Parallel::call sites of the photon phases and nothing else:
//   MonteCarloSimulation::runstellaremission     MonteCarloSimulation.cpp:251-261
//   PanMonteCarloSimulation::rundustselfabsorption (one call per cycle)   PanMonteCarloSimulation.cpp:144-145
//   PanMonteCarloSimulation::rundustemission     PanMonteCarloSimulation.cpp:260-261
// Everything around those calls stays the reference's: setup, the dust emission spectra (DustLib), the
// convergence loop, the cross-process sums (PanDustSystem::sumResults, Instrument::sumResults) and the
// output writers. The engine's tallies are handed to the items that own them in the reference's layouts,
// exactly where the CPU chunks would have added them (DustSystem::absorb, the instruments' detector arrays).
//
// Needs `friend class GpuPhotonEngine;` in the classes whose state it reads or fills (the patch that
// check_binding.sh applies to a scratch copy of the headers): DustMix (_asymmparv), TreeDustGrid (_tree,
// _cellnumberv, _eps), TreeNode (_neighbors), VoronoiDustGrid (_mesh), SersicGeometry (_sersicfunction,
// _rho0), SersicFunction (_sv, _Mv), PlummerGeometry and ExpDiskGeometry (_rho0), FullInstrument,
// SimpleInstrument, FrameInstrument, SEDInstrument (detector arrays).
#ifndef GPUPHOTONENGINE_HPP
#define GPUPHOTONENGINE_HPP

#include <cstdint>
#include <vector>

#include "skirt_mcrt.h"

class Array;
class DustSystem;
class InstrumentSystem;
class StellarSystem;
class WavelengthGrid;
struct SkirtVoronoi;

// Receives the engine's input descriptors as the binding extracts them from the set-up simulation items; the
// engine's upload is one such sink, a file dump (skirt_host_write_descriptors) another, which lets a test
// compare the binding's extraction with the .ski driver's without a device (tests/test_binding_describe.py)
class GpuDescriptorSink
{
public:
    virtual ~GpuDescriptorSink() = default;
    virtual void grid(const SkirtGridDesc& g) = 0;
    virtual void media(const SkirtMediaDesc& m) = 0;
    virtual void sources(const SkirtSourceDesc& s) = 0;
    virtual void instruments(const SkirtInstrDesc* d, int n) = 0;
};

class GpuPhotonEngine
{
public:
    // The descriptors the constructor would upload, handed to `sink` instead; needs no device
    static void describe(WavelengthGrid* lambdagrid, StellarSystem* ss, DustSystem* ds, InstrumentSystem* is,
                         GpuDescriptorSink& sink);

    // Describes the set-up simulation items to the engine on HIP device `device` (one engine per process;
    // the MPI rank picks its GPU). ds may be null (no dust system).
    GpuPhotonEngine(WavelengthGrid* lambdagrid, StellarSystem* ss, DustSystem* ds, InstrumentSystem* is,
                    int device);
    ~GpuPhotonEngine();
    GpuPhotonEngine(const GpuPhotonEngine&) = delete;
    GpuPhotonEngine& operator=(const GpuPhotonEngine&) = delete;

    // The MonteCarloSimulation properties of the photon loop (MonteCarloSimulation.cpp:31-35)
    void setPhaseParams(double minWeightReduction, int minScattEvents, double scattBias, bool continuousScattering);

    // dostellaremissionchunk over this process's share of every wavelength (rank of size, as the
    // reference's IdenticalAssigner hands out chunks); the absorbed stellar luminosities go into the dust
    // system through DustSystem::absorb(m, ell, L, true)
    void runStellar(uint64_t Npp, uint64_t seed, int rank, int size);

    // dodustselfabsorptionchunk for one self-absorption cycle (numbered 0, 1, ... over the whole
    // simulation). Labsbolv is the caller's _Labsbolv (PanMonteCarloSimulation.cpp:131-132) after
    // calculatedustemission and rebootLabsdust; the absorbed dust luminosities go into the dust system
    // through PanDustSystem::absorb(m, ell, L, false)
    void runSelfAbsorptionCycle(uint32_t cycle, const Array& Labsbolv, uint64_t Npp, uint64_t seed, int rank,
                                int size);

    // dodustemissionchunk for the dust emission phase (Labsbolv as above)
    void runDustEmission(const Array& Labsbolv, uint64_t Npp, uint64_t seed, int rank, int size);

    // After the last phase: the instrument tallies of all phases into the instruments' detector arrays
    // (summed over the processes later by Instrument::sumResults, in InstrumentSystem::write)
    void finish();
    // Optional, before the first phase: the cross-process sums on the GPUs instead of in MPI. ncclComm is
    // this process's RCCL communicator over the job's ranks (an ncclComm_t, e.g. from ncclCommInitRank with
    // the unique id broadcast over the reference's own ProcessCommunicator). Every phase's tallies are then
    // all-reduced over xGMI at the phase end (skirt_rccl_reducer, include/skirt_host.h), and only rank 0
    // hands them to the items: the reference's sumResults still runs and adds the other ranks' zeros.
    void sumOnDevices(void* ncclComm, int rank);

private:
    // describe(): the items only, no engine context
    GpuPhotonEngine(WavelengthGrid* lambdagrid, StellarSystem* ss, DustSystem* ds, InstrumentSystem* is,
                    GpuDescriptorSink* sink);
    void describeAll();
    void check(int rc) const;
    void describeGrid();
    void describeMedia();
    void describeSources();
    void describeInstruments();
    void uploadCellSources(const Array& Labsbolv);
    void runPhase(int phase, uint32_t cycle, uint64_t Npp, uint64_t seed, int rank, int size);
    bool handsTallies() const { return !_rccl || _sumRank == 0; }

    WavelengthGrid* _lambdagrid;
    StellarSystem* _ss;
    DustSystem* _ds;
    InstrumentSystem* _is;
    SkirtMcrt* _ctx{nullptr};
    GpuDescriptorSink* _sink{nullptr};  // where describeAll() sends the descriptors (the engine upload by default)
    SkirtVoronoi* _voronoi{nullptr};
    struct SkirtRccl* _rccl{nullptr};  // sumOnDevices
    int _sumRank{0};
    SkirtPhaseParams _params{};
    int _Nlambda{0};
    int _Ncells{0};
};

#endif
