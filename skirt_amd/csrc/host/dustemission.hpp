// Dust emission between photon phases: the equilibrium-temperature grey-body spectra of every dust
// cell (AllCellsDustLib + GreyBodyDustEmissivity) and the per-wavelength cell sources of the dust
// emission and self-absorption phases. Host code shared by the engine's host driver and the oracle,
// restating the reference operation for operation:
//   DustMix temperature grid + Planck-integrated absorption   SKIRTcore/DustMix.cpp:238-263, 674-712
//   PlanckFunction                                            SKIRTcore/PlanckFunction.cpp
//   DustSystem::meanintensityv                                SKIRTcore/DustSystem.cpp:935-957
//   DustLib::calculate / EmissionCalculator::body             SKIRTcore/DustLib.cpp:60-185
//   GreyBodyDustEmissivity::emissivity                        SKIRTcore/GreyBodyDustEmissivity.cpp:19-43
//   PanDustSystem::Labs(m), dustluminosity                    SKIRTcore/PanDustSystem.cpp:320-349, 408-411
//   cell luminosities and their cumulative distribution       PanMonteCarloSimulation.cpp:193-205, 273-294
#pragma once

#include <vector>

#include "model.hpp"

namespace skirt {

// DustMix::planckabs table of one dust mix: temperature grid (NR::powgrid(0, 5000, 1000, 500)) and the
// Planck-integrated absorption cross section at each temperature
struct PlanckTable {
    std::vector<double> Tv, planckabs;
};

// PlanckFunction B_lambda(T)
double planckFunction(double T, double lambda);

// one table per dust component (Pan simulations only)
std::vector<PlanckTable> planckTables(const Model& m);

// The absorbed luminosity Labs(m, ell) of PanDustSystem: stellar plus (when present) dust, row-major
// (cell, wavelength). labsDust may be null or empty.
std::vector<double> totalLabs(const Model& m, const std::vector<double>& labsStel, const std::vector<double>* labsDust);

// DustLib::calculate (AllCellsDustLib, GreyBodyDustEmissivity): the normalized emission spectrum
// dustluminosity(m, ell) of every cell, row-major (cell, wavelength), from Labs(m, ell)
void dustEmissionSpectra(const Model& m, const std::vector<PlanckTable>& tables, const std::vector<double>& labs,
                         std::vector<double>& lum);

// The sources of a dust phase at every wavelength: Lv[ell][m] = Labsbol(m) * dustluminosity(m, ell) for
// cells with Labsbol > 0, their sum Ltot[ell] and NR::cdf over the cells (Ncells + 1 values, only when
// Ltot > 0). Labsbol(m) = PanDustSystem::Labs(m): the stellar sum over wavelengths continued by the
// dust sum (labsDust may be null or empty).
struct CellSources {
    int ncells = 0, nlambda = 0;
    std::vector<double> lv;    // [ell][m]
    std::vector<double> cdf;   // [ell][m], Ncells + 1 per wavelength
    std::vector<double> ltot;  // [ell]
};
void cellSources(const Model& m, const std::vector<double>& labsStel, const std::vector<double>* labsDust,
                 const std::vector<double>& lum, CellSources& out);

// Labsdusttot / Labsstellartot of PanDustSystem (sums over cells, then wavelengths)
double tableTotal(const std::vector<double>& t);

// The self-absorption schedule of PanMonteCarloSimulation::rundustselfabsorption
// (PanMonteCarloSimulation.cpp:109-181): three stages with packet factors 1/10, 1/3, 1 and
// convergence thresholds 1 %, 0.7 %, 0.5 %; at most 100 cycles per stage, or exactly `cycles` when
// the dust system fixes them.
struct SelfAbsorptionSchedule {
    static constexpr int kStages = 3;
    static double factor(int stage) { return stage == 0 ? 1. / 10. : stage == 1 ? 1. / 3. : 1.; }
    static double epsmax(int stage) { return stage == 0 ? 0.010 : stage == 1 ? 0.007 : 0.005; }
    int fixedCycles = 0;
    int stage = 0, cycle = 1;       // the cycle about to run (1-based, as the reference counts)
    bool convergence = false;
    double prevLabsdusttot = 0.;
    int maxCycles() const { return fixedCycles ? fixedCycles : 100; }
    // true while another cycle of the current stage (or a later one) remains; advances stage/cycle
    bool next();
    // after a cycle: the convergence test of the reference on the new total absorbed dust luminosity
    void finishCycle(double Labsdusttot);
};

}  // namespace skirt
