// Dust emission spectra and dust-phase cell sources; see dustemission.hpp for the reference map.
#include "dustemission.hpp"

#include <cmath>
#include <stdexcept>

namespace skirt {

namespace {

constexpr double kH = 6.62606957e-34;  // Units.cpp:17-19
constexpr double kC = 2.99792458e8;
constexpr double kK = 1.3806488e-23;

// NR::locate_clip (NR.hpp): index j with xv[j] <= x < xv[j+1], clipped to [0, n-2]
int locateClip(const double* xv, int n, double x) {
    if (x < xv[0]) return 0;
    int jl = -1, ju = n - 1;
    while (ju - jl > 1) {
        int jm = (ju + jl) >> 1;
        if (x < xv[jm]) ju = jm;
        else jl = jm;
    }
    return jl;
}

double interpolateLinLin(double x, double x1, double x2, double f1, double f2) {
    return f1 + ((x - x1) / (x2 - x1)) * (f2 - f1);
}

// DustMix::equilibrium (DustMix.cpp:704-712) for a one-population mix
double equilibrium(const DustMix& mix, const PlanckTable& t, const WavelengthGrid& wl, const std::vector<double>& Jv) {
    double planckabs = 0.0;
    for (int ell = 0; ell < wl.n(); ell++) planckabs += mix.sigmaabs[ell] * Jv[ell] * wl.dlambda[ell];
    // DustMix::invplanckabs (DustMix.cpp:689-693)
    int n = (int)t.planckabs.size();
    int p = locateClip(t.planckabs.data(), n, planckabs);
    return interpolateLinLin(planckabs, t.planckabs[p], t.planckabs[p + 1], t.Tv[p], t.Tv[p + 1]);
}

// GreyBodyDustEmissivity::emissivity (GreyBodyDustEmissivity.cpp:19-43), one population
std::vector<double> greyBody(const DustMix& mix, const PlanckTable& t, const WavelengthGrid& wl,
                             const std::vector<double>& Jv) {
    int Nl = wl.n();
    std::vector<double> ev(Nl, 0.0);
    double T = equilibrium(mix, t, wl, Jv);
    for (int ell = 0; ell < Nl; ell++) ev[ell] += mix.sigmaabs[ell] * planckFunction(T, wl.lambda[ell]);
    for (int ell = 0; ell < Nl; ell++) ev[ell] /= mix.mu;
    return ev;
}

}  // namespace

double planckFunction(double T, double lambda) {
    double x = kH * kC / (lambda * kK * T);
    return 2.0 * kH * kC * kC / std::pow(lambda, 5) / (std::exp(x) - 1.0);
}

std::vector<PlanckTable> planckTables(const Model& m) {
    if (!m.pan || !m.wl.pan) throw std::runtime_error("dust emission needs a panchromatic wavelength grid");
    std::vector<PlanckTable> out;
    const int NT = 1000;
    for (const DustComp& dc : m.dust) {
        PlanckTable t;
        // NR::powgrid(_Tv, 0., 5000., NT, 500.) (NR.hpp:189-204)
        t.Tv.resize(NT + 1);
        double xmin = 0., xmax = 5000., ratio = 500.;
        double range = xmax - xmin;
        double q = std::pow(ratio, 1. / (NT - 1));
        double qn = std::pow(q, NT);
        for (int i = 0; i <= NT; ++i) t.Tv[i] = xmin + (1. - std::pow(q, i)) / (1. - qn) * range;
        t.planckabs.assign(NT + 1, 0.0);
        for (int p = 1; p <= NT; p++) {  // the value for p == 0 stays zero
            double planckabs = 0.0;
            for (int ell = 0; ell < m.wl.n(); ell++) {
                double lambda = m.wl.lambda[ell];
                double dlambda = m.wl.dlambda[ell];
                planckabs += dc.mix.sigmaabs[ell] * planckFunction(t.Tv[p], lambda) * dlambda;
            }
            t.planckabs[p] = planckabs;
        }
        out.push_back(std::move(t));
    }
    return out;
}

std::vector<double> totalLabs(const Model& m, const std::vector<double>& labsStel, const std::vector<double>* labsDust) {
    std::vector<double> out(labsStel.size());
    bool dust = labsDust && !labsDust->empty();
    for (size_t q = 0; q < out.size(); q++) {
        double sum = 0;
        sum += labsStel[q];
        if (dust) sum += (*labsDust)[q];
        out[q] = sum;
    }
    (void)m;
    return out;
}

void dustEmissionSpectra(const Model& m, const std::vector<PlanckTable>& tables, const std::vector<double>& labs,
                         std::vector<double>& lum) {
    int Ncells = m.ncells(), Nl = m.wl.n(), Ncomp = m.ncomp();
    lum.assign((size_t)Ncells * Nl, 0.0);
    std::vector<double> Jv(Nl);
    for (int c = 0; c < Ncells; c++) {
        // EmissionCalculator::body with one cell per library entry: Jv = 0 + meanintensityv(m), /= 1
        double fac = 4.0 * M_PI * m.volume[c];
        for (int ell = 0; ell < Nl; ell++) {
            double kappaabsrho = 0.0;
            for (int h = 0; h < Ncomp; h++) kappaabsrho += m.dust[h].mix.kabs[ell] * m.rho[(size_t)c * Ncomp + h];
            double J = labs[(size_t)c * Nl + ell] / (kappaabsrho * fac) / m.wl.dlambda[ell];
            Jv[ell] = 0.0 + (std::isfinite(J) ? J : 0.0);
            Jv[ell] /= 1;
        }
        double* Lv = &lum[(size_t)c * Nl];
        if (Ncomp > 1) {
            for (int h = 0; h < Ncomp; h++) {
                std::vector<double> ev = greyBody(m.dust[h].mix, tables[h], m.wl, Jv);
                double rho = m.rho[(size_t)c * Ncomp + h];
                for (int ell = 0; ell < Nl; ell++) Lv[ell] += ev[ell] * rho;
            }
        } else {
            std::vector<double> ev = greyBody(m.dust[0].mix, tables[0], m.wl, Jv);
            for (int ell = 0; ell < Nl; ell++) Lv[ell] = ev[ell];
        }
        for (int ell = 0; ell < Nl; ell++) Lv[ell] *= m.wl.dlambda[ell];
        double total = 0.0;
        for (int ell = 0; ell < Nl; ell++) total += Lv[ell];
        if (total > 0)
            for (int ell = 0; ell < Nl; ell++) Lv[ell] /= total;
    }
}

void cellSources(const Model& m, const std::vector<double>& labsStel, const std::vector<double>* labsDust,
                 const std::vector<double>& lum, CellSources& out) {
    int Ncells = m.ncells(), Nl = m.wl.n();
    out.ncells = Ncells;
    out.nlambda = Nl;
    // PanDustSystem::Labs(m) (PanDustSystem.cpp:337-349)
    bool dust = labsDust && !labsDust->empty();
    std::vector<double> Labsbol(Ncells, 0.0);
    for (int c = 0; c < Ncells; c++) {
        double sum = 0;
        for (int ell = 0; ell < Nl; ell++) sum += labsStel[(size_t)c * Nl + ell];
        if (dust)
            for (int ell = 0; ell < Nl; ell++) sum += (*labsDust)[(size_t)c * Nl + ell];
        Labsbol[c] = sum;
    }
    out.lv.assign((size_t)Nl * Ncells, 0.0);
    out.cdf.assign((size_t)Nl * (Ncells + 1), 0.0);
    out.ltot.assign(Nl, 0.0);
    for (int ell = 0; ell < Nl; ell++) {
        double* Lv = &out.lv[(size_t)ell * Ncells];
        for (int c = 0; c < Ncells; c++) {
            double Lb = Labsbol[c];
            if (Lb > 0.0) Lv[c] = Lb * lum[(size_t)c * Nl + ell];
        }
        double Ltot = 0.0;
        for (int c = 0; c < Ncells; c++) Ltot += Lv[c];
        out.ltot[ell] = Ltot;
        if (Ltot > 0) {
            // NR::cdf (NR.hpp:388-394)
            double* X = &out.cdf[(size_t)ell * (Ncells + 1)];
            X[0] = 0.0;
            for (int c = 0; c < Ncells; c++) X[c + 1] = X[c] + Lv[c];
            double norm = X[Ncells];
            for (int c = 0; c <= Ncells; c++) X[c] /= norm;
        }
    }
}

double tableTotal(const std::vector<double>& t) {
    double sum = 0;
    for (double v : t) sum += v;
    return sum;
}

bool SelfAbsorptionSchedule::next() {
    while (stage < kStages) {
        bool fixed = fixedCycles > 0;
        if (cycle <= maxCycles() && (!convergence || fixed)) return true;
        stage++;
        cycle = 1;
        convergence = false;
    }
    return false;
}

void SelfAbsorptionSchedule::finishCycle(double Labsdusttot) {
    double eps = std::fabs((Labsdusttot - prevLabsdusttot) / Labsdusttot);
    prevLabsdusttot = Labsdusttot;
    if ((stage < kStages - 1 || cycle > 1) && eps < epsmax(stage)) convergence = true;
    cycle++;
}

}  // namespace skirt
