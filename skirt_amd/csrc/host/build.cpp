// .ski file -> Model, including every setup step that consumes random numbers.
//
// The reference performs these steps in SimulationItem::setup() order (SimulationItem.cpp:18-31):
// wavelength grid, stellar system (StellarSystem.cpp:35-52), dust mixes (DustMix.cpp:44-264), the dust
// grid (TreeDustGrid.cpp:50-164 draws density samples while subdividing), then the cell densities
// (DustSystem.cpp:63-178, 100 random positions per cell) and the instruments. Random draws happen only
// in the tree subdivision and the cell density sampling, in that order; both are reproduced here on the
// caller's UniformSource so that a single-threaded reference run and this setup produce bit-identical
// densities and trees.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cfloat>
#include <limits>
#include <cstring>
#include <dlfcn.h>
#include <fstream>
#include <memory>
#include <numeric>
#include <sstream>
#include <stdexcept>
#include <thread>

#include "dustemission.hpp"
#include "model.hpp"
#include "mt_random.hpp"
#include "xml.hpp"

namespace skirt {

namespace {
// SKIRT_AMD_SETUP_TIMES=1 prints the duration of every setup stage to stderr
struct StageTimer {
    const char* name;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit StageTimer(const char* n) : name(n) {}
    ~StageTimer() {
        static const bool on = std::getenv("SKIRT_AMD_SETUP_TIMES") != nullptr;
        if (on)
            std::fprintf(stderr, "[setup] %-24s %.3f s\n", name,
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
};

// Runs fn(q, u) for the items q in [0, n) on worker threads, where u points to the `per` uniform
// deviates item q would have drawn had the items been processed one after the other, drawing as they
// go: the deviates are drawn ahead, in item order, one chunk at a time (the next chunk while the
// workers evaluate the current one). Results are therefore identical to the sequential loop's.
template <class Fn>
void parallelDraws(UniformSource& rng, size_t n, int per, Fn fn) {
    if (n == 0) return;
    const size_t chunk = std::max<size_t>(1, (size_t)(1 << 20) / std::max(1, per));
    const int T = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    // the Mersenne twister hands over raw words (the sequential part); the workers convert them
    MTRandom* mt = dynamic_cast<MTRandom*>(&rng);
    std::vector<uint32_t> wbuf[2];
    std::vector<double> dbuf[2];
    auto draw = [&](int k, size_t q0) {
        const size_t m = (std::min(n, q0 + chunk) - q0) * per;
        if (mt) {
            wbuf[k].resize(m);
            mt->words(wbuf[k].data(), m);
        } else {
            dbuf[k].resize(m);
            for (double& u : dbuf[k]) u = rng.uniform();
        }
    };
    draw(0, 0);
    for (size_t q0 = 0, k = 0; q0 < n; q0 += chunk, k ^= 1) {
        const size_t q1 = std::min(n, q0 + chunk);
        std::atomic<size_t> next{q0};
        std::vector<std::thread> th;
        std::vector<std::string> errs(T);
        for (int w = 0; w < T; w++)
            th.emplace_back([&, w] {
                try {
                    std::vector<double> u(per);
                    for (size_t q; (q = next.fetch_add(64)) < q1;)
                        for (size_t e = q; e < std::min(q1, q + 64); e++) {
                            if (mt) {
                                const uint32_t* y = &wbuf[k][(e - q0) * per];
                                for (int i = 0; i < per; i++) u[i] = MTRandom::deviate(y[i]);
                                fn(e, u.data());
                            } else {
                                fn(e, &dbuf[k][(e - q0) * per]);
                            }
                        }
                } catch (std::exception& ex) {
                    errs[w] = ex.what();
                }
            });
        if (q1 < n) draw((int)(k ^ 1), q1);
        for (auto& t : th) t.join();
        for (auto& e : errs)
            if (!e.empty()) throw std::runtime_error(e);
    }
}
}  // namespace

// ============================================================ small numeric helpers (Fundamentals/NR.hpp)
namespace nr {

// NR::locate_basic_impl / locate / locate_clip / locate_fail (NR.hpp Array versions)
static int locateBasic(const std::vector<double>& xv, double x, int n) {
    int jl = -1, ju = n;
    while (ju - jl > 1) {
        int jm = (ju + jl) >> 1;
        if (x < xv[jm]) ju = jm;
        else jl = jm;
    }
    return jl;
}
static int locate(const std::vector<double>& xv, double x) {
    int n = (int)xv.size();
    if (x == xv[n - 1]) return n - 2;
    return locateBasic(xv, x, n);
}
static int locateClip(const std::vector<double>& xv, double x) {
    if (x < xv[0]) return 0;
    return locateBasic(xv, x, (int)xv.size() - 1);
}
static int locateFail(const std::vector<double>& xv, double x) {
    int n = (int)xv.size();
    if (x > xv[n - 1]) return -1;
    return locateBasic(xv, x, n - 1);
}
static double interpolateLinLin(double x, double x1, double x2, double f1, double f2) {
    return f1 + ((x - x1) / (x2 - x1)) * (f2 - f1);
}
static double interpolateLogLin(double x, double x1, double x2, double f1, double f2) {
    x = std::log10(x);
    x1 = std::log10(x1);
    x2 = std::log10(x2);
    return f1 + ((x - x1) / (x2 - x1)) * (f2 - f1);
}
static double interpolateLogLog(double x, double x1, double x2, double f1, double f2) {
    x = std::log10(x);
    x1 = std::log10(x1);
    x2 = std::log10(x2);
    bool logf = f1 > 0 && f2 > 0;
    if (logf) {
        f1 = std::log10(f1);
        f2 = std::log10(f2);
    }
    double fx = f1 + ((x - x1) / (x2 - x1)) * (f2 - f1);
    if (logf) fx = std::pow(10, fx);
    return fx;
}
// NR::resample (NR.hpp:355-378)
template <double interp(double, double, double, double, double)>
static std::vector<double> resample(const std::vector<double>& xres, const std::vector<double>& xori,
                                    const std::vector<double>& yori) {
    int Nori = (int)xori.size();
    double xmin = xori[0], xmax = xori[Nori - 1];
    std::vector<double> yres(xres.size(), 0.0);
    for (size_t l = 0; l < xres.size(); l++) {
        double x = xres[l];
        if (std::fabs(1.0 - x / xmin) < 1e-5) yres[l] = yori[0];
        else if (std::fabs(1.0 - x / xmax) < 1e-5) yres[l] = yori[Nori - 1];
        else if (x < xmin || x > xmax) yres[l] = 0.0;
        else {
            int k = locate(xori, x);
            yres[l] = interp(x, xori[k], xori[k + 1], yori[k], yori[k + 1]);
        }
    }
    return yres;
}
// NR::cdf with a source vector (NR.hpp:388-394)
static void cdf(std::vector<double>& Pv, const std::vector<double>& pv) {
    size_t n = pv.size();
    Pv.assign(n + 1, 0.0);
    for (size_t i = 0; i < n; i++) Pv[i + 1] = Pv[i] + pv[i];
    double norm = Pv[n];
    for (auto& v : Pv) v /= norm;
}
static double sum(const std::vector<double>& v) { return std::accumulate(v.begin(), v.end(), 0.); }

}  // namespace nr

// ============================================================ model member functions

double Geometry::density(double x, double y, double z) const {
    switch (kind) {
    case GeometryKind::Plummer: {
        double r = std::sqrt(x * x + y * y + z * z);  // Position::radius -> Vec::norm
        double s = r / c;
        return rho0 * std::pow(1.0 + s * s, -2.5);
    }
    case GeometryKind::Point:  // PointGeometry::density
        return (x * x + y * y + z * z) == 0 ? std::numeric_limits<double>::infinity() : 0.0;
    case GeometryKind::Sersic: {
        // SpheGeometry::density(Position) -> SersicGeometry::density(r) = rho0 S(r/reff)
        const double r = std::sqrt(x * x + y * y + z * z);
        const double s = r / reff;
        const int Ns = (int)sv.size();
        if (s <= sv[0]) return rho0 * Sv[0];
        if (s >= sv[Ns - 1]) return rho0 * Sv[Ns - 1];
        const int i = nr::locateClip(sv, s);
        return rho0 * nr::interpolateLogLog(s, sv[i], sv[i + 1], Sv[i], Sv[i + 1]);
    }
    case GeometryKind::ExpDisk: {
        // AxGeometry::density(Position) -> ExpDiskGeometry::density(R, z) (Position::cylradius)
        const double R = std::sqrt(x * x + y * y);
        const double absz = std::fabs(z);
        if (Rmax > 0.0 && R > Rmax) return 0.0;
        else if (zmax > 0.0 && absz > zmax) return 0.0;
        else if (R < Rmin) return 0.0;
        return rho0 * std::exp(-R / hR) * std::exp(-absz / hz);
    }
    }
    return 0;
}

double Geometry::SigmaR() const {
    if (kind != GeometryKind::ExpDisk) throw std::runtime_error("Geometry is not axisymmetric");
    if (Rmax > 0.0) return rho0 * hR * (std::exp(-Rmin / hR) - std::exp(-Rmax / hR));
    return rho0 * hR * std::exp(-Rmin / hR);
}
double Geometry::SigmaZ() const {
    if (kind != GeometryKind::ExpDisk) throw std::runtime_error("Geometry is not axisymmetric");
    if (Rmin > 0.0) return 0.0;
    if (zmax > 0.0) return -2.0 * rho0 * hz * std::expm1(-zmax / hz);
    return 2.0 * rho0 * hz;
}
static double lngamma(double a);
double Geometry::Sigmar() const {
    if (kind == GeometryKind::Plummer) return 0.5 / (M_PI * c * c);
    if (kind == GeometryKind::Sersic)
        return 1.0 / (reff * reff) * std::pow(b, 2.0 * n) / (2.0 * M_PI * std::exp(lngamma(2.0 * n + 1.0)));
    throw std::runtime_error("Geometry is not spherically symmetric");
}

double Geometry::sersicInverseMass(double M) const {
    const int Ns = (int)sv.size();
    if (M <= Mv[0]) return sv[0];
    if (M >= Mv[Ns - 1]) return sv[Ns - 1];
    const int i = nr::locateClip(Mv, M);
    return nr::interpolateLogLog(M, Mv[i], Mv[i + 1], sv[i], sv[i + 1]);
}

// SpecialFunctions::lngamma / gamma (SpecialFunctions.cpp:16-40)
static double lngamma(double a) {
    static const double cof[6] = {76.18009172947146, -86.50532032941677, 24.01409824083091, -1.231739572450155,
                                  0.1208650973866179e-2, -0.5395239384953e-5};
    double y, xx, tmp, ser;
    y = xx = a;
    tmp = xx + 5.5;
    tmp -= (xx + 0.5) * std::log(tmp);
    ser = 1.000000000190015;
    for (int j = 0; j < 6; j++) ser += cof[j] / ++y;
    return -tmp + std::log(2.5066282746310005 * ser / xx);
}

// SersicFunction::SersicFunction(n) (SersicFunction.cpp): S(s) by the Abel-type integral on a
// 10001-point trapezoid, M(s) by a 33-point trapezoid per table interval, normalized
static void buildSersicTables(Geometry& g) {
    const double n = g.n;
    if (n < 0.5 || n > 10.0) throw std::runtime_error("The Sersic parameter should be between 0.5 and 10");
    const double b = 2.0 * n - 1.0 / 3.0 + 4.0 / 405.0 / n + 46.0 / 25515.0 / (n * n) + 131.0 / 1148175.0 / (n * n * n);
    g.b = b;  // SersicGeometry::setupSelfBefore computes the same expression
    const double I0 =std::pow(b, 2.0 * n) / (M_PI * std::exp(lngamma(2.0 * n + 1)));
    const int Ns = 101;
    g.sv.assign(Ns, 0.0);
    g.Sv.assign(Ns, 0.0);
    g.Mv.assign(Ns, 0.0);
    const double logsmin = -6.0, logsmax = 4.0;
    const double dlogs = (logsmax - logsmin) / (Ns - 1.0);
    for (int i = 0; i < Ns; i++) {
        const double logs = logsmin + i * dlogs;
        const double s = std::pow(10.0, logs);
        g.sv[i] = s;
        const double alpha = b * std::pow(s, 1.0 / n);
        double sum = 0.0;
        const int Nu = 10000;
        const double tmax = 100.0;
        const double umax = std::sqrt((tmax + 1.0) * (tmax - 1.0));
        const double du = umax / Nu;
        for (int j = 0; j <= Nu; j++) {
            double weight = 1.0;
            if (j == 0 || j == Nu) weight = 0.5;
            const double u = j * du;
            const double u2 = u * u;
            double w;
            if (u > 1e-3) w = (std::pow(1.0 + u2, 2.0 * n) - 1.0) / u2;
            else w = 2.0 * n + n * (2.0 * n - 1.0) * u2 + 2.0 / 3.0 * n * (2.0 * n - 1.0) * (n - 1.0) * u2 * u2;
            const double integrandum = 2.0 * std::exp(-alpha * (1.0 + u2)) / std::sqrt(w);
            sum += weight * integrandum;
        }
        g.Sv[i] = I0 * std::pow(b, n) * std::pow(alpha, 1.0 - n) / M_PI * du * sum;
    }
    auto S = [&](double s) {  // SersicFunction::operator()
        if (s <= g.sv[0]) return g.Sv[0];
        if (s >= g.sv[Ns - 1]) return g.Sv[Ns - 1];
        const int i = nr::locateClip(g.sv, s);
        return nr::interpolateLogLog(s, g.sv[i], g.sv[i + 1], g.Sv[i], g.Sv[i + 1]);
    };
    for (int i = 1; i < Ns; i++) {
        double sum = 0.0;
        for (int j = 0; j <= 32; j++) {
            double weight = 1.0;
            if (j == 0 || j == 32) weight = 0.5;
            const double ds = (g.sv[i] - g.sv[i - 1]) / 32.0;
            const double s = g.sv[i - 1] + j * ds;
            sum += weight * S(s) * s * s * ds;
        }
        const double dM = 4.0 * M_PI * sum;
        g.Mv[i] = g.Mv[i - 1] + dM;
    }
    for (int i = 0; i < Ns; i++) g.Mv[i] /= g.Mv[Ns - 1];
}

double lambertW1(double z) {
    const double eps = 1.0e-12;
    const double em1 = 0.3678794411714423215955237701614608;
    static const double c[12] = {-1.0, 2.331643981597124203363536062168, -1.812187885639363490240191647568,
                                 1.936631114492359755363277457668, -2.353551201881614516821543561516,
                                 3.066858901050631912893148922704, -4.175335600258177138854984177460,
                                 5.858023729874774148815053846119, -8.401032217523977370984161688514,
                                 12.250753501314460424, -18.100697012472442755, 27.029044799010561650};
    if (z < -em1 || z > 0.0 || std::isinf(z) || std::isnan(z)) throw std::runtime_error("LambertW1: bad argument");
    if (z == 0.0) return -DBL_MAX;
    const double q = z + em1;
    const double r = -std::sqrt(q);
    const double t8 = c[8] + r * (c[9] + r * (c[10] + r * c[11]));
    const double t5 = c[5] + r * (c[6] + r * (c[7] + r * t8));
    const double t1 = c[1] + r * (c[2] + r * (c[3] + r * (c[4] + r * t5)));
    const double w0 = c[0] + r * t1;
    if (q < 3.0e-3) return w0;
    double w;
    if (z < -1e-6) {
        w = w0;
    } else {
        const double l1 = std::log(-z);
        const double l2 = std::log(-l1);
        w = l1 - l2 + l2 / l1;
    }
    for (int i = 0; i < 10; i++) {  // Halley iteration
        const double e = std::exp(w);
        double t = w * e - z;
        const double p = w + 1.0;
        t /= e * p - 0.5 * (p + 1.0) * t / p;
        w -= t;
        if (std::fabs(t) < eps * (1.0 + std::fabs(w))) return w;
    }
    throw std::runtime_error("LambertW1: no convergence");
}

double WavelengthGrid::lambdamin(int ell) const {
    return (ell == 0) ? lambda[0] : std::sqrt(lambda[ell - 1] * lambda[ell]);
}
double WavelengthGrid::lambdamax(int ell) const {
    int N = n();
    return (ell == N - 1) ? lambda[N - 1] : std::sqrt(lambda[ell] * lambda[ell + 1]);
}

void DustGrid::cellBox(int m, double b[6]) const {
    if (kind == GridKind::Voronoi) {
        for (int q = 0; q < 6; q++) b[q] = vor.bbox[6 * (size_t)m + q];
        return;
    }
    if (kind == GridKind::Cartesian) {
        const CartesianGrid& g = cart;
        int i = m / (g.Nz * g.Ny), j = (m / g.Nz) % g.Ny, k = m % g.Nz;  // CartesianDustGrid::box
        b[0] = g.xv[i]; b[1] = g.yv[j]; b[2] = g.zv[k];
        b[3] = g.xv[i + 1]; b[4] = g.yv[j + 1]; b[5] = g.zv[k + 1];
    } else {
        int l = tree.idv[m];
        for (int q = 0; q < 6; q++) b[q] = tree.box[6 * (size_t)l + q];
    }
}

void DustGrid::cellCenter(int m, double c[3]) const {
    if (kind == GridKind::Voronoi) {
        for (int q = 0; q < 3; q++) c[q] = vor.centroid[3 * (size_t)m + q];
        return;
    }
    double b[6];
    cellBox(m, b);
    for (int q = 0; q < 3; q++) c[q] = 0.5 * (b[q] + b[3 + q]);
}

double DustGrid::cellVolume(int m) const {
    if (kind == GridKind::Voronoi) return vor.volume[m];
    double b[6];
    cellBox(m, b);
    return (b[3] - b[0]) * (b[4] - b[1]) * (b[5] - b[2]);
}

int DustGrid::whichcell(double x, double y, double z) const {
    if (kind == GridKind::Voronoi) return vor.cellIndex(x, y, z);
    if (kind == GridKind::Cartesian) {
        int i = nr::locateFail(cart.xv, x), j = nr::locateFail(cart.yv, y), k = nr::locateFail(cart.zv, z);
        if (i < 0 || j < 0 || k < 0) return -1;
        return k + cart.Nz * j + cart.Nz * cart.Ny * i;
    }
    const double* b = &tree.box[0];
    if (!(x >= b[0] && x <= b[3] && y >= b[1] && y <= b[4] && z >= b[2] && z <= b[5])) return -1;
    int l = 0;
    while (tree.firstChild[l] >= 0) l = tree.child(l, x, y, z);
    return tree.cellnumber[l];
}

int Instrument::pixel(double x, double y, double z) const {
    double xpp = -sinphi * x + cosphi * y;
    double ypp = -cosphi * costheta * x - sinphi * costheta * y + sintheta * z;
    double xp = cospa * xpp - sinpa * ypp;
    double yp = sinpa * xpp + cospa * ypp;
    int i = static_cast<int>(std::floor((xp - xpmin) / xpsiz));
    int j = static_cast<int>(std::floor((yp - ypmin) / ypsiz));
    if (i < 0 || i >= Nx || j < 0 || j >= Ny) return -1;
    return i + Nx * j;
}

double Model::kapparho(int m, int ell) const {
    if (m < 0) return 0;
    double result = 0;
    int nc = ncomp();
    for (int h = 0; h < nc; h++) result += dust[h].mix.kext[ell] * rho[(size_t)m * nc + h];
    return result;
}

// ============================================================ data tables

namespace {

struct Table {
    long nrows = 0, ncols = 0;
    std::vector<double> v;
    double at(long r, long c) const { return v[r * ncols + c]; }
};

Table readTable(const std::string& datadir, const std::string& name) {
    std::string path = datadir + "/" + name;
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open resource table " + path);
    Table t;
    int64_t hdr[2];
    if (std::fread(hdr, sizeof(int64_t), 2, f) != 2) { std::fclose(f); throw std::runtime_error("bad table " + path); }
    t.nrows = hdr[0];
    t.ncols = hdr[1];
    t.v.resize(t.nrows * t.ncols);
    size_t got = std::fread(t.v.data(), sizeof(double), t.v.size(), f);
    std::fclose(f);
    if (got != t.v.size()) throw std::runtime_error("truncated table " + path);
    return t;
}

// ============================================================ parsing helpers

struct Ctx {
    Units units;
    std::string datadir;
    UniformSource* rng;
    DensitySampler* sampler = nullptr;  // device density sampling (null: host threads)
};

// The density sampling of n items on the sampler's device, when there is one and the setup stream is the
// Mersenne twister: item q gets the 3 * nsample words the sequential loop would draw for it, in item
// order; the items go in chunks, the next chunk's words drawn while the device samples the current one.
// box(q, b) fills item q's box, apply(q, out) takes its sums. False: no device sampling (nothing drawn).
template <class BoxFn, class ApplyFn>
bool deviceSampling(const Ctx& c, const std::vector<DustComp>& dust, size_t n, int nsample, int mode, BoxFn box,
                    ApplyFn apply) {
    MTRandom* mt = dynamic_cast<MTRandom*>(c.rng);
    if (!c.sampler || !mt || n == 0) return false;
    const size_t per = 3 * (size_t)nsample;
    const size_t chunk = std::max<size_t>(1, ((size_t)1 << 26) / per);  // 64 Mi words (256 MiB) per call
    const size_t nout = mode == kDensNode ? 6 : dust.size();
    std::vector<uint32_t> w[2];
    std::vector<double> boxes, out;
    auto draw = [&](int k, size_t q0) {
        w[k].resize((std::min(n, q0 + chunk) - q0) * per);
        mt->words(w[k].data(), w[k].size());
    };
    draw(0, 0);
    for (size_t q0 = 0, k = 0; q0 < n; q0 += chunk, k ^= 1) {
        const size_t q1 = std::min(n, q0 + chunk);
        std::thread next;
        if (q1 < n) next = std::thread(draw, (int)(k ^ 1), q1);
        try {
            boxes.resize(6 * (q1 - q0));
            for (size_t q = q0; q < q1; q++) box(q, &boxes[6 * (q - q0)]);
            out.resize(nout * (q1 - q0));
            c.sampler->sample(dust, boxes.data(), q1 - q0, w[k].data(), nsample, mode, out.data());
            for (size_t q = q0; q < q1; q++) apply(q, &out[nout * (q - q0)]);
        } catch (...) {
            if (next.joinable()) next.join();
            throw;
        }
        if (next.joinable()) next.join();
    }
    return true;
}

double attr(const Ctx& c, const XmlElement* e, const char* key, const char* qty, double def) {
    if (!e->has(key)) return def;
    return c.units.parse(e->get(key), qty);
}
int attrInt(const XmlElement* e, const char* key, int def) {
    if (!e->has(key)) return def;
    return (int)std::lround(std::strtod(e->get(key).c_str(), nullptr));
}
bool attrBool(const XmlElement* e, const char* key, bool def) {
    if (!e->has(key)) return def;
    std::string v = e->get(key);
    std::transform(v.begin(), v.end(), v.begin(), ::tolower);
    return v == "true" || v == "yes" || v == "1";
}
std::vector<double> attrList(const Ctx& c, const XmlElement* e, const char* key, const char* qty) {
    std::vector<double> out;
    std::string s = e->get(key);
    std::stringstream ss(s);
    std::string item;
    while (std::getline(ss, item, ',')) out.push_back(c.units.parse(item, qty));
    return out;
}
const XmlElement* need(const XmlElement* e, const char* prop) {
    const XmlElement* it = e->item(prop);
    if (!it) throw std::runtime_error(std::string("missing property '") + prop + "' in " + e->name);
    return it;
}

Geometry parseGeometry(const Ctx& c, const XmlElement* g) {
    Geometry geo;
    if (g->name == "PlummerGeometry") {
        geo.kind = GeometryKind::Plummer;
        geo.c = attr(c, g, "scale", "length", 0);
        if (geo.c <= 0) throw std::runtime_error("the scale length c should be positive");
        geo.rho0 = 0.75 / std::pow(geo.c, 3) / M_PI;
    } else if (g->name == "PointGeometry") {
        geo.kind = GeometryKind::Point;
    } else if (g->name == "SersicGeometry") {
        // SersicGeometry::setupSelfBefore
        geo.kind = GeometryKind::Sersic;
        geo.n = attr(c, g, "index", "", 0);
        geo.reff = attr(c, g, "radius", "length", 0);
        if (geo.n <= 0.5 || geo.n > 10) throw std::runtime_error("the Sersic index n should be between 0.5 and 10");
        if (geo.reff <= 0) throw std::runtime_error("the effective radius should be positive");
        geo.rho0 = 1.0 / (geo.reff * geo.reff * geo.reff);
        buildSersicTables(geo);
    } else if (g->name == "ExpDiskGeometry") {
        // ExpDiskGeometry::setupSelfBefore (ExpDiskGeometry.cpp): checks and the normalization rho0
        geo.kind = GeometryKind::ExpDisk;
        geo.hR = attr(c, g, "radialScale", "length", 0);
        geo.hz = attr(c, g, "axialScale", "length", 0);
        geo.Rmax = attr(c, g, "radialTrunc", "length", 0);
        geo.zmax = attr(c, g, "axialTrunc", "length", 0);
        geo.Rmin = attr(c, g, "innerRadius", "length", 0);
        if (geo.hR <= 0) throw std::runtime_error("The radial scale length hR should be positive");
        if (geo.hz <= 0) throw std::runtime_error("The axial scale height hz should be positive");
        if (geo.Rmax < 0) throw std::runtime_error("The radial truncation length Rmax should be zero or positive");
        if (geo.zmax < 0) throw std::runtime_error("The axial truncation length zmax should be zero or positive");
        if (geo.Rmin < 0) throw std::runtime_error("The minimum radius Rmax should be zero or positive");
        else if (geo.Rmin > geo.Rmax && geo.Rmax > 0)
            throw std::runtime_error("The minimum radius Rmin should be larger than the truncation radius Rmax");
        const double intphi = 2.0 * M_PI;
        const double intz = (geo.zmax > 0) ? -2.0 * geo.hz * std::expm1(-geo.zmax / geo.hz) : 2.0 * geo.hz;
        const double tmin = (geo.Rmin > 0) ? std::exp(-geo.Rmin / geo.hR) * (1.0 + geo.Rmin / geo.hR) : 1.0;
        const double tmax = (geo.Rmax > 0) ? std::exp(-geo.Rmax / geo.hR) * (1.0 + geo.Rmax / geo.hR) : 0.0;
        const double intR = geo.hR * geo.hR * (tmin - tmax);
        geo.rho0 = 1.0 / (intR * intphi * intz);
    } else {
        throw std::runtime_error("unsupported geometry " + g->name);
    }
    return geo;
}

// ------------------------------------------------------------ wavelength grids
WavelengthGrid parseWavelengthGrid(const Ctx& c, const XmlElement* w) {
    WavelengthGrid wl;
    if (w->name == "OligoWavelengthGrid") {
        wl.pan = false;
        wl.lambda = attrList(c, w, "wavelengths", "wavelength");
        std::sort(wl.lambda.begin(), wl.lambda.end());
        wl.dlambda.resize(wl.lambda.size());
        for (size_t ell = 0; ell < wl.lambda.size(); ell++) wl.dlambda[ell] = 0.001 * wl.lambda[ell];
    } else if (w->name == "LogWavelengthGrid") {
        wl.pan = true;
        double lmin = attr(c, w, "minWavelength", "wavelength", 0);
        double lmax = attr(c, w, "maxWavelength", "wavelength", 0);
        int N = attrInt(w, "points", 0);
        if (lmin <= 0 || lmax <= lmin || N < 3) throw std::runtime_error("invalid LogWavelengthGrid");
        // NR::loggrid(_lambdav, lmin, lmax, N-1)  (LogWavelengthGrid.cpp, NR.hpp:269-275)
        int n = N - 1;
        wl.lambda.resize(n + 1);
        double logxmin = std::log10(lmin);
        double dlogx = std::log10(lmax / lmin) / n;
        for (int i = 0; i <= n; i++) wl.lambda[i] = std::pow(10, logxmin + i * dlogx);
        wl.dlambda.resize(N);
        for (int ell = 0; ell < N; ell++) wl.dlambda[ell] = wl.lambdamax(ell) - wl.lambdamin(ell);
    } else {
        throw std::runtime_error("unsupported wavelength grid " + w->name);
    }
    for (int ell = 1; ell < wl.n(); ell++)
        if (wl.lambda[ell] <= wl.lambda[ell - 1]) throw std::runtime_error("wavelengths should be sorted");
    return wl;
}

// ------------------------------------------------------------ dust mixes
// DustMix::setupSelfAfter part 1 (DustMix.cpp:47-89): population sums, albedo, g, kappa = sigma/mu
void finishMix(DustMix& mix, const std::vector<double>& muv, const std::vector<std::vector<double>>& sabs,
               const std::vector<std::vector<double>>& ssca, const std::vector<std::vector<double>>& gv, int Nlambda) {
    int Npop = (int)muv.size();
    if (Npop < 1) throw std::runtime_error("dust mixture must contain at least one dust population");
    std::vector<double> sigmaabs(Nlambda), sigmasca(Nlambda), sigmaext(Nlambda);
    mix.albedo.assign(Nlambda, 0);
    mix.g.assign(Nlambda, 0);
    for (int ell = 0; ell < Nlambda; ell++) {
        double sumabs = 0.0, sumsca = 0.0, sumgsca = 0.0;
        for (int c = 0; c < Npop; c++) {
            sumabs += sabs[c][ell];
            sumsca += ssca[c][ell];
            sumgsca += gv[c][ell] * ssca[c][ell];
        }
        double sumext = sumabs + sumsca;
        sigmaabs[ell] = sumabs;
        sigmasca[ell] = sumsca;
        sigmaext[ell] = sumext;
        mix.albedo[ell] = sumext ? sumsca / sumext : 0.;
        mix.g[ell] = sumsca ? sumgsca / sumsca : 0.;
    }
    double mu = 0.0;
    for (int c = 0; c < Npop; c++) mu += muv[c];
    mix.mu = mu;
    mix.sigmaabs = sigmaabs;
    mix.kabs.resize(Nlambda);
    mix.ksca.resize(Nlambda);
    mix.kext.resize(Nlambda);
    for (int ell = 0; ell < Nlambda; ell++) {
        mix.kabs[ell] = sigmaabs[ell] / mu;
        mix.ksca[ell] = sigmasca[ell] / mu;
        mix.kext[ell] = sigmaext[ell] / mu;
    }
}

DustMix parseMix(const Ctx& c, const XmlElement* e, const WavelengthGrid& wl) {
    DustMix mix;
    mix.type = e->name;
    int Nlambda = wl.n();
    std::vector<double> muv;
    std::vector<std::vector<double>> sabs, ssca, gv;
    if (e->name == "SimpleOligoDustMix") {
        // SimpleOligoDustMix.cpp setupSelfBefore: kappaabs = kext*(albedo+1), kappasca = kext*albedo,
        // population mass 1/kext[0] (the reference's quirk is kept on purpose)
        if (wl.pan) throw std::runtime_error("SimpleOligoDustMix requires an oligochromatic wavelength grid");
        std::vector<double> kext = attrList(c, e, "opacities", "opacity");
        std::vector<double> alb = attrList(c, e, "albedos", "");
        std::vector<double> asy = attrList(c, e, "asymmetryParameters", "");
        if ((int)kext.size() != Nlambda || (int)alb.size() != Nlambda || (int)asy.size() != Nlambda)
            throw std::runtime_error("SimpleOligoDustMix property list length differs from the number of wavelengths");
        std::vector<double> ka(Nlambda), ks(Nlambda), g(Nlambda);
        for (int ell = 0; ell < Nlambda; ell++) {
            ka[ell] = kext[ell] * (alb[ell] + 1.0);
            ks[ell] = kext[ell] * alb[ell];
            g[ell] = asy[ell];
        }
        double Mdust = 1.0 / kext[0];
        if (Mdust > 0) { muv.push_back(Mdust); sabs.push_back(ka); ssca.push_back(ks); gv.push_back(g); }
    } else if (e->name == "InterstellarDustMix") {
        // InterstellarDustMix.cpp setupSelfBefore + DustMix::addpopulation with resampling
        Table t = readTable(c.datadir, "InterstellarDustMix.bin");
        const int N = 1064;
        if (t.nrows != N || t.ncols != 6) throw std::runtime_error("unexpected InterstellarDustMix table shape");
        std::vector<double> lambdav(N), kabsv(N), kscav(N), gvv(N);
        for (int row = 0, k = N - 1; k >= 0; k--, row++) {
            double lambda = t.at(row, 0), albedo = t.at(row, 1), asymmpar = t.at(row, 2), Kabs = t.at(row, 4);
            lambda *= 1e-6;
            Kabs *= 1e-1;
            lambdav[k] = lambda;
            kabsv[k] = Kabs;
            kscav[k] = Kabs * albedo / (1.0 - albedo);
            gvv[k] = asymmpar;
        }
        double eps = 0.5e-5;
        if (wl.lambda[0] < lambdav[0] * (1 - eps) || wl.lambda[Nlambda - 1] > lambdav[N - 1] * (1 + eps))
            throw std::runtime_error("dust properties not defined over the simulation's wavelength range");
        muv.push_back(1.);
        sabs.push_back(nr::resample<nr::interpolateLogLog>(wl.lambda, lambdav, kabsv));
        ssca.push_back(nr::resample<nr::interpolateLogLog>(wl.lambda, lambdav, kscav));
        gv.push_back(nr::resample<nr::interpolateLogLin>(wl.lambda, lambdav, gvv));
    } else if (e->name == "MeanZubkoDustMix" || e->name == "DraineLiDustMix") {
        // MeanZubkoDustMix.cpp / DraineLiDustMix.cpp setupSelfBefore: cross sections per H atom, then
        // DustMix::addpopulation(mu, ...) (DustMix.cpp:300-321) with its wavelength check and resampling
        const bool zubko = e->name == "MeanZubkoDustMix";
        Table t = readTable(c.datadir, zubko ? "MeanZubkoDustMix.bin" : "DraineLiDustMix.bin");
        const int N = zubko ? 1201 : 800;
        if (t.nrows != N || t.ncols != 6) throw std::runtime_error("unexpected " + e->name + " table shape");
        std::vector<double> lambdav(N), sabsv(N), sscav(N), gvv(N);
        for (int k = 0; k < N; k++) {
            lambdav[k] = t.at(k, 0) * 1e-6;
            if (zubko) {
                const double sigmaext = t.at(k, 3) * 1e-4;
                const double albedo = t.at(k, 4);
                sabsv[k] = (1. - albedo) * sigmaext;
                sscav[k] = albedo * sigmaext;
            } else {
                sabsv[k] = t.at(k, 1) * 1e-4;
                sscav[k] = t.at(k, 2) * 1e-4;
            }
            gvv[k] = t.at(k, 5);
        }
        double eps = 0.5e-5;
        if (wl.lambda[0] < lambdav[0] * (1 - eps) || wl.lambda[Nlambda - 1] > lambdav[N - 1] * (1 + eps))
            throw std::runtime_error("dust properties not defined over the simulation's wavelength range");
        const double MdustoverMH = 5.4e-4 + 5.4e-4 + 1.8e-4 + 2.33e-3 + 8.27e-3;
        muv.push_back(zubko ? 1.44e-29 : MdustoverMH * constants::mproton);
        sabs.push_back(nr::resample<nr::interpolateLogLog>(wl.lambda, lambdav, sabsv));
        ssca.push_back(nr::resample<nr::interpolateLogLog>(wl.lambda, lambdav, sscav));
        gv.push_back(nr::resample<nr::interpolateLogLin>(wl.lambda, lambdav, gvv));
    } else {
        throw std::runtime_error("unsupported dust mix " + e->name);
    }
    finishMix(mix, muv, sabs, ssca, gv, Nlambda);
    return mix;
}

// DustMix::kappaext(lambda) (DustMix.cpp:482-522): log-log interpolation on a panchromatic grid, the
// matching wavelength (to 1e-5) of an oligochromatic one
double mixKappaext(const DustMix& mix, const WavelengthGrid& wl, double lambda) {
    if (wl.pan) {
        const int ell = nr::locateFail(wl.lambda, lambda);
        if (ell < 0) throw std::runtime_error("Optical properties are not defined for this wavelength");
        const double p = (std::log10(lambda) - std::log10(wl.lambda[ell])) /
                         (std::log10(wl.lambda[ell + 1]) - std::log10(wl.lambda[ell]));
        const double kL = mix.kext[ell], kR = mix.kext[ell + 1];
        if (kL > 0 && kR > 0) {
            const double lL = std::log10(kL), lR = std::log10(kR);
            return std::pow(10, lL + p * (lR - lL));
        }
        return kL + p * (kR - kL);
    }
    for (int ell = 0; ell < wl.n(); ell++)
        if (std::fabs(lambda / wl.lambda[ell] - 1.0) < 1e-5) return mix.kext[ell];
    throw std::runtime_error("Optical properties are not defined for this wavelength");
}

// ------------------------------------------------------------ stellar components
std::vector<double> sunLuminosityOligo(const Ctx& c, const WavelengthGrid& wl, const std::vector<double>& lum) {
    // OligoStellarComp.cpp setupSelfBefore
    Table t = readTable(c.datadir, "SunSED.bin");
    int Ns = (int)t.nrows;
    std::vector<double> lsun(Ns), Lsun(Ns);
    for (int k = 0; k < Ns; k++) {
        lsun[k] = t.at(k, 0) / 1e6;
        Lsun[k] = t.at(k, 1) * 1e6;
    }
    std::vector<double> Lv(wl.n());
    for (int ell = 0; ell < wl.n(); ell++) {
        double lambda = wl.lambda[ell];
        int k = nr::locateFail(lsun, lambda);
        if (k < 0) throw std::runtime_error("the sun does not emit at the wavelength of the simulation");
        double L = nr::interpolateLinLin(lambda, lsun[k], lsun[k + 1], Lsun[k], Lsun[k + 1]);
        Lv[ell] = lum[ell] * L * wl.dlambda[ell];
    }
    return Lv;
}

std::vector<double> sunSedNormalized(const Ctx& c, const WavelengthGrid& wl) {
    // SunSED.cpp setupSelfBefore -> SED::setemissivities (SED.cpp) -> setluminosities
    Table t = readTable(c.datadir, "SunSED.bin");
    int Ns = (int)t.nrows;
    std::vector<double> lv(Ns), jv(Ns);
    for (int k = 0; k < Ns; k++) {
        lv[k] = t.at(k, 0) / 1e6;
        jv[k] = t.at(k, 1);
    }
    std::vector<double> j = nr::resample<nr::interpolateLogLog>(wl.lambda, lv, jv);
    std::vector<double> Lv(wl.n());
    for (int ell = 0; ell < wl.n(); ell++) Lv[ell] = j[ell] * wl.dlambda[ell];
    double s = nr::sum(Lv);
    if (s <= 0) throw std::runtime_error("the total luminosity in the SED is zero or negative");
    for (auto& v : Lv) v /= s;
    return Lv;
}

// SED::setluminosities (SED.cpp): normalized to unit sum
static std::vector<double> normalizedSed(std::vector<double> Lv) {
    const double s = nr::sum(Lv);
    if (s <= 0) throw std::runtime_error("the total luminosity in the SED is zero or negative");
    for (auto& v : Lv) v /= s;
    return Lv;
}

std::vector<double> blackBodySedNormalized(double T, const WavelengthGrid& wl) {
    // BlackBodySED.cpp setupSelfBefore: per wavelength bin, the 101-point trapezoid rule of B(lambda)
    // lambda over log10(lambda) between lambdamin and lambdamax, times ln 10 dloglambda
    if (T <= 0) throw std::runtime_error("the black body temperature T should be positive");
    std::vector<double> Lv(wl.n());
    for (int ell = 0; ell < wl.n(); ell++) {
        const int N = 100;
        const double loglambdamin = std::log10(wl.lambdamin(ell));
        const double loglambdamax = std::log10(wl.lambdamax(ell));
        const double dloglambda = (loglambdamax - loglambdamin) / N;
        double sum = 0;
        for (int i = 0; i <= N; i++) {
            double weight = 1.0;
            if (i == 0 || i == N) weight = 0.5;
            const double loglambda = loglambdamin + i * dloglambda;
            const double lambda = std::pow(10, loglambda);
            sum += weight * planckFunction(T, lambda) * lambda;
        }
        Lv[ell] = sum * M_LN10 * dloglambda;
    }
    return normalizedSed(Lv);
}

std::vector<double> quasarSedNormalized(const WavelengthGrid& wl) {
    // QuasarSED.cpp setupSelfBefore: a broken power law in micron, then SED::setemissivities
    std::vector<double> Lv(wl.n());
    for (int ell = 0; ell < wl.n(); ell++) {
        double lambda = wl.lambda[ell];
        lambda *= 1e6;
        double j = 0.0;
        const double a = 1.0, b = 0.003981072, cq = 0.001258926, d = 0.070376103;
        if (lambda < 0.001) j = 0.0;
        else if (lambda < 0.01) j = a * std::pow(lambda, 0.2);
        else if (lambda < 0.1) j = b * std::pow(lambda, -1.0);
        else if (lambda < 5.0) j = cq * std::pow(lambda, -1.5);
        else if (lambda < 1000.0) j = d * std::pow(lambda, -4.0);
        else j = 0.0;
        Lv[ell] = j * wl.dlambda[ell];
    }
    return normalizedSed(Lv);
}

// ------------------------------------------------------------ octree
// TreeDustGrid::setupSelfBefore / subdivide (TreeDustGrid.cpp:50-233), OctTreeNode (OctTreeNode.cpp),
// TreeNode neighbor bookkeeping (TreeNode.cpp). Nodes are kept as indices into flat arrays; the
// neighbor lists are std::vector<int> per (node, wall) mutated in exactly the reference's order so that
// sortneighbors() (std::sort, not stable) sees identical input sequences.
enum Wall { BACK = 0, FRONT, LEFT, RIGHT, BOTTOM, TOP };

struct TreeBuilder {
    OctreeGrid& t;
    std::vector<std::vector<int>> nb;  // 6 per node, created lazily (ensureneighborlists)
    std::vector<char> hasLists;

    explicit TreeBuilder(OctreeGrid& tree) : t(tree) {}

    double* box(int l) { return &t.box[6 * (size_t)l]; }

    int addNode(int father, double x0, double y0, double z0, double x1, double y1, double z1) {
        int id = (int)t.firstChild.size();
        t.box.insert(t.box.end(), {x0, y0, z0, x1, y1, z1});
        t.firstChild.push_back(-1);
        t.father.push_back(father);
        t.level.push_back(father >= 0 ? t.level[father] + 1 : 0);
        if (t.binary) t.dir.push_back(-1);
        return id;
    }

    // OctTreeNode::createchildren_splitpoint (OctTreeNode.cpp:38-49): the box centre for
    // OctTreeNode::createchildren, the sampled barycentre for BaryOctTreeNode::createchildren
    void createChildren(int l, double rx, double ry, double rz) {
        double b[6];
        std::memcpy(b, box(l), sizeof b);
        int first = (int)t.firstChild.size();
        t.firstChild[l] = first;
        addNode(l, b[0], b[1], b[2], rx, ry, rz);
        addNode(l, rx, b[1], b[2], b[3], ry, rz);
        addNode(l, b[0], ry, b[2], rx, b[4], rz);
        addNode(l, rx, ry, b[2], b[3], b[4], rz);
        addNode(l, b[0], b[1], rz, rx, ry, b[5]);
        addNode(l, rx, b[1], rz, b[3], ry, b[5]);
        addNode(l, b[0], ry, rz, rx, b[4], b[5]);
        addNode(l, rx, ry, rz, b[3], b[4], b[5]);
    }

    // BinTreeNode::createchildren_splitdir (BinTreeNode.cpp:38-66): halves along one axis, child 0 below
    void createChildrenBin(int l, int d) {
        double b[6];
        std::memcpy(b, box(l), sizeof b);
        t.firstChild[l] = (int)t.firstChild.size();
        t.dir[l] = (signed char)d;
        double hi[6], lo[6];
        std::memcpy(lo, b, sizeof b);
        std::memcpy(hi, b, sizeof b);
        const double c = 0.5 * (b[d] + b[3 + d]);
        lo[3 + d] = c;
        hi[d] = c;
        addNode(l, lo[0], lo[1], lo[2], lo[3], lo[4], lo[5]);
        addNode(l, hi[0], hi[1], hi[2], hi[3], hi[4], hi[5]);
    }

    void ensure(int l) {
        if ((size_t)l >= hasLists.size()) { hasLists.resize(t.firstChild.size(), 0); nb.resize(6 * t.firstChild.size()); }
        hasLists[l] = 1;
    }
    std::vector<int>& lst(int l, int wall) { return nb[6 * (size_t)l + wall]; }
    void makeneighbors(int wall1, int n1, int n2) {
        static const int complementing[] = {FRONT, BACK, RIGHT, LEFT, TOP, BOTTOM};
        lst(n1, wall1).push_back(n2);
        lst(n2, complementing[wall1]).push_back(n1);
    }
    void deleteneighbor(int l, int wall, int node) {
        auto& v = lst(l, wall);
        for (size_t i = 0; i < v.size(); i++)
            if (v[i] == node) { v.erase(v.begin() + i); break; }
    }

    // OctTreeNode::addneighbors (OctTreeNode.cpp:51-182)
    void addneighbors(int l) {
        if (t.firstChild[l] < 0) return;
        int c0 = t.firstChild[l];
        int C[8];
        for (int k = 0; k < 8; k++) C[k] = c0 + k;
        ensure(l);
        for (int k = 0; k < 8; k++) ensure(C[k]);
        makeneighbors(FRONT, C[0], C[1]);
        makeneighbors(RIGHT, C[0], C[2]);
        makeneighbors(TOP, C[0], C[4]);
        makeneighbors(RIGHT, C[1], C[3]);
        makeneighbors(TOP, C[1], C[5]);
        makeneighbors(FRONT, C[2], C[3]);
        makeneighbors(TOP, C[2], C[6]);
        makeneighbors(TOP, C[3], C[7]);
        makeneighbors(FRONT, C[4], C[5]);
        makeneighbors(RIGHT, C[4], C[6]);
        makeneighbors(RIGHT, C[5], C[7]);
        makeneighbors(FRONT, C[6], C[7]);
        const double* cb = box(C[0]);
        double xc = cb[3], yc = cb[4], zc = cb[5];
        auto X0 = [&](int n) { return box(n)[0]; };
        auto Y0 = [&](int n) { return box(n)[1]; };
        auto Z0 = [&](int n) { return box(n)[2]; };
        auto X1 = [&](int n) { return box(n)[3]; };
        auto Y1 = [&](int n) { return box(n)[4]; };
        auto Z1 = [&](int n) { return box(n)[5]; };
        {
            std::vector<int> ns = lst(l, BACK);
            for (int n : ns) {
                deleteneighbor(n, FRONT, l);
                if (Y0(n) <= yc && Z0(n) <= zc) makeneighbors(FRONT, n, C[0]);
                if (Y1(n) >= yc && Z0(n) <= zc) makeneighbors(FRONT, n, C[2]);
                if (Y0(n) <= yc && Z1(n) >= zc) makeneighbors(FRONT, n, C[4]);
                if (Y1(n) >= yc && Z1(n) >= zc) makeneighbors(FRONT, n, C[6]);
            }
        }
        {
            std::vector<int> ns = lst(l, FRONT);
            for (int n : ns) {
                deleteneighbor(n, BACK, l);
                if (Y0(n) <= yc && Z0(n) <= zc) makeneighbors(BACK, n, C[1]);
                if (Y1(n) >= yc && Z0(n) <= zc) makeneighbors(BACK, n, C[3]);
                if (Y0(n) <= yc && Z1(n) >= zc) makeneighbors(BACK, n, C[5]);
                if (Y1(n) >= yc && Z1(n) >= zc) makeneighbors(BACK, n, C[7]);
            }
        }
        {
            std::vector<int> ns = lst(l, LEFT);
            for (int n : ns) {
                deleteneighbor(n, RIGHT, l);
                if (X0(n) <= xc && Z0(n) <= zc) makeneighbors(RIGHT, n, C[0]);
                if (X1(n) >= xc && Z0(n) <= zc) makeneighbors(RIGHT, n, C[1]);
                if (X0(n) <= xc && Z1(n) >= zc) makeneighbors(RIGHT, n, C[4]);
                if (X1(n) >= xc && Z1(n) >= zc) makeneighbors(RIGHT, n, C[5]);
            }
        }
        {
            std::vector<int> ns = lst(l, RIGHT);
            for (int n : ns) {
                deleteneighbor(n, LEFT, l);
                if (X0(n) <= xc && Z0(n) <= zc) makeneighbors(LEFT, n, C[2]);
                if (X1(n) >= xc && Z0(n) <= zc) makeneighbors(LEFT, n, C[3]);
                if (X0(n) <= xc && Z1(n) >= zc) makeneighbors(LEFT, n, C[6]);
                if (X1(n) >= xc && Z1(n) >= zc) makeneighbors(LEFT, n, C[7]);
            }
        }
        {
            std::vector<int> ns = lst(l, BOTTOM);
            for (int n : ns) {
                deleteneighbor(n, TOP, l);
                if (X0(n) <= xc && Y0(n) <= yc) makeneighbors(TOP, n, C[0]);
                if (X1(n) >= xc && Y0(n) <= yc) makeneighbors(TOP, n, C[1]);
                if (X0(n) <= xc && Y1(n) >= yc) makeneighbors(TOP, n, C[2]);
                if (X1(n) >= xc && Y1(n) >= yc) makeneighbors(TOP, n, C[3]);
            }
        }
        {
            std::vector<int> ns = lst(l, TOP);
            for (int n : ns) {
                deleteneighbor(n, BOTTOM, l);
                if (X0(n) <= xc && Y0(n) <= yc) makeneighbors(BOTTOM, n, C[4]);
                if (X1(n) >= xc && Y0(n) <= yc) makeneighbors(BOTTOM, n, C[5]);
                if (X0(n) <= xc && Y1(n) >= yc) makeneighbors(BOTTOM, n, C[6]);
                if (X1(n) >= xc && Y1(n) >= yc) makeneighbors(BOTTOM, n, C[7]);
            }
        }
    }

    // BinTreeNode::addneighbors (BinTreeNode.cpp:80-318): the two children become each other's neighbours
    // across the split wall; every neighbour of the node across the two walls perpendicular to the split
    // axis takes the child on its side, every other neighbour each child its extent along the axis
    // reaches. Walls visited in the reference's order BACK FRONT LEFT RIGHT BOTTOM TOP.
    void addneighborsBin(int l) {
        if (t.firstChild[l] < 0) return;
        static const int complementing[] = {FRONT, BACK, RIGHT, LEFT, TOP, BOTTOM};
        const int C0 = t.firstChild[l], C1 = C0 + 1, d = t.dir[l];
        const int lowWall = 2 * d, highWall = 2 * d + 1;
        ensure(l);
        ensure(C0);
        ensure(C1);
        const double c = box(C0)[3 + d];
        makeneighbors(highWall, C0, C1);
        for (int wall = BACK; wall <= TOP; wall++) {
            const int opp = complementing[wall];
            std::vector<int> ns = lst(l, wall);
            for (int n : ns) {
                deleteneighbor(n, opp, l);
                if (wall == lowWall) makeneighbors(opp, n, C0);
                else if (wall == highWall) makeneighbors(opp, n, C1);
                else {
                    if (box(n)[d] <= c) makeneighbors(opp, n, C0);
                    if (box(n)[3 + d] >= c) makeneighbors(opp, n, C1);
                }
            }
        }
    }

    // TreeNode::sortneighbors with the LargerOverlap functor (TreeNode.cpp:98-140)
    void sortneighbors(int l) {
        if (!hasLists[l]) return;
        const double* b = box(l);
        for (int wall = 0; wall < 6; wall++) {
            auto overlap = [&](int n) {
                const double* o = box(n);
                double a1, a2, b1, b2, c1, c2, d1, d2;  // rect (a1,b1)-(a2,b2) vs (c1,d1)-(c2,d2)
                switch (wall) {
                case BACK: case FRONT:
                    a1 = b[1]; b1 = b[2]; a2 = b[4]; b2 = b[5]; c1 = o[1]; d1 = o[2]; c2 = o[4]; d2 = o[5]; break;
                case LEFT: case RIGHT:
                    a1 = b[0]; b1 = b[2]; a2 = b[3]; b2 = b[5]; c1 = o[0]; d1 = o[2]; c2 = o[3]; d2 = o[5]; break;
                default:
                    a1 = b[0]; b1 = b[1]; a2 = b[3]; b2 = b[4]; c1 = o[0]; d1 = o[1]; c2 = o[3]; d2 = o[4]; break;
                }
                return std::max(std::min(a2, c2) - std::max(a1, c1), 0.) *
                       std::max(std::min(b2, d2) - std::max(b1, d1), 0.);
            };
            auto& v = lst(l, wall);
            std::sort(v.begin(), v.end(), [&](int n1, int n2) { return overlap(n1) > overlap(n2); });
        }
    }
};

// OctTreeDustGrid (binary = false) or BinTreeDustGrid (binary = true)
void buildOctree(const Ctx& c, const XmlElement* e, const Model& model, OctreeGrid& t, bool binary) {
    t.binary = binary;
    t.xmin = attr(c, e, "minX", "length", 0);
    t.xmax = attr(c, e, "maxX", "length", 0);
    t.ymin = attr(c, e, "minY", "length", 0);
    t.ymax = attr(c, e, "maxY", "length", 0);
    t.zmin = attr(c, e, "minZ", "length", 0);
    t.zmax = attr(c, e, "maxZ", "length", 0);
    if (t.xmax <= t.xmin || t.ymax <= t.ymin || t.zmax <= t.zmin) throw std::runtime_error("invalid grid extent");
    t.minLevel = attrInt(e, "minLevel", 2);
    t.maxLevel = attrInt(e, "maxLevel", 6);
    std::string search = e->get("searchMethod", "Neighbor");
    t.search = search == "TopDown" ? 0 : search == "Bookkeeping" ? 2 : 1;
    int Nrandom = attrInt(e, "sampleCount", 100);
    double maxOpticalDepth = attr(c, e, "maxOpticalDepth", "", 0);
    double maxMassFraction = attr(c, e, "maxMassFraction", "", 1e-6);
    double maxDensDispFraction = attr(c, e, "maxDensDispFraction", "", 0);
    // OctTreeDustGrid::barycentric (BaryOctTreeNode) / BinTreeDustGrid::directionMethod (BaryBinTreeNode)
    bool bary;
    if (binary) {
        const std::string method = e->get("directionMethod", "Alternating");
        if (method != "Alternating" && method != "Barycenter") throw std::runtime_error("unknown direction method " + method);
        bary = method == "Barycenter";
        if (t.search == 2) throw std::runtime_error("Bookkeeping method is not compatible with binary tree");  // BinTreeDustGrid.cpp:23-24
    } else {
        bary = attrBool(e, "barycentric", false);
    }
    if (t.minLevel < 0) throw std::runtime_error("The minimum tree level should be at least 0");
    if (t.maxLevel < 2) throw std::runtime_error("The maximum tree level should be at least 2");
    if (t.maxLevel <= t.minLevel) throw std::runtime_error("Maximum tree level should be larger than minimum tree level");
    if (Nrandom < 1) throw std::runtime_error("Number of random samples must be at least 1");

    double wx = t.xmax - t.xmin, wy = t.ymax - t.ymin, wz = t.zmax - t.zmin;
    t.eps = 1e-12 * std::sqrt(wx * wx + wy * wy + wz * wz);
    double totalmass = 0;
    for (auto& d : model.dust) totalmass += d.nf;  // CompDustDistribution::mass

    TreeBuilder tb(t);
    tb.addNode(-1, t.xmin, t.ymin, t.zmin, t.xmax, t.ymax, t.zmax);
    // TreeDustGrid::setupSelfBefore visits the nodes in creation order, subdividing as it goes. The nodes
    // that exist when a pass starts are decided together: the sampling ones draw their positions in
    // node order (parallelDraws), the subdivisions are then applied in node order, so that every node
    // number and every random draw is the reference's.
    const bool always = maxOpticalDepth == 0 && maxMassFraction == 0 && maxDensDispFraction == 0;
    std::unique_ptr<StageTimer> stage(new StageTimer("octree subdivision"));
    for (size_t l0 = 0; l0 < t.firstChild.size();) {
        const size_t l1 = t.firstChild.size();
        std::vector<int> sampled;  // nodes that sample the density, in node order
        for (size_t l = l0; l < l1; l++)
            if (t.level[l] > t.minLevel && t.level[l] < t.maxLevel) sampled.push_back((int)l);
        std::vector<char> divide(l1 - l0, 0);
        std::vector<std::array<double, 3>> bc(bary ? l1 - l0 : 0);  // sampled barycentres
        for (size_t l = l0; l < l1; l++) divide[l - l0] = t.level[l] <= t.minLevel;
        // the subdivision criteria of a sampled node from its mass, barycentre and density range
        auto decide = [&](int l, double sumrho, double sx, double sy, double sz, double mn, double mx) {
            const double* b = tb.box(l);
            if (bary) bc[l - l0] = {sx / sumrho, sy / sumrho, sz / sumrho};
            double vol = (b[3] - b[0]) * (b[4] - b[1]) * (b[5] - b[2]);
            double mass = sumrho / Nrandom * vol;
            bool needDivision = always;
            if (!needDivision && maxMassFraction > 0 && mass / totalmass >= maxMassFraction) needDivision = true;
            if (!needDivision && maxOpticalDepth > 0 &&
                constants::kappaV * mass / std::pow(vol, 2. / 3.) >= maxOpticalDepth)
                needDivision = true;
            if (!needDivision && maxDensDispFraction > 0) {
                double disp = mx > 0 ? (mx - mn) / mx : 0;
                if (disp >= maxDensDispFraction) needDivision = true;
            }
            divide[l - l0] = needDivision;
        };
        const bool onDevice = deviceSampling(
            c, model.dust, sampled.size(), Nrandom, kDensNode,
            [&](size_t q, double* b) { std::memcpy(b, tb.box(sampled[q]), 6 * sizeof(double)); },
            [&](size_t q, const double* o) { decide(sampled[q], o[0], o[1], o[2], o[3], o[4], o[5]); });
        if (!onDevice) parallelDraws(*c.rng, sampled.size(), 3 * Nrandom, [&](size_t q, const double* u) {
            // TreeNodeSampleDensityCalculator: Nrandom positions in the node, density of all components
            const int l = sampled[q];
            double b[6];
            std::memcpy(b, tb.box(l), sizeof b);
            std::vector<double> rhov(Nrandom);
            double sumrho = 0, sx = 0, sy = 0, sz = 0;  // TreeNodeSampleDensityCalculator::barycenter
            for (int n = 0; n < Nrandom; n++) {
                double fx = u[3 * n], fy = u[3 * n + 1], fz = u[3 * n + 2];
                double x = b[0] + fx * (b[3] - b[0]), y = b[1] + fy * (b[4] - b[1]), z = b[2] + fz * (b[5] - b[2]);
                double rho = 0;
                for (auto& d : model.dust) rho += d.density(x, y, z);
                rhov[n] = rho;
                sumrho += rho;
                sx += rho * x;
                sy += rho * y;
                sz += rho * z;
            }
            // sumrho is nr::sum(rhov): the same values accumulated in the same order
            decide(l, sumrho, sx, sy, sz, *std::min_element(rhov.begin(), rhov.end()),
                   *std::max_element(rhov.begin(), rhov.end()));
        });
        for (size_t l = l0; l < l1; l++) {
            if (!divide[l - l0]) continue;
            const double* b = tb.box((int)l);
            // at or below minLevel the node is split without a density calculator (TreeDustGrid.cpp:174-178)
            const bool useBary = bary && t.level[l] > t.minLevel;
            if (binary) {
                int d = t.level[l] % 3;  // BinTreeNode::createchildren: alternating x, y, z
                if (useBary) {
                    // BaryBinTreeNode::createchildren: the axis whose wall is nearest (relatively) to the
                    // barycentre; NaN distances (no mass sampled) fall through to z as in the reference
                    const auto& r = bc[l - l0];
                    double dx = std::min(r[0] - b[0], b[3] - r[0]) / (b[3] - b[0]);
                    double dy = std::min(r[1] - b[1], b[4] - r[1]) / (b[4] - b[1]);
                    double dz = std::min(r[2] - b[2], b[5] - r[2]) / (b[5] - b[2]);
                    if (dx < dy) d = dx < dz ? 0 : 2;
                    else d = dy < dz ? 1 : 2;
                }
                tb.createChildrenBin((int)l, d);
            } else if (useBary) {
                const auto& r = bc[l - l0];
                tb.createChildren((int)l, r[0], r[1], r[2]);
            } else {
                tb.createChildren((int)l, 0.5 * (b[0] + b[3]), 0.5 * (b[1] + b[4]), 0.5 * (b[2] + b[5]));
            }
        }
        l0 = l1;
    }
    stage.reset(new StageTimer("octree neighbours"));
    int Nnodes = t.nnodes();
    t.cellnumber.assign(Nnodes, -1);
    t.idv.clear();
    for (int l = 0; l < Nnodes; l++)
        if (t.firstChild[l] < 0) {
            t.cellnumber[l] = (int)t.idv.size();
            t.idv.push_back(l);
        }
    // neighbor lists, for the Neighbor search only, as the reference builds them (TreeDustGrid.cpp:158-163):
    // the TopDown and Bookkeeping walks (engine and oracle) never read them; empty lists otherwise
    tb.hasLists.assign(Nnodes, 0);
    tb.nb.assign(6 * (size_t)Nnodes, {});
    for (int l = 0; l < Nnodes && t.search == 1; l++) {
        if (binary) tb.addneighborsBin(l);
        else tb.addneighbors(l);
    }
    {
        // every node's lists sort on their own (TreeNode::sortneighbors): worker threads over node ranges
        stage.reset(new StageTimer("octree neighbour sort"));
        const int T = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
        std::atomic<int> next{0};
        std::vector<std::thread> th;
        for (int w = 0; w < T; w++)
            th.emplace_back([&] {
                for (int l0; (l0 = next.fetch_add(4096)) < Nnodes;)
                    for (int l = l0; l < std::min(Nnodes, l0 + 4096); l++) tb.sortneighbors(l);
            });
        for (auto& x : th) x.join();
    }
    stage.reset(new StageTimer("octree neighbour CSR"));
    t.nbrOffset.assign(6 * (size_t)Nnodes + 1, 0);
    size_t total = 0;
    for (size_t q = 0; q < 6 * (size_t)Nnodes; q++) total += tb.nb[q].size();
    t.nbrList.reserve(total);
    for (size_t q = 0; q < 6 * (size_t)Nnodes; q++) {
        t.nbrOffset[q] = (int)t.nbrList.size();
        t.nbrList.insert(t.nbrList.end(), tb.nb[q].begin(), tb.nb[q].end());
    }
    t.nbrOffset[6 * (size_t)Nnodes] = (int)t.nbrList.size();
}

// ------------------------------------------------------------ instruments
Instrument parseInstrument(const Ctx& c, const XmlElement* e) {
    Instrument ins;
    ins.name = e->get("instrumentName", "");
    if (e->name == "FullInstrument") ins.kind = InstrumentKind::Full;
    else if (e->name == "SimpleInstrument") ins.kind = InstrumentKind::Simple;
    else if (e->name == "SEDInstrument") ins.kind = InstrumentKind::SED;
    else if (e->name == "FrameInstrument") ins.kind = InstrumentKind::Frame;
    else throw std::runtime_error("unsupported instrument " + e->name);
    ins.distance = attr(c, e, "distance", "distance", 0);
    ins.inclination = attr(c, e, "inclination", "posangle", 0);
    ins.azimuth = attr(c, e, "azimuth", "posangle", 0);
    ins.positionAngle = attr(c, e, "positionAngle", "posangle", 0);
    if (ins.distance <= 0) throw std::runtime_error("instrument distance was not set");
    // DistantInstrument::setupSelfBefore (DistantInstrument.cpp:27-50)
    ins.costheta = std::cos(ins.inclination);
    ins.sintheta = std::sin(ins.inclination);
    ins.cosphi = std::cos(ins.azimuth);
    ins.sinphi = std::sin(ins.azimuth);
    ins.cospa = std::cos(ins.positionAngle);
    ins.sinpa = std::sin(ins.positionAngle);
    {
        // Direction(theta, phi) (Direction.cpp)
        double theta = ins.inclination, phi = ins.azimuth, eps = 1e-8;
        if (theta < -eps || theta > M_PI + eps) throw std::runtime_error("theta should be between 0 and pi");
        if (theta <= eps) { ins.kobs[0] = 0; ins.kobs[1] = 0; ins.kobs[2] = 1; }
        else if (theta >= M_PI - eps) { ins.kobs[0] = 0; ins.kobs[1] = 0; ins.kobs[2] = -1; }
        else {
            double st = std::sin(theta);
            ins.kobs[0] = st * std::cos(phi);
            ins.kobs[1] = st * std::sin(phi);
            ins.kobs[2] = std::cos(theta);
        }
    }
    ins.kx[0] = +ins.cosphi * ins.costheta * ins.sinpa - ins.sinphi * ins.cospa;
    ins.kx[1] = +ins.sinphi * ins.costheta * ins.sinpa + ins.cosphi * ins.cospa;
    ins.kx[2] = -ins.sintheta * ins.sinpa;
    ins.ky[0] = -ins.cosphi * ins.costheta * ins.cospa - ins.sinphi * ins.sinpa;
    ins.ky[1] = -ins.sinphi * ins.costheta * ins.cospa + ins.cosphi * ins.sinpa;
    ins.ky[2] = +ins.sintheta * ins.cospa;
    if (ins.kind != InstrumentKind::SED) {
        ins.fovx = attr(c, e, "fieldOfViewX", "length", 0);
        ins.fovy = attr(c, e, "fieldOfViewY", "length", 0);
        ins.Nx = attrInt(e, "pixelsX", 250);
        ins.Ny = attrInt(e, "pixelsY", 250);
        ins.xc = attr(c, e, "centerX", "length", 0);
        ins.yc = attr(c, e, "centerY", "length", 0);
        if (ins.Nx <= 0 || ins.Ny <= 0) throw std::runtime_error("number of pixels was not set");
        if (ins.fovx <= 0 || ins.fovy <= 0) throw std::runtime_error("field of view was not set");
        // SingleFrameInstrument::setupSelfBefore (SingleFrameInstrument.cpp:24-38)
        ins.xpmin = ins.xc - 0.5 * ins.fovx;
        ins.xpmax = ins.xc + 0.5 * ins.fovx;
        ins.xpsiz = ins.fovx / ins.Nx;
        ins.ypmin = ins.yc - 0.5 * ins.fovy;
        ins.ypmax = ins.yc + 0.5 * ins.fovy;
        ins.ypsiz = ins.fovy / ins.Ny;
    } else {
        ins.Nx = ins.Ny = 0;  // an SEDInstrument has no frame (SEDInstrument.cpp)
    }
    if (ins.kind == InstrumentKind::Full) ins.scatteringLevels = attrInt(e, "scatteringLevels", 0);
    return ins;
}

}  // namespace

// ============================================================ loadSki

// VoronoiDustGrid::setupSelfBefore (VoronoiDustGrid.cpp:28-138): the sites for the Uniform and
// DustDensity distributions, then the tessellation
static void buildVoronoiGrid(const Ctx& c, const XmlElement* ge, Model& m, UniformSource& rng) {
    const double xmin = attr(c, ge, "minX", "length", 0), xmax = attr(c, ge, "maxX", "length", 0);
    const double ymin = attr(c, ge, "minY", "length", 0), ymax = attr(c, ge, "maxY", "length", 0);
    const double zmin = attr(c, ge, "minZ", "length", 0), zmax = attr(c, ge, "maxZ", "length", 0);
    const int N = attrInt(ge, "numParticles", 0);
    if (N < 10) throw std::runtime_error("The number of particles should be at least 10");
    const std::string dist = ge->get("distribution", "DustDensity");
    auto contains = [&](double x, double y, double z) {  // Box::contains
        return x >= xmin && x <= xmax && y >= ymin && y <= ymax && z >= zmin && z <= zmax;
    };
    std::vector<double> sites(3 * (size_t)N);
    if (dist == "Uniform") {
        for (int q = 0; q < N; q++) {
            double fx = rng.uniform(), fy = rng.uniform(), fz = rng.uniform();  // Random::position(extent)
            sites[3 * q] = xmin + fx * (xmax - xmin);
            sites[3 * q + 1] = ymin + fy * (ymax - ymin);
            sites[3 * q + 2] = zmin + fz * (zmax - zmin);
        }
    } else if (dist == "DustDensity") {
        // CompDustDistribution::generatePosition: a component by mass (NR::locate_clip on the normalized
        // cumulative masses), then its geometry's generatePosition; points outside the domain are redrawn
        std::vector<double> masses, cum;
        for (const DustComp& d : m.dust) masses.push_back(d.nf);
        nr::cdf(cum, masses);
        for (int q = 0; q < N; q++) {
            while (true) {
                double X = rng.uniform();
                int h;
                if (X < cum[0]) h = 0;
                else h = nr::locateBasic(cum, X, (int)cum.size() - 1);
                const Geometry& geo = m.dust[h].geom;
                if (geo.kind != GeometryKind::Plummer) {
                    double x, y, z;
                    if (geo.kind == GeometryKind::ExpDisk) expDiskPosition(geo, rng, x, y, z);
                    else sersicPosition(geo, rng, x, y, z);
                    if (contains(x, y, z)) {
                        sites[3 * q] = x; sites[3 * q + 1] = y; sites[3 * q + 2] = z;
                        break;
                    }
                    continue;
                }
                // PlummerGeometry::randomradius, then SpheGeometry::generatePosition (Random::direction)
                double t = std::pow(rng.uniform(), 1.0 / 3.0);
                double r = geo.c * t / std::sqrt((1.0 - t) * (1.0 + t));
                double theta = std::acos(2.0 * rng.uniform() - 1.0);
                double phi = 2.0 * M_PI * rng.uniform();
                double kx, ky, kz;
                if (theta <= 1e-8) { kx = 0; ky = 0; kz = 1; }  // Direction(theta, phi), Direction.cpp
                else if (theta >= M_PI - 1e-8) { kx = 0; ky = 0; kz = -1; }
                else {
                    double st = std::sin(theta);
                    kx = st * std::cos(phi); ky = st * std::sin(phi); kz = std::cos(theta);
                }
                double x = r * kx, y = r * ky, z = r * kz;
                if (contains(x, y, z)) {
                    sites[3 * q] = x; sites[3 * q + 1] = y; sites[3 * q + 2] = z;
                    break;
                }
            }
        }
    } else {
        throw std::runtime_error("unsupported Voronoi particle distribution " + dist);
    }
    StageTimer st("tessellation");
    buildVoronoi(m.grid.vor, sites, xmin, xmax, ymin, ymax, zmin, zmax, c.sampler ? c.sampler->voronoiCells() : nullptr);
}

Model loadSki(const std::string& path, UniformSource& rng, const std::string& datadir, DensitySampler* sampler) {
    auto doc = parseXmlFile(path);
    if (doc->children.empty()) throw std::runtime_error("empty ski file");
    const XmlElement* sim = doc->children.front().get();
    Model m;
    if (sim->name == "OligoMonteCarloSimulation") m.pan = false;
    else if (sim->name == "PanMonteCarloSimulation") m.pan = true;
    else throw std::runtime_error("unsupported simulation type " + sim->name);

    const XmlElement* unitsEl = sim->item("units");
    m.units_system = unitsEl ? unitsEl->name : "ExtragalacticUnits";
    Ctx c{Units(m.units_system), datadir, &rng, sampler};

    if (const XmlElement* r = sim->item("random")) m.seed = (unsigned long)attrInt(r, "seed", 4357);
    m.packages = attr(c, sim, "packages", "", 1e6);
    m.minWeightReduction = attr(c, sim, "minWeightReduction", "", 1e4);
    m.minScattEvents = (int)attr(c, sim, "minScattEvents", "", 0);
    m.scattBias = attr(c, sim, "scattBias", "", 0.5);
    m.continuousScattering = attrBool(sim, "continuousScattering", false);
    if (m.packages < 0 || m.packages > 1e15) throw std::runtime_error("invalid number of photon packages");
    if (m.minWeightReduction < 1e3) throw std::runtime_error("the minimum weight reduction factor should be larger than 1000");
    if (m.scattBias < 0 || m.scattBias > 1) throw std::runtime_error("the scattering bias should be between 0 and 1");

    m.wl = parseWavelengthGrid(c, need(sim, "wavelengthGrid"));
    int Nlambda = m.wl.n();

    // ---- stellar system
    const XmlElement* ss = need(sim, "stellarSystem");
    m.starEmissionBias = attr(c, ss, "emissionBias", "", 0.5);
    for (const XmlElement* sc : ss->items("components")) {
        m.starGeom.push_back(parseGeometry(c, need(sc, "geometry")));
        if (sc->name == "OligoStellarComp") {
            if (m.pan) throw std::runtime_error("OligoStellarComp requires an oligochromatic simulation");
            std::vector<double> lum = attrList(c, sc, "luminosities", "");
            if ((int)lum.size() != Nlambda) throw std::runtime_error("number of luminosities differs from number of wavelengths");
            m.starL.push_back(sunLuminosityOligo(c, m.wl, lum));
        } else if (sc->name == "PanStellarComp") {
            const XmlElement* sed = need(sc, "sed");
            const XmlElement* norm = need(sc, "normalization");
            if (norm->name != "BolLuminosityStellarCompNormalization")
                throw std::runtime_error("unsupported stellar normalization " + norm->name);
            double Lsunits = attr(c, norm, "luminosity", "", 0);
            if (Lsunits <= 0) throw std::runtime_error("the bolometric luminosity should be positive");
            double Ltot = Lsunits * constants::Lsun;
            std::vector<double> sedL;
            if (sed->name == "SunSED") sedL = sunSedNormalized(c, m.wl);
            else if (sed->name == "BlackBodySED") sedL = blackBodySedNormalized(attr(c, sed, "temperature", "temperature", 0), m.wl);
            else if (sed->name == "QuasarSED") sedL = quasarSedNormalized(m.wl);
            else throw std::runtime_error("unsupported stellar SED " + sed->name);
            std::vector<double> Lv(Nlambda);
            for (int ell = 0; ell < Nlambda; ell++) Lv[ell] = Ltot * sedL[ell];
            m.starL.push_back(Lv);
        } else {
            throw std::runtime_error("unsupported stellar component " + sc->name);
        }
    }
    if (m.starL.empty()) throw std::runtime_error("there are no stellar components");
    {
        int Ncomp = (int)m.starL.size();
        m.starLtot.assign(Nlambda, 0.0);
        m.starX.assign(Nlambda, {});
        for (int ell = 0; ell < Nlambda; ell++) {
            for (int h = 0; h < Ncomp; h++) m.starLtot[ell] += m.starL[h][ell];
            std::vector<double> pv(Ncomp);
            for (int h = 0; h < Ncomp; h++) pv[h] = m.starL[h][ell];
            nr::cdf(m.starX[ell], pv);
        }
    }

    // ---- dust system
    const XmlElement* ds = sim->item("dustSystem");
    if (ds) {
        m.hasDust = true;
        bool pds = ds->name == "PanDustSystem";
        if (pds != m.pan) throw std::runtime_error("dust system type does not match the simulation type");
        m.sampleCount = attrInt(ds, "sampleCount", 100);
        m.writeConvergence = attrBool(ds, "writeConvergence", true);
        m.writeCellProperties = attrBool(ds, "writeCellProperties", false);
        m.writeCellsCrossed = attrBool(ds, "writeCellsCrossed", false);
        if (pds) {
            m.dustEmission = ds->item("dustEmissivity") != nullptr;
            m.selfAbsorption = m.dustEmission && attrBool(ds, "selfAbsorption", false);
            m.dustEmissionBias = attr(c, ds, "emissionBias", "", 0.5);
            m.emissionBoost = attr(c, ds, "emissionBoost", "", 1);
            m.cycles = attrInt(ds, "cycles", 0);
            m.writeISRF = attrBool(ds, "writeISRF", false);
            m.storeAbsorption = m.dustEmission;
        } else {
            m.writeMeanIntensity = attrBool(ds, "writeMeanIntensity", false);
            m.storeAbsorption = m.writeMeanIntensity;
        }
        const XmlElement* dd = need(ds, "dustDistribution");
        if (dd->name != "CompDustDistribution") throw std::runtime_error("unsupported dust distribution " + dd->name);
        for (const XmlElement* dc : dd->items("components")) {
            DustComp comp;
            comp.geom = parseGeometry(c, need(dc, "geometry"));
            if (comp.geom.kind == GeometryKind::Point)  // a delta density cannot be sampled on a dust grid
                throw std::runtime_error("PointGeometry is not supported for dust components");
            comp.mix = parseMix(c, need(dc, "mix"), m.wl);
            const XmlElement* nrm = need(dc, "normalization");
            if (nrm->name == "DustMassDustCompNormalization") {
                comp.nf = attr(c, nrm, "dustMass", "mass", 0);
            } else if (nrm->name == "FaceOnDustCompNormalization" || nrm->name == "EdgeOnDustCompNormalization" ||
                       nrm->name == "RadialDustCompNormalization") {
                // {FaceOn,EdgeOn,Radial}DustCompNormalization::normalizationFactor:
                // tau / (Sigma * kappaext(lambda)), Sigma = SigmaZ / SigmaR / Sigmar
                const double tau = attr(c, nrm, "opticalDepth", "", 0);
                const double lambda = attr(c, nrm, "wavelength", "wavelength", 0);
                const double Sigma = nrm->name[0] == 'F' ? comp.geom.SigmaZ()
                                     : nrm->name[0] == 'E' ? comp.geom.SigmaR() : comp.geom.Sigmar();
                comp.nf = tau / (Sigma * mixKappaext(comp.mix, m.wl, lambda));
            } else {
                throw std::runtime_error("unsupported dust normalization " + nrm->name);
            }
            m.dust.push_back(comp);
        }
        if (m.dust.empty()) throw std::runtime_error("dust distribution has no components");

        const XmlElement* ge = need(ds, "dustGrid");
        if (ge->name == "CartesianDustGrid") {
            m.grid.kind = GridKind::Cartesian;
            CartesianGrid& g = m.grid.cart;
            g.xmin = attr(c, ge, "minX", "length", 0);
            g.xmax = attr(c, ge, "maxX", "length", 0);
            g.ymin = attr(c, ge, "minY", "length", 0);
            g.ymax = attr(c, ge, "maxY", "length", 0);
            g.zmin = attr(c, ge, "minZ", "length", 0);
            g.zmax = attr(c, ge, "maxZ", "length", 0);
            if (g.xmax <= g.xmin || g.ymax <= g.ymin || g.zmax <= g.zmin) throw std::runtime_error("invalid grid extent");
            // the MoveableMesh of each axis on [0,1] (LinMesh.cpp, PowMesh.cpp, SymPowMesh.cpp; NR::lingrid,
            // NR::powgrid, NR::sympowgrid, Fundamentals/NR.hpp:171-261), then
            // _xv = mesh*(xmax-xmin) + xmin (CartesianDustGrid.cpp:34-36)
            auto mesh = [&](const char* prop, int& N, std::vector<double>& v, double lo, double hi) {
                const XmlElement* me = need(ge, prop);
                N = attrInt(me, "numBins", 100);
                if (N < 1) throw std::runtime_error("the number of mesh bins should be positive");
                std::vector<double> tv(N + 1);
                auto lingrid = [&](int n) {
                    const double dx = (1.0 - 0.0) / n;
                    for (int i = 0; i <= n; i++) tv[i] = 0.0 + i * dx;
                };
                if (me->name == "LinMesh") {
                    lingrid(N);
                } else if (me->name == "PowMesh" || me->name == "SymPowMesh") {
                    const double ratio = attr(c, me, "ratio", "", 1.0);
                    if (!(ratio > 0)) throw std::runtime_error("the bin width ratio should be positive");
                    const bool sym = me->name == "SymPowMesh";
                    if (sym ? N <= 2 : N <= 1) lingrid(N);
                    else if (std::fabs(ratio - 1.) < 1e-3) lingrid(N);
                    else if (!sym) {
                        const double range = 1.0 - 0.0;
                        const double q = std::pow(ratio, 1. / (N - 1));
                        const double qn = std::pow(q, N);
                        for (int i = 0; i <= N; ++i) tv[i] = 0.0 + (1. - std::pow(q, i)) / (1. - qn) * range;
                    } else {
                        const double xc = 0.5 * (0.0 + 1.0);
                        if (N % 2 == 0) {
                            const int M = N / 2;
                            const double q = std::pow(ratio, 1.0 / (M - 1.0));
                            const double qM = std::pow(q, M);
                            tv[M] = xc;
                            for (int i = 1; i <= M; ++i) {
                                const double dxi = (1.0 - std::pow(q, i)) / (1.0 - qM) * 0.5 * (1.0 - 0.0);
                                tv[M + i] = xc + dxi;
                                tv[M - i] = xc - dxi;
                            }
                        } else {
                            const int M = (N + 1) / 2;
                            const double q = std::pow(ratio, 1.0 / (M - 1.0));
                            const double qM = std::pow(q, M);
                            for (int i = 1; i <= M; ++i) {
                                const double dxi = (0.5 + 0.5 * q - std::pow(q, i)) / (0.5 + 0.5 * q - qM) * 0.5 * (1.0 - 0.0);
                                tv[M - 1 + i] = xc + dxi;
                                tv[M - i] = xc - dxi;
                            }
                        }
                    }
                } else {
                    throw std::runtime_error("unsupported mesh " + me->name);
                }
                v.resize(N + 1);
                for (int i = 0; i <= N; i++) v[i] = tv[i] * (hi - lo) + lo;
            };
            mesh("meshX", g.Nx, g.xv, g.xmin, g.xmax);
            mesh("meshY", g.Ny, g.yv, g.ymin, g.ymax);
            mesh("meshZ", g.Nz, g.zv, g.zmin, g.zmax);
            m.grid.ncells = g.Nx * g.Ny * g.Nz;
        } else if (ge->name == "OctTreeDustGrid" || ge->name == "BinTreeDustGrid") {
            m.grid.kind = GridKind::Octree;
            StageTimer st("octree");
            buildOctree(c, ge, m, m.grid.tree, ge->name == "BinTreeDustGrid");
            m.grid.ncells = (int)m.grid.tree.idv.size();
        } else if (ge->name == "VoronoiDustGrid") {
            m.grid.kind = GridKind::Voronoi;
            StageTimer st("voronoi");
            buildVoronoiGrid(c, ge, m, rng);
            m.grid.ncells = m.grid.vor.ncells();
        } else {
            throw std::runtime_error("unsupported dust grid " + ge->name);
        }

        // DustSystem::setupSelfAfter: volumes, then densities sampled at sampleCount random positions
        StageTimer st("cell densities");
        int Ncells = m.grid.ncells, Ncomp = m.ncomp();
        m.volume.resize(Ncells);
        for (int cell = 0; cell < Ncells; cell++) m.volume[cell] = m.grid.cellVolume(cell);
        m.rho.assign((size_t)Ncells * Ncomp, 0.0);
        if (m.grid.kind == GridKind::Voronoi) {
            // rejection sampling draws a data-dependent number of deviates, so the positions are drawn one
            // cell after the other (VoronoiMesh::randomPosition, the cell's neighbour sites gathered once);
            // their densities are then summed, in sample order, on worker threads, a chunk of cells at a time
            const VoronoiGrid& g = m.grid.vor;
            const int ns = m.sampleCount;
            MTRandom* mtr = dynamic_cast<MTRandom*>(&rng);  // a final class: its uniform() inlines
            auto uniform = [&]() { return mtr ? mtr->uniform() : rng.uniform(); };
            const int chunk = std::max(1, (1 << 22) / std::max(1, ns));
            std::vector<double> pos, nb;
            for (int c0 = 0; c0 < Ncells; c0 += chunk) {
                const int c1 = std::min(Ncells, c0 + chunk);
                pos.resize(3 * (size_t)(c1 - c0) * ns);
                std::unique_ptr<StageTimer> pst(new StageTimer("voronoi positions"));
                for (int cell = c0; cell < c1; cell++) {
                    nb.clear();
                    for (int q = g.nbrOffset[cell]; q < g.nbrOffset[cell + 1]; q++) {
                        const int id = g.nbrList[q];
                        if (id >= 0) nb.insert(nb.end(), &g.site[3 * (size_t)id], &g.site[3 * (size_t)id] + 3);
                    }
                    const double* b = &g.bbox[6 * (size_t)cell];
                    const double* sc = &g.site[3 * (size_t)cell];
                    const size_t nn = nb.size() / 3;
                    for (int n = 0; n < ns; n++) {
                        double x = 0, y = 0, z = 0;
                        bool in = false;
                        for (int t = 0; t < 10000 && !in; t++) {
                            // Random::position(box) then Box::fracpos; VoronoiMesh::isPointClosestTo (any
                            // closer neighbour rejects, so the order of the checks is free: the neighbour that
                            // rejected last is checked first)
                            const double fx = uniform();
                            const double fy = uniform();
                            const double fz = uniform();
                            x = b[0] + fx * (b[3] - b[0]);
                            y = b[1] + fy * (b[4] - b[1]);
                            z = b[2] + fz * (b[5] - b[2]);
                            const double tx = x - sc[0], ty = y - sc[1], tz = z - sc[2];
                            const double target = tx * tx + ty * ty + tz * tz;
                            in = true;
                            for (size_t q = 0; q < nn; q++) {
                                const double dx = x - nb[3 * q], dy = y - nb[3 * q + 1], dz = z - nb[3 * q + 2];
                                if (dx * dx + dy * dy + dz * dz < target) {
                                    in = false;
                                    if (q) for (int d = 0; d < 3; d++) std::swap(nb[3 * q + d], nb[d]);
                                    break;
                                }
                            }
                        }
                        if (!in) throw std::runtime_error("Can't find random position in cell");
                        double* o = &pos[3 * ((size_t)(cell - c0) * ns + n)];
                        o[0] = x; o[1] = y; o[2] = z;
                    }
                }
                pst.reset(new StageTimer("voronoi densities"));
                const int T = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
                std::atomic<int> next{c0};
                std::vector<std::thread> th;
                for (int w = 0; w < T; w++)
                    th.emplace_back([&] {
                        std::vector<double> sumv(Ncomp);
                        for (int q0; (q0 = next.fetch_add(256)) < c1;)
                            for (int cell = q0; cell < std::min(c1, q0 + 256); cell++) {
                                std::fill(sumv.begin(), sumv.end(), 0.0);
                                for (int n = 0; n < ns; n++) {
                                    const double* o = &pos[3 * ((size_t)(cell - c0) * ns + n)];
                                    for (int h = 0; h < Ncomp; h++) sumv[h] += m.dust[h].density(o[0], o[1], o[2]);
                                }
                                for (int h = 0; h < Ncomp; h++) m.rho[(size_t)cell * Ncomp + h] = 1.0 * sumv[h] / ns;
                            }
                    });
                for (auto& x : th) x.join();
            }
        } else {
            // Random::position(box) per sample: three deviates, drawn ahead in cell order
            const bool onDevice = deviceSampling(
                c, m.dust, (size_t)Ncells, m.sampleCount, kDensComponents,
                [&](size_t cell, double* b) { m.grid.cellBox((int)cell, b); },
                [&](size_t cell, const double* sumv) {
                    for (int h = 0; h < Ncomp; h++) m.rho[cell * Ncomp + h] = 1.0 * sumv[h] / m.sampleCount;
                });
            if (!onDevice) parallelDraws(rng, (size_t)Ncells, 3 * m.sampleCount, [&](size_t cell, const double* u) {
                double b[6];
                m.grid.cellBox((int)cell, b);
                std::vector<double> sumv(Ncomp, 0.0);
                for (int n = 0; n < m.sampleCount; n++) {
                    const double fx = u[3 * n], fy = u[3 * n + 1], fz = u[3 * n + 2];
                    const double x = b[0] + fx * (b[3] - b[0]), y = b[1] + fy * (b[4] - b[1]), z = b[2] + fz * (b[5] - b[2]);
                    for (int h = 0; h < Ncomp; h++) sumv[h] += m.dust[h].density(x, y, z);
                }
                for (int h = 0; h < Ncomp; h++) m.rho[cell * Ncomp + h] = 1.0 * sumv[h] / m.sampleCount;
            });
        }
    }

    // ---- instruments
    if (const XmlElement* is = sim->item("instrumentSystem"))
        for (const XmlElement* ie : is->items("instruments")) m.instruments.push_back(parseInstrument(c, ie));
    return m;
}

std::string defaultDataDir() {
    Dl_info info;
    if (dladdr((void*)&defaultDataDir, &info) && info.dli_fname) {
        std::string p(info.dli_fname);
        size_t s = p.rfind('/');
        std::string dir = (s == std::string::npos) ? "." : p.substr(0, s);
        // the library lives in skirt_amd/ (or skirt_amd/lib); data is skirt_amd/data
        for (const char* cand : {"/data", "/../data"}) {
            std::string d = dir + cand;
            std::ifstream f(d + "/SunSED.bin");
            if (f) return d;
        }
    }
    return "skirt_amd/data";
}

}  // namespace skirt
