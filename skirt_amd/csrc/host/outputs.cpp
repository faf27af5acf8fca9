#include "outputs.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <fstream>
#include <stdexcept>

#include "xml.hpp"

namespace skirt {

namespace {
// Qt rounds decimal ties away from zero (-101.5625 -> "-101.563" at 6 digits) where glibc's printf rounds
// them to even; resolve a tie from glibc's exact digit expansion before formatting.
double qtTieAdjust(double v, int sigdigits) {
    if (v == 0 || !std::isfinite(v) || sigdigits < 1) return v;
    char buf[128];
    std::snprintf(buf, sizeof buf, "%.60e", std::fabs(v));
    std::string s(buf);  // d.ddddd...e±XX
    std::string digits = s.substr(0, 1) + s.substr(2, s.find('e') - 2);
    if ((int)digits.size() <= sigdigits) return v;
    if (digits[sigdigits] != '5') return v;
    for (size_t i = sigdigits + 1; i < digits.size(); i++)
        if (digits[i] != '0') return v;
    // exact tie: nudge away from zero so that printf rounds up in magnitude
    return std::nextafter(v, v > 0 ? INFINITY : -INFINITY);
}
}  // namespace

std::string qtNumber(double v, char fmt, int prec) {
    if (fmt == 'f') {
        char buf[64];
        std::snprintf(buf, sizeof buf, "%.*f", prec, v);
        return buf;
    }
    char buf[64];
    if (fmt == 'e') std::snprintf(buf, sizeof buf, "%.*e", prec, qtTieAdjust(v, prec + 1));
    else std::snprintf(buf, sizeof buf, "%.*g", prec, qtTieAdjust(v, prec == 0 ? 1 : prec));
    // Qt writes the exponent without leading zeros ("5.5e-1", "0.00000000e+0")
    std::string s(buf);
    size_t e = s.find_first_of("eE");
    if (e != std::string::npos && e + 2 < s.size()) {
        std::string head = s.substr(0, e + 2);  // includes sign
        std::string digits = s.substr(e + 2);
        size_t nz = digits.find_first_not_of('0');
        digits = (nz == std::string::npos) ? "0" : digits.substr(nz);
        s = head + digits;
    }
    return s;
}

unsigned long readSkiSeed(const std::string& path) {
    auto doc = parseXmlFile(path);
    if (doc->children.empty()) return 4357;
    const XmlElement* r = doc->children.front()->item("random");
    if (!r || !r->has("seed")) return 4357;
    return (unsigned long)std::strtoul(r->get("seed").c_str(), nullptr, 10);
}

namespace {

class TextOut {
public:
    explicit TextOut(const std::string& path) : f_(path) {
        if (!f_) throw std::runtime_error("cannot create output file " + path);
    }
    void line(const std::string& s) { f_ << s << '\n'; }
    void column(const std::string& desc, char fmt = 'e', int prec = 6) {
        fmts_.push_back(fmt);
        precs_.push_back(prec);
        line("# column " + std::to_string(fmts_.size()) + ": " + desc);
    }
    void row(const std::vector<double>& v) {
        std::string s;
        for (size_t i = 0; i < v.size(); i++) {
            if (i) s += ' ';
            s += fmts_[i] == 'd' ? qtNumber(v[i], 'f', 0) : qtNumber(v[i], fmts_[i], precs_[i]);
        }
        line(s);
    }
private:
    std::ofstream f_;
    std::vector<char> fmts_;
    std::vector<int> precs_;
};

void fitsCard(std::string& hdr, const std::string& key, const std::string& value, const std::string& comment = "") {
    char card[81];
    std::string k = key;
    k.resize(8, ' ');
    std::string body = k + "= " + value;
    if (!comment.empty()) body += " / " + comment;
    std::snprintf(card, sizeof card, "%-80s", body.c_str());
    hdr.append(card, 80);
}

std::string fitsNum(double v) {
    char b[32];
    std::snprintf(b, sizeof b, "%20.10G", v);
    return b;
}

// FLOAT_IMG cube (FITSInOut.cpp:32-80): NAXIS1 = Nx, NAXIS2 = Ny, NAXIS3 = Nlambda (omitted when 1)
void writeFits(const std::string& path, const std::vector<double>& data, int nx, int ny, int nz,
               double xpsiz, double ypsiz, double xc, double yc, const std::string& bunit, const std::string& lunit) {
    std::string hdr;
    fitsCard(hdr, "SIMPLE", "                   T");
    fitsCard(hdr, "BITPIX", "                 -32");
    fitsCard(hdr, "NAXIS", nz > 1 ? "                   3" : "                   2");
    fitsCard(hdr, "NAXIS1", fitsNum(nx));
    fitsCard(hdr, "NAXIS2", fitsNum(ny));
    if (nz > 1) fitsCard(hdr, "NAXIS3", fitsNum(nz));
    fitsCard(hdr, "BSCALE", "                  1.");
    fitsCard(hdr, "BZERO", "                  0.");
    fitsCard(hdr, "ORIGIN", "'SKIRT MI355X engine'");
    fitsCard(hdr, "BUNIT", "'" + bunit + "'");
    fitsCard(hdr, "CRPIX1", fitsNum((nx + 1) / 2.0));
    fitsCard(hdr, "CRVAL1", fitsNum(xc));
    fitsCard(hdr, "CDELT1", fitsNum(xpsiz));
    fitsCard(hdr, "CTYPE1", "'" + lunit + "'");
    fitsCard(hdr, "CRPIX2", fitsNum((ny + 1) / 2.0));
    fitsCard(hdr, "CRVAL2", fitsNum(yc));
    fitsCard(hdr, "CDELT2", fitsNum(ypsiz));
    fitsCard(hdr, "CTYPE2", "'" + lunit + "'");
    {
        char card[81];
        std::snprintf(card, sizeof card, "%-80s", "END");
        hdr.append(card, 80);
    }
    while (hdr.size() % 2880) hdr.push_back(' ');
    std::vector<unsigned char> body(data.size() * 4);
    for (size_t i = 0; i < data.size(); i++) {
        float f = (float)data[i];
        uint32_t u;
        std::memcpy(&u, &f, 4);
        body[4 * i] = (unsigned char)(u >> 24);
        body[4 * i + 1] = (unsigned char)(u >> 16);
        body[4 * i + 2] = (unsigned char)(u >> 8);
        body[4 * i + 3] = (unsigned char)u;
    }
    while (body.size() % 2880) body.push_back(0);
    std::ofstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot create output file " + path);
    f.write(hdr.data(), hdr.size());
    f.write((const char*)body.data(), body.size());
}

}  // namespace

void writeOutputs(const Model& m, const std::string& prefix, const std::vector<std::vector<double>>& frames,
                  const std::vector<std::vector<double>>& seds, const std::vector<double>& labs) {
    Units units(m.units_system);
    int Nl = m.wl.n();
    for (size_t i = 0; i < m.instruments.size(); i++) {
        const Instrument& ins = m.instruments[i];
        size_t NF = (size_t)ins.nframe() * Nl;
        auto fslot = [&](int s) {
            if (frames[i].empty()) return std::vector<double>();
            return std::vector<double>(frames[i].begin() + s * NF, frames[i].begin() + (s + 1) * NF);
        };
        auto Fslot = [&](int s) {
            if (seds[i].empty()) return std::vector<double>();
            return std::vector<double>(seds[i].begin() + (size_t)s * Nl, seds[i].begin() + (size_t)(s + 1) * Nl);
        };
        std::vector<std::vector<double>> farr, Farr;
        std::vector<std::string> fnames, Fnames;
        if (ins.kind == InstrumentKind::Full) {
            // FullInstrument::write (FullInstrument.cpp:176-237)
            std::vector<double> ftrav = fslot(SlotTrav), fdir = fslot(SlotStrDir), fsca = fslot(SlotStrSca);
            std::vector<double> fdd = fslot(SlotDusDir), fds = fslot(SlotDusSca);
            std::vector<double> Ftrav = Fslot(SlotTrav), Fdir = Fslot(SlotStrDir), Fsca = Fslot(SlotStrSca);
            std::vector<double> Fdd = Fslot(SlotDusDir), Fds = Fslot(SlotDusSca);
            std::vector<double> ftot, Ftot, ftotdus, Ftotdus;
            if (m.dustEmission) {
                ftot.resize(NF); Ftot.resize(Nl); ftotdus.resize(NF); Ftotdus.resize(Nl);
                for (size_t q = 0; q < NF; q++) { ftot[q] = fdir[q] + fsca[q] + fdd[q] + fds[q]; ftotdus[q] = fdd[q] + fds[q]; }
                for (int q = 0; q < Nl; q++) { Ftot[q] = Fdir[q] + Fsca[q] + Fdd[q] + Fds[q]; Ftotdus[q] = Fdd[q] + Fds[q]; }
            } else if (m.hasDust) {
                ftot.resize(NF); Ftot.resize(Nl);
                for (size_t q = 0; q < NF; q++) ftot[q] = fdir[q] + fsca[q];
                for (int q = 0; q < Nl; q++) Ftot[q] = Fdir[q] + Fsca[q];
                fdd.clear(); fds.clear(); Fdd.clear(); Fds.clear();
            } else {
                ftot = ftrav; ftrav.clear(); Ftot = Ftrav; Fdir = Ftrav;
                fdir.clear(); fsca.clear(); fdd.clear(); fds.clear(); Fsca.clear(); Fdd.clear(); Fds.clear();
            }
            if (!m.dustEmission) { fdd.clear(); fds.clear(); Fdd.clear(); Fds.clear(); }
            farr = {ftot, fdir, fsca, ftotdus, fds, ftrav};
            Farr = {Ftot, Fdir, Fsca, Ftotdus, Fds, Ftrav};
            fnames = {"total", "direct", "scattered", "dust", "dustscattered", "transparent"};
            Fnames = {"total flux", "direct stellar flux", "scattered stellar flux", "total dust emission flux",
                      "dust emission scattered flux", "transparent flux"};
            for (int n = 0; n < ins.scatteringLevels; n++) {
                farr.push_back(fslot(SlotLevel0 + n));
                Farr.push_back(Fslot(SlotLevel0 + n));
                fnames.push_back("scatteringlevel" + std::to_string(n + 1));
                Fnames.push_back(std::to_string(n + 1) + "-times scattered flux");
            }
        } else {
            if (ins.hasFrames()) { farr.push_back(fslot(0)); fnames.push_back("total"); }
            if (ins.hasSeds()) { Farr.push_back(Fslot(0)); Fnames.push_back("total flux"); }
        }

        // frames: SingleFrameInstrument::calibrateAndWriteDataCubes
        if (ins.hasFrames()) {
            int Nframep = ins.nframe();
            for (int ell = 0; ell < Nl; ell++) {
                double dlambda = m.wl.dlambda[ell];
                for (int ii = 0; ii < ins.Nx; ii++)
                    for (int jj = 0; jj < ins.Ny; jj++) {
                        size_t q = ii + (size_t)ins.Nx * jj + (size_t)Nframep * ell;
                        for (auto& f : farr)
                            if (!f.empty()) f[q] /= dlambda;
                    }
            }
            double xpsizang = 2.0 * atan(ins.xpsiz / (2.0 * ins.distance));
            double ypsizang = 2.0 * atan(ins.ypsiz / (2.0 * ins.distance));
            double area = xpsizang * ypsizang;
            for (auto& f : farr) for (auto& v : f) v /= area;
            double fourpid2 = 4.0 * M_PI * ins.distance * ins.distance;
            for (auto& f : farr) for (auto& v : f) v /= fourpid2;
            for (int ell = 0; ell < Nl; ell++) {
                double lambda = m.wl.lambda[ell];
                for (int ii = 0; ii < ins.Nx; ii++)
                    for (int jj = 0; jj < ins.Ny; jj++) {
                        size_t q = ii + (size_t)ins.Nx * jj + (size_t)Nframep * ell;
                        for (auto& f : farr)
                            if (!f.empty()) f[q] = units.osurfacebrightness(lambda, f[q]);
                    }
            }
            double lf = Units::factor("length", units.unitFor("length"));
            for (size_t q = 0; q < farr.size(); q++) {
                if (farr[q].empty()) continue;
                writeFits(prefix + "_" + ins.name + "_" + fnames[q] + ".fits", farr[q], ins.Nx, ins.Ny, Nl,
                          ins.xpsiz / lf, ins.ypsiz / lf, ins.xc / lf, ins.yc / lf, units.unitFor("neutralsurfacebrightness"),
                          units.unitFor("length"));
            }
        }
        // SEDs: DistantInstrument::calibrateAndWriteSEDs
        if (ins.hasSeds()) {
            for (int ell = 0; ell < Nl; ell++) {
                double dlambda = m.wl.dlambda[ell];
                for (auto& F : Farr)
                    if (!F.empty()) F[ell] /= dlambda;
            }
            double fourpid2 = 4.0 * M_PI * ins.distance * ins.distance;
            for (auto& F : Farr) for (auto& v : F) v /= fourpid2;
            TextOut sed(prefix + "_" + ins.name + "_sed.dat");
            sed.column("lambda (" + units.unitFor("wavelength") + ")", 'e', 8);
            for (auto& n : Fnames) sed.column(n + "; lambda*F_lambda (" + units.unitFor("neutralfluxdensity") + ")", 'e', 8);
            for (int ell = 0; ell < Nl; ell++) {
                double lambda = m.wl.lambda[ell];
                std::vector<double> vals{units.owavelength(lambda)};
                for (auto& F : Farr) vals.push_back(F.empty() ? 0. : units.ofluxdensity(lambda, F[ell]));
                sed.row(vals);
            }
        }
    }

    int Ncells = m.ncells(), Ncomp = m.ncomp();
    if (m.hasDust && m.pan && m.writeISRF && !labs.empty()) {
        // PanDustSystem::write, ISRF part
        TextOut f(prefix + "_ds_isrf.dat");
        f.line("# Mean field intensities for all dust cells with nonzero absorption");
        f.column("dust cell index", 'd');
        f.column("x coordinate of cell center (" + units.unitFor("length") + ")", 'g');
        f.column("y coordinate of cell center (" + units.unitFor("length") + ")", 'g');
        f.column("z coordinate of cell center (" + units.unitFor("length") + ")", 'g');
        for (int ell = 0; ell < Nl; ell++)
            f.column("J_lambda (W/m3/sr) for lambda = " + qtNumber(units.owavelength(m.wl.lambda[ell]), 'g', 6) + " " +
                         units.unitFor("wavelength"), 'g');
        for (int c = 0; c < Ncells; c++) {
            double Ltot = 0;
            for (int ell = 0; ell < Nl; ell++) Ltot += labs[(size_t)c * Nl + ell];
            if (!(Ltot > 0.0)) continue;
            double ctr[3];
            m.grid.cellCenter(c, ctr);
            std::vector<double> vals{(double)c, units.olength(ctr[0]), units.olength(ctr[1]), units.olength(ctr[2])};
            double fac = 4.0 * M_PI * m.volume[c];
            for (int ell = 0; ell < Nl; ell++) {
                double kappaabsrho = 0.0;
                for (int h = 0; h < Ncomp; h++) kappaabsrho += m.dust[h].mix.kabs[ell] * m.rho[(size_t)c * Ncomp + h];
                double J = labs[(size_t)c * Nl + ell] / (kappaabsrho * fac) / m.wl.dlambda[ell];
                vals.push_back(std::isfinite(J) ? J : 0.0);
            }
            f.row(vals);
        }
    }
    if (m.hasDust && m.writeCellProperties) {
        // DustSystem::writecellproperties (statistics lines omitted)
        TextOut f(prefix + "_ds_cellprops.dat");
        f.column("volume (" + units.unitFor("volume") + ")");
        f.column("density (" + units.unitFor("massvolumedensity") + ")");
        f.column("mass fraction");
        f.column("optical depth");
        double totalmass = 0;
        for (auto& d : m.dust) totalmass += d.nf;
        for (int c = 0; c < Ncells; c++) {
            double rho = 0;
            for (int h = 0; h < Ncomp; h++) rho += m.rho[(size_t)c * Ncomp + h];
            double V = m.volume[c];
            double delta = (rho * V) / totalmass;
            double tau = constants::kappaV * rho * std::pow(V, 1. / 3.);
            f.row({units.ovolume(V), units.omassvolumedensity(rho), delta, tau});
        }
    }
}

void writeCellsCrossed(const Model& m, const std::string& prefix, const std::vector<uint64_t>& hist) {
    size_t n = hist.size();
    while (n > 0 && hist[n - 1] == 0) n--;
    TextOut f(prefix + "_ds_crossed.dat");
    f.line("# total number of cells in grid: " + std::to_string(m.ncells()));
    f.column("number of cells crossed", 'd');
    f.column("number of paths that crossed this number of cells", 'd');
    for (size_t i = 0; i < n; i++) f.row({(double)i, (double)hist[i]});
}

void writeConvergence(const Model& m, const std::string& prefix, const double sigma[3]) {
    Units units(m.units_system);
    const int Ncomp = (int)m.dust.size();
    double M = 0.0;  // the grid's mass, in the reference's cell order
    for (int c = 0; c < m.ncells(); c++) {
        double rho = 0;
        for (int h = 0; h < Ncomp; h++) rho += m.rho[(size_t)c * Ncomp + h];
        M += rho * m.volume[c];
    }
    // CompDustDistribution: the sums over the components of nf times the geometry's value
    // (DustComp.cpp:119-141; SpheGeometry.cpp:49-71 and AxGeometry.cpp:34-47 for the x and y axes)
    int dim = 1;
    double ref[3] = {0, 0, 0}, Mref = 0;
    for (auto& d : m.dust) {
        const bool ax = d.geom.kind == GeometryKind::ExpDisk;
        dim = std::max(dim, ax ? 2 : 1);
        const double sxy = ax ? 2.0 * d.geom.SigmaR() : 2.0 * d.geom.Sigmar();
        ref[0] += d.nf * sxy;
        ref[1] += d.nf * sxy;
        ref[2] += d.nf * (ax ? d.geom.SigmaZ() : 2.0 * d.geom.Sigmar());
        Mref += d.nf;
    }
    const std::string us = " " + units.unitFor("masssurfacedensity");
    auto num = [&](double v) { return qtNumber(units.omasssurfacedensity(v), 'g', 6) + us; };
    TextOut f(prefix + "_ds_convergence.dat");
    f.line("Convergence check on the grid: ");
    auto pair = [&](const std::string& what, double expected, double actual) {
        f.line("   - " + what);
        f.line("         expected value = " + num(expected));
        f.line("         actual value =   " + num(actual));
    };
    if (dim == 1) {
        pair("radial (r-axis) surface density", 0.5 * ref[0], 0.5 * sigma[0]);
    } else {
        pair("edge-on (R-axis) surface density", 0.5 * ref[0], 0.5 * sigma[0]);
        pair("face-on (Z-axis) surface density", ref[2], sigma[2]);
    }
    f.line("   - total dust mass");
    f.line("         expected value = " + qtNumber(units.omass(Mref), 'g', 6) + " " + units.unitFor("mass"));
    f.line("         actual value =   " + qtNumber(units.omass(M), 'g', 6) + " " + units.unitFor("mass"));
}

}  // namespace skirt
