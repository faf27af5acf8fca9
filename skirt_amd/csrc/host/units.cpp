#include "units.hpp"

#include <cmath>
#include <cstdlib>
#include <sstream>
#include <stdexcept>
#include <vector>

namespace skirt {

namespace {

const std::map<std::string, double>& table() {
    using namespace constants;
    static const std::map<std::string, double> t = [] {
        std::map<std::string, double> f;
        const double arcsec = M_PI / (180. * 3600.);
        f["length m"] = 1.;
        f["length cm"] = 1e-2;
        f["length km"] = 1e3;
        f["length AU"] = AU;
        f["length pc"] = pc;
        f["length kpc"] = 1e3 * pc;
        f["length Mpc"] = 1e6 * pc;
        f["distance m"] = 1.;
        f["distance cm"] = 1e-2;
        f["distance km"] = 1e3;
        f["distance AU"] = AU;
        f["distance pc"] = pc;
        f["distance kpc"] = 1e3 * pc;
        f["distance Mpc"] = 1e6 * pc;
        f["wavelength m"] = 1.;
        f["wavelength cm"] = 1e-2;
        f["wavelength mm"] = 1e-3;
        f["wavelength micron"] = 1e-6;
        f["wavelength nm"] = 1e-9;
        f["wavelength A"] = 1e-10;
        f["grainsize m"] = 1.;
        f["grainsize cm"] = 1e-2;
        f["grainsize mm"] = 1e-3;
        f["grainsize micron"] = 1e-6;
        f["grainsize nm"] = 1e-9;
        f["grainsize A"] = 1e-10;
        f["section m2"] = 1.;
        f["volume m3"] = 1.;
        f["volume AU3"] = std::pow(AU, 3);
        f["volume pc3"] = std::pow(pc, 3);
        f["velocity m/s"] = 1.;
        f["velocity km/s"] = 1e3;
        f["mass kg"] = 1.;
        f["mass g"] = 1e-3;
        f["mass Msun"] = Msun;
        f["bulkmass kg"] = 1.;
        f["bulkmassdensity kg/m3"] = 1.;
        f["bulkmassdensity g/cm3"] = 1e3;
        f["masssurfacedensity kg/m2"] = 1.;
        f["masssurfacedensity Msun/AU2"] = Msun / std::pow(AU, 2);
        f["masssurfacedensity Msun/pc2"] = Msun / std::pow(pc, 2);
        f["massvolumedensity kg/m3"] = 1.;
        f["massvolumedensity g/cm3"] = 1e3;
        f["massvolumedensity Msun/AU3"] = Msun / std::pow(AU, 3);
        f["massvolumedensity Msun/pc3"] = Msun / std::pow(pc, 3);
        f["opacity m2/kg"] = 1.;
        f["energy J"] = 1.;
        f["bolluminosity W"] = 1.;
        f["bolluminosity Lsun"] = Lsun;
        f["monluminosity W/m"] = 1.;
        f["monluminosity W/micron"] = 1e6;
        f["monluminosity Lsun/micron"] = Lsun * 1e6;
        f["neutralfluxdensity W/m2"] = 1.;
        f["neutralsurfacebrightness W/m2/sr"] = 1.;
        f["neutralsurfacebrightness W/m2/arcsec2"] = 1. / std::pow(arcsec, 2);
        f["wavelengthfluxdensity W/m3"] = 1.;
        f["wavelengthfluxdensity W/m2/micron"] = 1e6;
        f["wavelengthsurfacebrightness W/m3/sr"] = 1.;
        f["wavelengthsurfacebrightness W/m2/micron/sr"] = 1e6;
        f["wavelengthsurfacebrightness W/m2/micron/arcsec2"] = 1e6 / std::pow(arcsec, 2);
        f["frequencyfluxdensity W/m2/Hz"] = 1.;
        f["frequencyfluxdensity Jy"] = 1e-26;
        f["frequencyfluxdensity mJy"] = 1e-29;
        f["frequencyfluxdensity MJy"] = 1e-20;
        f["frequencysurfacebrightness W/m2/Hz/sr"] = 1.;
        f["frequencysurfacebrightness W/m2/Hz/arcsec2"] = 1. / std::pow(arcsec, 2);
        f["frequencysurfacebrightness Jy/sr"] = 1e-26;
        f["frequencysurfacebrightness Jy/arcsec2"] = 1e-26 / std::pow(arcsec, 2);
        f["frequencysurfacebrightness MJy/sr"] = 1e-20;
        f["frequencysurfacebrightness MJy/arcsec2"] = 1e-20 / std::pow(arcsec, 2);
        f["temperature K"] = 1.;
        f["angle rad"] = 1.;
        f["angle deg"] = M_PI / 180.;
        f["angle arcsec"] = M_PI / (180. * 3600.);
        f["posangle rad"] = 1.;
        f["posangle deg"] = M_PI / 180.;
        f["solidangle sr"] = 1.;
        f["solidangle arcsec2"] = std::pow(arcsec, 2);
        f["pressure Pa"] = 1.;
        f["pressure K/m3"] = k;
        return f;
    }();
    return t;
}

std::vector<std::string> splitWs(const std::string& s) {
    std::istringstream in(s);
    std::vector<std::string> out;
    std::string w;
    while (in >> w) out.push_back(w);
    return out;
}

}  // namespace

Units::Units(const std::string& system) : system_(system) {
    auto& u = unitForQty_;
    if (system == "SIUnits") {
        u = {{"length", "m"}, {"distance", "m"}, {"wavelength", "m"}, {"grainsize", "m"}, {"section", "m2"},
             {"volume", "m3"}, {"velocity", "m/s"}, {"mass", "kg"}, {"bulkmass", "kg"},
             {"bulkmassdensity", "kg/m3"}, {"masssurfacedensity", "kg/m2"}, {"massvolumedensity", "kg/m3"},
             {"opacity", "m2/kg"}, {"energy", "J"}, {"bolluminosity", "W"}, {"monluminosity", "W/m"},
             {"neutralfluxdensity", "W/m2"}, {"neutralsurfacebrightness", "W/m2/sr"},
             {"wavelengthfluxdensity", "W/m3"}, {"wavelengthsurfacebrightness", "W/m3/sr"},
             {"frequencyfluxdensity", "W/m2/Hz"}, {"frequencysurfacebrightness", "W/m2/Hz/sr"},
             {"temperature", "K"}, {"angle", "rad"}, {"posangle", "rad"}, {"solidangle", "sr"}, {"pressure", "Pa"}};
    } else if (system == "StellarUnits") {
        u = {{"length", "AU"}, {"distance", "pc"}, {"wavelength", "micron"}, {"grainsize", "micron"},
             {"section", "m2"}, {"volume", "AU3"}, {"velocity", "km/s"}, {"mass", "Msun"}, {"bulkmass", "kg"},
             {"bulkmassdensity", "kg/m3"}, {"masssurfacedensity", "Msun/AU2"}, {"massvolumedensity", "Msun/AU3"},
             {"opacity", "m2/kg"}, {"energy", "J"}, {"bolluminosity", "Lsun"}, {"monluminosity", "Lsun/micron"},
             {"neutralfluxdensity", "W/m2"}, {"neutralsurfacebrightness", "W/m2/arcsec2"},
             {"wavelengthfluxdensity", "W/m2/micron"}, {"wavelengthsurfacebrightness", "W/m2/micron/arcsec2"},
             {"frequencyfluxdensity", "Jy"}, {"frequencysurfacebrightness", "MJy/sr"}, {"temperature", "K"},
             {"angle", "arcsec"}, {"posangle", "deg"}, {"solidangle", "arcsec2"}, {"pressure", "K/m3"}};
    } else if (system == "ExtragalacticUnits") {
        u = {{"length", "pc"}, {"distance", "Mpc"}, {"wavelength", "micron"}, {"grainsize", "micron"},
             {"section", "m2"}, {"volume", "pc3"}, {"velocity", "km/s"}, {"mass", "Msun"}, {"bulkmass", "kg"},
             {"bulkmassdensity", "kg/m3"}, {"masssurfacedensity", "Msun/pc2"}, {"massvolumedensity", "Msun/pc3"},
             {"opacity", "m2/kg"}, {"energy", "J"}, {"bolluminosity", "Lsun"}, {"monluminosity", "Lsun/micron"},
             {"neutralfluxdensity", "W/m2"}, {"neutralsurfacebrightness", "W/m2/arcsec2"},
             {"wavelengthfluxdensity", "W/m2/micron"}, {"wavelengthsurfacebrightness", "W/m2/micron/arcsec2"},
             {"frequencyfluxdensity", "Jy"}, {"frequencysurfacebrightness", "MJy/sr"}, {"temperature", "K"},
             {"angle", "arcsec"}, {"posangle", "deg"}, {"solidangle", "arcsec2"}, {"pressure", "K/m3"}};
    } else {
        throw std::runtime_error("unsupported unit system " + system);
    }
}

double Units::factor(const std::string& qty, const std::string& unit) {
    auto it = table().find(qty + " " + unit);
    if (it == table().end()) throw std::runtime_error("unknown quantity " + qty + " and/or unit " + unit);
    return it->second;
}

const std::string& Units::unitFor(const std::string& qty) const {
    auto it = unitForQty_.find(qty);
    if (it == unitForQty_.end()) throw std::runtime_error("unknown quantity " + qty);
    return it->second;
}

double Units::parse(const std::string& value, const std::string& qty) const {
    std::vector<std::string> seg = splitWs(value);
    if (seg.empty() || seg.size() > 2) throw std::runtime_error("malformed value '" + value + "'");
    char* end = nullptr;
    double x = std::strtod(seg[0].c_str(), &end);
    if (end == seg[0].c_str() || *end != 0) throw std::runtime_error("malformed number in '" + value + "'");
    if (qty.empty()) {
        if (seg.size() != 1) throw std::runtime_error("dimensionless value with unit: '" + value + "'");
        return x;
    }
    if (seg.size() == 1) return x * factor(qty, unitFor(qty));
    return x * factor(qty, seg[1]);
}

double Units::owavelength(double lambda) const { return lambda / factor("wavelength", unitFor("wavelength")); }

double Units::ofluxdensity(double lambda, double Flambda) const {
    return lambda * Flambda / factor("neutralfluxdensity", unitFor("neutralfluxdensity"));
}

double Units::osurfacebrightness(double lambda, double flambda) const {
    return lambda * flambda / factor("neutralsurfacebrightness", unitFor("neutralsurfacebrightness"));
}

double Units::olength(double x) const { return x / factor("length", unitFor("length")); }
double Units::ovolume(double v) const { return v / factor("volume", unitFor("volume")); }
double Units::omasssurfacedensity(double sigma) const {
    return sigma / factor("masssurfacedensity", unitFor("masssurfacedensity"));
}

double Units::omass(double M) const {
    return M / factor("mass", unitFor("mass"));
}

double Units::omassvolumedensity(double rho) const {
    return rho / factor("massvolumedensity", unitFor("massvolumedensity"));
}
double Units::obolluminosity(double L) const { return L / factor("bolluminosity", unitFor("bolluminosity")); }

}  // namespace skirt
