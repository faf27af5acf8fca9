// Physical constants and unit conversion for .ski input and SKIRT-format output.
//
// Restates SKIRTcore/Units.cpp: the SI constants (Units.cpp:9-24 of the stripped listing, the anonymous
// namespace at the top of the file), the "<quantity> <unit>" factor table (Units.cpp initialize()),
// the default unit per quantity of each unit system (ExtragalacticUnits.cpp, SIUnits.cpp,
// StellarUnits.cpp) and the string conversion of Discover/DoublePropertyHandler.cpp:169-198
// (value * factor, default unit when none is given). Output conversion follows Units.cpp:973-1030
// (the "Neutral" flux output style, lambda*F_lambda, which is the default).
#pragma once

#include <map>
#include <string>

namespace skirt {

namespace constants {
constexpr double c = 2.99792458e8;
constexpr double h = 6.62606957e-34;
constexpr double k = 1.3806488e-23;
constexpr double AU = 1.49597871e11;
constexpr double pc = 3.08567758e16;
constexpr double Msun = 1.9891e30;
constexpr double Lsun = 3.839e26;
constexpr double mproton = 1.67262178e-27;  // Units.cpp _Mproton
constexpr double lambdaV = 550e-9;
constexpr double kappaV = 2600.;
}  // namespace constants

class Units {
public:
    // system: "ExtragalacticUnits", "SIUnits" or "StellarUnits"
    explicit Units(const std::string& system = "ExtragalacticUnits");

    // factor converting `unit` of quantity `qty` to SI; throws for unknown combinations
    static double factor(const std::string& qty, const std::string& unit);
    // converts "<number> [<unit>]" for quantity qty ("" = dimensionless) to SI
    double parse(const std::string& value, const std::string& qty) const;
    const std::string& unitFor(const std::string& qty) const;

    // output conversions used by the SED / frame writers
    double owavelength(double lambda) const;
    double ofluxdensity(double lambda, double Flambda) const;       // lambda*F_lambda in W/m2
    double osurfacebrightness(double lambda, double flambda) const;  // lambda*f_lambda per unit solid angle
    double olength(double x) const;
    double ovolume(double v) const;
    double omassvolumedensity(double rho) const;
    double omasssurfacedensity(double sigma) const;
    double omass(double M) const;
    double obolluminosity(double L) const;

    const std::string& system() const { return system_; }

private:
    std::string system_;
    std::map<std::string, std::string> unitForQty_;
};

}  // namespace skirt
