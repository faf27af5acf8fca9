// SKIRT-format outputs: calibrated instrument SEDs (text) and frames (FITS), ds_isrf and ds_cellprops.
//
// Restates the host-side write path of the reference, which runs after the photon phases:
//   FullInstrument::write (FullInstrument.cpp:176-237) -- which arrays are combined and written,
//   SingleFrameInstrument::calibrateAndWriteDataCubes (SingleFrameInstrument.cpp:151-226),
//   DistantInstrument::calibrateAndWriteSEDs (DistantInstrument.cpp:131-183),
//   PanDustSystem::write ISRF part (PanDustSystem.cpp:613-640) and DustSystem::meanintensityv (:935-957),
//   DustSystem::writecellproperties (DustSystem.cpp:636-660),
//   TextOutFile column formats (TextOutFile.cpp:46-90, Qt QString::number formatting).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "model.hpp"

namespace skirt {

// frames[i] = instrument i's accumulators [nslots][nlambda][nframe]; seds[i] = [nslots][nlambda];
// labs = Ncells x Nlambda row-major (may be empty). Writes <prefix>_<instr>_sed.dat,
// <prefix>_<instr>_<name>.fits, and <prefix>_ds_isrf.dat / _ds_cellprops.dat when the model asks for them.
void writeOutputs(const Model& m, const std::string& prefix, const std::vector<std::vector<double>>& frames,
                  const std::vector<std::vector<double>>& seds, const std::vector<double>& labs);

// DustSystem::write (DustSystem.cpp:1004-1024): <prefix>_ds_crossed.dat, hist[n] = paths that crossed n
// cells, written up to the last nonzero bin
void writeCellsCrossed(const Model& m, const std::string& prefix, const std::vector<uint64_t>& hist);

// DustSystem::writeconvergence (DustSystem.cpp:195-305): <prefix>_ds_convergence.dat, the grid's mass and
// column densities through the origin (sigma: x, y and z axes, each the sum of its two half axes) beside
// the dust distribution's analytic values. The geometries here are spherical (dimension 1) or axisymmetric
// (ExpDisk, dimension 2); the dimension-3 branch of the reference has no geometry to reach it.
void writeConvergence(const Model& m, const std::string& prefix, const double sigma[3]);

// Qt-compatible number formatting: QString::number(v, 'e', prec) and QString::number(v, 'g', prec)
std::string qtNumber(double v, char fmt, int prec);

// reads the Random seed from a ski file without running setup (4357 when absent)
unsigned long readSkiSeed(const std::string& path);

}  // namespace skirt
