// skirt-mi355x: runs the stellar emission phase of a .ski file on one MI355X and writes SKIRT-format
// outputs (the counterpart of `skirt <file.ski>` for the photon-shooting path, SKIRTmain/SkirtMain.cpp).
//   skirt-mi355x [-d device | -g ngpus] [-o outprefix] [-p packages] [-s seed] file.ski
// -g N runs the simulation on devices 0 .. N-1 of this node: each shoots its slice of every wavelength and
// the tallies are summed over xGMI by RCCL all-reduces at each phase end (skirt_sim_run_devices).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../../include/skirt_host.h"

int main(int argc, char** argv) {
    int device = 0, ngpus = 0;
    double packages = 0;
    unsigned long long seed = 0;
    std::string out, ski;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "-d") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "-g") && i + 1 < argc) ngpus = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
        else if (!std::strcmp(argv[i], "-p") && i + 1 < argc) packages = std::atof(argv[++i]);
        else if (!std::strcmp(argv[i], "-s") && i + 1 < argc) seed = std::strtoull(argv[++i], nullptr, 10);
        else ski = argv[i];
    }
    if (ski.empty()) {
        std::fprintf(stderr, "usage: skirt-mi355x [-d device | -g ngpus] [-o outprefix] [-p packages] [-s seed] file.ski\n");
        return 2;
    }
    if (out.empty()) {
        out = ski;
        if (out.size() > 4 && out.substr(out.size() - 4) == ".ski") out.resize(out.size() - 4);
    }
    if (ngpus > 0) {
        SkirtStats st;
        double secs = 0;
        if (skirt_sim_run_devices(ski.c_str(), nullptr, ngpus, packages, seed, out.c_str(), &st, &secs)) {
            std::fprintf(stderr, "*** Error: %s\n", skirt_sim_error());
            return 1;
        }
        std::printf("%d GPUs (RCCL all-reduce of the tallies): rank 0 shot %llu packets; photon phases %.3f s\n",
                    ngpus, (unsigned long long)st.packets, secs);
        return 0;
    }
    SkirtSim* sim = skirt_sim_load(ski.c_str(), nullptr, packages, seed);
    if (!sim) { std::fprintf(stderr, "*** Error: %s\n", skirt_sim_error()); return 1; }
    SkirtSimInfo info;
    skirt_sim_info(sim, &info);
    std::printf("Setup: %d cells, %d wavelengths, %llu packets per wavelength (%.2f s)\n", info.ncells, info.nlambda,
                (unsigned long long)info.npp, info.setup_seconds);
    if (skirt_sim_attach(sim, device) || skirt_sim_run_stellar(sim, 0, 0)) {
        std::fprintf(stderr, "*** Error: %s\n", skirt_sim_error());
        skirt_sim_free(sim);
        return 1;
    }
    SkirtStats st;
    skirt_mcrt_stats(skirt_sim_engine(sim), &st);
    std::printf("Stellar emission phase: %llu packets in %.3f ms (%.3g packets/s)\n", (unsigned long long)st.packets,
                st.kernel_ms, st.packets / (st.kernel_ms * 1e-3));
    // PanMonteCarloSimulation::runSelf (PanMonteCarloSimulation.cpp:96-104): the self-absorption cycles and
    // the dust emission phase follow the stellar phase (a no-op for Oligo models and Pan models without
    // dust emission), so the written outputs hold every phase the model asks for
    const double* dustTot = nullptr;
    if (skirt_sim_run_dust(sim) || skirt_sim_fetch(sim)) {
        std::fprintf(stderr, "*** Error: %s\n", skirt_sim_error());
        skirt_sim_free(sim);
        return 1;
    }
    int ncycles = skirt_sim_selfabs_totals(sim, &dustTot);
    for (int c = 0; c < ncycles; c++)
        std::printf("Self-absorption cycle %d: total absorbed dust luminosity %.9g\n", c + 1, dustTot[c]);
    if (skirt_sim_write(sim, out.c_str())) { std::fprintf(stderr, "*** Error: %s\n", skirt_sim_error()); return 1; }
    skirt_sim_free(sim);
    return 0;
}
