// The cross-GPU sums of the photon phases in C++ (include/skirt_host.h, skirt_rccl_*): one RCCL
// communicator per device of the process, the engine's reducer callback an in-place ncclAllReduce
// (ncclDouble, ncclSum) on the stream the engine hands it -- the reference's MPI_Allreduce of Labs and
// the instrument arrays at each phase end (PanDustSystem.cpp:394-404, Instrument.cpp:57-66,
// MPIsupport/ProcessManager.cpp:133-137) over xGMI. skirt_sim_run_devices drives one engine per device
// from its own thread (IdenticalAssigner slices, skirt_sim_run_*_shard) and writes the outputs once.
#include <chrono>
#include <exception>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "../../../include/skirt_host.h"

namespace skirt {
void setSimError(const std::string& msg);  // sim.cpp
}

struct SkirtRccl {
    std::vector<ncclComm_t> comms;
    bool owned = true;
};

namespace {

int reduceTally(void* user, int /*tally*/, double* buf, size_t n, void* stream) {
    ncclComm_t comm = *static_cast<ncclComm_t*>(user);
    return ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, comm, static_cast<hipStream_t>(stream)) == ncclSuccess ? 0
                                                                                                                : 1;
}

}  // namespace

extern "C" {

int skirt_rccl_create(int ndev, const int* devices, SkirtRccl** out) {
    if (!out || ndev < 1 || !devices) return SKIRT_ERR_ARG;
    *out = nullptr;
    auto* r = new SkirtRccl;
    r->comms.resize(ndev);
    if (ncclCommInitAll(r->comms.data(), ndev, devices) != ncclSuccess) {
        delete r;
        return SKIRT_ERR_HIP;
    }
    *out = r;
    return SKIRT_OK;
}

int skirt_rccl_wrap(void* nccl_comm, SkirtRccl** out) {
    if (!out || !nccl_comm) return SKIRT_ERR_ARG;
    auto* r = new SkirtRccl;
    r->comms.push_back(static_cast<ncclComm_t>(nccl_comm));
    r->owned = false;
    *out = r;
    return SKIRT_OK;
}

void* skirt_rccl_rank(SkirtRccl* r, int rank) {
    if (!r || rank < 0 || rank >= (int)r->comms.size()) return nullptr;
    return &r->comms[rank];
}

SkirtReduceTallyFn skirt_rccl_reducer(void) { return reduceTally; }

void skirt_rccl_destroy(SkirtRccl* r) {
    if (!r) return;
    if (r->owned)
        for (ncclComm_t c : r->comms) ncclCommDestroy(c);
    delete r;
}

int skirt_sim_run_devices(const char* ski, const char* datadir, int ndev, double packages, uint64_t seed,
                          const char* outprefix, SkirtStats* stats, double* seconds) {
    if (!ski || ndev < 1) return SKIRT_ERR_ARG;
    std::vector<int> devs(ndev);
    for (int d = 0; d < ndev; d++) devs[d] = d;
    SkirtRccl* rccl = nullptr;
    int rc = skirt_rccl_create(ndev, devs.data(), &rccl);
    if (rc) {
        skirt::setSimError("ncclCommInitAll over " + std::to_string(ndev) + " devices failed");
        return rc;
    }
    // one model per device: the setup draws are the reference's, so every rank builds the same grid
    std::vector<SkirtSim*> sims(ndev, nullptr);
    std::vector<int> rcs(ndev, SKIRT_OK);
    std::vector<std::string> errs(ndev);
    {
        std::vector<std::thread> th;
        for (int d = 0; d < ndev; d++)
            th.emplace_back([&, d] {
                sims[d] = skirt_sim_load(ski, datadir, packages, seed);
                if (!sims[d]) { rcs[d] = SKIRT_ERR_ARG; errs[d] = skirt_sim_error(); }
            });
        for (auto& t : th) t.join();
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (int d = 0; d < ndev && rc == SKIRT_OK; d++)
        if ((rc = rcs[d])) skirt::setSimError("device " + std::to_string(d) + ": " + errs[d]);
    if (rc == SKIRT_OK) {
        // one host thread per device: the engine's phase loop runs on its thread, and the ranks' all-reduces
        // meet on the devices
        std::vector<std::thread> th;
        for (int d = 0; d < ndev; d++)
            th.emplace_back([&, d] {
                SkirtSim* s = sims[d];
                int r = skirt_sim_attach(s, d);
                if (!r) r = skirt_mcrt_set_reducer(skirt_sim_engine(s), skirt_rccl_reducer(), skirt_rccl_rank(rccl, d));
                if (!r) r = skirt_sim_run_stellar_shard(s, d, ndev);
                if (!r) r = skirt_sim_run_dust_shard(s, d, ndev);
                if (!r) r = skirt_sim_fetch(s);  // sums the instruments over the ranks
                rcs[d] = r;
                if (r) errs[d] = skirt_sim_error();
            });
        for (auto& t : th) t.join();
        for (int d = 0; d < ndev && rc == SKIRT_OK; d++)
            if ((rc = rcs[d])) skirt::setSimError("device " + std::to_string(d) + ": " + errs[d]);
    }
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (rc == SKIRT_OK && stats) rc = skirt_mcrt_stats(skirt_sim_engine(sims[0]), stats);
    if (rc == SKIRT_OK && outprefix && *outprefix) rc = skirt_sim_write(sims[0], outprefix);
    for (SkirtSim* s : sims)
        if (s) skirt_sim_free(s);
    skirt_rccl_destroy(rccl);
    return rc;
}

}  // extern "C"
