// The cross-GPU sums of the photon phases in C++ (include/skirt_host.h, skirt_rccl_*): one RCCL
// communicator per device of the process, the engine's reducer callback an in-place ncclAllReduce
// (ncclDouble, ncclSum) on the stream the engine hands it -- the reference's MPI_Allreduce of Labs and
// the instrument arrays at each phase end (PanDustSystem.cpp:394-404, Instrument.cpp:57-66,
// MPIsupport/ProcessManager.cpp:133-137) over xGMI. skirt_sim_run_devices drives one engine per device
// from its own thread (IdenticalAssigner slices, skirt_sim_run_*_shard) and writes the outputs once.
//
// Failure semantics (Parallel.cpp:181-193: the first exception stops every worker and is rethrown in the
// parent): the device threads pass a RankGate before every all-reduce, so that once one of them has failed no
// other enqueues a collective it would wait in for ever, and the failing thread aborts the communicators
// (ncclCommAbort, not Destroy), which returns peers already waiting on the device. The parent reports the
// first failure.
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <exception>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "../../../include/skirt_host.h"
#include "rank_gate.hpp"

namespace skirt {
void setSimError(const std::string& msg);  // sim.cpp
}

struct SkirtRccl;

namespace {
struct RankCtx {  // the reducer's user pointer of one rank (skirt_rccl_rank)
    SkirtRccl* owner;
    int rank;
};
}  // namespace

struct SkirtRccl {
    std::vector<ncclComm_t> comms;
    std::vector<RankCtx> ranks;
    bool owned = true;
    std::unique_ptr<skirt::RankGate> gate;
    std::atomic<bool> aborted{false};
};

namespace {

int reduceTally(void* user, int /*tally*/, double* buf, size_t n, void* stream) {
    auto* rk = static_cast<RankCtx*>(user);
    SkirtRccl* r = rk->owner;
    // no collective once a rank has failed; with several ranks in this process, not before all have arrived
    if (r->gate->ranks() > 1 ? !r->gate->arrive() : r->gate->failed()) return 1;
    if (r->aborted.load()) return 1;
    if (ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, r->comms[rk->rank], static_cast<hipStream_t>(stream)) !=
        ncclSuccess) {
        skirt_rccl_abort(r, ("ncclAllReduce failed on rank " + std::to_string(rk->rank)).c_str());
        return 1;
    }
    return 0;
}

// SKIRT_AMD_FAIL_DEVICE=d: the thread of device d fails before its first phase (tests of the failure path)
bool injectedFailure(int d) {
    const char* e = getenv("SKIRT_AMD_FAIL_DEVICE");
    return e && *e && atoi(e) == d;
}

}  // namespace

extern "C" {

static void initRanks(SkirtRccl* r) {
    const int n = (int)r->comms.size();
    r->ranks.resize(n);
    for (int d = 0; d < n; d++) r->ranks[d] = RankCtx{r, d};
    r->gate.reset(new skirt::RankGate(n));
}

int skirt_rccl_create(int ndev, const int* devices, SkirtRccl** out) {
    if (!out || ndev < 1 || !devices) return SKIRT_ERR_ARG;
    *out = nullptr;
    auto* r = new SkirtRccl;
    r->comms.resize(ndev);
    if (ncclCommInitAll(r->comms.data(), ndev, devices) != ncclSuccess) {
        delete r;
        return SKIRT_ERR_HIP;
    }
    initRanks(r);
    *out = r;
    return SKIRT_OK;
}

int skirt_rccl_wrap(void* nccl_comm, SkirtRccl** out) {
    if (!out || !nccl_comm) return SKIRT_ERR_ARG;
    auto* r = new SkirtRccl;
    r->comms.push_back(static_cast<ncclComm_t>(nccl_comm));
    r->owned = false;
    initRanks(r);
    *out = r;
    return SKIRT_OK;
}

void* skirt_rccl_rank(SkirtRccl* r, int rank) {
    if (!r || rank < 0 || rank >= (int)r->comms.size()) return nullptr;
    return &r->ranks[rank];
}

SkirtReduceTallyFn skirt_rccl_reducer(void) { return reduceTally; }

int skirt_rccl_abort(SkirtRccl* r, const char* why) {
    if (!r) return SKIRT_ERR_ARG;
    r->gate->fail(why ? why : "aborted");  // no rank enqueues another collective
    if (r->aborted.exchange(true)) return SKIRT_OK;
    // returns the ranks already waiting in an all-reduce on the device; a wrapped communicator belongs to its
    // job, which aborts it itself
    if (r->owned)
        for (ncclComm_t c : r->comms) ncclCommAbort(c);
    return SKIRT_OK;
}

void skirt_rccl_destroy(SkirtRccl* r) {
    if (!r) return;
    if (r->owned && !r->aborted.load())
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
        // a failing thread stops the others: each checks the gate before its next stage, the reducer before
        // every collective, and the first failure aborts the communicators (peers waiting on the device return)
        skirt::RankGate& gate = *rccl->gate;
        std::vector<std::thread> th;
        for (int d = 0; d < ndev; d++)
            th.emplace_back([&, d] {
                SkirtSim* s = sims[d];
                auto stopped = [&] { return gate.failed() ? SKIRT_ERR_STATE : SKIRT_OK; };
                int r = injectedFailure(d) ? SKIRT_ERR_STATE : SKIRT_OK;
                if (r) skirt::setSimError("failure injected (SKIRT_AMD_FAIL_DEVICE)");
                if (!r) r = skirt_sim_attach(s, d);
                if (!r) r = skirt_mcrt_set_reducer(skirt_sim_engine(s), skirt_rccl_reducer(), skirt_rccl_rank(rccl, d));
                if (!r && !(r = stopped())) r = skirt_sim_run_stellar_shard(s, d, ndev);
                if (!r && !(r = stopped())) r = skirt_sim_run_dust_shard(s, d, ndev);
                if (!r && !(r = stopped())) r = skirt_sim_fetch(s);  // sums the instruments over the ranks
                rcs[d] = r;
                if (r && !gate.failed()) {  // this thread failed first (not stopped by another's failure)
                    errs[d] = skirt_sim_error();
                    skirt_rccl_abort(rccl, ("device " + std::to_string(d) + ": " + errs[d]).c_str());
                }
            });
        for (auto& t : th) t.join();
        for (int d = 0; d < ndev && rc == SKIRT_OK; d++) rc = rcs[d];
        if (rc) skirt::setSimError(gate.failed() ? gate.message() : "a device thread failed");
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
