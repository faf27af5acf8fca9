// The failure semantics of the multi-device driver (skirt_sim_run_devices): the reference's Parallel::call
// stops every worker at the first exception and rethrows it in the parent (SKIRTcore/Parallel.cpp:181-193).
// Ranks that sum their tallies with collectives cannot simply stop: a peer already waiting in an all-reduce
// would wait for ever. So the ranks pass a gate before every collective. The gate opens when every rank has
// arrived; once any rank has failed it stays shut, and every rank waiting at it or arriving later gets
// `false` and enqueues no collective. The first failure's message is kept for the parent to report.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <string>

namespace skirt {

class RankGate {
public:
    explicit RankGate(int ranks) : n_(ranks < 1 ? 1 : ranks) {}

    // waits until every rank has arrived at this gate (true), or until some rank has failed (false)
    bool arrive() {
        std::unique_lock<std::mutex> lk(m_);
        if (failed_) return false;
        if (++count_ == n_) {
            count_ = 0;
            ++gen_;
            cv_.notify_all();
            return true;
        }
        const uint64_t g = gen_;
        cv_.wait(lk, [&] { return failed_ || gen_ != g; });
        // every rank arrived before the failure (the generation moved on): the collective goes ahead
        return gen_ != g;
    }

    // marks the job failed (the first call's message is kept) and releases every waiting rank;
    // returns true for the first failure
    bool fail(const std::string& msg) {
        std::lock_guard<std::mutex> lk(m_);
        const bool first = !failed_;
        if (first) msg_ = msg;
        failed_ = true;
        cv_.notify_all();
        return first;
    }

    bool failed() {
        std::lock_guard<std::mutex> lk(m_);
        return failed_;
    }

    std::string message() {
        std::lock_guard<std::mutex> lk(m_);
        return msg_;
    }

    int ranks() const { return n_; }

private:
    std::mutex m_;
    std::condition_variable cv_;
    const int n_;
    int count_ = 0;
    uint64_t gen_ = 0;
    bool failed_ = false;
    std::string msg_;
};

}  // namespace skirt
