// CPU check of skirt_amd/csrc/host/rank_gate.hpp (tests/test_rank_gate.py): the gate the device threads of
// skirt_sim_run_devices pass before every all-reduce. Prints one line per rank: the results of its arrivals.
//   rank_gate_check RANKS COLLECTIVES FAIL_RANK FAIL_AFTER
// rank FAIL_RANK fails after FAIL_AFTER collectives (-1: nobody fails); every other rank arrives COLLECTIVES
// times or until the gate refuses it.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../skirt_amd/csrc/host/rank_gate.hpp"

int main(int argc, char** argv) {
    if (argc != 5) return 2;
    const int n = atoi(argv[1]), colls = atoi(argv[2]), failRank = atoi(argv[3]), failAfter = atoi(argv[4]);
    skirt::RankGate gate(n);
    std::vector<std::string> log(n);
    std::vector<std::thread> th;
    for (int r = 0; r < n; r++)
        th.emplace_back([&, r] {
            for (int c = 0; c < colls; c++) {
                if (r == failRank && c == failAfter) {
                    gate.fail("rank " + std::to_string(r) + " failed");
                    log[r] += "F";
                    return;
                }
                // a little work between collectives, different per rank
                std::this_thread::sleep_for(std::chrono::microseconds(200 * ((r * 7 + c) % 5)));
                const bool ok = gate.arrive();
                log[r] += ok ? "1" : "0";
                if (!ok) return;
            }
        });
    for (auto& t : th) t.join();
    for (int r = 0; r < n; r++) std::printf("%d %s\n", r, log[r].c_str());
    std::printf("failed %d %s\n", gate.failed() ? 1 : 0, gate.message().c_str());
    return 0;
}
