// Host check of skirt_amd/csrc/host/mt_random.hpp: the SSE2 refill and the batched words() against a plain
// one-word-at-a-time restatement of the reference's generator (Random.cpp:41-126: 69069 seeding, the 1998
// MT19937 genrand recurrence and tempering, deviates 0 and 1 rejected), over several seeds and request
// sizes that cross the 624-word refills at odd offsets. Also uniform() against words() + deviate().
//   g++ -O2 -std=c++17 -I skirt_amd/csrc/host tools/mt_check.cpp -o /tmp/mt_check && /tmp/mt_check
#include <cstdio>
#include <vector>

#include "mt_random.hpp"

namespace {
struct PlainMT {  // the reference's arithmetic on unsigned long, one word at a time
    unsigned long mt[624];
    int mti = 624;
    explicit PlainMT(unsigned long seed) {
        mt[0] = seed & 0xffffffffUL;
        for (mti = 1; mti < 624; mti++) mt[mti] = (69069 * mt[mti - 1]) & 0xffffffffUL;
    }
    unsigned long next() {
        static const unsigned long mag01[2] = {0x0UL, 0x9908b0dfUL};
        if (mti >= 624) {
            int kk;
            unsigned long y;
            for (kk = 0; kk < 227; kk++) {
                y = (mt[kk] & 0x80000000UL) | (mt[kk + 1] & 0x7fffffffUL);
                mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 0x1];
            }
            for (; kk < 623; kk++) {
                y = (mt[kk] & 0x80000000UL) | (mt[kk + 1] & 0x7fffffffUL);
                mt[kk] = mt[kk - 227] ^ (y >> 1) ^ mag01[y & 0x1];
            }
            y = (mt[623] & 0x80000000UL) | (mt[0] & 0x7fffffffUL);
            mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 0x1];
            mti = 0;
        }
        unsigned long y = mt[mti++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680UL;
        y ^= (y << 15) & 0xefc60000UL;
        y ^= (y >> 18);
        return y;
    }
    unsigned long word() {  // the next word uniform() accepts
        for (;;) {
            const unsigned long y = next();
            if (y != 0 && y != 0xffffffffUL) return y;
        }
    }
};
}  // namespace

int main() {
    long bad = 0, checked = 0;
    // (seed 0 seeds an all-zero state: every word is 0 and rejected; skirt_sim_load refuses it)
    const unsigned long seeds[] = {4357, 1, 123456789, 0xffffffffUL, 0x100000001UL};
    const size_t sizes[] = {1, 3, 7, 623, 624, 625, 1000, 4095, 100003};
    for (unsigned long seed : seeds) {
        skirt::MTRandom fast(seed);
        skirt::MTRandom slow(seed);
        PlainMT plain(seed);
        std::vector<uint32_t> w;
        for (int rep = 0; rep < 3; rep++)
            for (size_t n : sizes) {
                w.assign(n, 0);
                fast.words(w.data(), n);
                for (size_t i = 0; i < n; i++) {
                    const unsigned long ref = plain.word();
                    const double u = slow.uniform();
                    checked++;
                    if (w[i] != (uint32_t)ref || u != skirt::MTRandom::deviate(w[i])) bad++;
                }
            }
    }
    std::printf("mt_check: %ld words checked, %ld mismatches\n", checked, bad);
    return bad ? 1 : 0;
}
