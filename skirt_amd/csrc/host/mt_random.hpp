// Host-side Mersenne-twister uniform deviates, used only during model SETUP (cell density sampling and
// octree subdivision sampling), so that the product's setup consumes random numbers exactly like the
// reference's and yields identical cell densities and trees.
//
// Restates SKIRTcore/Random.cpp: seeding with the 69069 linear congruential generator
// (Random.cpp:41-56), the 1998 MT19937 genrand recurrence and tempering, and the rejection of exactly 0
// and 1 (Random.cpp:89-126); position(box) draws x, y, z in that order (Random.cpp:226-234).
// The photon-shooting hot path on the GPU uses Philox (see device/philox.hpp), not this generator.
#pragma once

#include <cstddef>
#include <cstdint>

namespace skirt {

class UniformSource {
public:
    virtual ~UniformSource() = default;
    virtual double uniform() = 0;
};

class MTRandom final : public UniformSource {
public:
    explicit MTRandom(unsigned long seed = 4357) { seed_(seed); }

    // the tempered 32-bit outputs behind the next n deviates: uniform() == word / 0xffffffff, and the
    // words it rejects (0 and 0xffffffff, the deviates 0 and 1) are skipped here as there
    void words(uint32_t* out, size_t n) {
        for (size_t q = 0; q < n;) {
            if (mti_ >= 624) refill_();
            unsigned long y = mt_[mti_++];
            y ^= (y >> 11);
            y ^= (y << 7) & 0x9d2c5680UL;
            y ^= (y << 15) & 0xefc60000UL;
            y ^= (y >> 18);
            if (y != 0 && y != 0xffffffffUL) out[q++] = (uint32_t)y;
        }
    }
    static double deviate(uint32_t y) { return static_cast<double>(y) / static_cast<unsigned long>(0xffffffffUL); }

    double uniform() override {
        double ans;
        do {
            unsigned long y;
            if (mti_ >= 624) refill_();
            y = mt_[mti_++];
            y ^= (y >> 11);
            y ^= (y << 7) & 0x9d2c5680UL;
            y ^= (y << 15) & 0xefc60000UL;
            y ^= (y >> 18);
            ans = static_cast<double>(y) / static_cast<unsigned long>(0xffffffffUL);
        } while (ans <= 0.0 || ans >= 1.0);
        return ans;
    }

private:
    unsigned long mt_[624];
    int mti_ = 624;

    void seed_(unsigned long seed) {
        mt_[0] = seed & 0xffffffffUL;
        for (mti_ = 1; mti_ < 624; mti_++) mt_[mti_] = (69069 * mt_[mti_ - 1]) & 0xffffffffUL;
    }

    void refill_() {
        static const unsigned long mag01[2] = {0x0UL, 0x9908b0dfUL};
        unsigned long y;
        int kk;
        for (kk = 0; kk < 227; kk++) {
            y = (mt_[kk] & 0x80000000UL) | (mt_[kk + 1] & 0x7fffffffUL);
            mt_[kk] = mt_[kk + 397] ^ (y >> 1) ^ mag01[y & 0x1];
        }
        for (; kk < 623; kk++) {
            y = (mt_[kk] & 0x80000000UL) | (mt_[kk + 1] & 0x7fffffffUL);
            mt_[kk] = mt_[kk - 227] ^ (y >> 1) ^ mag01[y & 0x1];
        }
        y = (mt_[623] & 0x80000000UL) | (mt_[0] & 0x7fffffffUL);
        mt_[623] = mt_[396] ^ (y >> 1) ^ mag01[y & 0x1];
        mti_ = 0;
    }
};

}  // namespace skirt
