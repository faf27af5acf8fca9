// Host-side Mersenne-twister uniform deviates, used only during model SETUP (cell density sampling and
// octree subdivision sampling), so that the product's setup consumes random numbers exactly like the
// reference's and yields identical cell densities and trees.
//
// Restates SKIRTcore/Random.cpp: seeding with the 69069 linear congruential generator
// (Random.cpp:41-56), the 1998 MT19937 genrand recurrence and tempering, and the rejection of exactly 0
// and 1 (Random.cpp:89-126); position(box) draws x, y, z in that order (Random.cpp:226-234).
// The photon-shooting hot path on the GPU uses Philox (see device/philox.hpp), not this generator.
#pragma once

#include <emmintrin.h>

#include <algorithm>
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
    // words it rejects (0 and 0xffffffff, the deviates 0 and 1) are skipped here as there. A round tempers
    // at most as many state words as outputs are still wanted (each yields at most one), four at a time
    // (SSE2), so the sequence is the one-at-a-time sequence.
    void words(uint32_t* out, size_t n) {
        for (size_t q = 0; q < n;) {
            if (mti_ >= 624) refill_();
            const int take = (int)std::min<size_t>((size_t)(624 - mti_), n - q);
            uint32_t* o = out + q;
            int i = 0;
            __m128i bad = _mm_setzero_si128();
            const __m128i ones = _mm_set1_epi32(-1);
            for (; i + 4 <= take; i += 4) {
                const __m128i y = temper4_(_mm_loadu_si128(reinterpret_cast<const __m128i*>(mt_ + mti_ + i)));
                _mm_storeu_si128(reinterpret_cast<__m128i*>(o + i), y);
                bad = _mm_or_si128(bad, _mm_or_si128(_mm_cmpeq_epi32(y, _mm_setzero_si128()), _mm_cmpeq_epi32(y, ones)));
            }
            for (; i < take; i++) {
                o[i] = temper_(mt_[mti_ + i]);
                if (o[i] == 0u || o[i] == 0xffffffffu) bad = ones;
            }
            mti_ += take;
            if (_mm_movemask_epi8(bad) == 0) {
                q += take;
            } else {  // a rejected word (probability 2^-31 per word): compact the round
                size_t k = q;
                for (int j = 0; j < take; j++)
                    if (o[j] != 0u && o[j] != 0xffffffffu) out[k++] = o[j];
                q = k;
            }
        }
    }
    static double deviate(uint32_t y) { return static_cast<double>(y) / static_cast<unsigned long>(0xffffffffUL); }

    double uniform() override {
        double ans;
        do {
            if (mti_ >= 624) refill_();
            const uint32_t y = temper_(mt_[mti_++]);
            ans = static_cast<double>(y) / static_cast<unsigned long>(0xffffffffUL);
        } while (ans <= 0.0 || ans >= 1.0);
        return ans;
    }

private:
    // 32-bit state words: the reference's unsigned long arithmetic masked to 32 bits (Random.cpp:41-126)
    uint32_t mt_[624];
    int mti_ = 624;

    static __m128i temper4_(__m128i y) {
        y = _mm_xor_si128(y, _mm_srli_epi32(y, 11));
        y = _mm_xor_si128(y, _mm_and_si128(_mm_slli_epi32(y, 7), _mm_set1_epi32((int)0x9d2c5680u)));
        y = _mm_xor_si128(y, _mm_and_si128(_mm_slli_epi32(y, 15), _mm_set1_epi32((int)0xefc60000u)));
        return _mm_xor_si128(y, _mm_srli_epi32(y, 18));
    }
    static uint32_t temper_(uint32_t y) {
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }

    void seed_(unsigned long seed) {
        mt_[0] = (uint32_t)(seed & 0xffffffffUL);
        for (mti_ = 1; mti_ < 624; mti_++) mt_[mti_] = 69069u * mt_[mti_ - 1];
    }

    // the genrand recurrence; mag01[y & 1] as a mask
    static uint32_t twist_(uint32_t a, uint32_t b, uint32_t c) {
        const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
        return c ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
    static __m128i twist4_(__m128i a, __m128i b, __m128i c) {
        const __m128i y = _mm_or_si128(_mm_and_si128(a, _mm_set1_epi32((int)0x80000000u)),
                                       _mm_and_si128(b, _mm_set1_epi32(0x7fffffff)));
        const __m128i odd = _mm_sub_epi32(_mm_setzero_si128(), _mm_and_si128(y, _mm_set1_epi32(1)));
        return _mm_xor_si128(_mm_xor_si128(c, _mm_srli_epi32(y, 1)), _mm_and_si128(odd, _mm_set1_epi32((int)0x9908b0dfu)));
    }
    // four words at a time: word kk reads words kk+1 (not yet updated) and kk+397 (old) or kk-227 (updated
    // earlier in this refill), so each group of four loads its operands before it stores
    void refill_() {
        auto ld = [&](int k) { return _mm_loadu_si128(reinterpret_cast<const __m128i*>(mt_ + k)); };
        for (int kk = 0; kk < 224; kk += 4)  // words 0..226: 56 groups and 3 single words
            _mm_storeu_si128(reinterpret_cast<__m128i*>(mt_ + kk), twist4_(ld(kk), ld(kk + 1), ld(kk + 397)));
        for (int kk = 224; kk < 227; kk++) mt_[kk] = twist_(mt_[kk], mt_[kk + 1], mt_[kk + 397]);
        for (int kk = 227; kk < 623; kk += 4)  // words 227..622: 99 groups
            _mm_storeu_si128(reinterpret_cast<__m128i*>(mt_ + kk), twist4_(ld(kk), ld(kk + 1), ld(kk - 227)));
        mt_[623] = twist_(mt_[623], mt_[0], mt_[396]);
        mti_ = 0;
    }
};

}  // namespace skirt
