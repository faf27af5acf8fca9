// Counter-based per-packet random numbers for the photon engine.
//
// The reference draws from one MT19937 stream per thread (SKIRTcore/Random.cpp:89-126), which makes a
// packet's random numbers depend on thread scheduling. Here every photon packet owns an independent
// Philox4x32-10 stream (Salmon et al. 2011) so that results depend only on (seed, phase tag, global
// packet index) -- not on the GPU count, the kernel geometry or the lane that happens to run it:
//   key     = (seed mod 2^32, seed / 2^32)
//   counter = (block, tag, packet mod 2^32, packet / 2^32), block = 0, 1, 2, ...
// Each block gives four 32-bit words; a uniform deviate takes two of them, a then b, as the 53-bit
// integer (a>>5)*2^26 + (b>>6) mapped to ((x + 0.5) * 2^-53), strictly inside (0,1) like the reference's
// uniform() which rejects 0 and 1.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace skirt_dev {

struct PacketRng {
    uint32_t k0, k1;     // key
    uint32_t tag;
    uint32_t plo, phi;   // packet index
    uint32_t block;
    uint32_t w2, w3;     // cached second half of the last block
    uint32_t have;       // 0 or 2 cached words

    __host__ __device__ inline void start(uint64_t seed, uint32_t t, uint64_t packet) {
        k0 = (uint32_t)seed;
        k1 = (uint32_t)(seed >> 32);
        tag = t;
        plo = (uint32_t)packet;
        phi = (uint32_t)(packet >> 32);
        block = 0;
        have = 0;
    }

    __host__ __device__ static inline void philox(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                                  uint32_t key0, uint32_t key1) {
#pragma unroll
        for (int r = 0; r < 10; r++) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
            const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ key0;
            const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ key1;
            c1 = (uint32_t)p1;
            c3 = (uint32_t)p0;
            c0 = n0;
            c2 = n2;
            key0 += 0x9E3779B9u;
            key1 += 0xBB67AE85u;
        }
    }

    __host__ __device__ inline double uniform() {
        uint32_t a, b;
        if (have) {
            a = w2;
            b = w3;
            have = 0;
        } else {
            uint32_t c0 = block++, c1 = tag, c2 = plo, c3 = phi;
            philox(c0, c1, c2, c3, k0, k1);
            a = c0;
            b = c1;
            w2 = c2;
            w3 = c3;
            have = 2;
        }
        const uint64_t x = ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
        return ((double)x + 0.5) * (1.0 / 9007199254740992.0);
    }
};

}  // namespace skirt_dev
