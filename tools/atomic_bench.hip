// Microbenchmark for the Labs tally: scattered 8-byte atomic adds (one random address per lane, the
// trace kernel's pattern) in several instruction flavours, and plain scattered stores for comparison.
// Build: hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics -o tools/atomic_bench tools/atomic_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int KIND>
__global__ void kAdd(double* buf, size_t n, int iters, unsigned seed) {
    unsigned x = (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u + seed;
    for (int i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        double* p = buf + (x % n);
        if (KIND == 0) {
            __hip_atomic_fetch_add((__attribute__((address_space(1))) double*)p, 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (KIND == 1) {
            double v = 1.0;
            asm volatile("global_atomic_add_f64 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
        } else if (KIND == 2) {
            double v = 1.0;
            asm volatile("global_atomic_add_f64 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
        } else if (KIND == 3) {
            __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned long long*)p, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (KIND == 4) {
            __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned long long*)p, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            *p = 1.0;
        }
    }
    if (KIND == 1 || KIND == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main() {
    const int blocks = 256 * 8, threads = 256, iters = 64;
    const double total = (double)blocks * threads * iters;
    const size_t n = (size_t)1 << 24;  // 128 MiB of doubles, about the C3 Labs table
    double* buf;
    CHECK(hipMalloc(&buf, n * 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char* names[] = {"f64 atomic (agent)", "f64 atomic nt", "f64 atomic sc1", "u64 atomic (agent)",
                           "u64 atomic (workgroup)", "plain 8-B store"};
    for (int kind = 0; kind < 6; kind++) {
        CHECK(hipMemset(buf, 0, n * 8));
        float best = 1e9;
        for (int rep = 0; rep < 3; rep++) {
            CHECK(hipEventRecord(e0));
            switch (kind) {
            case 0: kAdd<0><<<blocks, threads>>>(buf, n, iters, rep); break;
            case 1: kAdd<1><<<blocks, threads>>>(buf, n, iters, rep); break;
            case 2: kAdd<2><<<blocks, threads>>>(buf, n, iters, rep); break;
            case 3: kAdd<3><<<blocks, threads>>>(buf, n, iters, rep); break;
            case 4: kAdd<4><<<blocks, threads>>>(buf, n, iters, rep); break;
            default: kAdd<5><<<blocks, threads>>>(buf, n, iters, rep); break;
            }
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        std::vector<double> h(n);
        CHECK(hipMemcpy(h.data(), buf, n * 8, hipMemcpyDeviceToHost));
        double sum = 0;
        for (size_t q = 0; q < n; q++) sum += (kind == 3 || kind == 4) ? (double)reinterpret_cast<unsigned long long&>(h[q]) : h[q];
        printf("%-24s %8.3f ms  %.3g adds/s  sum/expected %.6f\n", names[kind], best, total / (best * 1e-3),
               kind < 5 ? sum / (3 * total) : 0.0);
    }
    return 0;
}
