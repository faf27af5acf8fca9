// Microbenchmark, second set: what a 64-byte atomic request costs when several lanes of one wave
// instruction add into the same line, whether the Labs footprint matters, returning reservation
// atomics on a few counters (a bucketed add log), LDS f64 atomics and 16-byte record stores in runs.
// Build: hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics -o tools/atomic_bench2 tools/atomic_bench2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ void gadd(double* p, double v) {
    __hip_atomic_fetch_add((__attribute__((address_space(1))) double*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// K consecutive lanes add into the same 64-byte line (K distinct doubles of it)
template <int K>
__global__ void kLine(double* buf, size_t nlines, int iters, unsigned seed) {
    const int lane = threadIdx.x & 63;
    unsigned x = ((blockIdx.x * blockDim.x + threadIdx.x) / K) * 2654435761u + seed;
    for (int i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        gadd(buf + (size_t)(x % nlines) * 8 + (lane % K) * (8 / K), 1.0);
    }
}

// returning atomics on nb counters (a bucket reservation per lane)
__global__ void kReserve(unsigned* cnt, int nb, int iters, unsigned seed, unsigned* sink) {
    unsigned x = (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u + seed;
    unsigned acc = 0;
    for (int i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        acc += atomicAdd(cnt + (x % nb) * 16, 8u);
    }
    if (acc == 0xdeadbeef) sink[0] = acc;
}

// LDS f64 atomics over a 64 KB table
__global__ void kLds(double* out, int iters, unsigned seed) {
    __shared__ double t[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) t[i] = 0;
    __syncthreads();
    unsigned x = (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u + seed;
    for (int i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        atomicAdd(&t[x & 8191], 1.0);
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = t[seed & 8191];
}

// 16-byte records stored in runs of R consecutive lanes at random positions
template <int R>
__global__ void kRec(double2* buf, size_t nrec, int iters, unsigned seed) {
    const int lane = threadIdx.x & 63;
    unsigned x = ((blockIdx.x * blockDim.x + threadIdx.x) / R) * 2654435761u + seed;
    for (int i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        buf[(size_t)(x % (nrec / R)) * R + lane % R] = make_double2((double)i, 1.0);
    }
}

int main() {
    const int blocks = 256 * 8, threads = 256, iters = 64;
    const double total = (double)blocks * threads * iters;
    const size_t n = (size_t)1 << 24;  // 128 MiB of doubles
    double* buf;
    unsigned* cnt;
    CHECK(hipMalloc(&buf, n * 8 * 2));
    CHECK(hipMalloc(&cnt, 1 << 20));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch) {
        float best = 1e9;
        for (int rep = 0; rep < 3; rep++) {
            (void)hipEventRecord(e0);
            launch(rep);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("%-44s %8.3f ms  %.3g ops/s\n", name, best, total / (best * 1e-3));
    };
    CHECK(hipMemset(buf, 0, n * 8));
    for (size_t lines : {(size_t)1 << 21, (size_t)655360 / 8, (size_t)1 << 13}) {
        char nm[96];
        snprintf(nm, sizeof nm, "f64 add, 1 lane/line, %6.1f MB", lines * 64 / 1e6);
        timeit(nm, [&](int r) { kLine<1><<<blocks, threads>>>(buf, lines, iters, r); });
        snprintf(nm, sizeof nm, "f64 add, 2 lanes/line, %6.1f MB", lines * 64 / 1e6);
        timeit(nm, [&](int r) { kLine<2><<<blocks, threads>>>(buf, lines, iters, r); });
        snprintf(nm, sizeof nm, "f64 add, 4 lanes/line, %6.1f MB", lines * 64 / 1e6);
        timeit(nm, [&](int r) { kLine<4><<<blocks, threads>>>(buf, lines, iters, r); });
        snprintf(nm, sizeof nm, "f64 add, 8 lanes/line, %6.1f MB", lines * 64 / 1e6);
        timeit(nm, [&](int r) { kLine<8><<<blocks, threads>>>(buf, lines, iters, r); });
    }
    for (int nb : {152, 1024, 16384}) {
        char nm[96];
        CHECK(hipMemset(cnt, 0, 1 << 20));
        snprintf(nm, sizeof nm, "u32 returning add, %d counters", nb);
        timeit(nm, [&](int r) { kReserve<<<blocks, threads>>>(cnt, nb, iters, r, cnt); });
    }
    timeit("LDS f64 atomic add, 64 KB table", [&](int r) { kLds<<<blocks, threads>>>(buf, iters, r); });
    double2* rec = reinterpret_cast<double2*>(buf);
    const size_t nrec = n;  // 256 MiB of records
    timeit("16-B record store, runs of 1", [&](int r) { kRec<1><<<blocks, threads>>>(rec, nrec, iters, r); });
    timeit("16-B record store, runs of 4", [&](int r) { kRec<4><<<blocks, threads>>>(rec, nrec, iters, r); });
    timeit("16-B record store, runs of 8", [&](int r) { kRec<8><<<blocks, threads>>>(rec, nrec, iters, r); });
    timeit("16-B record store, runs of 16", [&](int r) { kRec<16><<<blocks, threads>>>(rec, nrec, iters, r); });
    return 0;
}
