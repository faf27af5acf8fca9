// FETCH_SIZE calibration for the trace kernel's access pattern. MI355X_MICROARCH.md calibrates FETCH_SIZE
// only for wide coalesced streaming reads (it reports half their bytes); the trace kernel's dominant
// loads are scattered 16-byte gathers (one leaf-map entry per lane, random lines). Each kernel below
// reads a known number of bytes; run under `rocprofv3 --pmc FETCH_SIZE` and divide FETCH_SIZE (KiB) x 1024
// by the printed byte count to get the factor bench.py's traffic figure uses.
//   streamKernel    16 B per lane, coalesced, every byte of the table once          (reference: 0.5)
//   gather16Kernel  16 B per lane at random 16-B-aligned slots: one 64-B line per lane (bytes = 64 per load)
//   gather8Kernel   8 B per lane at random 8-B slots: one 64-B line per lane (bytes = 64 per load)
// Tables of 1 GiB (beyond the 256 MiB Infinity Cache) and 32 MiB (the C3 leaf map, cache-resident).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/gather_bench tools/gather_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void streamKernel(const double2* t, size_t n, double* out) {
    double acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = t[i];
        acc += v.x + v.y;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename T>
__global__ void gatherKernel(const T* t, size_t n, int iters, unsigned seed, double* out) {
    unsigned x = (blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u + seed;
    double acc = 0;
    for (int i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        const T v = t[(size_t)x % n];
        if constexpr (sizeof(T) == 16) acc += v.x + v.y;
        else acc += v;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    const int blocks = 256 * 8, threads = 256, iters = 64;
    const size_t lanes = (size_t)blocks * threads;
    double* out;
    CHECK(hipMalloc(&out, lanes * sizeof(double)));
    for (size_t bytes : {(size_t)1 << 30, (size_t)32 << 20}) {
        void* t;
        CHECK(hipMalloc(&t, bytes));
        CHECK(hipMemset(t, 0, bytes));
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        float ms;
        // warm the table into whatever cache level holds it
        hipLaunchKernelGGL(streamKernel, dim3(blocks), dim3(threads), 0, 0, (const double2*)t, bytes / 16, out);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(streamKernel, dim3(blocks), dim3(threads), 0, 0, (const double2*)t, bytes / 16, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("streamKernel    table %5zu MiB  bytes %.6g  %.3f ms  %.0f GB/s\n", bytes >> 20, (double)bytes, ms,
               bytes / ms / 1e6);
        const double lines = (double)lanes * iters;
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL((gatherKernel<double2>), dim3(blocks), dim3(threads), 0, 0, (const double2*)t, bytes / 16,
                           iters, 1u, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("gather16 (16 B) table %5zu MiB  loads %.6g  lines x 64 B %.6g  %.3f ms  %.3g loads/s\n", bytes >> 20,
               lines, lines * 64, ms, lines / ms * 1e3);
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL((gatherKernel<double>), dim3(blocks), dim3(threads), 0, 0, (const double*)t, bytes / 8,
                           iters, 2u, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("gather8  (8 B)  table %5zu MiB  loads %.6g  lines x 64 B %.6g  %.3f ms  %.3g loads/s\n", bytes >> 20,
               lines, lines * 64, ms, lines / ms * 1e3);
        CHECK(hipFree(t));
    }
    CHECK(hipDeviceSynchronize());
    return 0;
}
