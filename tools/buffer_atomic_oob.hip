// Does MI355X drop an out-of-range buffer_atomic_add_f64 (raw buffer, offset >= num_records)? The trace
// kernel's Labs drain relies on it to issue its atomics unconditionally (every lane, the empty ones out of
// range), so the compiler's waitcnt pass sees a fixed number of vector-memory operations per step. The test
// keeps every access inside its own allocation: num_records covers the first N doubles, the out-of-range
// offsets point into a guard region behind them, which must stay zero.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/boob tools/buffer_atomic_oob.hip && /tmp/boob
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ double buf_atomic_add_f64(double v, __amdgpu_buffer_rsrc_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.ptr.buffer.atomic.fadd.f64");

__global__ void k(double* p, unsigned n, int iters) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, 0, n * 8u, 0x00020000);
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int it = 0; it < iters; it++) {
        // even lanes: in range (element i mod n); odd lanes: out of range, into the guard behind the table
        const unsigned off = (i & 1u) ? (n + (i % 64u)) * 8u : (i % n) * 8u;
        buf_atomic_add_f64(1.0, r, (int)off, 0, 0);
    }
}

int main() {
    const unsigned n = 1024, guard = 128;
    const int blocks = 256, threads = 256, iters = 16;
    double* d = nullptr;
    if (hipMalloc(&d, (n + guard) * sizeof(double)) != hipSuccess) return 2;
    hipMemset(d, 0, (n + guard) * sizeof(double));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, n, iters);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
    std::vector<double> h(n + guard);
    hipMemcpy(h.data(), d, h.size() * sizeof(double), hipMemcpyDeviceToHost);
    double in = 0, out = 0;
    for (unsigned q = 0; q < n; q++) in += h[q];
    for (unsigned q = n; q < n + guard; q++) out += h[q];
    const double expect = (double)blocks * threads / 2 * iters;
    printf("in-range sum %.0f (expected %.0f), guard sum %.0f (expected 0): %s\n", in, expect, out,
           (in == expect && out == 0) ? "out-of-range buffer atomics are dropped" : "NOT DROPPED");
    hipFree(d);
    return (in == expect && out == 0) ? 0 : 1;
}
