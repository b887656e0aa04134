// LDS random-gather ceiling (diagnostics): lanes walk C independent chains
// x = tab[x] through an 8 KiB table of random u32 indices (the decode
// table's size and access pattern), at several workgroup sizes.  Reports
// lane-lookups per cycle per CU -- the roof for tANS table lookups.
// Build: hipcc -O3 --offload-arch=gfx950 lds_gather.hip -o lds_gather
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int C>
__global__ void gather_kernel(const uint32_t* __restrict__ init, uint32_t* out, int steps, uint32_t mask) {
    __shared__ uint32_t tab[2048];
    for (uint32_t i = threadIdx.x; i < 2048; i += blockDim.x) tab[i] = init[i];
    __syncthreads();
    uint32_t x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = (threadIdx.x * 7919u + c * 104729u + blockIdx.x * 31u) & mask;
    for (int s = 0; s < steps; ++s) {
#pragma unroll
        for (int c = 0; c < C; ++c) x[c] = tab[x[c]] & mask;
    }
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) acc += x[c];
    if (acc == 0xFFFFFFFFu) out[0] = acc;
}

template <int C>
void run(const uint32_t* d_init, uint32_t* d_out, int threads, int wgs_per_cu) {
    const int cus = 256, steps = 4096;
    const int grid = cus * wgs_per_cu * 4;  // several rounds
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(gather_kernel<C>, dim3(grid), dim3(threads), 0, 0, d_init, d_out, 64, 2047u);
    hipDeviceSynchronize();
    hipEventRecord(a);
    hipLaunchKernelGGL(gather_kernel<C>, dim3(grid), dim3(threads), 0, 0, d_init, d_out, steps, 2047u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lookups = (double)grid * threads * C * steps;
    const double clk = 2.3e9;
    printf("chains=%d threads=%4d grid=%6d  %.3f ms  %.2f lane-lookups/cycle/CU (at %.1f GHz)\n", C, threads, grid,
           ms, lookups / (ms * 1e-3 * clk) / cus, clk / 1e9);
}

int main() {
    uint32_t h[2048];
    uint64_t z = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 2048; ++i) {
        z += 0x9E3779B97F4A7C15ull;
        uint64_t y = z;
        y = (y ^ (y >> 30)) * 0xBF58476D1CE4E5B9ull;
        y = (y ^ (y >> 27)) * 0x94D049BB133111EBull;
        h[i] = (uint32_t)(y ^ (y >> 31));
    }
    uint32_t *d_init, *d_out;
    hipMalloc(&d_init, sizeof h);
    hipMalloc(&d_out, 64);
    hipMemcpy(d_init, h, sizeof h, hipMemcpyHostToDevice);
    for (int threads : {256, 512, 1024}) {
        run<1>(d_init, d_out, threads, 4);
        run<2>(d_init, d_out, threads, 4);
        run<4>(d_init, d_out, threads, 4);
        run<8>(d_init, d_out, threads, 4);
    }
    return 0;
}
