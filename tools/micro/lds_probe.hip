// LDS access-pattern probe (diagnostics, not product code): throughput of the
// random table reads and histogram atomics the FSE kernels are built from,
// in lane-operations per cycle per CU (clock from s_memtime over the launch).
//   gather_u32    x = tab32[x]           (decode table reads, ds_read_b32)
//   gather_u16    x = tab16[x]           (encoder stateTable reads, ds_read_u16)
//   gather_b64    x = tab64[x >> 1].half (the same table read 8 bytes wide)
//   gather_u16_16 x = tab16[x], 16-bank half-tables by lane bit 4
//   hist_cur      ds_add_u32 in the encoder's histogram layout (16 copies, 16-bit halves)
//   hist_lane     ds_add_u32, one private 8-bit-counter column per lane (bank = lane)
//   bperm2        two ds_bpermute_b32 per step from 64-entry register tables
//                 (the symbol transforms of a block with <= 64 symbols held in
//                 two VGPRs instead of an LDS array: dNB and dFS)
// Byte values for the histograms: geometric p = 1/2 (skewed) or uniform.
// Build: hipcc -O3 --offload-arch=gfx950 lds_probe.hip -o lds_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int STEPS = 2048;
constexpr int C = 4;  // independent chains per lane

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    return x;
}

template <int V>
__global__ __launch_bounds__(256) void probe(const uint32_t* __restrict__ init, const uint8_t* __restrict__ lut,
                                             uint32_t* out, uint64_t* clk) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[2048 * 4];  // 32 KiB
    for (uint32_t i = threadIdx.x; i < 2048 * 4; i += blockDim.x) tab[i] = (V >= 4) ? 0u : init[i & 2047];
    __syncthreads();
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = mix(threadIdx.x * 7919u + c * 104729u + blockIdx.x * 31u);
    uint32_t acc = 0;
    if (V == 0) {
        for (int s = 0; s < STEPS; ++s)
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = tab[x[c] & 2047u];
    } else if (V == 1) {
        const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tab);
        for (int s = 0; s < STEPS; ++s)
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = t16[x[c] & 2047u] ^ (x[c] >> 11);
    } else if (V == 2) {
        const uint2* t64 = reinterpret_cast<const uint2*>(tab);
        for (int s = 0; s < STEPS; ++s)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const uint2 v = t64[(x[c] & 2047u) >> 1];
                x[c] = (x[c] & 1u) ? v.y : v.x;
            }
    } else if (V == 3) {
        // 16-bank half tables: lanes with bit 4 clear read banks 0-15, set read 16-31
        const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tab);
        const uint32_t half = (lane >> 4) & 1u;
        for (int s = 0; s < STEPS; ++s)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const uint32_t i = x[c] & 2047u;  // entry i: word (i / 2) -> row (i / 32), bank (i / 2) % 16
                const uint32_t w = ((i >> 5) << 5) + half * 16u + ((i >> 1) & 15u);
                x[c] = t16[2u * w + (i & 1u)] ^ (x[c] >> 11);
            }
    } else if (V == 6) {
        const uint32_t r0 = init[lane], r1 = init[64 + lane];  // two 64-entry register tables
        for (int s = 0; s < STEPS; ++s)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int a = (int)((x[c] & 63u) << 2);
                const uint32_t u = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)r0);
                const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)r1);
                x[c] = u ^ (v >> 3);
            }
    } else if (V == 4 || V == 5) {
        uint32_t r = mix(threadIdx.x + blockIdx.x * 256u);
        for (int s = 0; s < STEPS; ++s)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                r = r * 1664525u + 1013904223u;
                // bytes from registers (a table read would add an LDS / memory op per add):
                // lut != nullptr -> geometric p = 1/2 (skewed, like C2's head), else uniform
                const uint32_t b = lut ? (uint32_t)__clz(r | 1u) : (r >> 24);
                if (V == 4) {
                    // encoder layout: 16 copies bin-major, 16-bit halves: word b * 8 + ((lane >> 1) & 7)
                    __hip_atomic_fetch_add(&tab[b * 8u + ((lane >> 1) & 7u) + 2048u * (threadIdx.x >> 6)],
                                           1u << (16u * (lane & 1u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {
                    // one 8-bit column per lane: word (b >> 2) * 64 + lane, byte b & 3 (bank = lane)
                    __hip_atomic_fetch_add(&tab[(b >> 2) * 64u + lane + 0u * (threadIdx.x >> 6)], 1u << (8u * (b & 3u)),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        __syncthreads();
        acc = tab[threadIdx.x];
    }
#pragma unroll
    for (int c = 0; c < C; ++c) acc += x[c];
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (acc == 0x12345u) out[0] = acc;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int V>
void run(const char* name, const uint32_t* d_init, const uint8_t* d_lut, uint32_t* d_out, uint64_t* d_clk, int wg_per_cu) {
    const int cus = 256, grid = cus * wg_per_cu;
    hipLaunchKernelGGL(probe<V>, dim3(grid), dim3(256), 0, 0, d_init, d_lut, d_out, d_clk);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(probe<V>, dim3(grid), dim3(256), 0, 0, d_init, d_lut, d_out, d_clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    uint64_t* h = new uint64_t[grid];
    hipMemcpy(h, d_clk, grid * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < grid; ++i) mean += (double)h[i];
    mean /= grid;
    delete[] h;
    // lane-ops per cycle per CU: every WG's ops over its mean in-kernel cycles x WGs per CU resident
    const double ops_wg = 256.0 * C * STEPS;
    printf("%-14s wg/cu=%d  %.3f ms  cycles/wg %.0f  lane-ops/cycle/CU %.2f  (wave-instr cycles %.2f)\n", name, wg_per_cu,
           ms, mean, ops_wg * wg_per_cu / mean, 64.0 / (ops_wg * wg_per_cu / mean));
}

int main() {
    uint32_t h[2048];
    for (int i = 0; i < 2048; ++i) {
        uint32_t z = (uint32_t)i * 0x9E3779B9u + 12345u;
        h[i] = ((z ^ (z >> 13)) * 0x85ebca6bu);
    }
    uint8_t lut[2][4096];
    {  // LUT generator p = 0.155 (C2) and uniform
        size_t remaining = 4096, idx = 0;
        uint32_t s = 0;
        while (remaining > 0) {
            size_t cnt = (size_t)((double)remaining * 0.155);
            if (cnt < 1) cnt = 1;
            for (size_t k = 0; k < cnt; ++k) lut[0][idx + k] = (uint8_t)s;
            idx += cnt;
            remaining -= cnt;
            ++s;
        }
        for (int i = 0; i < 4096; ++i) lut[1][i] = (uint8_t)(i * 251 >> 4);
    }
    uint32_t *d_init, *d_out;
    uint8_t* d_lut;
    uint64_t* d_clk;
    hipMalloc(&d_init, sizeof h);
    hipMalloc(&d_out, 64);
    hipMalloc(&d_lut, sizeof lut);
    hipMalloc(&d_clk, 256 * 8 * 8);
    hipMemcpy(d_init, h, sizeof h, hipMemcpyHostToDevice);
    hipMemcpy(d_lut, lut, sizeof lut, hipMemcpyHostToDevice);
    for (int w : {2, 4}) {
        run<0>("gather_u32", d_init, d_lut, d_out, d_clk, w);
        run<1>("gather_u16", d_init, d_lut, d_out, d_clk, w);
        run<2>("gather_b64", d_init, d_lut, d_out, d_clk, w);
        run<3>("gather_u16_16", d_init, d_lut, d_out, d_clk, w);
        run<6>("bperm2", d_init, d_lut, d_out, d_clk, w);
        run<4>("hist_cur_geo", d_init, d_lut, d_out, d_clk, w);
        run<5>("hist_lane_geo", d_init, d_lut, d_out, d_clk, w);
        run<4>("hist_cur_uni", d_init, nullptr, d_out, d_clk, w);
        run<5>("hist_lane_uni", d_init, nullptr, d_out, d_clk, w);
    }
    return 0;
}
