// Serial-chain latency probe (diagnostics): cycles per dependent table
// lookup x = T[x] for one wave-uniform chain (the single-stream decode's
// critical path), with the 2048-entry table
//   lds    in LDS, uniform address (ds_read_b32 + v_readfirstlane)
//   vgpr   in 32 VGPRs x 64 lanes, read by a uniform dynamic index (movrel)
//          + v_readlane
//   smem   in global memory through the scalar cache (s_load_dword)
// plus "lds2": two independent chains interleaved (the 2-state decoder).
// Build: hipcc -O3 --offload-arch=gfx950 chain_probe.hip -o chain_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int STEPS = 1 << 20;

typedef __attribute__((address_space(4))) const uint32_t cst_u32;

template <int V>
__global__ __launch_bounds__(64) void chain(const uint32_t* __restrict__ tab_g, uint32_t* out, uint64_t* clk) {
    __shared__ uint32_t tab[2048];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 2048; i += 64) tab[i] = tab_g[i];
    uint32_t vt[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) vt[k] = tab_g[k * 64 + lane];
    __syncthreads();
    uint32_t x = 7u, y = 1234u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (V == 0) {
        for (int s = 0; s < STEPS; ++s) x = __builtin_amdgcn_readfirstlane(tab[x & 2047u]);
    } else if (V == 1) {
        for (int s = 0; s < STEPS; ++s) {
            const uint32_t i = x & 2047u;
            x = __builtin_amdgcn_readlane(vt[i >> 6], i & 63u);
        }
    } else if (V == 2) {
        cst_u32* tc = (cst_u32*)tab_g;
        for (int s = 0; s < STEPS; ++s) x = tc[x & 2047u];
    } else if (V == 3) {
        for (int s = 0; s < STEPS; ++s) {
            const uint32_t a = tab[x & 2047u], b = tab[y & 2047u];
            x = __builtin_amdgcn_readfirstlane(a) + (y >> 3);
            y = __builtin_amdgcn_readfirstlane(b) ^ (x >> 5);
        }
    } else if (V == 4) {
        for (int s = 0; s < STEPS; ++s) {
            const uint32_t i = x & 2047u, j = y & 2047u;
            const uint32_t a = __builtin_amdgcn_readlane(vt[i >> 6], i & 63u);
            const uint32_t b = __builtin_amdgcn_readlane(vt[j >> 6], j & 63u);
            x = a + (y >> 3);
            y = b ^ (x >> 5);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[blockIdx.x] = x + y;
        clk[blockIdx.x] = t1 - t0;
    }
}


// Issue-rate probe for one lone wave: 8 independent or 1 dependent chain of
// SALU (s_add / s_xor) or VALU (v_add / v_xor) per step.
template <int V>
__global__ __launch_bounds__(64) void issue(uint32_t* out, uint64_t* clk, uint32_t seed) {
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = seed * (i + 3);
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * (i + 5) + seed;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < STEPS / 8; ++s) {
        if (V == 0) {  // 8 independent SALU adds per step
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("s_add_u32 %0, %0, 0x9e37" : "+s"(a[i]));
        } else if (V == 1) {  // 8 dependent SALU ops
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("s_add_u32 %0, %0, 0x9e37" : "+s"(a[0]));
        } else if (V == 2) {  // 8 independent VALU
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, 0x9e37, %0" : "+v"(v[i]));
        } else if (V == 3) {  // 8 dependent VALU
#pragma unroll
            for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, 0x9e37, %0" : "+v"(v[0]));
        } else if (V == 4) {  // alternating independent SALU / VALU
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                asm volatile("s_add_u32 %0, %0, 0x9e37" : "+s"(a[i]));
                asm volatile("v_add_u32 %0, 0x9e37, %0" : "+v"(v[i]));
            }
        } else if (V == 5) {  // VALU -> SALU round trip: v_readfirstlane then s_add
#pragma unroll
            for (int i = 0; i < 8; ++i) a[0] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(v[0] + a[0])) + 1u;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] + v[i];
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) clk[0] = t1 - t0;
}

template <int V>
void run_issue(const char* name, uint32_t* d_out, uint64_t* d_clk) {
    hipLaunchKernelGGL(issue<V>, dim3(1), dim3(64), 0, 0, d_out, d_clk, 7u);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(issue<V>, dim3(1), dim3(64), 0, 0, d_out, d_clk, 7u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t c = 0;
    (void)hipMemcpy(&c, d_clk, 8, hipMemcpyDeviceToHost);
    // whole-kernel time per instruction (one wave on the GPU), and s_memtime cycles
    printf("%-14s %.3f ns/instruction (kernel time)  %.2f cycles/instruction (s_memtime)\n", name,
           ms * 1e6 / STEPS, (double)c / STEPS);
}

template <int V>
void run(const char* name, const uint32_t* d_tab, uint32_t* d_out, uint64_t* d_clk) {
    hipLaunchKernelGGL(chain<V>, dim3(1), dim3(64), 0, 0, d_tab, d_out, d_clk);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(chain<V>, dim3(1), dim3(64), 0, 0, d_tab, d_out, d_clk);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    uint64_t c = 0;
    (void)hipMemcpy(&c, d_clk, 8, hipMemcpyDeviceToHost);
    printf("%-6s %.3f ms  %.1f ns/step  %.1f cycles/step (s_memtime)\n", name, ms, ms * 1e6 / STEPS, (double)c / STEPS);
}

int main() {
    uint32_t h[2048];
    for (int i = 0; i < 2048; ++i) h[i] = (uint32_t)((i * 1103515245u + 12345u) >> 5) & 2047u;
    uint32_t *d_tab, *d_out;
    uint64_t* d_clk;
    (void)hipMalloc(&d_tab, sizeof h);
    (void)hipMalloc(&d_out, 4096);
    (void)hipMalloc(&d_clk, 64);
    (void)hipMemcpy(d_tab, h, sizeof h, hipMemcpyHostToDevice);
    run<0>("lds", d_tab, d_out, d_clk);
    run<1>("vgpr", d_tab, d_out, d_clk);
    run<2>("smem", d_tab, d_out, d_clk);
    run<3>("lds2", d_tab, d_out, d_clk);
    run<4>("vgpr2", d_tab, d_out, d_clk);
    run_issue<0>("salu_indep", d_out, d_clk);
    run_issue<1>("salu_dep", d_out, d_clk);
    run_issue<2>("valu_indep", d_out, d_clk);
    run_issue<3>("valu_dep", d_out, d_clk);
    run_issue<4>("salu_valu_mix", d_out, d_clk);
    run_issue<5>("valu_to_salu", d_out, d_clk);
    return 0;
}
