// Probe: do same-address LDS atomics with return (ds_add_rtn_u32) of one
// wave instruction hand out their old values in ascending lane order?  If
// so, one atomic per 64 positions gives each position its rank among the
// earlier positions holding the same symbol (the rank pass of the table
// builds, fse_device.hpp wave_build_spread).  Every lane of every wave draws
// a key (1..64 distinct keys, skewed or uniform) and an activity bit, reads
// the key's counter, does the atomic, and checks the returned value against
// counter-before + active lanes below with the same key (ballot peers).
// Build: hipcc -O3 --offload-arch=gfx950 lds_atomic_order.hip -o lds_atomic_order
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(256) void probe(uint32_t iters, uint32_t nkeys, uint32_t skew, uint32_t* bad, uint32_t* total) {
    __shared__ uint32_t cnt[4][64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    cnt[w][lane] = 0;
    __syncthreads();
    uint32_t nbad = 0, nops = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t h = mix(it * 0x9E3779B9u ^ (blockIdx.x * 256u + threadIdx.x) * 0x85EBCA6Bu);
        uint32_t key = h % nkeys;
        if (skew) key = min((uint32_t)__builtin_ctz((h >> 8) | 0x80000000u), nkeys - 1u);  // geometric
        const bool act = ((h >> 7) & 7u) != 0u || (it & 1u);  // ~7/8 active on odd iterations... all on even
        const uint32_t before = cnt[w][key];
        __builtin_amdgcn_wave_barrier();
        uint32_t r = 0;
        if (act) r = atomicAdd(&cnt[w][key], 1u);
        // expected: before + active lanes below with the same key
        uint64_t peers = 0;
        for (uint32_t k = 0; k < nkeys; ++k) {
            const uint64_t m = __ballot(act && key == k);
            if (key == k) peers = m;
        }
        const uint32_t below = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (act) {
            nops += 1;
            if (r != before + below) nbad += 1;
        }
        __builtin_amdgcn_wave_barrier();
    }
    atomicAdd(bad, nbad);
    atomicAdd(total, nops);
}

int main() {
    uint32_t *bad, *total;
    hipMalloc(&bad, 4);
    hipMalloc(&total, 4);
    uint32_t all_bad = 0;
    for (uint32_t skew = 0; skew < 2; ++skew)
        for (uint32_t nk : {1u, 2u, 5u, 16u, 48u, 64u}) {
            hipMemset(bad, 0, 4);
            hipMemset(total, 0, 4);
            hipLaunchKernelGGL(probe, dim3(2048), dim3(256), 0, 0, 256u, nk, skew, bad, total);
            uint32_t hb = 0, ht = 0;
            hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
            hipMemcpy(&ht, total, 4, hipMemcpyDeviceToHost);
            printf("keys %2u %s: %u out-of-order of %u atomics\n", nk, skew ? "geometric" : "uniform  ", hb, ht);
            all_bad += hb;
        }
    printf(all_bad ? "ORDER VIOLATED\n" : "lane order held in every case\n");
    return all_bad ? 1 : 0;
}
