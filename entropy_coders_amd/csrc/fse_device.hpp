// fse_device.hpp -- CDNA4 (gfx950) device building blocks of the FSE coder.
//
// Everything here runs inside one 64-lane wavefront: statistics, the
// normalised histogram, the NCount header and the tANS tables are produced
// by a single wave per block with LDS scratch, so kernels need no
// cross-wave synchronisation.  Each function cites the reference
// (Cognoscan/entropy_coders) lines whose behaviour it reproduces bit-exactly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fse_status.h"

namespace fsehip {

// Diagnostics (the libfsehip_diag.so build, -DFSEHIP_DIAG=1, for tools/ only):
// phase stamps when P.stamps is set by the host, and the encoder's phase
// ablations (FSE_ABLATE, EncParams::debug).  Both compile to nothing in the
// product library.
#ifdef FSEHIP_DIAG
constexpr bool kDiag = true;
#else
constexpr bool kDiag = false;
#endif
#define FSE_ABLATE(P, bits) (kDiag && ((P).debug & (bits)) != 0u)
#define FSE_STAMP(P, slot)                                                                     \
    do {                                                                                       \
        if (kDiag && (P).stamps && threadIdx.x == 0)                                           \
            (P).stamps[(uint64_t)blockIdx.x * kStamps + (slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)

#ifndef FSEHIP_KSTAMPS
#define FSEHIP_KSTAMPS
constexpr int kStamps = 10;  // stamp slots per workgroup (diagnostics; also in fse_kernels.h)
#endif
constexpr uint32_t LOG_MIN = 5;       // lib.rs:9
constexpr uint32_t LOG_MAX_REF = 15;  // lib.rs:10
constexpr uint32_t LOG_DEFAULT = 11;  // lib.rs:12
constexpr uint32_t HDR_MAX = 512;     // header bytes kept in LDS
constexpr uint32_t WAVE = 64;

__device__ __forceinline__ uint32_t ilog2u(uint32_t x) { return 31u - (uint32_t)__clz(x); }
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Synchronise the lanes of one wave around LDS traffic.  A wave's LDS
// operations execute in order, so only compiler reordering must be stopped;
// this lets the wave-level builders below run inside multi-wave workgroups.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Inclusive scans across the wave on DPP (VALU lane moves, a few cycles
// each) instead of ds_bpermute shuffles (an LDS round trip each): row_shr
// 1/2/4/8 within each 16-lane row, then row_bcast:15 and row_bcast:31 carry
// the row totals (GFX9 DPP).  Identity 0 (unsigned sum and max); out-of-row
// sources and masked rows read 0.  Call with every lane of the wave active.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, true);
}
template <class Op>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, Op op) {
    v = op(v, dpp0<0x111, 0xf>(v));  // row_shr:1
    v = op(v, dpp0<0x112, 0xf>(v));  // row_shr:2
    v = op(v, dpp0<0x114, 0xf>(v));  // row_shr:4
    v = op(v, dpp0<0x118, 0xf>(v));  // row_shr:8
    v = op(v, dpp0<0x142, 0xa>(v));  // row_bcast:15 into rows 1 and 3
    v = op(v, dpp0<0x143, 0xc>(v));  // row_bcast:31 into rows 2 and 3
    return v;
}
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    return wave_incl_scan(v, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    return wave_incl_scan(v, [](uint32_t a, uint32_t b) { return max(a, b); });
}
// Lane 63's value on the scalar unit (wave-uniform).
__device__ __forceinline__ uint32_t bcast63(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }
// Reductions: the scan's last lane, read on the scalar unit (wave-uniform).
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(v), 63);
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max(v), 63);
}

// Lanes of the wave holding the same key (one ballot per key bit),
// restricted to the active lanes.  Keys are symbols < table_len, so only
// kbits = bits of (table_len - 1) need comparing (wave-uniform; 6 for C2's
// 48 symbols instead of 8).
__device__ __forceinline__ uint64_t match_key(uint32_t key, uint64_t active, uint32_t kbits) {
    uint64_t peers = active;
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) {
        if (b >= kbits) break;
        uint64_t bal = __ballot((key >> b) & 1u);
        peers &= ((key >> b) & 1u) ? bal : ~bal;
    }
    return peers;
}
__device__ __forceinline__ uint32_t key_bits(uint32_t tl) { return tl <= 1u ? 1u : 32u - (uint32_t)__clz(tl - 1u); }

// The same peer mask for keys < 64 through LDS: every lane clears slot
// `lane` of the 64 u64 masks `pm`, ORs its lane bit into pm[key] and reads
// pm[key] back.  Three LDS instructions instead of ~9 VALU per key bit; one
// wave's LDS instructions complete in order, so each step sees the whole
// previous one (the compiler keeps their order: the slots may alias).
__device__ __forceinline__ uint64_t lds_peers(uint32_t key, uint64_t* pm, uint64_t lanebit) {
    pm[lane_id()] = 0;
    __hip_atomic_fetch_or(&pm[key], lanebit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    return __hip_atomic_load(&pm[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// ---------------------------------------------------------------------------
// Histogram::new (histogram.rs:18-66): 256-bin count of one block by one
// wave.  HS LDS sub-histograms (lane % HS), interleaved bin-major
// ([bin][sub]): the copies of a bin sit on consecutive banks, so a skewed
// block's same-symbol atomics neither serialise on one address nor pile
// onto one bank.  Measured against 4 copies at a 257-word stride
// (tools/micro/hist_bench.hip, 1 GiB): C2 0.46 -> 0.29 ms with 8 copies,
// uniform 0.24 -> 0.21 ms, LUT p=0.77 0.95 -> 0.43 ms; 16 copies (8 KiB)
// halve the lanes behind each counter word again (round 3).
// Counters are 16-bit: a bin's HS copies are HS/2 words of two halves (copy
// c = lane % HS counts in word c / 2, half c % 2), so the increment is a
// per-lane constant and a byte's address is one shift-or.  A copy counts at
// most 1/8 of a segment's bytes, so segments of HIST_SEG bytes cannot
// overflow a half; each segment is folded into the u32 counts[].
// Returns table_len (1 + largest symbol, 1 for an empty block).  counts
// must not alias hs.
// ---------------------------------------------------------------------------
#ifndef FSE_HSUB
#define FSE_HSUB 16
#endif
constexpr uint32_t HSUB = FSE_HSUB;  // default sub-histogram count
#ifndef FSE_HIST_U16
#define FSE_HIST_U16 1
#endif
constexpr bool HIST_U16 = FSE_HIST_U16 != 0;
// hot_words: the hot symbol's own counters after the bins (two lanes per word;
// the 16-copy layout of one block per wave only)
template <uint32_t HS>
constexpr uint32_t hot_words() { return HS == 16 ? 32u : 0u; }
template <uint32_t HS>
constexpr uint32_t hist_words() { return (HIST_U16 ? 256 * HS / 2 : 256 * HS) + hot_words<HS>(); }
constexpr uint32_t HIST_WORDS = hist_words<HSUB>();
constexpr uint32_t HIST_SEG = 1u << 18;

// The counting loop is a call of its own (noinline): inlined, it raised the
// encoder's VGPR count from 119 to 210.  Across the call the pointers are
// generic, so they are cast back to their address spaces here (a generic
// sub-histogram pointer would make every increment a FLAT atomic).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gbl_u4;
typedef __attribute__((address_space(1))) const uint8_t gbl_u8;

template <uint32_t HS>
__device__ __attribute__((noinline)) void wave_histogram_seg(const uint8_t* __restrict__ src_generic, uint32_t n,
                                                             uint32_t* hs_generic) {
    static_assert(HS == 8 || HS == 16, "sub-histograms");
    constexpr bool HOT = hot_words<HS>() != 0;
    static_assert(HIST_U16 || !HOT, "hot words hold two u16 halves");
    constexpr uint32_t WPB = (hist_words<HS>() - hot_words<HS>()) / 256u;  // words per bin
    const uint32_t lane = lane_id();
    // byte address of this lane's copy: ((lane / 2) % (HS / 2)) words into each bin's
    lds_u32* mine = (lds_u32*)hs_generic + (HIST_U16 ? ((lane >> 1) & (HS / 2u - 1u)) : (lane & (HS - 1u)));
    const uint32_t inc = HIST_U16 ? 1u << (16u * (lane & 1u)) : 1u;
    gbl_u8* src = (gbl_u8*)src_generic;
    // The hot symbol (the segment's first byte, wave-uniform) counts in words
    // of its own, two lanes per word, instead of its bin's 8 words shared by
    // 8 lanes each: a skewed block's dominant-symbol atomics stop queueing on
    // the same addresses.  One compare and one select per byte, no branch.
    const uint32_t hot = HOT && n ? __builtin_amdgcn_readfirstlane((uint32_t)src[0]) : 0x100u;
    lds_u32* hot_word = (lds_u32*)hs_generic + 256u * WPB + (lane >> 1);
    auto add_plain = [&](uint32_t byte) {
        __hip_atomic_fetch_add(&mine[byte * WPB], inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto add_hot = [&](uint32_t byte) {
        lds_u32* a = byte == hot ? hot_word : &mine[byte * WPB];
        __hip_atomic_fetch_add(a, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    uint32_t done = 0;
    if ((reinterpret_cast<uintptr_t>(src_generic) & 15u) == 0) {
        // batches of 8 x 16-byte loads per lane, double-buffered: the next
        // batch is in flight while the current one is counted
        constexpr uint32_t U = 8;
        const uint32_t nvec = n >> 4;
        gbl_u4* v4 = (gbl_u4*)src_generic;
        uint32_t v = 0;
        auto batches = [&](auto add) {
            auto count = [&](const u32x4* d) {
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t w[4] = {d[u].x, d[u].y, d[u].z, d[u].w};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
#pragma unroll
                        for (int b = 0; b < 4; ++b) add((w[k] >> (8 * b)) & 0xFFu);
                    }
                }
            };
            if (U * WAVE <= nvec) {
                u32x4 d[U];
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) d[u] = v4[u * WAVE + lane];
                for (; v + 2u * U * WAVE <= nvec; v += U * WAVE) {
                    u32x4 e[U];
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) e[u] = v4[v + U * WAVE + u * WAVE + lane];
                    count(d);
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) d[u] = e[u];
                }
                count(d);
                v += U * WAVE;
            }
            for (v += lane; v < nvec; v += WAVE) {
                const u32x4 d = v4[v];
                const uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
#pragma unroll
                    for (int b = 0; b < 4; ++b) add((w[k] >> (8 * b)) & 0xFFu);
                }
            }
        };
        // a block takes the hot path when at least half of a 1 KiB sample
        // (each lane's first 16 bytes) is the hot symbol; the others keep the
        // plain loop, with no per-byte compare
        bool skew = false;
        if (HOT && nvec >= WAVE) {
            const u32x4 q = v4[lane];
            const uint32_t w[4] = {q.x, q.y, q.z, q.w};
            uint32_t c = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int b = 0; b < 4; ++b) c += ((w[k] >> (8 * b)) & 0xFFu) == hot ? 1u : 0u;
            skew = bcast63(wave_incl_sum(c)) >= 8u * WAVE;
        }
        if (skew) batches(add_hot);
        else batches(add_plain);
        done = nvec << 4;
    }
    for (uint32_t i = done + lane; i < n; i += WAVE) add_plain(src[i]);
}

template <uint32_t HS = HSUB>
__device__ inline uint32_t wave_histogram(const uint8_t* __restrict__ src, uint32_t n,
                                          uint32_t* hs /*LDS [hist_words<HS>()]*/, uint32_t* counts /*LDS[256]*/) {
    constexpr uint32_t HW = hot_words<HS>(), NW = hist_words<HS>(), Q = (NW - HW) / 256u / 4u;  // uint4 per bin
    const uint32_t lane = lane_id();
    for (uint32_t s = lane; s < 256; s += WAVE) counts[s] = 0;
    uint32_t seg = 0;
    do {
        for (uint32_t i = lane; i < NW; i += WAVE) hs[i] = 0;
        wave_sync();
        const uint32_t m = min(n - seg, HIST_SEG);
        wave_histogram_seg<HS>(src + seg, m, hs);
        wave_sync();
        if (HW) {  // the hot symbol's own words
            const uint32_t x = lane < HW ? hs[NW - HW + lane] : 0u;
            const uint32_t t = bcast63(wave_incl_sum((x & 0xFFFFu) + (x >> 16)));
            if (lane == 0 && m) counts[src[seg]] += t;
        }
        for (uint32_t s = lane; s < 256; s += WAVE) {
            uint32_t c = 0;
#pragma unroll
            for (uint32_t k = 0; k < Q; ++k) {
                const uint4 q = reinterpret_cast<const uint4*>(hs)[Q * s + k];
                if (HIST_U16)
                    c += (q.x & 0xFFFFu) + (q.x >> 16) + (q.y & 0xFFFFu) + (q.y >> 16) + (q.z & 0xFFFFu) + (q.z >> 16) +
                         (q.w & 0xFFFFu) + (q.w >> 16);
                else
                    c += q.x + q.y + q.z + q.w;
            }
            counts[s] += c;
        }
        wave_sync();
        seg += m;
    } while (seg < n);
    uint32_t tl = 0;
    for (uint32_t s = lane; s < 256; s += WAVE)
        if (counts[s]) tl = max(tl, s + 1u);
    tl = wave_max(tl);
    wave_sync();
    return tl == 0 ? 1u : tl;
}

// ---------------------------------------------------------------------------
// optimal_log2 (histogram.rs:264-277), release-build u32 semantics.
// ---------------------------------------------------------------------------
__device__ inline int optimal_log2(uint32_t size, uint32_t table_len, uint32_t* L) {
    if (size == 0) return FSE_ERR_EMPTY;
    uint32_t min_src = ilog2u(size) + 1u;
    if (table_len <= 1) return FSE_ERR_ALL_ZERO_SYMBOL0;
    uint32_t min_sym = ilog2u(table_len - 1u) + 2u;
    uint32_t min_bits = min(min_src, min_sym);
    if (size == 1) return FSE_ERR_TOO_SHORT;
    uint32_t max_bits = ilog2u(size - 1u) - 2u;  // wraps for size 2..4
    uint32_t r = max(min(LOG_DEFAULT, max_bits), min_bits);
    r = min(max(r, LOG_MIN), LOG_MAX_REF);
    *L = r;
    return FSE_OK;
}

constexpr int32_t UNASSIGNED = -2;

// normalize_slow (histogram.rs:157-261): rare, single lane.
__device__ inline int normalize_slow_lane(const uint32_t* counts, uint32_t size, uint32_t tl, uint32_t L,
                                          int32_t* norm) {
    uint32_t low_t = size >> L;
    uint32_t low_one = (uint32_t)(size * 3u) >> (L + 1u);
    uint32_t td = 1u << L;
    uint32_t total = size;
    for (uint32_t s = 0; s < 256; ++s) norm[s] = 0;
    for (uint32_t s = 0; s < tl; ++s) {
        uint32_t t = counts[s];
        if (t == 0) continue;
        if (t <= low_t) { norm[s] = -1; td -= 1; total -= t; }
        else if (t <= low_one) { norm[s] = 1; td -= 1; total -= t; }
        else norm[s] = UNASSIGNED;
    }
    if (td == 0) return FSE_OK;
    if (total / td > low_one) {
        uint32_t low = (uint32_t)(total * 3u) / (uint32_t)(td * 2u);
        for (uint32_t s = 0; s < tl; ++s)
            if (norm[s] == UNASSIGNED && counts[s] <= low) { norm[s] = 1; td -= 1; total -= counts[s]; }
    }
    if ((uint32_t)((1u << L) - td) == tl) {
        uint32_t vmax = 0, imax = 0;
        for (uint32_t s = 0; s < 256; ++s)
            if (counts[s] > vmax) { vmax = counts[s]; imax = s; }
        norm[imax] += (int32_t)td;
        return FSE_OK;
    }
    if (total == 0) {
        while (td != 0) {
            bool moved = false;
            for (uint32_t s = 0; s < tl; ++s) {
                if (norm[s] > 0) {
                    norm[s] += 1; td -= 1; moved = true;
                    if (td == 0) break;
                }
            }
            if (!moved) return FSE_ERR_CURSED;
        }
        return FSE_OK;
    }
    const uint32_t vsl = 62u - L;
    const uint64_t mid = (1ull << (vsl - 1u)) - 1ull;
    const uint64_t r_step = (((1ull << vsl) * (uint64_t)td) + mid) / (uint64_t)total;
    uint64_t acc = mid;
    for (uint32_t s = 0; s < tl; ++s) {
        if (norm[s] == UNASSIGNED) {
            uint64_t end = acc + (uint64_t)counts[s] * r_step;
            uint64_t w = (end >> vsl) - (acc >> vsl);
            if (w < 1) return FSE_ERR_CURSED;
            norm[s] = (int32_t)w;
            acc = end;
        }
    }
    return FSE_OK;
}

// ---------------------------------------------------------------------------
// Histogram::normalize (histogram.rs:95-155), wave-parallel fast path: each
// lane owns 4 symbols; the residual goes to the first largest symbol (strict
// `>` at 135) found by a (prob, -index) max-reduction; the slow path runs on
// lane 0.  Returns status; *L_out = effective tableLog.
// ---------------------------------------------------------------------------
__device__ inline int wave_normalize(const uint32_t* counts, uint32_t size, uint32_t tl, uint32_t log2_req,
                                     int32_t* norm, uint32_t* L_out, uint32_t* used_slow, int* scratch) {
    const uint32_t lane = lane_id();
    if (tl <= 1) return FSE_ERR_ALL_ZERO_SYMBOL0;  // ilog2(0) at 98
    if (size == 0) return FSE_ERR_EMPTY;
    uint32_t L = min(max(log2_req, LOG_MIN), LOG_MAX_REF);
    L = max(L, ilog2u(tl - 1u) + 2u);
    const uint32_t scale = 62u - L;
    const uint64_t step = (1ull << 62) / (uint64_t)size;
    const uint64_t v_step = 1ull << (scale - 20u);
    const uint32_t low_t = size >> L;
    const uint32_t RTB[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};

    uint32_t local_sum = 0, best = 0, single = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        uint32_t s = lane * 4u + k;
        int32_t v = 0;
        if (s < tl) {
            uint32_t t = counts[s];
            if (t == size) {
                single = s + 1u;
            } else if (t == 0) {
                v = 0;
            } else if (t <= low_t) {
                v = -1;
                local_sum += 1;
            } else {
                uint64_t p = ((uint64_t)t * step) >> scale;
                if (p < 8) p += (((uint64_t)t * step - (p << scale)) > v_step * (uint64_t)RTB[p]) ? 1u : 0u;
                v = (int32_t)p;
                local_sum += (uint32_t)p;
                uint32_t key = ((uint32_t)p << 8) | (255u - s);
                if (p > 0) best = max(best, key);
            }
        }
        norm[s] = v;
    }
    single = wave_max(single);
    uint32_t sum = wave_sum(local_sum);
    best = wave_max(best);
    *used_slow = 0;
    if (single) {  // t == size returns immediately (113-120); other counts are 0
        if (lane == 0) norm[single - 1u] = (int32_t)(1u << L);
        wave_sync();
        *L_out = L;
        return FSE_OK;
    }
    const int32_t to_distribute = (int32_t)(1u << L) - (int32_t)sum;
    const int32_t largest_prob = (int32_t)(best >> 8);
    const uint32_t largest = best ? 255u - (best & 255u) : 0u;
    wave_sync();
    int rc = FSE_OK;
    if (to_distribute != 0 && -to_distribute >= (largest_prob >> 1)) {
        *used_slow = 1;
        if (lane == 0) scratch[0] = normalize_slow_lane(counts, size, tl, L, norm);
        wave_sync();
        rc = scratch[0];
    } else {
        if (lane == 0) norm[largest] += to_distribute;
    }
    wave_sync();
    *L_out = L;
    return rc;
}

// ---------------------------------------------------------------------------
// NormHistogram::write (histogram.rs:376-431), one lane.  Writes the header
// bytes into hdr[] (LDS) and returns the byte length (<= HDR_MAX) or < 0.
// ---------------------------------------------------------------------------
struct ByteWriter {
    uint8_t* buf;
    uint32_t byte;
    uint64_t acc;
    uint32_t nacc;
    bool overflow;
    __device__ void put(uint32_t v, uint32_t nb) {
        acc |= (uint64_t)(v & ((1u << nb) - 1u)) << nacc;
        nacc += nb;
        while (nacc >= 8) {
            if (byte < HDR_MAX) buf[byte] = (uint8_t)acc; else overflow = true;
            byte++;
            acc >>= 8;
            nacc -= 8;
        }
    }
    __device__ uint32_t finish() {
        if (nacc) {
            if (byte < HDR_MAX) buf[byte] = (uint8_t)acc; else overflow = true;
            byte++;
        }
        return byte;
    }
};

__device__ inline int header_write_lane(const int32_t* norm, uint32_t L, uint32_t tl, uint8_t* hdr,
                                       uint32_t* bits_out = nullptr) {
    ByteWriter w{hdr, 0, 0, 0, false};
    w.put(L - LOG_MIN, 4);
    int32_t thr = 1 << L;
    int32_t rem = thr + 1;
    uint32_t zc = 0;
    uint32_t nb = L + 1u;
    for (uint32_t i = 0; i < tl; ++i) {
        int32_t s = norm[i];
        if (rem <= 1) break;
        if (zc != 0) {
            if (s == 0) { zc += 1; continue; }
            zc -= 1;
            while (zc >= 24) { w.put(0xFFFF, 16); zc -= 24; }
            while (zc >= 3) { w.put(3, 2); zc -= 3; }
            w.put(zc, 2);
        }
        int32_t mx = (2 * thr - 1) - rem;
        rem -= (s < 0 ? -s : s);
        int32_t c = s + 1;
        if (c >= thr) c += mx;
        w.put((uint32_t)c, nb - (c < mx ? 1u : 0u));
        zc = (c == 1) ? 1u : 0u;
        if (rem < 1) return FSE_ERR_BAD_TABLE;
        while (rem < thr) { nb -= 1; thr >>= 1; }
    }
    if (bits_out) *bits_out = w.byte * 8u + w.nacc;  // BitStackWriter::finish's count (writer.rs:201-222)
    uint32_t len = w.finish();
    if (w.overflow) return FSE_ERR_DST_TOO_SMALL;
    return (int)len;
}

// Wave-parallel NormHistogram::write (histogram.rs:376-431), same bytes as
// header_write_lane.  The writer's state before symbol i depends only on
// prefix quantities, so every field is placed independently:
//   remaining_i = 2^L + 1 - sum_{j<i} |norm_j|, threshold_i = the largest
//   power of two <= remaining_i, nb_i = log2(threshold_i) + 1 (the shrink
//   loop at 424-427); a zero is written only when it starts a run (391-395);
//   the 2-bit/16-bit repeat markers for a run of r zeros (r-1 repeats) go
//   right before the next non-zero symbol (397-408).
// Field lengths are prefix-summed and the bits OR-ed into the LDS words.
__device__ __forceinline__ void or_bits(uint32_t* words, uint32_t pos, uint32_t v, uint32_t nb) {
    if (nb == 0) return;
    const uint32_t w = pos >> 5, sh = pos & 31u;
    atomicOr(&words[w], v << sh);
    if (sh + nb > 32u) atomicOr(&words[w + 1], v >> (32u - sh));
}

__device__ inline int wave_header_write(const int32_t* norm, uint32_t L, uint32_t tl, uint32_t* hw /*LDS, HDR_MAX/4 words*/) {
    const uint32_t lane = lane_id();
    for (uint32_t i = lane; i < HDR_MAX / 4; i += WAVE) hw[i] = 0;
    int32_t v[4];
    uint32_t absum = 0, lastnz = 0;  // lastnz: 1 + index of the last non-zero among this lane's symbols
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t i = lane * 4u + k;
        v[k] = (i < tl) ? norm[i] : 0;
        absum += (uint32_t)(v[k] < 0 ? -v[k] : v[k]);
        if (i < tl && v[k] != 0) lastnz = i + 1u;
    }
    const uint32_t ex_abs = wave_incl_sum(absum) - absum;
    const uint32_t prev_nz = max((uint32_t)__shfl_up(wave_incl_max(lastnz), 1, 64), 0u) * (lane ? 1u : 0u);
    // pass 1: field lengths
    uint32_t len[4], nbits = 0;
    {
        uint32_t rem = (1u << L) + 1u - ex_abs, lnz = prev_nz;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = lane * 4u + k;
            uint32_t l = 0;
            if (i < tl && rem > 1u) {
                const bool prev_zero = i > 0 && lnz != i;  // symbol i-1 is zero
                if (v[k] == 0 && prev_zero) {
                    l = 0;  // inside a zero run: not written
                } else {
                    if (v[k] != 0 && prev_zero) {  // markers for r zeros before i
                        const uint32_t r = i - lnz;  // lnz = 1 + index of last non-zero
                        const uint32_t z = r - 1u;
                        l += 16u * (z / 24u) + 2u * ((z % 24u) / 3u) + 2u;
                    }
                    const uint32_t thr = 1u << ilog2u(rem);
                    const uint32_t nb = ilog2u(thr) + 1u;
                    const int32_t mx = (int32_t)(2u * thr - 1u - rem);
                    int32_t c = v[k] + 1;
                    if (c >= (int32_t)thr) c += mx;
                    l += nb - (c < mx ? 1u : 0u);
                }
            }
            len[k] = l;
            nbits += l;
            rem -= (uint32_t)(v[k] < 0 ? -v[k] : v[k]);
            if (i < tl && v[k] != 0) lnz = i + 1u;
        }
    }
    const uint32_t ex_bits = wave_incl_sum(nbits) - nbits;
    const uint32_t total = 4u + bcast63(ex_bits + nbits);
    const uint32_t bytes = (total + 7u) >> 3;
    if (bytes > HDR_MAX) return FSE_ERR_DST_TOO_SMALL;
    wave_sync();
    // pass 2: place the bits
    if (lane == 0) or_bits(hw, 0, L - LOG_MIN, 4);
    {
        uint32_t pos = 4u + ex_bits;
        uint32_t rem = (1u << L) + 1u - ex_abs, lnz = prev_nz;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = lane * 4u + k;
            if (len[k]) {
                const bool prev_zero = i > 0 && lnz != i;
                if (v[k] != 0 && prev_zero) {
                    uint32_t z = i - lnz - 1u;
                    while (z >= 24u) { or_bits(hw, pos, 0xFFFFu, 16); pos += 16; z -= 24u; }
                    const uint32_t q3 = z / 3u;
                    if (q3) { or_bits(hw, pos, (1u << (2u * q3)) - 1u, 2u * q3); pos += 2u * q3; }
                    or_bits(hw, pos, z % 3u, 2);
                    pos += 2;
                }
                const uint32_t thr = 1u << ilog2u(rem);
                const uint32_t nb = ilog2u(thr) + 1u;
                const int32_t mx = (int32_t)(2u * thr - 1u - rem);
                int32_t c = v[k] + 1;
                if (c >= (int32_t)thr) c += mx;
                const uint32_t w = nb - (c < mx ? 1u : 0u);
                or_bits(hw, pos, (uint32_t)c & ((1u << w) - 1u), w);
                pos += w;
            }
            rem -= (uint32_t)(v[k] < 0 ? -v[k] : v[k]);
            if (i < tl && v[k] != 0) lnz = i + 1u;
        }
    }
    wave_sync();
    return (int)bytes;
}

// ---------------------------------------------------------------------------
// NormHistogram::read (histogram.rs:436-505) as wave-uniform code: every lane
// of the calling wave holds the same values, so the serial parse runs on the
// scalar unit (s_lshr_b64 window, s_flbit for the threshold) instead of one
// VALU lane.  norm[] must be zeroed by the caller.  Results and statuses are
// the reference's (stream_reader.rs:16-135 read / peek / advance semantics).
//
// The scalar unit is shared by the CU's waves, and the decode-table kernel is
// bound by its issue rate (the parse is ~90% of that kernel's scalar
// instructions), so the common field is a straight run of scalar code: every
// error here is BAD_HEADER, so the end-of-data check is deferred (left only
// falls; reads past the data see zeros and the loop still ends within 256
// symbols), the threshold is recomputed unconditionally (thr = 2^ilog2(rem)
// holds throughout, the closed form of 492-495), every lane stores the same
// norm value (no exec-mask change), and the zero-run marks (456-464) and the
// loop's end conditions leave the common path through one branch.
// ---------------------------------------------------------------------------
// The parse itself, over a word source ld(i) (word i of the header, zero
// past the block) and a sink put(sym, value) for the normalised counts:
// header_read_wave runs it wave-uniform on the scalar unit, header_read_row
// one header per lane (hdr_parse_kernel).
template <class LD, class PUT>
__device__ __forceinline__ int header_read_core(LD ld, PUT put, uint32_t n, uint32_t lmax, uint32_t* L_out,
                                                uint32_t* tl_out) {
    if (n == 0) return FSE_ERR_EMPTY;
    // a header is at most ~420 bytes: bounding the bit count keeps it in
    // int32 for any block (n*8 overflows above 2^28 bytes) without changing
    // where the header can run out
    const int32_t total = (int32_t)(min(n, 1u << 20) * 8u);
    // window: words bw, bw+1; next bit = 32*bw + off; left = bits after it
    uint32_t bw = 0, off = 0;
    int32_t left = total;
    uint64_t buf = (uint64_t)ld(0) | ((uint64_t)ld(1) << 32);
    auto refill = [&]() {  // fields are <= 16 bits, so one word per field suffices
        if (off >= 32u) {
            off -= 32u;
            ++bw;
            buf = (buf >> 32) | ((uint64_t)ld(bw + 1u) << 32);
        }
    };
    if (left < 4) return FSE_ERR_BAD_HEADER;
    const uint32_t L = ((uint32_t)buf & 15u) + LOG_MIN;
    off = 4;
    left -= 4;
    if (L > LOG_MAX_REF) return FSE_ERR_BAD_HEADER;  // TableLogTooLarge
    if (L > lmax) return FSE_ERR_UNSUPPORTED;          // valid for the crate, beyond this build's tables
    uint32_t sym = 0, rem = (1u << L) + 1u, lg = L, thr = 1u << L;  // read width = lg + 1
    for (;;) {  // entered with rem > 1 and sym < 256
        refill();
        // peek(nb) falling back to peek(nb-1) (471-473): the short path only
        // uses the low nb-1 bits and the long path needs all nb, so "left <
        // the advance" is the reference's error for both
        const uint32_t raw = (uint32_t)(buf >> off);
        const uint32_t t2 = 2u * thr - 1u;
        const uint32_t mx = t2 - rem;
        const uint32_t low = raw & (thr - 1u);
        uint32_t vlong = raw & t2;
        vlong = vlong >= thr ? vlong - mx : vlong;
        const bool lng = low >= mx;
        const uint32_t val = lng ? vlong : low;
        const uint32_t adv = lg + (lng ? 1u : 0u);
        off += adv;
        left -= (int32_t)adv;
        const int32_t sv = (int32_t)val - 1;
        rem -= (uint32_t)__builtin_abs(sv);  // stays >= 1 (val <= rem)
        put(sym, sv);
        sym += 1u;
        lg = 31u - (uint32_t)__builtin_clz(rem);
        thr = 1u << lg;
        // leave the common path after a 0 (val == 1), at rem == 1 or at
        // symbol 256, as one test: rem <= 2^15 + 1 and val <= 2^16, so bit 31
        // of rem - 2 and of (val ^ 1) - 1 is set exactly when rem < 2, val == 1
        if ((((rem - 2u) | ((val ^ 1u) - 1u)) >> 31 | (sym >> 8)) == 0u) continue;
        if (rem <= 1u || sym >= 256u) break;
        // zero-run marks after a 0 (456-464): peek(..).unwrap_or(0)
        for (;;) {
            refill();
            if (left < 16 || ((uint32_t)(buf >> off) & 0xFFFFu) != 0xFFFFu) break;
            off += 16u;
            left -= 16;
            sym += 24u;
        }
        for (;;) {
            refill();
            if (left < 2 || ((uint32_t)(buf >> off) & 3u) != 3u) break;
            off += 2u;
            left -= 2;
            sym += 3u;
        }
        if (left < 2) return FSE_ERR_BAD_HEADER;
        sym += (uint32_t)(buf >> off) & 3u;
        off += 2u;
        left -= 2;
        if (sym >= 256u) break;
    }
    if (left < 0) return FSE_ERR_BAD_HEADER;   // a field ran past the data (UnexpectedEof)
    if (rem != 1u) return FSE_ERR_BAD_HEADER;  // TooManySymbols
    *L_out = L;
    *tl_out = sym;
    return (total - left + 7) >> 3;
}

__device__ inline int header_read_wave(uint32_t r0, uint32_t r1, uint32_t n, uint32_t lmax, int32_t* norm,
                                       uint32_t* L_out, uint32_t* tl_out) {
    // r0 / r1 hold header words lane / 64 + lane (zero past the block): a
    // word is one v_readlane.  Headers of L <= 12 fit in 417 bytes, so the
    // 512 bytes held always cover them (L > lmax returns before reading on).
    auto ld = [&](uint32_t i) -> uint32_t {
        const uint32_t a = __builtin_amdgcn_readlane(r0, i & 63u);
        const uint32_t b = __builtin_amdgcn_readlane(r1, i & 63u);
        return i < 64u ? a : (i < 128u ? b : 0u);
    };
    // every lane stores the same norm value (no exec-mask change)
    return header_read_core(ld, [&](uint32_t sym, int32_t sv) { norm[sym] = sv; }, n, lmax, L_out, tl_out);
}

// One header per lane: words from this lane's 128-word LDS row (the first nw
// staged, as header_read_wave holds 512 bytes; word i at (i + rot) % 128, so
// lanes at the same word read different banks), the counts as int16 into its
// 256-entry LDS norm row, rotated the same way (zeroed by the caller).
__device__ inline int header_read_row(const lds_u32* row, uint32_t rot, uint32_t nw, uint32_t n, uint32_t lmax,
                                      __attribute__((address_space(3))) int16_t* norm, uint32_t* L_out,
                                      uint32_t* tl_out) {
    auto ld = [&](uint32_t i) -> uint32_t { return i < nw ? row[(i + rot) & 127u] : 0u; };
    return header_read_core(
        ld, [&](uint32_t sym, int32_t sv) { norm[(sym + 2u * rot) & 255u] = (int16_t)sv; }, n, lmax, L_out, tl_out);
}

// ---------------------------------------------------------------------------
// Symbol spread and per-position occurrence rank (fse.rs:110-162, 294-337),
// wave-parallel.  After the call:
//   sym_at[i]  = symbol at table position i            (LDS, 2^L bytes)
//   cumul[s]   = sum_{t<s} c'(t), c' = 1 for -1         (LDS, 256)
// and `visit(i, s, base(s) + rank)` is invoked once per position with the
// rank of position i among the positions holding s in ascending position
// order (stateTable order, fse.rs:158-162; DecodeTable order, fse.rs:329-337)
// plus the caller's per-symbol base (cumul[s] for the stateTable, the
// symbol's first x for the decode table), folded into the rank counters so
// that a visit reads no per-symbol array.
//
// The spread walks multipliers m = 0..2^L-1: position (m*step) mod 2^L is
// visited iff it is <= the high threshold, and the j-th visited position
// gets the j-th positive occurrence in symbol order (fse.rs:139-150).  The
// owner of occurrence j comes from a forward max-fill of symbol start marks.
// Both walks take 4 consecutive entries per lane, so a 2^11 table needs 8
// wave steps per walk instead of 32.
// Ranks come from ballot peer matching over 64 consecutive positions.  With
// RK (LDS, 2 x 2^L bytes) and table_len <= 64 they take two passes without
// a serial chain: per-chunk symbol counts, a per-symbol prefix over chunks,
// then rank = prefix + peers below; otherwise running per-symbol counters
// (an LDS read-modify-write per chunk).
// ---------------------------------------------------------------------------
// Exclusive scan helpers on DPP: wave_shr:1 (lane 0 reads 0).
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) { return dpp0<0x138, 0xf>(v); }

struct NoStamps {
    uint64_t* stamps = nullptr;
};

// Atomic ranks (below) and how a table built with them checks itself.
struct RankAtomic {
    bool on;              // atomic ranks allowed (else the peer-mask ranks)
    uint8_t* inv8;        // inverse mode: 2^L bytes of dead scratch (lane | last-in-chunk << 6 per slot)
    const uint16_t* st;   // stateTable mode (inv8 == nullptr): the visit's stateTable, entries st_off + position
    uint32_t st_off;
    uint32_t* fallbacks;  // global count of tables whose check failed (rebuilt with peer-mask ranks), or nullptr
    uint32_t inject;      // diagnostics build only: chunk 0's ranks in descending lane order (fault injection)
};

// Is slot x the first slot of some symbol (x == cumul[s] for an s with
// slots)?  cumul is non-decreasing over all 256 symbols (a symbol without
// slots repeats the next start), so a lower-bound search answers it.
__device__ __forceinline__ bool is_start_slot(const uint16_t* cumul, uint32_t x) {
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t h = 128; h; h >>= 1)
        if ((uint32_t)cumul[lo + h - 1u] < x) lo += h;
    return lo < 256u && (uint32_t)cumul[lo] == x;
}

// MAXCH: 2^LMAX / 64 chunks (two-pass ranks); INV: the atomic ranks' check in
// inverse mode (RankAtomic::inv8), else in stateTable mode (RankAtomic::st);
// GSYM: sym_at is in global memory (the encoder at L >= 13, whose LDS then
// holds two or more workgroups per CU): its writes are fenced before other
// lanes read them, the rank pass keeps several chunks' loads in flight, and
// the stateTable check tests slot starts in cumul instead of reading symbols
template <uint32_t MAXCH = 64, bool INV = false, bool GSYM = false, typename Visit, typename Base,
          class SP = NoStamps>
__device__ inline int wave_build_spread(const int32_t* norm, uint32_t L, uint32_t tl, uint8_t* sym_at,
                                        uint8_t* occ_sym, uint16_t* cumul, uint32_t* cnt, Visit visit, Base base,
                                        const RankAtomic& ra, uint16_t* RK = nullptr, uint64_t* PM = nullptr,
                                        const SP* SPp = nullptr) {
    // SPp: diagnostics only, a params struct with `stamps` (phase stamps 3..7)
#define SPREAD_STAMP(k)                                  \
    do {                                                 \
        if (SPp) FSE_STAMP(*SPp, k);                     \
    } while (0)
    const uint32_t lane = lane_id();
    const uint32_t size = 1u << L;
    const uint32_t mask = size - 1u;
    // per-lane 4 symbols: c'(s), positive count, -1 flag
    uint32_t cp[4], pos_n[4], neg[4];
    uint32_t sum_c = 0, sum_p = 0, sum_neg = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t s = lane * 4u + k;
        int32_t v = (s < tl) ? norm[s] : 0;
        neg[k] = (v == -1 || v < -1) ? 1u : 0u;
        pos_n[k] = v > 0 ? (uint32_t)v : 0u;
        cp[k] = (v == -1) ? 1u : pos_n[k];
        sum_c += cp[k];
        sum_p += pos_n[k];
        sum_neg += neg[k];
    }
    const uint32_t ex_c = wave_incl_sum(sum_c) - sum_c;
    const uint32_t ex_p = wave_incl_sum(sum_p) - sum_p;
    const uint32_t ex_n = wave_incl_sum(sum_neg) - sum_neg;
    const uint32_t total_neg = bcast63(ex_n + sum_neg);
    const uint32_t total_pos = bcast63(ex_p + sum_p);
    if (total_pos + total_neg > size || total_neg > size) return FSE_ERR_BAD_TABLE;
    const int32_t ht = (int32_t)size - 1 - (int32_t)total_neg;
    SPREAD_STAMP(3);
    for (uint32_t i = lane; i < size / 16u; i += WAVE) {  // size >= 32: whole 16-byte stores
        reinterpret_cast<uint4*>(occ_sym)[i] = make_uint4(0, 0, 0, 0);
        reinterpret_cast<uint4*>(sym_at)[i] = make_uint4(0, 0, 0, 0);
    }
    if (GSYM) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    wave_sync();
    {
        uint32_t c = ex_c, p = ex_p, ng = ex_n;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t s = lane * 4u + k;
            cumul[s] = (uint16_t)c;
            if (pos_n[k]) occ_sym[p] = (uint8_t)s;  // start mark of s's occurrences
            if (neg[k]) sym_at[size - 1u - ng] = (uint8_t)s;  // -1 symbols from the top (122-125)
            c += cp[k];
            p += pos_n[k];
            ng += neg[k];
        }
    }
    if (GSYM) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    wave_sync();
    // forward max-fill: occ_sym[j] = owner of positive occurrence j (4 per
    // lane; entries at and above total_pos are filled too and never read)
    {
        uint32_t* occ4 = reinterpret_cast<uint32_t*>(occ_sym);
        uint32_t carry = 0;
        for (uint32_t base = 0; base * 4u < total_pos; base += WAVE) {
            const uint32_t q = base + lane;
            const uint32_t w = q * 4u < size ? occ4[q] : 0u;
            const uint32_t m0 = w & 0xFFu, m1 = max(m0, (w >> 8) & 0xFFu), m2 = max(m1, (w >> 16) & 0xFFu),
                           m3 = max(m2, w >> 24);
            const uint32_t incl = wave_incl_max(m3);
            const uint32_t b = max(carry, wave_shr1(incl));
            if (q * 4u < size) occ4[q] = max(b, m0) | (max(b, m1) << 8) | (max(b, m2) << 16) | (max(b, m3) << 24);
            carry = max(carry, bcast63(incl));
        }
    }
    wave_sync();
    SPREAD_STAMP(4);
    // spread: j-th valid multiplier -> position (multipliers 4q..4q+3 per lane)
    const uint32_t step = (size >> 3) * 5u + 3u;  // table_step: size*5/8+3 (fse.rs:67-70)
    {
        uint32_t j0 = 0;
        for (uint32_t base = 0; base < size; base += 4u * WAVE) {
            const uint32_t m = base + 4u * lane;
            uint32_t p[4], nv = 0;
            bool v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                p[k] = ((m + k) * step) & mask;
                v[k] = m + k < size && (int32_t)p[k] <= ht;
                nv += v[k] ? 1u : 0u;
            }
            const uint32_t incl = wave_incl_sum(nv);
            uint32_t j = j0 + incl - nv;
            // owners of occurrences j .. j + 3: one read of the two words
            // holding them (a 2^L-byte array sits in a larger LDS region or
            // at the end of LDS, where reads past it return 0)
            const uint32_t ja = j & ~3u;
            const uint32_t* o4 = reinterpret_cast<const uint32_t*>(occ_sym) + (ja >> 2);
            const uint64_t ow = (((uint64_t)o4[1] << 32) | o4[0]) >> (8u * (j - ja));
            uint32_t c = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (v[k] && j < total_pos) sym_at[p[k]] = (uint8_t)(ow >> (8u * c));
                j += v[k] ? 1u : 0u;
                c += v[k] ? 1u : 0u;
            }
            j0 += bcast63(incl);
        }
        if (j0 != total_pos) return FSE_ERR_BAD_TABLE;  // position != 0 assert
    }
    if (GSYM) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    wave_sync();
    SPREAD_STAMP(5);
    if (ra.on) {
        // Ranks by one LDS atomic per 64 positions: the old values that a
        // ds_add_rtn_u32 hands to the lanes of one instruction hitting the
        // same counter come in ascending lane order on gfx950 (tools/micro/
        // lds_atomic_order.hip: 1.5e9 atomics, uniform and skewed keys,
        // partial exec masks, none out of order), and a wave's LDS
        // instructions run in order, so the value is the count of s at
        // earlier positions -- the rank -- on top of the caller's base.  The
        // lane order is not documented, so every table checks the result
        // (below) and is rebuilt with the peer-mask ranks if it fails.
        //
        // Inverse mode (inv8): the counters carry the symbol's slot in the
        // high half (cumul[s] + rank, the stateTable order of fse.rs:157-162)
        // and base + rank in the low half, so one atomic gives both; slot g
        // records the lane that took it and whether it was the last slot its
        // chunk took for that symbol (the counter read back after the
        // instruction).
        constexpr uint32_t step = INV ? 0x10001u : 1u;
        for (uint32_t s = lane; s < 256u; s += WAVE) cnt[s] = INV ? ((uint32_t)cumul[s] << 16) | base(s) : base(s);
        wave_sync();
        // the next chunk's symbols are read while this chunk's atomics are in
        // flight; in inverse mode the counter is read back right behind the
        // atomic (a wave's LDS instructions run in order), one wait for both
        // (GSYM: GD chunks' symbols in flight, a global load's latency being
        // several iterations long)
        constexpr uint32_t GD = GSYM ? 8u : 1u;
        uint32_t sy_q[GD];
#pragma unroll
        for (uint32_t k = 0; k < GD; ++k) sy_q[k] = k * WAVE + lane < size ? sym_at[k * WAVE + lane] : 0u;
        for (uint32_t i0 = 0; i0 < size; i0 += WAVE) {
            const uint32_t i = i0 + lane;
            const bool act = i < size;
            const uint32_t sy = sy_q[0];
            if constexpr (GSYM) {
#pragma unroll
                for (uint32_t k = 0; k + 1u < GD; ++k) sy_q[k] = sy_q[k + 1u];
                sy_q[GD - 1u] = i + GD * WAVE < size ? sym_at[i + GD * WAVE] : 0u;
            } else {
                if (i + WAVE < size) sy_q[0] = sym_at[i + WAVE];
            }
            uint32_t r = 0, endw = 0;
            if (act) {
                r = __hip_atomic_fetch_add((lds_u32*)cnt + sy, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (INV) endw = __hip_atomic_load((lds_u32*)cnt + sy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (kDiag && ra.inject && i0 == 0) {  // fault injection: the lanes' order reversed
                const uint64_t peers = match_key(sy, __ballot(act), key_bits(tl));
                const uint32_t bl = (uint32_t)__popcll(peers & lanemask_lt()), k = (uint32_t)__popcll(peers);
                r += (k - 1u - 2u * bl) * step;
            }
            if (act) {
                if (INV) {
                    const uint32_t g = r >> 16;
                    ra.inv8[g] = (uint8_t)(lane | (g + 1u == (endw >> 16) ? 0x40u : 0u));
                    visit(i, sy, r & 0xFFFFu);
                } else {
                    visit(i, sy, r);
                }
            }
        }
        wave_sync();
        // The check: the ranks of one symbol must follow its positions.  A
        // wave's instructions keep their order, so only lanes of one
        // instruction can be out of order, and only among themselves.
        bool bad = false;
        if (INV) {
            // consecutive slots g, g + 1 of one chunk's range for one symbol
            // (g not flagged last) must hold ascending lanes
            for (uint32_t q0 = 0; q0 < size; q0 += 8u * WAVE) {
                const uint32_t g = q0 + 8u * lane;
                if (g < size) {
                    const uint2 w = *reinterpret_cast<const uint2*>(ra.inv8 + g);
                    const uint64_t b8 = ((uint64_t)w.y << 32) | w.x;
                    const uint32_t nx = g + 8u < size ? (uint32_t)ra.inv8[g + 8u] : 0x40u;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint32_t cur = (uint32_t)(b8 >> (8 * j)) & 0xFFu;
                        const uint32_t nxt = j < 7 ? (uint32_t)(b8 >> (8 * j + 8)) & 0xFFu : nx;
                        bad |= !(cur & 0x40u) && (cur & 63u) >= (nxt & 63u);
                    }
                }
            }
        } else {
            // the stateTable (slot -> st_off + position): positions ascend
            // within a symbol's slots; a descent must be a symbol boundary
            for (uint32_t q0 = 0; q0 < size; q0 += 4u * WAVE) {
                const uint32_t g = q0 + 4u * lane;
                if (g < size) {
                    const uint2 w = *reinterpret_cast<const uint2*>(ra.st + g);
                    const uint32_t v[5] = {w.x & 0xFFFFu, w.x >> 16, w.y & 0xFFFFu, w.y >> 16,
                                           g + 4u < size ? (uint32_t)ra.st[g + 4u] : 0xFFFFFu};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (GSYM) {
                            if (v[j] > v[j + 1] && !is_start_slot(cumul, g + (uint32_t)j + 1u)) bad = true;
                        } else {
                            if (v[j] > v[j + 1] && sym_at[v[j] - ra.st_off] == sym_at[v[j + 1] - ra.st_off]) bad = true;
                        }
                    }
                }
            }
        }
        if (__ballot(bad) == 0ull) return FSE_OK;
        if (lane == 0 && ra.fallbacks) atomicAdd(ra.fallbacks, 1u);
        wave_sync();
        // rebuilt below with the peer-mask ranks (every position visited again)
    }
    if (RK != nullptr && tl <= 64u && size >= WAVE) {
        // pass 1: per 64-position chunk t, each symbol's count at RK[t][s]
        // (written by its lowest lane) and each lane's peers below, packed
        // four chunks per register
        const uint32_t nch = size / WAVE, kb = key_bits(tl);
        const uint64_t lanebit = 1ull << lane;
        for (uint32_t i = lane; i < nch * 64u / 8u; i += WAVE) reinterpret_cast<uint4*>(RK)[i] = make_uint4(0, 0, 0, 0);
        wave_sync();
        uint32_t below[(MAXCH + 3) / 4];
#pragma unroll
        for (uint32_t t = 0; t < MAXCH; ++t) {
            if ((t & 3u) == 0) below[t >> 2] = 0;
            if (t < nch) {
                const uint32_t sy = sym_at[t * WAVE + lane];
                const uint64_t peers = PM ? lds_peers(sy, PM, lanebit) : match_key(sy, ~0ull, kb);
                const uint32_t bl = (uint32_t)__popcll(peers & lanemask_lt());
                if (bl == 0) RK[t * 64u + sy] = (uint16_t)__popcll(peers);
                below[t >> 2] |= bl << (8u * (t & 3u));
            }
        }
        wave_sync();
        SPREAD_STAMP(6);
        // per-symbol exclusive prefix over the chunks (lane = symbol), from
        // the symbol's base
        {
            uint32_t run = base(lane);
#pragma unroll
            for (uint32_t t = 0; t < MAXCH; ++t) {
                if (t < nch) {
                    const uint32_t c = RK[t * 64u + lane];
                    RK[t * 64u + lane] = (uint16_t)run;
                    run += c;
                }
            }
        }
        wave_sync();
        SPREAD_STAMP(7);
        // pass 2: rank = the symbol's count in earlier chunks + peers below
#pragma unroll
        for (uint32_t t = 0; t < MAXCH; ++t) {
            if (t < nch) {
                const uint32_t i = t * WAVE + lane;
                const uint32_t sy = sym_at[i];
                visit(i, sy, (uint32_t)RK[t * 64u + sy] + ((below[t >> 2] >> (8u * (t & 3u))) & 0xFFu));
            }
        }
        wave_sync();
        return FSE_OK;
    }
    // occurrence ranks in ascending position order (PM: occ_sym is dead by
    // now, so the caller may alias the masks into it)
    const bool lds_match = PM != nullptr && tl <= 64u && size >= WAVE;
    const uint64_t lanebit = 1ull << lane;
    for (uint32_t s = lane; s < 256; s += WAVE) cnt[s] = base(s);
    wave_sync();
    for (uint32_t i0 = 0; i0 < size; i0 += WAVE) {
        uint32_t i = i0 + lane;
        bool act = i < size;
        uint64_t active = __ballot(act);
        uint32_t s = act ? sym_at[i] : 0u;
        uint64_t peers = lds_match ? lds_peers(s, PM, lanebit) : match_key(s, active, key_bits(tl));
        uint32_t before = act ? cnt[s] : 0u;
        uint32_t r = before + (uint32_t)__popcll(peers & lanemask_lt());
        wave_sync();
        bool leader = act && ((peers & lanemask_lt()) == 0);
        if (leader) cnt[s] = before + (uint32_t)__popcll(peers);
        if (act) visit(i, s, r);
        wave_sync();
    }
    return FSE_OK;
#undef SPREAD_STAMP
}

}  // namespace fsehip
