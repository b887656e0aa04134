// fse_kernels.hip -- batched FSE (tANS) block codec kernels for gfx950.
//
// Wire format: exactly the reference's fse_compress2 block (lib.rs:146-183):
// NCount header || 2-state payload (backward bit stack + marker bit).
//
// Encode (one 64-lane workgroup = BPW blocks x T lanes):
//   1. per block, one wave: histogram -> normalise -> header -> tables (LDS)
//   2. per block, T lanes, each owning S contiguous pairs:
//        spec  : state-only pass from a guessed state (warms the boundary)
//        count : exact bit count from the neighbour's spec end state
//        verify: redo any lane whose assumed start state was wrong (exact)
//        scan  : per-lane bit offsets (the stack writes high pairs first)
//        emit  : bits written straight to the output slot; the two partial
//                words at each lane boundary are OR-merged through LDS
//      The encoder also records decode checkpoints (the sidecar index).
// Decode (one 64-lane workgroup per block): header parse, decode table in
//   LDS, then each lane decodes the checkpoint segments assigned to it.
//   Without a sidecar one lane decodes the block serially (reference mode).
#include "fse_device.hpp"
#include "fse_kernels.h"

namespace fsehip {

// ------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------
__device__ __forceinline__ uint4 load_chunk(const uint8_t* blk, uint32_t n, uint32_t c) {
    const uint32_t off = c << 4;
    if (off + 16u <= n) return *reinterpret_cast<const uint4*>(blk + off);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t i = 0; i < 16u && off + i < n; ++i) w[i >> 2] |= (uint32_t)blk[off + i] << (8u * (i & 3u));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Encoder state step (Encoder::encode_raw, fse.rs:227-239).
struct EncTab {
    const uint16_t* st;
    const uint2* tt;  // {deltaNbBits, deltaFindState}
};

// Bit emitter into a 32-bit-word view of the output slot.  Bits are
// appended LSB-first (writer.rs:140-180); the first word is partial when the
// lane's offset is not word aligned and is handed to the merge step.
struct Emit {
    uint64_t acc;
    uint32_t nacc;
    uint32_t word;
    uint32_t* gw;
    bool head;
    uint32_t head_word, head_val;
    __device__ __forceinline__ void start(uint32_t* g, uint32_t off) {
        gw = g;
        acc = 0;
        nacc = off & 31u;
        word = off >> 5;
        head = nacc != 0;
        head_word = 0xFFFFFFFFu;
        head_val = 0;
    }
    __device__ __forceinline__ void put(uint32_t v, uint32_t nb) {
        acc |= (uint64_t)v << nacc;
        nacc += nb;
    }
    __device__ __forceinline__ void flush() {
        if (nacc >= 32) {
            uint32_t val = (uint32_t)acc;
            if (head) {
                head = false;
                head_word = word;
                head_val = val;
            } else {
                gw[word] = val;
            }
            word++;
            acc >>= 32;
            nacc -= 32;
        }
    }
    __device__ __forceinline__ uint32_t pos() const { return word * 32u + nacc; }
};

struct Ckpt {
    uint64_t* base;  // this block's sidecar entries, or nullptr
    uint32_t mask;   // interval - 1 (interval is a power of two)
    uint32_t shift;  // log2(interval)
    uint32_t hdr_bits;
    uint32_t L;
};

enum { PASS_SPEC = 0, PASS_COUNT = 1, PASS_EMIT = 2 };

template <int MODE>
__device__ __forceinline__ void enc_sym(uint32_t& x, uint32_t s, const EncTab& T, uint32_t& bits, Emit& em) {
    const uint2 t = T.tt[s];
    const uint32_t nb = (t.x + x) >> 16;
    if (MODE == PASS_COUNT) bits += nb;
    if (MODE == PASS_EMIT) em.put(x & ((1u << nb) - 1u), nb);
    x = T.st[(int32_t)(x >> nb) + (int32_t)t.y];
}

// Encode pairs pb-1 down to pa (lib.rs:167-176: E1 then E0 per pair).
template <int MODE>
__device__ void enc_range(const uint8_t* __restrict__ blk, uint32_t n, uint32_t pa, uint32_t pb, uint32_t& x0,
                          uint32_t& x1, const EncTab& T, uint32_t& bits, Emit& em, const Ckpt& ck) {
    if (pb <= pa) return;
    const int32_t c_hi = (int32_t)((pb - 1u) >> 3), c_lo = (int32_t)(pa >> 3);
    uint4 cur = load_chunk(blk, n, (uint32_t)c_hi);
    for (int32_t c = c_hi; c >= c_lo; --c) {
        uint4 nxt = (c > c_lo) ? load_chunk(blk, n, (uint32_t)(c - 1)) : make_uint4(0, 0, 0, 0);
        const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
        for (int j = 7; j >= 0; --j) {
            const uint32_t p = (uint32_t)c * 8u + (uint32_t)j;
            if (p < pb && p >= pa) {
                const uint32_t sh = 16u * (uint32_t)(j & 1);
                const uint32_t s0 = (w[j >> 1] >> sh) & 0xFFu;
                const uint32_t s1 = (w[j >> 1] >> (sh + 8u)) & 0xFFu;
                enc_sym<MODE>(x1, s1, T, bits, em);
                enc_sym<MODE>(x0, s0, T, bits, em);
                if (MODE == PASS_EMIT) {
                    em.flush();
                    if (ck.base && (p & ck.mask) == 0u) {
                        const uint64_t e = (uint64_t)(em.pos() - ck.hdr_bits) |
                                           ((uint64_t)(x0 - (1u << ck.L)) << 32) |
                                           ((uint64_t)(x1 - (1u << ck.L)) << 48);
                        ck.base[p >> ck.shift] = e;
                    }
                }
            }
        }
        cur = nxt;
    }
}

// Encoder::new_first_symbol, fse.rs:210-218
__device__ __forceinline__ uint32_t enc_init(const EncTab& T, uint32_t s) {
    const uint2 t = T.tt[s];
    const uint32_t bo = (t.x + (1u << 15)) >> 16;
    const uint32_t v = (bo << 16) - t.x;
    return T.st[(int32_t)(v >> bo) + (int32_t)t.y];
}

// ------------------------------------------------------------------------
// Encode kernel
// ------------------------------------------------------------------------
template <int LMAX, int T>
struct EncSmem {
    static constexpr int BPW = 64 / T;
    static constexpr uint32_t SIZE = 1u << LMAX;
    uint16_t st[BPW][SIZE];
    uint2 tt[BPW][256];
    uint8_t hdr[BPW][HDR_MAX];
    union {
        uint32_t h4[1024];
        struct {
            uint8_t sym_at[SIZE];
            uint8_t occ_sym[SIZE];
        } sp;
    } tmp;
    uint32_t counts[256];
    int32_t norm[256];
    uint16_t cumul[256];
    uint32_t cnt[256];
    int32_t info_status[BPW];
    uint32_t info_L[BPW];
    uint32_t info_hl[BPW];
    uint32_t specF[BPW][T + 1];
    uint32_t cntF[BPW][T + 1];
    uint32_t mword[BPW][2 * (T + 1)];
    uint32_t mval[BPW][2 * (T + 1)];
    int scratch[4];
};

template <int LMAX, int T>
__global__ __launch_bounds__(64) void encode_blocks_kernel(EncParams P) {
    constexpr int BPW = 64 / T;
    __shared__ EncSmem<LMAX, T> sm;
    const uint32_t lane = lane_id();

    // ---- phase 1: statistics, header and tables, one block at a time
    for (int b = 0; b < BPW; ++b) {
        const uint64_t gb = (uint64_t)blockIdx.x * BPW + b;
        if (gb >= P.n_blocks) {
            if (lane == 0) sm.info_status[b] = 1;  // no block
            continue;
        }
        const uint64_t off = gb * P.block_size;
        const uint32_t n = (uint32_t)min((uint64_t)P.block_size, P.n_total - off);
        const uint8_t* blk = P.src + off;
        const uint32_t tl = wave_histogram(blk, n, sm.tmp.h4, sm.counts);
        int rc = FSE_OK;
        uint32_t Lreq = P.table_log, L = 0, slow = 0;
        if (n == 0) rc = FSE_ERR_EMPTY;
        if (rc == FSE_OK && P.table_log == 0) rc = optimal_log2(n, tl, &Lreq);  // histogram.rs:301
        if (rc == FSE_OK) rc = wave_normalize(sm.counts, n, tl, Lreq, sm.norm, &L, &slow, sm.scratch);
        if (rc == FSE_OK && n < 2) rc = FSE_ERR_TOO_SHORT;  // lib.rs:154/156 unwrap
        if (rc == FSE_OK && L > (uint32_t)LMAX) rc = FSE_ERR_UNSUPPORTED;
        if (rc == FSE_OK) {
            if (lane == 0) sm.scratch[1] = header_write_lane(sm.norm, L, tl, sm.hdr[b]);
            __syncthreads();
            if (sm.scratch[1] < 0) rc = sm.scratch[1];
        }
        if (rc == FSE_OK) {
            const uint32_t size = 1u << L;
            uint16_t* st = sm.st[b];
            const uint16_t* cumul = sm.cumul;
            rc = wave_build_spread(sm.norm, L, tl, sm.tmp.sp.sym_at, sm.tmp.sp.occ_sym, sm.cumul, sm.cnt,
                                   [&](uint32_t i, uint32_t s, uint32_t r) {
                                       st[cumul[s] + r] = (uint16_t)(size + i);  // fse.rs:157-162
                                   });
            // symbol transforms, fse.rs:165-188 (total == cumul[s])
            for (uint32_t s = lane; s < 256; s += WAVE) {
                int32_t x = (s < tl) ? sm.norm[s] : 0;
                uint2 t = make_uint2(0, 0);
                if (s < tl) {
                    const int32_t tot = (int32_t)sm.cumul[s];
                    if (x == 0) {
                        t.x = ((L + 1u) << 16) - (1u << L);
                    } else if (x == -1 || x == 1) {
                        t.x = (L << 16) - (1u << L);
                        t.y = (uint32_t)(tot - 1);
                    } else {
                        const uint32_t mb = L - ilog2u((uint32_t)(x - 1));
                        t.x = (mb << 16) - ((uint32_t)x << mb);
                        t.y = (uint32_t)(tot - x);
                    }
                }
                sm.tt[b][s] = t;
            }
        }
        if (lane == 0) {
            sm.info_status[b] = rc;
            sm.info_L[b] = L;
            sm.info_hl[b] = (rc == FSE_OK) ? (uint32_t)sm.scratch[1] : 0u;
            if (rc != FSE_OK) {
                P.status[gb] = rc;
                P.comp_len[gb] = 0;
                if (P.payload_bits) P.payload_bits[gb] = 0;
            }
        }
        __syncthreads();
    }

    // ---- phase 2: T lanes per block
    const int b = (int)(lane / T);
    const uint32_t k = lane % T;
    const uint64_t gb = (uint64_t)blockIdx.x * BPW + b;
    const bool live = sm.info_status[b] == FSE_OK;
    const uint64_t boff = gb * P.block_size;
    const uint32_t n = live ? (uint32_t)min((uint64_t)P.block_size, P.n_total - boff) : 0u;
    const uint8_t* blk = P.src + boff;
    const uint32_t L = sm.info_L[b];
    const EncTab tab{sm.st[b], sm.tt[b]};
    const uint32_t Pm = live ? ((n & 1u) ? (n - 3u) / 2u : n / 2u - 1u) : 0u;
    uint32_t S = (Pm + T - 1u) / T;
    S = max(8u, (S + 7u) & ~7u);
    const uint32_t ktop = Pm ? (Pm - 1u) / S : 0u;
    const bool act = live && k <= ktop;
    const uint32_t pa = k * S, pb = min(pa + S, Pm);
    Emit em;
    em.start(nullptr, 0);
    Ckpt ck{nullptr, 0, 0, 0, L};
    uint32_t bits = 0;

    // exact start of the top lane: init states (+ odd-length extra step)
    auto top_start = [&](uint32_t& x0, uint32_t& x1, uint32_t& bts, Emit& e, bool emit, bool count) {
        if (n & 1u) {  // lib.rs:155-160
            x0 = enc_init(tab, blk[n - 1u]);
            x1 = enc_init(tab, blk[n - 2u]);
            const uint32_t s = blk[n - 3u];
            const uint2 t = tab.tt[s];
            const uint32_t nb = (t.x + x0) >> 16;
            if (count) bts += nb;
            if (emit) {
                e.put(x0 & ((1u << nb) - 1u), nb);
                e.flush();
            }
            x0 = tab.st[(int32_t)(x0 >> nb) + (int32_t)t.y];
        } else {  // lib.rs:161-165
            x0 = enc_init(tab, blk[n - 2u]);
            x1 = enc_init(tab, blk[n - 1u]);
        }
    };

    // spec pass: lanes 1..ktop (the top lane runs exactly)
    uint32_t x0 = 0, x1 = 0;
    if (act && k >= 1) {
        if (k == ktop) {
            top_start(x0, x1, bits, em, false, false);
        } else {
            x0 = x1 = 1u << L;
        }
        enc_range<PASS_SPEC>(blk, n, pa, pb, x0, x1, tab, bits, em, ck);
        sm.specF[b][k] = x0 | (x1 << 16);
    }
    __syncthreads();

    // count pass from the neighbour's spec end state
    uint32_t start = 0;
    auto count_pass = [&](uint32_t st0) {
        uint32_t y0, y1, bt = 0;
        if (k == ktop) {
            top_start(y0, y1, bt, em, false, true);
        } else {
            y0 = st0 & 0xFFFFu;
            y1 = st0 >> 16;
        }
        enc_range<PASS_COUNT>(blk, n, pa, pb, y0, y1, tab, bt, em, ck);
        if (k == 0) bt += 2u * L + 1u;  // finals + marker (lib.rs:178-181)
        sm.cntF[b][k] = y0 | (y1 << 16);
        return bt;
    };
    if (act) {
        start = (k < ktop) ? sm.specF[b][k + 1] : 0u;
        bits = count_pass(start);
    }
    // verify: a lane's start must equal its neighbour's exact end state.
    // Iterates to the unique fixed point (the top lane is exact).
    for (;;) {
        __syncthreads();
        bool bad = false;
        uint32_t nbF = 0;
        if (act && k < ktop) {
            nbF = sm.cntF[b][k + 1];
            bad = nbF != start;
        }
        __syncthreads();
        if (__ballot(bad) == 0) break;
        if (bad) {
            start = nbF;
            bits = count_pass(start);
        }
    }

    // offsets: lane k writes after every lane j > k (stack order)
    const uint32_t hl = sm.info_hl[b];
    const uint32_t hdr_bits = hl * 8u;
    uint32_t mybits = act ? bits : 0u;
    uint32_t suffix = mybits;  // inclusive suffix sum over lanes >= k within the block
#pragma unroll
    for (int d = 1; d < T; d <<= 1) {
        uint32_t o = __shfl_down(suffix, d, T);
        if (k + d < T) suffix += o;
    }
    const uint32_t total_bits = hdr_bits + __shfl(suffix, 0, T);
    const uint32_t off = hdr_bits + suffix - mybits;
    const bool fits = (uint64_t)total_bits <= P.slot_bytes * 8ull;
    uint32_t* gw = reinterpret_cast<uint32_t*>(P.out + gb * P.slot_bytes);

    // emit pass
    for (uint32_t e = k; e < 2u * (T + 1u); e += T) {
        if (b < BPW) sm.mword[b][e] = 0xFFFFFFFFu;
    }
    __syncthreads();
    if (act && fits) {
        em.start(gw, off);
        if (P.sidecar && P.ckpt_interval) {
            ck.base = P.sidecar + gb * P.ckpt_per_block;
            ck.mask = P.ckpt_interval - 1u;
            ck.shift = 31u - __clz(P.ckpt_interval);
            ck.hdr_bits = hdr_bits;
        }
        uint32_t y0, y1, bt = 0;
        if (k == ktop) {
            top_start(y0, y1, bt, em, true, false);
            if (ck.base && (Pm & ck.mask) == 0u) {  // checkpoint "before pair Pm"
                ck.base[Pm >> ck.shift] = (uint64_t)(em.pos() - hdr_bits) | ((uint64_t)(y0 - (1u << L)) << 32) |
                                          ((uint64_t)(y1 - (1u << L)) << 48);
            }
        } else {
            y0 = start & 0xFFFFu;
            y1 = start >> 16;
        }
        enc_range<PASS_EMIT>(blk, n, pa, pb, y0, y1, tab, bt, em, ck);
        if (k == 0) {  // Encoder::finish x2 + marker (lib.rs:178-181)
            const uint32_t m = (1u << L) - 1u;
            em.put(y1 & m, L);
            em.flush();
            em.put(y0 & m, L);
            em.flush();
            em.put(1u, 1u);
            em.flush();
        }
        // boundary words -> merge list (entry order = stream order)
        const uint32_t slot = 2u * (T - k);
        if (!em.head) {
            sm.mword[b][slot] = em.head_word;
            sm.mval[b][slot] = em.head_val;
        }
        if (em.nacc) {
            sm.mword[b][slot + 1] = em.word;
            sm.mval[b][slot + 1] = (uint32_t)em.acc;
        }
    }
    // header: whole words stored directly, the last partial word merged
    if (live && fits) {
        const uint8_t* h = sm.hdr[b];
        for (uint32_t w = k; w < hl / 4u; w += T)
            gw[w] = (uint32_t)h[4 * w] | ((uint32_t)h[4 * w + 1] << 8) | ((uint32_t)h[4 * w + 2] << 16) |
                    ((uint32_t)h[4 * w + 3] << 24);
        if (k == 0 && (hl & 3u)) {
            uint32_t v = 0;
            for (uint32_t i = hl & ~3u; i < hl; ++i) v |= (uint32_t)h[i] << (8u * (i & 3u));
            sm.mword[b][0] = hl / 4u;
            sm.mval[b][0] = v;
        }
    }
    __syncthreads();
    // merge: each run of equal word indices is OR-ed by its first entry
    if (live && fits) {
        constexpr uint32_t NE = 2u * (T + 1u);
        for (uint32_t e = k; e < NE; e += T) {
            const uint32_t w = sm.mword[b][e];
            if (w == 0xFFFFFFFFu) continue;
            bool first = true;
            for (int q = (int)e - 1; q >= 0; --q) {
                const uint32_t wq = sm.mword[b][q];
                if (wq == 0xFFFFFFFFu) continue;
                first = (wq != w);
                break;
            }
            if (!first) continue;
            uint32_t v = sm.mval[b][e];
            for (uint32_t q = e + 1; q < NE; ++q) {
                const uint32_t wq = sm.mword[b][q];
                if (wq == 0xFFFFFFFFu) continue;
                if (wq != w) break;
                v |= sm.mval[b][q];
            }
            gw[w] = v;
        }
    }
    if (live && k == 0) {
        if (fits) {
            P.status[gb] = FSE_OK;
            P.comp_len[gb] = (total_bits + 7u) >> 3;
            if (P.payload_bits) P.payload_bits[gb] = total_bits - hdr_bits;
        } else {
            P.status[gb] = FSE_ERR_DST_TOO_SMALL;
            P.comp_len[gb] = 0;
        }
    }
}

// ------------------------------------------------------------------------
// Decode
// ------------------------------------------------------------------------
// Backward bit reader over the block's 32-bit words (BitStackReader
// semantics, stack_reader.rs:17-215): `pos` = bits remaining above the
// block start; buf holds stream bits [base, base+64).
struct BitReader {
    const uint32_t* words;
    uint64_t buf;
    int32_t base;
    int32_t pos;
    __device__ __forceinline__ void init(const uint32_t* w, int32_t p) {
        words = w;
        pos = p;
        int32_t top = (p + 31) & ~31;
        base = top - 64;
        if (base < 0) base = 0;
        buf = (uint64_t)words[base >> 5] | ((uint64_t)words[(base >> 5) + 1] << 32);
    }
    __device__ __forceinline__ uint32_t pop(uint32_t nb) {
        pos -= (int32_t)nb;
        return (uint32_t)(buf >> (uint32_t)(pos - base)) & ((1u << nb) - 1u);
    }
    __device__ __forceinline__ void refill() {
        if (pos - base < 32 && base > 0) {
            base -= 32;
            buf = (buf << 32) | (uint64_t)words[base >> 5];
        }
    }
};

template <int LMAX>
struct DecSmem {
    static constexpr uint32_t SIZE = 1u << LMAX;
    // dt[i] = new_state | symbol << 16 | nb << 24; the spread scratch lives
    // in the top half of the same array (see wave_build_spread call).
    uint32_t dt[SIZE];
    int32_t norm[256];
    uint16_t cumul[256];
    uint32_t cnt[256];
    int scratch[4];
};

__device__ __forceinline__ void store_byte(uint8_t* out, uint32_t i, uint32_t lim, uint32_t v) {
    if (i < lim) out[i] = (uint8_t)v;
}

template <int LMAX>
__global__ __launch_bounds__(64) void decode_blocks_kernel(DecParams P) {
    __shared__ DecSmem<LMAX> sm;
    const uint32_t lane = lane_id();
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = P.comp_len[gb];
    const uint64_t ooff = gb * (uint64_t)P.block_size;
    // raw length: container length, or unknown (reference mode) with cap
    const bool known = P.n_total != 0;
    const uint32_t n = known ? (uint32_t)min((uint64_t)P.block_size, P.n_total - ooff) : 0u;
    const uint32_t cap = known ? n : P.out_cap;
    uint8_t* out = P.out + ooff;

    uint32_t L = 0, tl = 0;
    if (lane == 0) {
        int hl = header_read_lane(in, clen, sm.norm, &L, &tl);  // lib.rs:219
        sm.scratch[0] = hl;
        sm.scratch[1] = (int)L;
        sm.scratch[2] = (int)tl;
    }
    __syncthreads();
    int rc = FSE_OK;
    const int hl = sm.scratch[0];
    L = (uint32_t)sm.scratch[1];
    tl = (uint32_t)sm.scratch[2];
    if (hl < 0) rc = hl;
    if (rc == FSE_OK && L > (uint32_t)LMAX) rc = FSE_ERR_UNSUPPORTED;
    if (rc == FSE_OK && ((uint32_t)hl >= clen || in[clen - 1] == 0)) rc = FSE_ERR_NO_MARKER;  // lib.rs:222
    const uint32_t size = 1u << L;
    bool single = false;
    if (rc == FSE_OK) {
        uint8_t* scr = reinterpret_cast<uint8_t*>(sm.dt);
        const int32_t* norm = sm.norm;
        uint32_t* dt = sm.dt;
        rc = wave_build_spread(sm.norm, L, tl, scr + 3u * size, scr + 2u * size, sm.cumul, sm.cnt,
                               [&](uint32_t i, uint32_t s, uint32_t r) {  // fse.rs:329-337
                                   const int32_t v = norm[s];
                                   const uint32_t nx = (v == -1 || v < -1 ? 1u : (uint32_t)v) + r;
                                   const uint32_t nb = L - ilog2u(nx);
                                   dt[i] = (((nx << nb) - size) & 0xFFFFu) | (s << 16) | (nb << 24);
                               });
        for (uint32_t s = lane; s < 256; s += WAVE)
            if (s < tl && sm.norm[s] == (int32_t)size) single = true;
        single = __ballot(single) != 0;
    }
    __syncthreads();
    if (rc == FSE_OK && single && !known) rc = FSE_ERR_SINGLE_SYMBOL;
    if (rc == FSE_OK && known && n < 2) rc = FSE_ERR_LENGTH_MISMATCH;
    if (rc != FSE_OK) {
        if (lane == 0) {
            P.status[gb] = rc;
            if (P.out_len) P.out_len[gb] = 0;
        }
        return;
    }
    const int32_t hdr_bits = hl * 8;
    const int32_t top = (int32_t)(clen - 1u) * 8 + (int32_t)ilog2u(in[clen - 1]);
    const uint32_t* words = reinterpret_cast<const uint32_t*>(in);
    const uint32_t* dt = sm.dt;
    const uint32_t smask = size - 1u;

    if (P.sidecar && known) {
        // ---- parallel: lane j decodes checkpoint segments j, j+64, ...
        const uint32_t Pm = (n & 1u) ? (n - 3u) / 2u : n / 2u - 1u;
        const uint32_t I = P.ckpt_interval;
        const uint32_t nseg = Pm / I + 1u;
        const uint64_t* sc = P.sidecar + gb * P.ckpt_per_block;
        int32_t err = FSE_OK;
        for (uint32_t seg = lane; seg < nseg; seg += WAVE) {
            const uint64_t e = sc[seg];
            BitReader br;
            br.init(words, hdr_bits + (int32_t)(uint32_t)e);
            uint32_t s0 = (uint32_t)(e >> 32) & 0xFFFFu, s1 = (uint32_t)(e >> 48);
            const uint32_t p0 = seg * I;
            const uint32_t p1 = min(p0 + I, Pm);
            uint32_t p = p0;
            // whole 8-pair chunks: 16-byte stores
            for (; p + 8u <= p1; p += 8u) {
                uint32_t w[4];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t e0 = dt[s0 & smask], e1 = dt[s1 & smask];
                    const uint32_t nb0 = e0 >> 24;
                    const uint32_t v0 = br.pop(nb0);
                    const uint32_t nb1 = e1 >> 24;
                    const uint32_t v1 = br.pop(nb1);
                    s0 = ((e0 & 0xFFFFu) + v0) & 0xFFFFu;
                    s1 = ((e1 & 0xFFFFu) + v1) & 0xFFFFu;
                    const uint32_t pr = ((e0 >> 16) & 0xFFu) | (e1 & 0xFF0000u) >> 8;
                    if (j & 1) w[j >> 1] |= pr << 16; else w[j >> 1] = pr;
                    br.refill();
                }
                *reinterpret_cast<uint4*>(out + 2u * p) = make_uint4(w[0], w[1], w[2], w[3]);
            }
            for (; p < p1; ++p) {
                const uint32_t e0 = dt[s0 & smask], e1 = dt[s1 & smask];
                const uint32_t v0 = br.pop(e0 >> 24);
                const uint32_t v1 = br.pop(e1 >> 24);
                s0 = ((e0 & 0xFFFFu) + v0) & 0xFFFFu;
                s1 = ((e1 & 0xFFFFu) + v1) & 0xFFFFu;
                out[2u * p] = (uint8_t)(e0 >> 16);
                out[2u * p + 1u] = (uint8_t)(e1 >> 16);
                br.refill();
            }
            if (seg == nseg - 1u) {
                // termination in container mode (oracle decompress2_impl),
                // mirroring lib.rs:227-244
                uint32_t o = 2u * Pm;
                for (;;) {
                    if (o + 2u == n) {
                        out[o++] = (uint8_t)(dt[s0 & smask] >> 16);
                        out[o++] = (uint8_t)(dt[s1 & smask] >> 16);
                        break;
                    }
                    if (o + 1u == n) {
                        out[o++] = (uint8_t)(dt[s0 & smask] >> 16);
                        break;
                    }
                    uint32_t e0 = dt[s0 & smask];
                    uint32_t nb = e0 >> 24;
                    if (br.pos - (int32_t)nb < hdr_bits) {
                        out[o++] = (uint8_t)(e0 >> 16);
                        if (o < n) out[o++] = (uint8_t)(dt[s1 & smask] >> 16);
                        break;
                    }
                    s0 = ((e0 & 0xFFFFu) + br.pop(nb)) & 0xFFFFu;
                    br.refill();
                    out[o++] = (uint8_t)(e0 >> 16);
                    if (o >= n) { err = FSE_ERR_LENGTH_MISMATCH; break; }
                    uint32_t e1 = dt[s1 & smask];
                    nb = e1 >> 24;
                    if (br.pos - (int32_t)nb < hdr_bits) {
                        out[o++] = (uint8_t)(e1 >> 16);
                        if (o < n) out[o++] = (uint8_t)(dt[s0 & smask] >> 16);
                        break;
                    }
                    s1 = ((e1 & 0xFFFFu) + br.pop(nb)) & 0xFFFFu;
                    br.refill();
                    out[o++] = (uint8_t)(e1 >> 16);
                    if (o >= n) { err = FSE_ERR_LENGTH_MISMATCH; break; }
                }
                if (o != n) err = FSE_ERR_LENGTH_MISMATCH;
            }
        }
        err = (int32_t)wave_max((uint32_t)(-err));
        if (lane == 0) {
            P.status[gb] = -err;
            if (P.out_len) P.out_len[gb] = err ? 0u : n;
        }
        return;
    }

    // ---- serial (reference mode or no sidecar): one lane, every read
    // checked (lib.rs:215-248); optionally records the sidecar index.
    if (lane != 0) return;
    BitReader br;
    br.init(words, top);
    int32_t err = FSE_OK;
    uint32_t o = 0;
    if (br.pos - (int32_t)L < hdr_bits) err = FSE_ERR_TOO_SHORT;  // lib.rs:224
    uint32_t s0 = 0, s1 = 0;
    if (err == FSE_OK) {
        s0 = br.pop(L);
        br.refill();
        if (br.pos - (int32_t)L < hdr_bits) err = FSE_ERR_TOO_SHORT;  // lib.rs:225
    }
    if (err == FSE_OK) {
        s1 = br.pop(L);
        br.refill();
        const uint32_t I = P.ckpt_interval;
        uint64_t* rec = (P.sidecar_out && I) ? P.sidecar_out + gb * P.ckpt_per_block : nullptr;
        const uint32_t ckmask = I ? I - 1u : 0u;
        for (uint32_t pidx = 0;; ++pidx) {
            if (rec && (pidx & ckmask) == 0u && pidx / I < P.ckpt_per_block)
                rec[pidx / I] = (uint64_t)(uint32_t)(br.pos - hdr_bits) | ((uint64_t)s0 << 32) |
                                ((uint64_t)s1 << 48);
            if (known && o + 2u == n) {
                store_byte(out, o++, cap, dt[s0 & smask] >> 16);
                store_byte(out, o++, cap, dt[s1 & smask] >> 16);
                break;
            }
            if (known && o + 1u == n) {
                store_byte(out, o++, cap, dt[s0 & smask] >> 16);
                break;
            }
            const uint32_t e0 = dt[s0 & smask];
            uint32_t nb = e0 >> 24;
            if (br.pos - (int32_t)nb < hdr_bits) {  // decode0 fails: 242-243
                if (o + 2u > cap) { err = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL; break; }
                store_byte(out, o++, cap, e0 >> 16);
                store_byte(out, o++, cap, dt[s1 & smask] >> 16);
                break;
            }
            s0 = ((e0 & 0xFFFFu) + br.pop(nb)) & 0xFFFFu;
            br.refill();
            if (o >= cap) { err = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL; break; }
            store_byte(out, o++, cap, e0 >> 16);
            const uint32_t e1 = dt[s1 & smask];
            nb = e1 >> 24;
            if (br.pos - (int32_t)nb < hdr_bits) {  // decode1 fails: 235-239
                if (o + 2u > cap) { err = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL; break; }
                store_byte(out, o++, cap, e1 >> 16);
                store_byte(out, o++, cap, dt[s0 & smask] >> 16);
                break;
            }
            s1 = ((e1 & 0xFFFFu) + br.pop(nb)) & 0xFFFFu;
            br.refill();
            if (o >= cap) { err = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL; break; }
            store_byte(out, o++, cap, e1 >> 16);
        }
    }
    if (err == FSE_OK && known && o != n) err = FSE_ERR_LENGTH_MISMATCH;
    P.status[gb] = err;
    if (P.out_len) P.out_len[gb] = err ? 0u : o;
}

// ------------------------------------------------------------------------
// Histogram::new per block (histogram::count), one wave per block.
// ------------------------------------------------------------------------
__global__ __launch_bounds__(64) void histogram_blocks_kernel(const uint8_t* src, uint64_t n_total,
                                                              uint32_t block_size, uint32_t n_blocks,
                                                              uint32_t* counts, uint32_t* table_len) {
    __shared__ uint32_t h4[1024];
    __shared__ uint32_t cnts[256];
    const uint64_t gb = blockIdx.x;
    if (gb >= n_blocks) return;
    const uint64_t off = gb * block_size;
    const uint32_t n = (uint32_t)min((uint64_t)block_size, n_total - off);
    const uint32_t tl = wave_histogram(src + off, n, h4, cnts);
    for (uint32_t s = lane_id(); s < 256; s += WAVE) counts[gb * 256 + s] = cnts[s];
    if (lane_id() == 0 && table_len) table_len[gb] = tl;
}

// ------------------------------------------------------------------------
// Synthetic generator (same definition as oracle fo_generate).
// ------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void generate_kernel(GenParams G) {
    const uint64_t GOLDEN = 0x9E3779B97F4A7C15ull;
    const uint64_t i16 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16ull;
    if (i16 >= G.n_total) return;
    uint32_t w[4] = {0, 0, 0, 0};
    for (int j = 0; j < 16; ++j) {
        const uint64_t i = i16 + j;
        if (i >= G.n_total) break;
        const uint64_t b = i / G.block_size, r = i - b * G.block_size;
        const uint64_t sb = G.seed ^ (b * GOLDEN);
        const uint64_t x = mix64(sb + (r + 1ull) * GOLDEN);
        uint32_t v;
        if (G.kind == 0) {
            const uint32_t idx = (uint32_t)(x & 4095u);
            uint32_t lo = 0, hi = G.nsym - 1u;  // last symbol whose LUT start <= idx
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1u) >> 1;
                if (G.bound[mid] <= idx) lo = mid; else hi = mid - 1u;
            }
            v = lo & 0xFFu;
        } else if (G.kind == 1) {
            const uint32_t c = (uint32_t)__builtin_ctzll(x | (1ull << 63));
            v = c > 255u ? 255u : c;
        } else {
            v = (uint32_t)(((x >> 32) * 240ull) >> 32);
        }
        w[j >> 2] |= v << (8 * (j & 3));
    }
    if (i16 + 16 <= G.n_total) {
        *reinterpret_cast<uint4*>(G.out + i16) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
        for (uint64_t j = 0; i16 + j < G.n_total; ++j) G.out[i16 + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    }
}

// ------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------
hipError_t launch_encode(const EncParams& P, uint32_t lmax, hipStream_t stream) {
    const uint32_t grid = (P.n_blocks + 1u) / 2u;  // T = 32 lanes, 2 blocks per workgroup
    if (lmax <= 11) {
        hipLaunchKernelGGL((encode_blocks_kernel<11, 32>), dim3(grid), dim3(64), 0, stream, P);
    } else {
        hipLaunchKernelGGL((encode_blocks_kernel<12, 32>), dim3(grid), dim3(64), 0, stream, P);
    }
    return hipGetLastError();
}

hipError_t launch_decode(const DecParams& P, uint32_t lmax, hipStream_t stream) {
    if (lmax <= 11) {
        hipLaunchKernelGGL((decode_blocks_kernel<11>), dim3(P.n_blocks), dim3(64), 0, stream, P);
    } else {
        hipLaunchKernelGGL((decode_blocks_kernel<12>), dim3(P.n_blocks), dim3(64), 0, stream, P);
    }
    return hipGetLastError();
}

hipError_t launch_histogram(const uint8_t* src, uint64_t n_total, uint32_t block_size, uint32_t n_blocks,
                            uint32_t* counts, uint32_t* table_len, hipStream_t stream) {
    hipLaunchKernelGGL(histogram_blocks_kernel, dim3(n_blocks), dim3(64), 0, stream, src, n_total, block_size,
                       n_blocks, counts, table_len);
    return hipGetLastError();
}

hipError_t launch_generate(const GenParams& G, hipStream_t stream) {
    const uint64_t threads = (G.n_total + 15) / 16;
    const uint32_t grid = (uint32_t)((threads + 255) / 256);
    hipLaunchKernelGGL(generate_kernel, dim3(grid), dim3(256), 0, stream, G);
    return hipGetLastError();
}

}  // namespace fsehip
