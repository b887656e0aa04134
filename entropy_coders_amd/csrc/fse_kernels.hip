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
#include <type_traits>

#include "fse_device.hpp"
#include "fse_kernels.h"

namespace fsehip {

// ------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------
// Diagnostic phase stamps (only when P.stamps is set by the host).
#define FSE_STAMP(P, slot)                                                                     \
    do {                                                                                       \
        if ((P).stamps && threadIdx.x == 0)                                                    \
            (P).stamps[(uint64_t)blockIdx.x * kStamps + (slot)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// Decode output group: pairs per lane between stores (32 pairs = 64 B, one
// HBM burst).  Segment starts are multiples of ckpt_interval, so groups are
// 64 B aligned whenever ckpt_interval >= 32.
constexpr uint32_t DEC_GROUP = 32;

__device__ __forceinline__ uint4 load_chunk(const uint8_t* blk, uint32_t n, uint32_t c) {
    const uint32_t off = c << 4;
    if (off + 16u <= n) return *reinterpret_cast<const uint4*>(blk + off);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t i = 0; i < 16u && off + i < n; ++i) w[i >> 2] |= (uint32_t)blk[off + i] << (8u * (i & 3u));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Encoder tables in LDS: stateTable (u16 entries, fse.rs:157-162) and the
// symbol transforms {deltaNbBits, LDS byte address of
// stateTable[deltaFindState]} (fse.rs:165-188): the block's table base is
// folded into the transform, so one state step is add, shift, shift-add,
// ds_read_u16 whichever table of the workgroup the lane uses.
struct EncTab {
    const uint2* tt;  // {deltaNbBits, LDS address of stateTable + 2 * deltaFindState}
};
typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
__device__ __forceinline__ uint32_t st_at(uint32_t lds_addr) {
    return *(lds_cu16*)(uintptr_t)lds_addr;
}
// LDS byte address of a __shared__ object
template <class P>
__device__ __forceinline__ uint32_t lds_addr_of(P* p) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) P*)p;
}

// Bit emitter into a 32-bit-word view of the output slot.  Bits are
// appended LSB-first (writer.rs:140-180); every completed word is stored,
// including the lane's first word, whose low bits belong to the previous
// lane: the merge step later rewrites each boundary word with the OR of both
// lanes' bits.
// Bit writer of one lane's range: BitStackWriter order (writer.rs:140-222),
// words through a 16-word LDS ring (RING_STRIDE words per lane: 16-byte
// aligned, conflict-free dwordx4 reads).  Every 8-word group of the slot
// that lies wholly inside the lane's range leaves as one 32-byte store (two
// dwordx4; L2 merges a lane's consecutive groups into whole lines) once the
// lane has moved past it; the partial groups at either end leave as dword
// stores.  (A 32-word ring with 64-byte groups needed 9 KiB of LDS per
// workgroup, which held the encoder at 8 workgroups per CU.)  The lane's first word, when
// it shares it with the lane above (off % 32 != 0), is never stored: its
// value (head_val) goes to the merge list, like the lane's last partial
// word.  Stores stay below wlim (the slot's words).
struct Emit {
    uint32_t lo, hi;    // pending bits: lo = the word being filled, hi = bits past it
    uint32_t nacc;
    uint32_t word;      // index of the word being filled
    uint32_t w0;        // first word index of the lane
    uint32_t head_val;  // lane's bits of word w0 (valid once word > w0 and the head group left)
    uint32_t wlim;      // words in the slot: stores never leave it
    uint32_t gs;        // next 8-word group to store
    bool skip_head;
    uint32_t* gw;
    uint32_t* ring;     // LDS, 16 words, 16-byte aligned
    __device__ __forceinline__ void start(uint32_t* g, uint32_t off, uint32_t lim = 0xFFFFFFFFu,
                                          uint32_t* r = nullptr) {
        gw = g;
        wlim = lim;
        ring = r;
        lo = hi = 0;
        nacc = off & 31u;
        word = off >> 5;
        w0 = word;
        gs = word >> 3;
        skip_head = (off & 31u) != 0u;
        head_val = 0;
    }
    __device__ __forceinline__ void put(uint32_t v, uint32_t nb) {
        const uint64_t t = (uint64_t)v << nacc;  // nacc < 64
        lo |= (uint32_t)t;
        hi |= (uint32_t)(t >> 32);
        nacc += nb;
    }
    // The ring slot of the word being filled is written every time: until
    // the word completes nothing reads it, so no branch is needed.  Callers
    // flush before nacc can reach 64 (<= 2 x 12 bits per flush).
    __device__ __forceinline__ void flush() {
        const bool f = nacc >= 32u;
        ring[word & 15u] = lo;
        lo = f ? hi : lo;
        hi = 0;  // nacc < 32 after the flush
        nacc &= 31u;
        word += f ? 1u : 0u;
    }
    __device__ __forceinline__ uint32_t pos() const { return word * 32u + nacc; }
    __device__ __forceinline__ void store_words(uint32_t a, uint32_t b) {
        for (uint32_t i = a; i < b; ++i)
            if (i < wlim) gw[i] = ring[i & 15u];
    }
    __device__ __forceinline__ void store_group(uint32_t g) {
        const uint32_t base = g << 3;
        if (g == (w0 >> 3) && ((w0 & 7u) != 0u || skip_head)) {  // the lane's first group: its own words only
            if (skip_head) head_val = ring[w0 & 15u];
            store_words(skip_head ? w0 + 1u : w0, base + 8u);
        } else if (base + 8u <= wlim) {
            const uint4* r = reinterpret_cast<const uint4*>(ring + (base & 15u));
            uint4* o = reinterpret_cast<uint4*>(gw + base);
            const uint4 a = r[0], b = r[1];
            o[0] = a;
            o[1] = b;
        }
    }
    // Store the group the lane has moved past, if any (called every <= 8
    // pairs: <= 6 new words, fewer than a group, so the ring never overruns
    // a pending group and at most one group completes between calls).
    __device__ __forceinline__ void drain() {
        if (word >= (gs + 1u) << 3) {
            store_group(gs);
            ++gs;
        }
    }
    // End of the lane: remaining whole groups, then the whole words of the
    // last group (the partial word stays in acc for the merge list).
    __device__ __forceinline__ void finish() {
        while (word >= (gs + 1u) << 3) {
            store_group(gs);
            ++gs;
        }
        uint32_t lo = gs << 3;
        if (gs == (w0 >> 3)) {
            lo = w0;
            if (skip_head) {
                lo = w0 + 1u;
                if (word > w0) head_val = ring[w0 & 15u];
            }
        }
        store_words(lo, word);
    }
};

// Words per lane of the emit ring in LDS: 16 used; the stride of 20 puts
// the 16 lanes of each dwordx4 read group on distinct 16-byte bank slots.
constexpr uint32_t RING_STRIDE = 20;

struct Ckpt {
    uint64_t* base;  // this block's sidecar entries, or nullptr
    uint32_t mask;   // interval - 1 (interval is a power of two, >= 8)
    uint32_t shift;  // log2(interval)
    uint32_t hdr_bits;
    uint32_t L;
};

// PASS_STATE: state chain only (the scratch path's count pass, no bits and
// no trajectory).
enum { PASS_STATE = 0, PASS_COUNT = 1, PASS_EMIT = 2, PASS_REPAIR = 3 };

// Trajectory of a count pass, for convergence-based repair: the state pair
// and running bit count after every ckc-th chunk (at most TRACK_SLOTS slots per lane,
// slot 0 = the lane's end).  A repair re-encodes from the corrected start
// state only until it meets the recorded trajectory: from there on states
// and bits are identical, so the lane's total follows from the record and
// its end state (its neighbour's start) is unchanged.
// Slots hold {x0 | x1 << 16, bits still to come after the slot}: a pass
// writes its running count there, and track_fixup turns the slots it wrote
// into remaining counts once the pass total is known, so every slot stays
// consistent with the lane's current trajectory.
// Trajectory slots per lane.  16 (repairs stop sooner) measured slower
// than 8 on C2: the count pass writes twice as many slots.
constexpr uint32_t TRACK_SLOTS = 8;
struct Track {
    uint2* cp;        // this lane's slots (LDS)
    uint32_t ckc;     // chunks per slot
    bool done;        // REPAIR: met the recorded trajectory
    uint32_t jstar;   // REPAIR: the slot where it did (slots above it were rewritten)
};

// After a pass with total `total`: slots above `jlo` (exclusive) hold
// running counts; make them remaining counts.
__device__ __forceinline__ void track_fixup(Track& tr, uint32_t nslot, int32_t jlo, uint32_t total) {
    for (int32_t j = (int32_t)nslot - 1; j > jlo; --j) tr.cp[j].y = total - tr.cp[j].y;
}

struct EncState {
    uint32_t x0, x1, bits;
};

// Encoder::encode_raw (fse.rs:227-239): returns nb, updates x.
__device__ __forceinline__ uint32_t enc_step(uint32_t& x, uint32_t s, const EncTab& T) {
    const uint2 t = T.tt[s];
    const uint32_t nb = (t.x + x) >> 16;
    x = st_at(((x >> nb) << 1) + t.y);
    return nb;
}

// One 16-byte chunk.  NS = 2 (fse_compress2): pairs c8+7 .. c8 (lib.rs:167-176:
// E1 then E0 per pair).  NS = 1 (fse_compress): symbols c8+15 .. c8 with one
// state (lib.rs:127-138).  FULL chunks need no guard; only the topmost chunk
// of the topmost lane can extend past the last main-loop step pb.
template <int MODE, bool FULL, int NS>
__device__ __forceinline__ void enc_chunk(const uint4& q, uint32_t c8, uint32_t pb, uint32_t& x0, uint32_t& x1,
                                          const EncTab& T, uint32_t& bits, Emit& em) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    // all 16 symbol transforms depend only on the chunk: issue their LDS
    // reads up front so only the stateTable reads sit on the state chain
    uint2 t0[8], t1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t sh = 16u * (uint32_t)(j & 1);
        t0[j] = T.tt[(w[j >> 1] >> sh) & 0xFFu];
        t1[j] = T.tt[(w[j >> 1] >> (sh + 8u)) & 0xFFu];
    }
    if (NS == 1) {
#pragma unroll
        for (int j = 15; j >= 0; --j) {
            if (!FULL && c8 + (uint32_t)j >= pb) continue;
            const uint2 t = (j & 1) ? t1[j >> 1] : t0[j >> 1];
            const uint32_t v0 = x0;
            const uint32_t nb0 = (t.x + x0) >> 16;
            x0 = st_at(((x0 >> nb0) << 1) + t.y);
            if (MODE == PASS_COUNT || MODE == PASS_REPAIR) bits += nb0;
            if (MODE == PASS_EMIT) {
                em.put(__builtin_amdgcn_ubfe(v0, 0u, nb0), nb0);
                if (j & 1) em.flush();  // <= 2 x 12 bits between flushes
            }
        }
        if (MODE == PASS_EMIT) em.flush();
        return;
    }
#pragma unroll
    for (int j = 7; j >= 0; --j) {
        if (!FULL && c8 + (uint32_t)j >= pb) continue;
        const uint32_t v1 = x1, v0 = x0;
        const uint32_t nb1 = (t1[j].x + x1) >> 16;
        x1 = st_at(((x1 >> nb1) << 1) + t1[j].y);
        const uint32_t nb0 = (t0[j].x + x0) >> 16;
        x0 = st_at(((x0 >> nb0) << 1) + t0[j].y);
        if (MODE == PASS_COUNT || MODE == PASS_REPAIR) bits += nb1 + nb0;
        if (MODE == PASS_EMIT) {
            const uint32_t pairbits = (__builtin_amdgcn_ubfe(v0, 0u, nb0) << nb1) | __builtin_amdgcn_ubfe(v1, 0u, nb1);
            em.put(pairbits, nb1 + nb0);
            em.flush();
        }
    }
}

// Sidecar entry for the decoder state before pair p (= encoder state after
// encoding pair p): bit position (payload-relative) and both states.
// (NS = 1: one state, s1 = 0.)
template <int NS>
__device__ __forceinline__ void ckpt_record(const Ckpt& ck, uint32_t p, uint32_t pos, uint32_t x0, uint32_t x1) {
    ck.base[p >> ck.shift] = (uint64_t)(pos - ck.hdr_bits) | ((uint64_t)(x0 - (1u << ck.L)) << 32) |
                             (NS == 2 ? ((uint64_t)(x1 - (1u << ck.L)) << 48) : 0ull);
}

// Encode pairs pb-1 down to pa.  Source chunks (16 B = 8 pairs) stream
// through four fixed registers, each reloaded right after it is consumed,
// so three loads stay in flight and no register copy forces an early
// s_waitcnt.  Loads are unconditional (the index is clamped to the
// segment); the partial topmost chunk is peeled and loaded byte-wise.
template <int MODE, int NS>
__device__ __forceinline__ EncState enc_range(const uint8_t* __restrict__ blk, uint32_t n, uint32_t pa, uint32_t pb,
                                              EncState st, const EncTab& T, Emit& em, const Ckpt& ck, Track& tr) {
    constexpr bool TRACK = MODE == PASS_COUNT || MODE == PASS_REPAIR;
    uint32_t x0 = st.x0, x1 = st.x1, bits = st.bits;
    if (pb <= pa) return st;
    const uint4* v = reinterpret_cast<const uint4*>(blk);
    constexpr uint32_t CS = NS == 2 ? 3u : 4u;  // log2 steps per 16-byte chunk
    int32_t c_hi = (int32_t)((pb - 1u) >> CS);
    const int32_t c_lo = (int32_t)(pa >> CS);
    // checkpoint after chunk c when (c - c_lo) % ckc == 0; slot (c - c_lo) / ckc
    uint32_t rem = 0, slot = 0;
    if (TRACK) {
        rem = (uint32_t)(c_hi - c_lo) % tr.ckc;
        slot = (uint32_t)(c_hi - c_lo) / tr.ckc;
    }
    auto track = [&]() {
        if (rem == 0u) {
            const uint32_t sv = x0 | (x1 << 16);
            if (MODE == PASS_REPAIR) {
                const uint2 r = tr.cp[slot];
                if (r.x == sv) {
                    tr.done = true;
                    tr.jstar = slot;
                    bits += r.y;  // the rest of the trajectory is the recorded one
                } else {
                    tr.cp[slot] = make_uint2(sv, bits);
                }
            } else {
                tr.cp[slot] = make_uint2(sv, bits);
            }
            slot -= 1u;
            rem = tr.ckc - 1u;
        } else {
            rem -= 1u;
        }
    };
    if (pb & ((1u << CS) - 1u)) {  // partial topmost chunk
        const uint4 q = load_chunk(blk, n, (uint32_t)c_hi);
        enc_chunk<MODE, false, NS>(q, (uint32_t)c_hi << CS, pb, x0, x1, T, bits, em);
        if (MODE == PASS_EMIT) em.drain();
        if (MODE == PASS_EMIT && ck.base && (((uint32_t)c_hi << CS) & ck.mask) == 0u)
            ckpt_record<NS>(ck, (uint32_t)c_hi << CS, em.pos(), x0, x1);
        if (TRACK) track();
        c_hi -= 1;
    }
    if (c_hi < c_lo || (MODE == PASS_REPAIR && tr.done)) return EncState{x0, x1, bits};
    auto ld = [&](int32_t c) { return v[c < c_lo ? c_lo : c]; };
    uint4 q0 = ld(c_hi), q1 = ld(c_hi - 1), q2 = ld(c_hi - 2), q3 = ld(c_hi - 3);
    auto body = [&](const uint4& q, int32_t c) {
        enc_chunk<MODE, true, NS>(q, (uint32_t)c << CS, pb, x0, x1, T, bits, em);
        if (MODE == PASS_EMIT) em.drain();
        if (MODE == PASS_EMIT && ck.base && (((uint32_t)c << CS) & ck.mask) == 0u)
            ckpt_record<NS>(ck, (uint32_t)c << CS, em.pos(), x0, x1);
        if (TRACK) track();
    };
    auto stop = [&](int32_t cn) { return cn < c_lo || (MODE == PASS_REPAIR && tr.done); };
    for (int32_t c = c_hi;; c -= 4) {
        body(q0, c);
        if (stop(c - 1)) break;
        q0 = ld(c - 4);
        body(q1, c - 1);
        if (stop(c - 2)) break;
        q1 = ld(c - 5);
        body(q2, c - 2);
        if (stop(c - 3)) break;
        q2 = ld(c - 6);
        body(q3, c - 3);
        if (stop(c - 4)) break;
        q3 = ld(c - 7);
    }
    return EncState{x0, x1, bits};
}

// Encoder::new_first_symbol, fse.rs:210-218
__device__ __forceinline__ uint32_t enc_init(const EncTab& T, uint32_t s) {
    const uint2 t = T.tt[s];
    const uint32_t bo = (t.x + (1u << 15)) >> 16;
    const uint32_t v = (bo << 16) - t.x;
    return st_at(((v >> bo) << 1) + t.y);
}

// Exact state of the topmost lane before the main loop.  NS = 2: both
// encoders seeded with the last symbols, plus the odd-length extra step
// (lib.rs:153-165).  NS = 1: the state seeded with the last symbol; the
// main loop then covers symbols n-2 .. 0 (lib.rs:120-126).
template <int MODE, int NS>
__device__ __forceinline__ EncState top_start(const uint8_t* blk, uint32_t n, const EncTab& tab, Emit& em) {
    EncState e;
    e.bits = 0;
    if (NS == 1) {
        e.x0 = enc_init(tab, blk[n - 1u]);
        e.x1 = 0;  // unused; 0 in every lane so packed states compare equal
        return e;
    }
    if (n & 1u) {  // lib.rs:155-160
        e.x0 = enc_init(tab, blk[n - 1u]);
        e.x1 = enc_init(tab, blk[n - 2u]);
        const uint32_t v0 = e.x0;
        const uint32_t nb = enc_step(e.x0, blk[n - 3u], tab);
        if (MODE == PASS_COUNT) e.bits = nb;
        if (MODE == PASS_EMIT) {
            em.put(v0 & ((1u << nb) - 1u), nb);
            em.flush();
        }
    } else {  // lib.rs:161-165
        e.x0 = enc_init(tab, blk[n - 2u]);
        e.x1 = enc_init(tab, blk[n - 1u]);
    }
    return e;
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
    // phase-1 scratch (statistics, header, spread) and phase-2 scratch
    // (trajectories, end states, merge list) share the same LDS: 13.4 KB per
    // workgroup at L <= 11, so 12 workgroups fit a CU (the VGPR limit)
    union {
        struct {
            union {
                uint32_t hs[HIST_WORDS];  // sub-histograms (counts[] go to cnt[], free until the spread)
                uint32_t hdrw[HDR_MAX / 4];  // NCount header, stored to the slot before the spread
                struct {
                    __attribute__((aligned(16))) uint8_t sym_at[SIZE];
                    __attribute__((aligned(16))) uint8_t occ_sym[SIZE];
                } sp;
            } u;
            int32_t norm[256];
            uint16_t cumul[256];
            uint32_t cnt[256];
        } p1;
        struct {
            union {
                uint2 cp[64 * TRACK_SLOTS];  // count-pass trajectories (Track)
                uint32_t ring[64 * RING_STRIDE];  // emit: 16-word output ring per lane (Emit)
            } u;
            uint32_t cntF[BPW][T + 1];
            uint32_t emF[BPW][T + 1];  // scratch path: end states of the emit pass
            uint32_t mword[BPW][2 * (T + 1)];
            uint32_t mval[BPW][2 * (T + 1)];
        } p2;
    } ph;
    int32_t info_status[BPW];
    uint32_t info_new[BPW];  // block takes the scratch path
    uint32_t info_L[BPW];
    uint32_t info_hl[BPW];
    uint32_t info_hv[BPW];  // the header's last partial word (merged with the payload's first bits)
    int scratch[4];
};

template <int LMAX, int T, int NS, bool SCR = false>
__global__ __launch_bounds__(64) void encode_blocks_kernel(EncParams P) {
    constexpr int BPW = 64 / T;
    __shared__ EncSmem<LMAX, T> sm;
    const uint32_t lane = lane_id();

    FSE_STAMP(P, 0);
    // ---- phase 1: statistics, header and tables, one block at a time
    for (int b = 0; b < BPW; ++b) {
        const uint64_t gb = (uint64_t)blockIdx.x * BPW + b;
        if (gb >= P.n_blocks) {
            if (lane == 0) {
                sm.info_status[b] = 1;  // no block
                sm.info_new[b] = 1u;
            }
            continue;
        }
        const uint64_t off = gb * P.block_size;
        const uint32_t n = (uint32_t)min((uint64_t)P.block_size, P.n_total - off);
        const uint8_t* blk = P.src + off;
        uint32_t* counts = sm.ph.p1.cnt;  // the spread reuses cnt[] after normalize
        const uint32_t tl = wave_histogram(blk, n, sm.ph.p1.u.hs, counts);
        FSE_STAMP(P, 1);
        if (P.debug & 8u) {  // ablation: histogram only
            if (lane == 0) P.status[gb] = (int32_t)tl;
            continue;
        }
        int rc = FSE_OK;
        uint32_t Lreq = P.table_log, L = 0, slow = 0;
        if (n == 0) rc = FSE_ERR_EMPTY;
        if (rc == FSE_OK && P.table_log == 0) rc = optimal_log2(n, tl, &Lreq);  // histogram.rs:301
        if (rc == FSE_OK) rc = wave_normalize(counts, n, tl, Lreq, sm.ph.p1.norm, &L, &slow, sm.scratch);
        if (rc == FSE_OK && n < 2) rc = FSE_ERR_TOO_SHORT;  // lib.rs:154/156 unwrap
        if (rc == FSE_OK && L > (uint32_t)LMAX) rc = FSE_ERR_UNSUPPORTED;
        // scratch path unless the distribution is skewed (its encoder
        // trajectories merge slowly, so start states from the count pass
        // would often be wrong and every wrong one costs a whole re-emit)
        bool newp = SCR && P.scratch != nullptr && P.path != 1u;
        if (newp && P.path == 0u && rc == FSE_OK) {
            uint32_t mx = 0;
            for (uint32_t s = lane; s < tl; s += WAVE) mx = max(mx, (uint32_t)max(sm.ph.p1.norm[s], 0));
            mx = wave_max(mx);
            newp = (uint64_t)mx * 256u <= ((uint64_t)P.pmax256 << L);
        }
        if (lane == 0) sm.info_new[b] = newp ? 1u : 0u;
        FSE_STAMP(P, 2);
        if (rc == FSE_OK) {
            const int hl = wave_header_write(sm.ph.p1.norm, L, tl, sm.ph.p1.u.hdrw);
            if (lane == 0) sm.scratch[1] = hl;
            if (hl < 0) {
                rc = hl;
            } else {
                // whole header words go to the slot now (no payload store
                // touches them); the last partial word is merged at the end
                const uint32_t* h = sm.ph.p1.u.hdrw;
                uint32_t* gw = reinterpret_cast<uint32_t*>(P.out + gb * P.slot_bytes);
                for (uint32_t w = lane; w < (uint32_t)hl / 4u; w += WAVE) gw[w] = h[w];
                if (lane == 0) sm.info_hv[b] = (hl & 3) ? h[hl / 4] & ((1u << (8u * (hl & 3))) - 1u) : 0u;
            }
            wave_sync();  // the spread reuses the header's LDS
        }
        FSE_STAMP(P, 3);
        if (rc == FSE_OK) {
            const uint32_t size = 1u << L;
            uint16_t* st = sm.st[b];
            const uint16_t* cumul = sm.ph.p1.cumul;
            rc = wave_build_spread(sm.ph.p1.norm, L, tl, sm.ph.p1.u.sp.sym_at, sm.ph.p1.u.sp.occ_sym, sm.ph.p1.cumul, sm.ph.p1.cnt,
                                   [&](uint32_t i, uint32_t s, uint32_t r) {
                                       st[cumul[s] + r] = (uint16_t)(size + i);  // fse.rs:157-162
                                   });
            // symbol transforms, fse.rs:165-188 (total == cumul[s]), with
            // the stateTable's LDS address folded into deltaFindState
            const uint32_t stb = lds_addr_of(&sm.st[b][0]);
            for (uint32_t s = lane; s < 256; s += WAVE) {
                int32_t x = (s < tl) ? sm.ph.p1.norm[s] : 0;
                uint2 t = make_uint2(0, stb);
                if (s < tl) {
                    const int32_t tot = (int32_t)sm.ph.p1.cumul[s];
                    if (x == 0) {
                        t.x = ((L + 1u) << 16) - (1u << L);
                    } else if (x == -1 || x == 1) {
                        t.x = (L << 16) - (1u << L);
                        t.y = stb + (uint32_t)(2 * (tot - 1));
                    } else {
                        const uint32_t mb = L - ilog2u((uint32_t)(x - 1));
                        t.x = (mb << 16) - ((uint32_t)x << mb);
                        t.y = stb + (uint32_t)(2 * (tot - x));
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

    FSE_STAMP(P, 4);
    if (P.debug & 9u) return;  // ablation: statistics + tables only (1), histogram only (8)
    // ---- phase 2: T lanes per block
    const int b = BPW == 1 ? 0 : (int)(lane / T);
    const uint32_t k = BPW == 1 ? lane : lane % T;
    const uint64_t gb = (uint64_t)blockIdx.x * BPW + b;
    const bool live = sm.info_status[b] == FSE_OK;
    const uint64_t boff = gb * P.block_size;
    const uint32_t n = live ? (uint32_t)min((uint64_t)P.block_size, P.n_total - boff) : 0u;
    const uint8_t* blk = P.src + boff;
    const uint32_t L = sm.info_L[b];
    const EncTab tab{sm.tt[b]};
    // main-loop steps: pairs (NS = 2) or symbols below the seed (NS = 1)
    const uint32_t Pm = live ? (NS == 2 ? ((n & 1u) ? (n - 3u) / 2u : n / 2u - 1u) : n - 1u) : 0u;
    constexpr uint32_t SPC = NS == 2 ? 8u : 16u;  // steps per 16-byte chunk
    uint32_t S = (Pm + T - 1u) / T;
    S = max(SPC, (S + SPC - 1u) & ~(SPC - 1u));
    const uint32_t ktop = Pm ? (Pm - 1u) / S : 0u;
    const bool act = live && k <= ktop;
    const uint32_t pa = k * S, pb = min(pa + S, Pm);
    Emit em;
    em.start(nullptr, 0);
    Ckpt ck{nullptr, 0, 0, 0, L};

    // Two ways to the exact start state of every lane (the lane above's end
    // state) and the exact bit offset of every lane:
    //  * repair path: count pass from guessed starts with trajectories, then
    //    convergence repair (re-encode from the corrected start until the
    //    recorded trajectory is met) until the fixed point, then the emit
    //    pass writes straight to the final offsets.  A repair round costs the
    //    slowest lane's convergence distance.
    //  * scratch path: count pass (state chains only, from a guessed start
    //    `warm` pairs above the lane's range), then the emit pass from those
    //    end states into lane-private scratch streams, which also yields the
    //    exact lengths.  A lane's start was right iff the emit end state of
    //    the lane above equals the count end state it was given (by
    //    induction from the exact top lane); a wrong one re-emits.  A copy
    //    pass then moves every stream to its final bit offset.
    bool newp = SCR;
#pragma unroll
    for (int bb = 0; bb < BPW; ++bb) newp = newp && sm.info_new[bb] != 0u;  // wave-uniform
    Track tr{&sm.ph.p2.u.cp[lane * TRACK_SLOTS], max(1u, (S / SPC + TRACK_SLOTS - 1u) / TRACK_SLOTS), false, 0u};
    const uint32_t nslot = pb > pa ? (((pb - 1u) / SPC) - (pa / SPC)) / tr.ckc + 1u : 0u;
    uint32_t start = (1u << L) | (NS == 2 ? (1u << L) << 16 : 0u);
    uint32_t bits = 0;
    uint32_t* sw = nullptr;  // scratch path: this lane's stream
    uint32_t n_iter = 0, n_rerun = 0;  // diagnostics (stamps counters)
    if (newp) {
        sw = P.scratch + ((uint64_t)gb * T + k) * P.scr_lane_words;
        if (act) {
            EncState e0;
            uint32_t ptop = pb;
            if (k == ktop) {
                e0 = top_start<PASS_STATE, NS>(blk, n, tab, em);
            } else {
                e0 = EncState{start & 0xFFFFu, start >> 16, 0u};
                ptop = min(pb + P.warm, Pm);
            }
            e0 = enc_range<PASS_STATE, NS>(blk, n, pa, ptop, e0, tab, em, ck, tr);
            sm.ph.p2.cntF[b][k] = e0.x0 | (e0.x1 << 16);
        }
        FSE_STAMP(P, 5);
        __syncthreads();
        if (act && k < ktop) start = sm.ph.p2.cntF[b][k + 1];
        Ckpt ckl{nullptr, 0, 0, 0, L};
        if (P.sidecar && P.ckpt_interval) {
            ckl.base = P.sidecar + gb * P.ckpt_per_block;
            ckl.mask = P.ckpt_interval - 1u;
            ckl.shift = 31u - __clz(P.ckpt_interval);
            ckl.hdr_bits = 0;  // lane-local positions until the copy pass
        }
        // the lane's whole stream (including the finals and marker of lane 0)
        // into its scratch words; checkpoints at lane-local bit positions
        auto emit_lane = [&]() -> uint32_t {
            em.start(sw, 0, P.scr_lane_words, &sm.ph.p2.u.ring[lane * RING_STRIDE]);
            EncState e0;
            if (k == ktop) {
                e0 = top_start<PASS_EMIT, NS>(blk, n, tab, em);
                if (ckl.base && (Pm & ckl.mask) == 0u) ckpt_record<NS>(ckl, Pm, em.pos(), e0.x0, e0.x1);
            } else {
                e0 = EncState{start & 0xFFFFu, start >> 16, 0u};
            }
            e0 = enc_range<PASS_EMIT, NS>(blk, n, pa, pb, e0, tab, em, ckl, tr);
            sm.ph.p2.emF[b][k] = e0.x0 | (e0.x1 << 16);
            if (k == 0) {  // Encoder::finish (x2 for NS = 2) + marker (lib.rs:178-181 / 139-141)
                const uint32_t m = (1u << L) - 1u;
                if (NS == 2) {
                    em.put(e0.x1 & m, L);
                    em.flush();
                }
                em.put(e0.x0 & m, L);
                em.flush();
                em.put(1u, 1u);
                em.flush();
            }
            em.finish();
            if (em.nacc) sw[em.word] = em.lo;  // the partial last word (lane-private)
            return em.pos();
        };
        if (act) bits = emit_lane();
        for (;;) {
            __syncthreads();
            const bool bad = act && k < ktop && sm.ph.p2.emF[b][k + 1] != start;
            __syncthreads();
            if (__ballot(bad) == 0) break;
            ++n_iter;
            n_rerun += (uint32_t)__popcll(__ballot(bad));
            if (bad) {
                start = sm.ph.p2.emF[b][k + 1];
                bits = emit_lane();
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // scratch and sidecar stores land before the copy reads
    } else {
        // count pass: the top lane from its exact start (init states + the
        // odd-length extra step), every other lane from a guessed start state,
        // recording its trajectory.  Then verify against the neighbour's end
        // state and repair by convergence (Track) until the fixed point.
        if (act) {
            EncState e0 = (k == ktop) ? top_start<PASS_COUNT, NS>(blk, n, tab, em) : EncState{start & 0xFFFFu, start >> 16, 0u};
            e0 = enc_range<PASS_COUNT, NS>(blk, n, pa, pb, e0, tab, em, ck, tr);
            bits = e0.bits;
            sm.ph.p2.cntF[b][k] = e0.x0 | (e0.x1 << 16);
            track_fixup(tr, nslot, -1, bits);
        }
        FSE_STAMP(P, 5);
        for (;;) {
            if (P.debug & 16u) break;  // ablation: no repair (wrong output)
            __syncthreads();
            bool bad = false;
            uint32_t nbF = 0;
            if (act && k < ktop) {
                nbF = sm.ph.p2.cntF[b][k + 1];
                bad = nbF != start;
            }
            __syncthreads();
            if (__ballot(bad) == 0) break;
            ++n_iter;
            n_rerun += (uint32_t)__popcll(__ballot(bad));
            if (bad) {
                start = nbF;
                tr.done = false;
                const EncState e0 = enc_range<PASS_REPAIR, NS>(blk, n, pa, pb, EncState{start & 0xFFFFu, start >> 16, 0u},
                                                           tab, em, ck, tr);
                bits = e0.bits;
                if (!tr.done) sm.ph.p2.cntF[b][k] = e0.x0 | (e0.x1 << 16);  // did not converge: new end state
                track_fixup(tr, nslot, tr.done ? (int32_t)tr.jstar : -1, bits);
            }
        }
        if (k == 0) bits += (uint32_t)NS * L + 1u;  // finals + marker (lib.rs:178-181 / 139-141)
    }

    FSE_STAMP(P, 6);
    if (P.stamps && lane == 0)
        P.stamps[(uint64_t)blockIdx.x * kStamps + kStamps - 1] = (uint64_t)n_iter | ((uint64_t)n_rerun << 32);
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
    const bool fits = (uint64_t)total_bits <= P.slot_bytes * 8ull && !(P.debug & 2u);
    uint32_t* gw = reinterpret_cast<uint32_t*>(P.out + gb * P.slot_bytes);

    // emit pass (repair path) or copy pass (scratch path)
    for (uint32_t e = k; e < 2u * (T + 1u); e += T) {
        if (b < BPW) sm.ph.p2.mword[b][e] = 0xFFFFFFFFu;
    }
    __syncthreads();
    if (act && fits) {
        em.start(gw, off, (P.debug & 4u) ? 0u : (uint32_t)(P.slot_bytes >> 2),  // debug bit 2: no payload stores (ablation)
                 &sm.ph.p2.u.ring[lane * RING_STRIDE]);
        if (newp) {
            // the lane's stream at its final offset: whole words through the
            // emitter (ring, 64-byte groups, merge list), then the tail bits
            // (four 16-byte loads in flight ahead of the words being moved)
            const uint32_t nw = bits >> 5, rb = bits & 31u, nq = nw >> 2;
            const uint4* s4 = reinterpret_cast<const uint4*>(sw);
            auto put4 = [&](const uint4& q) {
                em.put(q.x, 32u);
                em.flush();
                em.put(q.y, 32u);
                em.flush();
                em.put(q.z, 32u);
                em.flush();
                em.put(q.w, 32u);
                em.flush();
                em.drain();
            };
            if (nq) {
                auto ldq = [&](uint32_t q) { return s4[min(q, nq - 1u)]; };
                uint4 c0 = ldq(0), c1 = ldq(1), c2 = ldq(2), c3 = ldq(3);
                for (uint32_t q = 0; q < nq; q += 4u) {
                    const uint4 n0 = ldq(q + 4u), n1 = ldq(q + 5u), n2 = ldq(q + 6u), n3 = ldq(q + 7u);
                    put4(c0);
                    if (q + 1u < nq) put4(c1);
                    if (q + 2u < nq) put4(c2);
                    if (q + 3u < nq) put4(c3);
                    c0 = n0;
                    c1 = n1;
                    c2 = n2;
                    c3 = n3;
                }
            }
            for (uint32_t i = nq << 2; i < nw; ++i) {
                em.put(sw[i], 32u);
                em.flush();
            }
            em.drain();
            if (rb) {
                em.put(sw[nw] & ((1u << rb) - 1u), rb);
                em.flush();
            }
            // sidecar: lane-local positions -> payload-relative ones
            if (P.sidecar && P.ckpt_interval) {
                uint64_t* base = P.sidecar + gb * P.ckpt_per_block;
                const uint32_t I = P.ckpt_interval;
                const uint32_t i0 = (pa + I - 1u) / I;
                uint32_t i1 = (pb + I - 1u) / I;
                if (k == ktop && (Pm & (I - 1u)) == 0u) i1 = Pm / I + 1u;
                const uint32_t delta = off - hdr_bits;
                for (uint32_t j = i0; j < i1; ++j) {
                    const uint64_t v = base[j];
                    base[j] = (v & ~0xFFFFFFFFull) | (uint64_t)((uint32_t)v + delta);
                }
            }
        } else {
            if (P.sidecar && P.ckpt_interval) {
                ck.base = P.sidecar + gb * P.ckpt_per_block;
                ck.mask = P.ckpt_interval - 1u;
                ck.shift = 31u - __clz(P.ckpt_interval);
                ck.hdr_bits = hdr_bits;
            }
            EncState e0;
            if (k == ktop) {
                e0 = top_start<PASS_EMIT, NS>(blk, n, tab, em);
                if (ck.base && (Pm & ck.mask) == 0u)  // checkpoint "before step Pm"
                    ckpt_record<NS>(ck, Pm, em.pos(), e0.x0, e0.x1);
            } else {
                e0 = EncState{start & 0xFFFFu, start >> 16, 0u};
            }
            e0 = enc_range<PASS_EMIT, NS>(blk, n, pa, pb, e0, tab, em, ck, tr);
            const uint32_t y0 = e0.x0, y1 = e0.x1;
            if (k == 0) {  // Encoder::finish (x2 for NS = 2) + marker (lib.rs:178-181 / 139-141)
                const uint32_t m = (1u << L) - 1u;
                if (NS == 2) {
                    em.put(y1 & m, L);
                    em.flush();
                }
                em.put(y0 & m, L);
                em.flush();
                em.put(1u, 1u);
                em.flush();
            }
        }
        em.finish();
        // boundary words -> merge list (entry order = stream order)
        const uint32_t slot = 2u * (T - k);
        if ((off & 31u) != 0u && em.word > em.w0) {  // first word stored with the low bits empty
            sm.ph.p2.mword[b][slot] = em.w0;
            sm.ph.p2.mval[b][slot] = em.head_val;
        }
        if (em.nacc) {  // last word never stored
            sm.ph.p2.mword[b][slot + 1] = em.word;
            sm.ph.p2.mval[b][slot + 1] = em.lo;
        }
    }
    // header: whole words were stored in phase 1; the last partial word is merged
    if (live && fits && k == 0 && (hl & 3u)) {
        sm.ph.p2.mword[b][0] = hl / 4u;
        sm.ph.p2.mval[b][0] = sm.info_hv[b];
    }
    FSE_STAMP(P, 7);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stores above land before the merge rewrites
    __syncthreads();
    // merge: each run of equal word indices is OR-ed by its first entry
    if (live && fits) {
        constexpr uint32_t NE = 2u * (T + 1u);
        for (uint32_t e = k; e < NE; e += T) {
            const uint32_t w = sm.ph.p2.mword[b][e];
            if (w == 0xFFFFFFFFu) continue;
            bool first = true;
            for (int q = (int)e - 1; q >= 0; --q) {
                const uint32_t wq = sm.ph.p2.mword[b][q];
                if (wq == 0xFFFFFFFFu) continue;
                first = (wq != w);
                break;
            }
            if (!first) continue;
            uint32_t v = sm.ph.p2.mval[b][e];
            for (uint32_t q = e + 1; q < NE; ++q) {
                const uint32_t wq = sm.ph.p2.mword[b][q];
                if (wq == 0xFFFFFFFFu) continue;
                if (wq != w) break;
                v |= sm.ph.p2.mval[b][q];
            }
            if (w < (uint32_t)(P.slot_bytes >> 2)) gw[w] = v;
        }
    }
    FSE_STAMP(P, 8);
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
// Backward bit readers (BitStackReader semantics, stack_reader.rs:17-215):
// `pos` = bits remaining above the block start, buf holds stream bits
// [base, base+64) of the block; refills pull the next lower 32-bit word.
// LdsReader reads the block staged in LDS; GlobalReader reads global memory
// directly (blocks whose payload does not fit the LDS stage).
struct LdsReader {
    const uint32_t* w;
    uint64_t buf;
    int32_t base;
    int32_t pos;
    __device__ __forceinline__ void init(const uint32_t* words, int32_t p) {
        w = words;
        pos = p;
        base = ((p + 31) & ~31) - 64;
        if (base < 0) base = 0;
        buf = (uint64_t)w[base >> 5] | ((uint64_t)w[(base >> 5) + 1] << 32);
    }
    __device__ __forceinline__ uint32_t pop(uint32_t nb) {
        pos -= (int32_t)nb;
        return (uint32_t)(buf >> (uint32_t)(pos - base)) & ((1u << nb) - 1u);
    }
    __device__ __forceinline__ void refill() {
        if (pos - base < 32 && base > 0) {
            base -= 32;
            buf = (buf << 32) | (uint64_t)w[base >> 5];
        }
    }
};
using GlobalReader = LdsReader;  // same code, words in global memory

__device__ __forceinline__ void store_byte(uint8_t* out, uint32_t i, uint32_t lim, uint32_t v) {
    if (i < lim) out[i] = (uint8_t)v;
}

// Decode table entry (fse.rs:260-265 DecodeTransform, repacked for the
// decode loop): nb | symbol << 8 | (4 * new_state) << 16.  nb in bits 0-4
// lets an entry serve directly as a v_bfe width/offset operand, the byte
// sum of two entries' low bytes is nb0 + nb1, and the high half is the LDS
// byte offset of the next state's base entry.
__device__ __forceinline__ uint32_t dte_make(uint32_t nb, uint32_t sym, uint32_t ns) {
    return nb | (sym << 8) | (ns << 18);
}
__device__ __forceinline__ uint32_t dte_nb(uint32_t e) { return e & 0xFFu; }
__device__ __forceinline__ uint32_t dte_sym(uint32_t e) { return (e >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t dte_ns(uint32_t e) { return e >> 18; }

// Decode main-loop pairs [p0, p1) of one segment without read checks (the
// sidecar guarantees the bits) through a windowed reader (global-memory
// blocks); when `last`, finish with the reference termination in container
// mode (the oracle's decompress2_impl; lib.rs:227-244).  Returns a status.
template <class RD>
__device__ __forceinline__ int32_t decode_segment(RD& br, uint32_t s0, uint32_t s1, uint32_t p0, uint32_t p1,
                                                  bool last, uint32_t n, uint32_t Pm, uint8_t* __restrict__ out,
                                                  const uint32_t* dt, uint32_t smask, int32_t hdr_bits) {
    uint32_t p = p0;
    for (; p + 8u <= p1; p += 8u) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t e0 = dt[s0 & smask], e1 = dt[s1 & smask];
            const uint32_t v0 = br.pop(dte_nb(e0));
            const uint32_t v1 = br.pop(dte_nb(e1));
            s0 = dte_ns(e0) + v0;
            s1 = dte_ns(e1) + v1;
            const uint32_t pr = __builtin_amdgcn_perm(e1, e0, 0x0c0c0501u);
            if (j & 1) w[j >> 1] |= pr << 16; else w[j >> 1] = pr;
            br.refill();
        }
        *reinterpret_cast<uint4*>(out + 2u * p) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    for (; p < p1; ++p) {
        const uint32_t e0 = dt[s0 & smask], e1 = dt[s1 & smask];
        const uint32_t v0 = br.pop(dte_nb(e0));
        const uint32_t v1 = br.pop(dte_nb(e1));
        s0 = dte_ns(e0) + v0;
        s1 = dte_ns(e1) + v1;
        out[2u * p] = (uint8_t)dte_sym(e0);
        out[2u * p + 1u] = (uint8_t)dte_sym(e1);
        br.refill();
    }
    if (!last) return FSE_OK;
    uint32_t o = 2u * Pm;
    for (;;) {
        if (o + 2u == n) {
            out[o++] = (uint8_t)dte_sym(dt[s0 & smask]);
            out[o++] = (uint8_t)dte_sym(dt[s1 & smask]);
            break;
        }
        if (o + 1u == n) {
            out[o++] = (uint8_t)dte_sym(dt[s0 & smask]);
            break;
        }
        const uint32_t e0 = dt[s0 & smask];
        uint32_t nb = dte_nb(e0);
        if (br.pos - (int32_t)nb < hdr_bits) {
            out[o++] = (uint8_t)dte_sym(e0);
            if (o < n) out[o++] = (uint8_t)dte_sym(dt[s1 & smask]);
            break;
        }
        s0 = dte_ns(e0) + br.pop(nb);
        br.refill();
        out[o++] = (uint8_t)dte_sym(e0);
        const uint32_t e1 = dt[s1 & smask];
        nb = dte_nb(e1);
        if (br.pos - (int32_t)nb < hdr_bits) {
            out[o++] = (uint8_t)dte_sym(e1);
            if (o < n) out[o++] = (uint8_t)dte_sym(dt[s0 & smask]);
            break;
        }
        s1 = dte_ns(e1) + br.pop(nb);
        br.refill();
        out[o++] = (uint8_t)dte_sym(e1);
    }
    return o == n ? FSE_OK : FSE_ERR_LENGTH_MISMATCH;
}

// Bits [pos, pos + 32) of an LDS-staged block (pos >= 0): one ds_read2 of
// the two words holding them and a v_alignbit.  Bits above the block's end
// are garbage; callers only use the low nb0 + nb1 <= 24 bits.
__device__ __forceinline__ uint32_t lds_bits32(const uint32_t* pay, int32_t pos) {
    const uint32_t* wp = pay + ((uint32_t)pos >> 5);
    return __builtin_amdgcn_alignbit(wp[1], wp[0], (uint32_t)pos);
}

// Padded LDS image of a block (VAR 3): source word w lives at LDS word
// w + w/32, and the dword after each 32-word row repeats the next row's
// first word, so words w and w+1 are always adjacent (one ds_read2).  Lanes
// that walk equal-size segments in lockstep then land on different banks:
// a segment stride of S words puts lane l at bank ~(S * 33/32 * l) mod 32
// instead of (S * l) mod 32, which for S ~ 32 (C2) collapsed onto a handful
// of banks.
__device__ __forceinline__ uint32_t pad_word(uint32_t w) { return w + (w >> 5); }
__device__ __forceinline__ uint32_t lds_bits32_pad(const uint32_t* pay, int32_t pos) {
    const uint32_t* wp = pay + pad_word((uint32_t)pos >> 5);
    return __builtin_amdgcn_alignbit(wp[1], wp[0], (uint32_t)pos);
}
template <int VAR>
__device__ __forceinline__ uint32_t lds_bits(const uint32_t* pay, int32_t pos) {
    return (VAR == 3 || VAR == 5) ? lds_bits32_pad(pay, pos) : lds_bits32(pay, pos);
}

// Segment decode for a block staged in LDS.  One LdsChain = one segment's
// decoder pair (two tANS states + the shared bit position).  Per pair:
// pos -= nb0 + nb1 (byte sum of the two entries), the pair's bits at pos,
// v1 = low nb1 bits and v0 = the nb0 bits above (stack order: decoder 0
// pops first), and the next states' LDS offsets a0/a1 (4 * state).
//   VAR 0: one ds_read2 of the two words at pos per pair;
//   VAR 1: the same window fetched from pos_prev - 24 alongside the table
//          reads (one LDS latency on the chain instead of two);
//   VAR 12 (default in decode_pre_kernel): VAR 9 reading one payload dword
//          per pair (the upper word of the window is one of the previous
//          pair's two words): C3 0.64 -> 0.60 ms.
//   VAR 9: VAR 1 without the clamp (the image
//          has a pad below it), with segments permuted over the lanes (lane
//          t takes segment 33t mod NT) so that lockstep reads spread over the
//          banks: branch-free, ~13 VALU + 3 LDS reads per pair (VAR 2: ~23
//          VALU, an exec-masked refill and a wait on it every pair); C3
//          0.66 -> 0.62 ms.
//   VAR 2: a per-lane 64-bit window over words (k, k+1), B = 32k, holding
//          >= 32 bits below pos at each pair start; refills are exec-masked
//          to the lanes that need one, the next word prefetched a refill
//          ahead.  Lanes walk equal-size segments in lockstep, so unmasked
//          per-pair payload reads pile onto a few banks.
template <int VAR>
struct LdsChain {
    int32_t pos, B;
    uint32_t wlo, whi, wnx, a0, a1;
    __device__ __forceinline__ void init(const uint32_t* pay, int32_t p, uint32_t s0, uint32_t s1) {
        pos = p;
        a0 = s0 << 2;
        a1 = s1 << 2;
        B = 0;
        wlo = whi = wnx = 0;
        if (VAR == 2 || VAR == 6) {
            const int32_t k = max((p >> 5) - 1, 0);
            B = k << 5;
            wlo = pay[k];
            whi = pay[k + 1];
            wnx = pay[max(k - 1, 0)];
        }
        if (VAR == 12) {  // the first pair reads word lo/32 and takes word lo/32 + 1 from here
            B = (p - 24) & ~31;
            whi = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(pay) + (B >> 3) + 4);
        }
    }
    __device__ __forceinline__ uint32_t pair(const uint32_t* pay, const uint8_t* dtb) {
        uint32_t x, e0, e1;
        if (VAR == 2) {
            e0 = *reinterpret_cast<const uint32_t*>(dtb + a0);
            e1 = *reinterpret_cast<const uint32_t*>(dtb + a1);
            pos -= (int32_t)((e0 + e1) & 0xFFu);
            x = (uint32_t)((((uint64_t)whi << 32) | wlo) >> (uint32_t)(pos - B));
            if (pos < B + 32) {
                B -= 32;
                whi = wlo;
                wlo = wnx;
                wnx = pay[max((B >> 5) - 1, 0)];
            }
        } else if (VAR == 6) {
            // VAR 2's window with a branch-free refill: selects instead of an
            // exec-masked branch, and the prefetch of the word below the
            // window issued every pair (when no refill happened it re-reads
            // the same word).  No SALU, no phi copies of in-flight loads.
            e0 = *reinterpret_cast<const uint32_t*>(dtb + a0);
            e1 = *reinterpret_cast<const uint32_t*>(dtb + a1);
            pos -= (int32_t)((e0 + e1) & 0xFFu);
            const uint32_t d = (uint32_t)(pos - B);  // in [8, 64]
            x = (uint32_t)((((uint64_t)whi << 32) | wlo) >> d);
            const bool c = d < 32u;
            B = c ? B - 32 : B;
            whi = c ? wlo : whi;
            wlo = c ? wnx : wlo;
            // word B/32 - 1 (B >= -32: the image has a 16-byte pad below it)
            wnx = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(pay) + (B >> 3) - 4);
        } else if (VAR == 5) {
            // padded image + the window for this pair fetched together with
            // the table entries (its <= 24 bits lie in [pos - 24, pos))
            const int32_t lo = max(pos - 24, 0);
            const uint32_t* wp = pay + pad_word((uint32_t)lo >> 5);
            const uint32_t w0 = wp[0], w1 = wp[1];
            const uint32_t base = (uint32_t)lo & ~31u;
            e0 = *reinterpret_cast<const uint32_t*>(dtb + a0);
            e1 = *reinterpret_cast<const uint32_t*>(dtb + a1);
            pos -= (int32_t)((e0 + e1) & 0xFFu);
            x = (uint32_t)((((uint64_t)w1 << 32) | w0) >> ((uint32_t)pos - base));
        } else if (VAR == 12) {
            // VAR 9 with one payload dword per pair instead of two: a pair
            // consumes <= 24 < 32 bits, so the window base lo moves down by at
            // most one word per pair and the upper word is always one of the
            // previous pair's two words (B = previous lo)
            const int32_t lo = (pos - 24) & ~31;
            const uint32_t w0 = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(pay) + (lo >> 3));
            e0 = *reinterpret_cast<const uint32_t*>(dtb + a0);
            e1 = *reinterpret_cast<const uint32_t*>(dtb + a1);
            const uint32_t w1 = lo == B ? whi : wlo;
            pos -= (int32_t)((e0 + e1) & 0xFFu);
            x = (uint32_t)((((uint64_t)w1 << 32) | w0) >> (uint32_t)(pos - lo));
            B = lo;
            whi = w1;
            wlo = w0;
        } else if (VAR == 9) {
            // VAR 1 without the clamp: the decode_pre_kernel image has a
            // 16-byte pad below it, so the window may start at word -1
            const int32_t lo = (pos - 24) & ~31;
            const uint32_t* wp = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(pay) + (lo >> 3));
            const uint32_t w0 = wp[0], w1 = wp[1];
            e0 = *reinterpret_cast<const uint32_t*>(dtb + a0);
            e1 = *reinterpret_cast<const uint32_t*>(dtb + a1);
            pos -= (int32_t)((e0 + e1) & 0xFFu);
            x = (uint32_t)((((uint64_t)w1 << 32) | w0) >> (uint32_t)(pos - lo));
        } else if (VAR == 1) {
            const int32_t lo = max(pos - 24, 0);
            const uint32_t* wp = pay + ((uint32_t)lo >> 5);
            const uint32_t w0 = wp[0], w1 = wp[1];
            const uint32_t base = (uint32_t)lo & ~31u;
            e0 = *reinterpret_cast<const uint32_t*>(dtb + a0);
            e1 = *reinterpret_cast<const uint32_t*>(dtb + a1);
            pos -= (int32_t)((e0 + e1) & 0xFFu);
            x = (uint32_t)((((uint64_t)w1 << 32) | w0) >> ((uint32_t)pos - base));
        } else {
            e0 = *reinterpret_cast<const uint32_t*>(dtb + a0);
            e1 = *reinterpret_cast<const uint32_t*>(dtb + a1);
            pos -= (int32_t)((e0 + e1) & 0xFFu);
            x = lds_bits<VAR>(pay, pos);
        }
        const uint32_t v1 = __builtin_amdgcn_ubfe(x, 0u, e1);
        const uint32_t v0 = __builtin_amdgcn_ubfe(x, e1, e0);
        a0 = (e0 >> 16) + (v0 << 2);
        a1 = (e1 >> 16) + (v1 << 2);
        return __builtin_amdgcn_perm(e1, e0, 0x0c0c0501u);  // sym0 | sym1 << 8
    }
};

// 32 pairs = one whole 64-byte segment of output per lane, stored back to
// back (full HBM write bursts instead of masked partial ones).
template <uint32_t GRP = DEC_GROUP>
__device__ __forceinline__ void store_group(uint8_t* __restrict__ dst, const uint32_t* w) {
    uint4* o4 = reinterpret_cast<uint4*>(dst);
#pragma unroll
    for (uint32_t q = 0; q < GRP / 8u; ++q) o4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// Pairs [p, p1) of one chain, then (when `last`) the reference termination
// in container mode (the oracle's decompress2_impl; lib.rs:227-244).
template <int VAR>
__device__ __forceinline__ int32_t run_chain(LdsChain<VAR>& c, const uint32_t* pay, const uint8_t* dtb, uint32_t p,
                                             uint32_t p1, bool last, uint32_t n, uint32_t Pm,
                                             uint8_t* __restrict__ out, int32_t hdr_bits) {
    for (; p + DEC_GROUP <= p1; p += DEC_GROUP) {
        uint32_t w[DEC_GROUP / 2u];
#pragma unroll
        for (uint32_t j = 0; j < DEC_GROUP; j += 2u) {
            const uint32_t lo = c.pair(pay, dtb);
            const uint32_t hi = c.pair(pay, dtb);
            w[j >> 1] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);  // lo.b0 lo.b1 hi.b0 hi.b1
        }
        store_group(out + 2u * p, w);
    }
    for (; p < p1; ++p) {
        const uint32_t pr = c.pair(pay, dtb);
        out[2u * p] = (uint8_t)pr;
        out[2u * p + 1u] = (uint8_t)(pr >> 8);
    }
    if (!last) return FSE_OK;
    auto ent = [&](uint32_t a) { return *reinterpret_cast<const uint32_t*>(dtb + a); };
    uint32_t o = 2u * Pm;
    int32_t pos = c.pos;
    uint32_t a0 = c.a0, a1 = c.a1;
    for (;;) {
        if (o + 2u == n) {
            out[o++] = (uint8_t)dte_sym(ent(a0));
            out[o++] = (uint8_t)dte_sym(ent(a1));
            break;
        }
        if (o + 1u == n) {
            out[o++] = (uint8_t)dte_sym(ent(a0));
            break;
        }
        const uint32_t e0 = ent(a0);
        uint32_t nb = dte_nb(e0);
        if (pos - (int32_t)nb < hdr_bits) {
            out[o++] = (uint8_t)dte_sym(e0);
            if (o < n) out[o++] = (uint8_t)dte_sym(ent(a1));
            break;
        }
        pos -= (int32_t)nb;
        a0 = (e0 >> 16) + (__builtin_amdgcn_ubfe(lds_bits<VAR>(pay, pos), 0u, nb) << 2);
        out[o++] = (uint8_t)dte_sym(e0);
        const uint32_t e1 = ent(a1);
        nb = dte_nb(e1);
        if (pos - (int32_t)nb < hdr_bits) {
            out[o++] = (uint8_t)dte_sym(e1);
            if (o < n) out[o++] = (uint8_t)dte_sym(ent(a0));
            break;
        }
        pos -= (int32_t)nb;
        a1 = (e1 >> 16) + (__builtin_amdgcn_ubfe(lds_bits<VAR>(pay, pos), 0u, nb) << 2);
        out[o++] = (uint8_t)dte_sym(e1);
    }
    return o == n ? FSE_OK : FSE_ERR_LENGTH_MISMATCH;
}

// Two segments per lane, interleaved pair by pair (independent state
// chains: one chain's LDS and VALU latency hides behind the other's work).
template <int VAR>
__device__ __forceinline__ int32_t decode_dual(const uint32_t* pay, const uint8_t* dtb, LdsChain<VAR>& A, uint32_t pa,
                                               uint32_t pa1, bool lastA, LdsChain<VAR>& Bc, uint32_t pb, uint32_t pb1,
                                               bool lastB, uint32_t n, uint32_t Pm, uint8_t* __restrict__ out,
                                               int32_t hdr_bits) {
    // 16 pairs (32 B) per chain between stores: two chains' output buffers
    // in registers at once
    constexpr uint32_t GRP = 16u;
    const uint32_t common = min(pa1 - pa, pb1 - pb) / GRP * GRP;
    for (uint32_t k = 0; k < common; k += GRP) {
        uint32_t wa[GRP / 2u], wb[GRP / 2u];
#pragma unroll
        for (uint32_t j = 0; j < GRP; j += 2u) {
            const uint32_t la = A.pair(pay, dtb);
            const uint32_t lb = Bc.pair(pay, dtb);
            const uint32_t ha = A.pair(pay, dtb);
            const uint32_t hb = Bc.pair(pay, dtb);
            wa[j >> 1] = __builtin_amdgcn_perm(ha, la, 0x05040100u);
            wb[j >> 1] = __builtin_amdgcn_perm(hb, lb, 0x05040100u);
        }
        store_group<GRP>(out + 2u * (pa + k), wa);
        store_group<GRP>(out + 2u * (pb + k), wb);
    }
    const int32_t ra = run_chain(A, pay, dtb, pa + common, pa1, lastA, n, Pm, out, hdr_bits);
    const int32_t rb = run_chain(Bc, pay, dtb, pb + common, pb1, lastB, n, Pm, out, hdr_bits);
    return ra != FSE_OK ? ra : rb;
}

// One workgroup of NW waves per block.  The compressed block (<= PMAX bytes)
// is staged into LDS by one coalesced copy; wave 0 parses the header and
// builds the decode table (fse.rs:280-338) while the block lands; then every
// lane decodes the checkpoint segments assigned to it.  Without a sidecar
// (or in reference mode) lane 0 decodes the block serially with every read
// checked (lib.rs:215-248) and may record the sidecar index.
template <int LMAX, int NW, uint32_t PMAX>
struct DecSmem {
    static constexpr uint32_t SIZE = 1u << LMAX;
    // dt[i] = dte_make(nb, symbol, new_state); the spread scratch lives
    // in the top half of the same array (see the wave_build_spread call).
    uint32_t pay[PMAX / 4];  // first: LDS offset 0, so payload addresses need no base add
    uint32_t dt[SIZE];
    int32_t norm[256];
    uint16_t cumul[256];
    uint32_t cnt[NW * 256];
    uint32_t wscr[NW + 4];
    int scratch[8];
    int err[NW];
};

template <int LMAX, int NW, uint32_t PMAX>
__global__ __launch_bounds__(64 * NW) void decode_blocks_kernel(DecParams P) {
    __shared__ DecSmem<LMAX, NW, PMAX> sm;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = P.comp_len[gb];
    const uint64_t ooff = gb * (uint64_t)P.block_size;
    // raw length: container length, or unknown (reference mode) with a cap
    const bool known = P.n_total != 0;
    const uint32_t n = known ? (uint32_t)min((uint64_t)P.block_size, P.n_total - ooff) : 0u;
    const uint32_t cap = known ? n : P.out_cap;
    uint8_t* out = P.out + ooff;
    // prebuilt decode tables (dtable_blocks_kernel / C3): no header parse, no table build
    const bool pre = P.dt != nullptr;
    const int32_t info = pre ? P.dtinfo[gb] : 0;
    const bool padded = pre && P.variant == 3;
    const uint32_t nwords = (clen + 3u) >> 2;
    const bool in_lds = padded ? (pad_word(nwords) + 2u) * 4u <= PMAX : clen <= PMAX;
    FSE_STAMP(P, 0);

    {  // stage the block (or at least its header) in LDS, plus a prebuilt table
        if (padded && in_lds && info >= 0) {
            // dword LDS-DMA: LDS word d <- source word d - d/33 (the 33rd
            // dword of each row repeats the next row's first word)
            const uint32_t nd = pad_word(nwords) + 2u;
            const uint32_t wmax = (uint32_t)min((uint64_t)nwords + 1u, P.slot_bytes / 4u) - 1u;
            const uint32_t* src = reinterpret_cast<const uint32_t*>(in);
            for (uint32_t i = wv * 64u; i < nd; i += 64u * NW) {
                const uint32_t d = i + lane;
                const uint32_t w = min(d - d / 33u, wmax);
                if (d < nd) __builtin_amdgcn_global_load_lds(src + w, sm.pay + i, 4, 0, 0);
            }
        } else {
            const uint32_t ncopy = in_lds ? clen : min(clen, (uint32_t)min((uint64_t)HDR_MAX, P.slot_bytes));
            const uint32_t nvec = (pre && info < 0) ? 0u : (ncopy + 15u) >> 4;
            const uint4* src4 = reinterpret_cast<const uint4*>(in);
            uint4* dst4 = reinterpret_cast<uint4*>(sm.pay);
            // LDS-DMA: each wave-instruction moves 1 KiB, lane-linear in LDS
            for (uint32_t i = wv * 64u; i < nvec; i += 64u * NW) {
                if (i + lane < nvec)
                    __builtin_amdgcn_global_load_lds(src4 + i + lane, dst4 + i, 16, 0, 0);
            }
        }
        if (pre && info >= 0) {
            const uint32_t dvec = 1u << ((uint32_t)info >> 16) >> 2;  // 4 << L bytes
            const uint4* t4 = reinterpret_cast<const uint4*>(P.dt + gb * (uint64_t)(1u << LMAX));
            uint4* d4 = reinterpret_cast<uint4*>(sm.dt);
            for (uint32_t i = wv * 64u; i < dvec; i += 64u * NW) {
                if (i + lane < dvec)
                    __builtin_amdgcn_global_load_lds(t4 + i + lane, d4 + i, 16, 0, 0);
            }
        }
        if (!pre)
            for (uint32_t i = tid; i < 256u; i += 64u * NW) sm.norm[i] = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    FSE_STAMP(P, 1);
    int rc;
    int32_t hdr_bits;
    uint32_t L;
    if (pre) {
        rc = info < 0 ? info : FSE_OK;
        if (rc == FSE_OK && (!known || n < 2)) rc = FSE_ERR_LENGTH_MISMATCH;
        hdr_bits = (info & 0xFFFF) * 8;
        L = (uint32_t)info >> 16;
    } else {
        if (__builtin_amdgcn_readfirstlane(wv) == 0) {  // NormHistogram::read (lib.rs:219), scalar unit
            uint32_t Lh = 0, tl = 0;
            const uint32_t availw = (min(clen, PMAX) + 3u) >> 2;
            const uint32_t r0 = lane < availw ? sm.pay[lane] : 0u;
            const uint32_t r1 = lane + 64u < availw ? sm.pay[lane + 64u] : 0u;
            const int hl = header_read_wave(r0, r1, clen, (uint32_t)LMAX, sm.norm, &Lh, &tl);
            int r = hl < 0 ? hl : FSE_OK;
            if (r == FSE_OK && ((uint32_t)hl >= clen || in[clen - 1] == 0)) r = FSE_ERR_NO_MARKER;  // lib.rs:222
            if (lane == 0) {
                sm.scratch[0] = hl;
                sm.scratch[1] = (int)Lh;
                sm.scratch[2] = (int)tl;
                sm.scratch[3] = r;
            }
        }
        __syncthreads();
        FSE_STAMP(P, 2);
        if (sm.scratch[3] == FSE_OK) {  // DecodeTable::update (lib.rs:223, fse.rs:280-338)
            const uint32_t Lt = (uint32_t)sm.scratch[1], tl = (uint32_t)sm.scratch[2];
            const uint32_t size = 1u << Lt;
            uint8_t* scr = reinterpret_cast<uint8_t*>(sm.dt);
            const int32_t* norm = sm.norm;
            uint32_t* dt = sm.dt;
            const int r = block_build_spread<NW, LMAX>(sm.norm, Lt, tl, scr + 3u * size, scr + 2u * size, sm.cumul,
                                                       sm.cnt, sm.wscr, [&](uint32_t i, uint32_t s, uint32_t rk) {
                                                           const int32_t v = norm[s];
                                                           const uint32_t nx = (v < 0 ? 1u : (uint32_t)v) + rk;
                                                           const uint32_t nb = Lt - ilog2u(nx);
                                                           dt[i] = dte_make(nb, s, (nx << nb) - size);
                                                       });
            if (tid == 0) {
                int r2 = r;
                bool single = false;
                for (uint32_t q = 0; q < tl; ++q)
                    if (sm.norm[q] == (int32_t)size) single = true;
                if (r2 == FSE_OK && single && !known) r2 = FSE_ERR_SINGLE_SYMBOL;
                if (r2 == FSE_OK && known && n < 2) r2 = FSE_ERR_LENGTH_MISMATCH;
                sm.scratch[3] = r2;
            }
        }
        __syncthreads();
        rc = sm.scratch[3];
        hdr_bits = sm.scratch[0] * 8;
        L = (uint32_t)sm.scratch[1];
    }
    FSE_STAMP(P, 3);
    if (rc != FSE_OK) {
        if (tid == 0) {
            P.status[gb] = rc;
            if (P.out_len) P.out_len[gb] = 0;
        }
        return;
    }
    const uint32_t smask = (1u << L) - 1u;
    const uint32_t* dt = sm.dt;
    if (P.debug & 1u) {
        if (tid == 0) P.status[gb] = FSE_OK;
        return;
    }
    const uint32_t* gwords = reinterpret_cast<const uint32_t*>(in);

    if (P.sidecar && known) {
        const uint32_t Pm = (n & 1u) ? (n - 3u) / 2u : n / 2u - 1u;
        const uint32_t I = P.ckpt_interval;
        const uint32_t nseg = Pm / I + 1u;
        const uint64_t* sc = P.sidecar + gb * P.ckpt_per_block;
        int32_t err = FSE_OK;
        const uint32_t maxbp = clen * 8u - (uint32_t)hdr_bits;
        const uint8_t* dtb = reinterpret_cast<const uint8_t*>(dt);
        constexpr uint32_t NT = 64u * NW;
        auto seg_ok = [&](uint64_t e) { return (uint32_t)e <= maxbp; };  // corrupt index: never read outside
        {
            for (uint32_t seg = tid; seg < nseg; seg += NT) {
                const uint64_t e = sc[seg];
                const uint32_t p0 = seg * I;
                const uint32_t p1 = min(p0 + I, Pm);
                const uint32_t bp = (uint32_t)e;
                const uint32_t s0 = (uint32_t)(e >> 32) & smask, s1 = (uint32_t)(e >> 48) & smask;
                int32_t r;
                if (!seg_ok(e)) {
                    r = FSE_ERR_BAD_ARG;
                } else if (in_lds) {
                    const bool lastseg = seg == nseg - 1u;
                    if (padded) {
                        LdsChain<3> c;
                        c.init(sm.pay, hdr_bits + (int32_t)bp, s0, s1);
                        r = run_chain(c, sm.pay, dtb, p0, p1, lastseg, n, Pm, out, hdr_bits);
                    } else {
                        LdsChain<2> c;
                        c.init(sm.pay, hdr_bits + (int32_t)bp, s0, s1);
                        r = run_chain(c, sm.pay, dtb, p0, p1, lastseg, n, Pm, out, hdr_bits);
                    }
                } else {
                    GlobalReader br;  // LDS and global paths stay separate (no flat loads)
                    br.init(gwords, hdr_bits + (int32_t)bp);
                    r = decode_segment(br, s0, s1, p0, p1, seg == nseg - 1u, n, Pm, out, dt, smask, hdr_bits);
                }
                if (r != FSE_OK) err = r;
            }
        }
        err = -(int32_t)wave_max((uint32_t)(-err));
        if (lane == 0) sm.err[wv] = err;
        __syncthreads();
        FSE_STAMP(P, 4);
        if (tid == 0) {
            int32_t e = FSE_OK;
            for (int w = 0; w < NW; ++w)
                if (sm.err[w] != FSE_OK) e = sm.err[w];
            P.status[gb] = e;
            if (P.out_len) P.out_len[gb] = e ? 0u : n;
        }
        return;
    }

    // ---- serial (reference mode / no sidecar): lane 0, every read checked
    if (tid != 0) return;
    const int32_t top = (int32_t)(clen - 1u) * 8 + (int32_t)ilog2u(in[clen - 1]);
    LdsReader br;
    br.init(gwords, top);  // serial path reads global memory (rare; any length)
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
                store_byte(out, o++, cap, dte_sym(dt[s0 & smask]));
                store_byte(out, o++, cap, dte_sym(dt[s1 & smask]));
                break;
            }
            if (known && o + 1u == n) {
                store_byte(out, o++, cap, dte_sym(dt[s0 & smask]));
                break;
            }
            const uint32_t e0 = dt[s0 & smask];
            uint32_t nb = dte_nb(e0);
            if (br.pos - (int32_t)nb < hdr_bits) {  // decode0 fails: 242-243
                if (o + 2u > cap) { err = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL; break; }
                store_byte(out, o++, cap, dte_sym(e0));
                store_byte(out, o++, cap, dte_sym(dt[s1 & smask]));
                break;
            }
            s0 = dte_ns(e0) + br.pop(nb);
            br.refill();
            if (o >= cap) { err = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL; break; }
            store_byte(out, o++, cap, dte_sym(e0));
            const uint32_t e1 = dt[s1 & smask];
            nb = dte_nb(e1);
            if (br.pos - (int32_t)nb < hdr_bits) {  // decode1 fails: 235-239
                if (o + 2u > cap) { err = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL; break; }
                store_byte(out, o++, cap, dte_sym(e1));
                store_byte(out, o++, cap, dte_sym(dt[s0 & smask]));
                break;
            }
            s1 = dte_ns(e1) + br.pop(nb);
            br.refill();
            if (o >= cap) { err = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL; break; }
            store_byte(out, o++, cap, dte_sym(e1));
        }
    }
    if (err == FSE_OK && known && o != n) err = FSE_ERR_LENGTH_MISMATCH;
    P.status[gb] = err;
    if (P.out_len) P.out_len[gb] = err ? 0u : o;
}

// ------------------------------------------------------------------------
// Segment decode with prebuilt tables (the default sidecar decode and C3):
// no header parse, no table build, no serial path, so the kernel is small
// and its LDS is the block image plus the table.  VAR 3 stages the block as
// the padded image (pad_word), VAR 2 linearly with per-lane windows.
// ------------------------------------------------------------------------
// ------------------------------------------------------------------------
// 1-state decode (fse_decompress, lib.rs:187-211): one state chain, one
// symbol per step, same tables and sidecar layout (s1 = 0).  The per-lane
// window reader is the VAR 2 one.
// ------------------------------------------------------------------------
struct LdsChain1 {
    int32_t pos, B;
    uint32_t wlo, whi, wnx, a;
    __device__ __forceinline__ void init(const uint32_t* pay, int32_t p, uint32_t s) {
        pos = p;
        a = s << 2;
        const int32_t k = max((p >> 5) - 1, 0);
        B = k << 5;
        wlo = pay[k];
        whi = pay[k + 1];
        wnx = pay[max(k - 1, 0)];
    }
    // one symbol; returns the table entry (symbol in bits 8-15)
    __device__ __forceinline__ uint32_t step(const uint32_t* pay, const uint8_t* dtb) {
        const uint32_t e = *reinterpret_cast<const uint32_t*>(dtb + a);
        pos -= (int32_t)(e & 0xFFu);
        const uint32_t x = (uint32_t)((((uint64_t)whi << 32) | wlo) >> (uint32_t)(pos - B));
        if (pos < B + 32) {
            B -= 32;
            whi = wlo;
            wlo = wnx;
            wnx = pay[max((B >> 5) - 1, 0)];
        }
        a = (e >> 16) + (__builtin_amdgcn_ubfe(x, 0u, e) << 2);
        return e;
    }
};

// Steps [p, p1) of one 1-state segment; the last segment then emits the
// final state's symbol if, as in the reference loop, the next read fails.
__device__ __forceinline__ int32_t run_chain1(LdsChain1& c, const uint32_t* pay, const uint8_t* dtb, uint32_t p,
                                              uint32_t p1, bool last, uint32_t n, uint8_t* __restrict__ out,
                                              int32_t hdr_bits) {
    constexpr uint32_t G = 2u * DEC_GROUP;  // 64 symbols = one 64-byte segment of output
    for (; p + G <= p1; p += G) {
        uint32_t w[G / 4u];
#pragma unroll
        for (uint32_t j = 0; j < G; j += 4u) {
            const uint32_t e0 = c.step(pay, dtb), e1 = c.step(pay, dtb);
            const uint32_t e2 = c.step(pay, dtb), e3 = c.step(pay, dtb);
            w[j >> 2] = __builtin_amdgcn_perm(__builtin_amdgcn_perm(e3, e2, 0x0c0c0501u),
                                              __builtin_amdgcn_perm(e1, e0, 0x0c0c0501u), 0x05040100u);
        }
        uint4* o4 = reinterpret_cast<uint4*>(out + p);
#pragma unroll
        for (uint32_t q = 0; q < G / 16u; ++q) o4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    }
    for (; p < p1; ++p) out[p] = (uint8_t)dte_sym(c.step(pay, dtb));
    // container mode: the raw length ends the block (as the 2-state path
    // does); for a valid stream the reference's next read fails right here
    if (last) out[n - 1u] = (uint8_t)dte_sym(*reinterpret_cast<const uint32_t*>(dtb + c.a));  // finish (lib.rs:208)
    return FSE_OK;
}

// The same for blocks read from global memory (windowed reader).
template <class RD>
__device__ __forceinline__ int32_t decode_segment1(RD& br, uint32_t s, uint32_t p, uint32_t p1, bool last, uint32_t n,
                                                   uint8_t* __restrict__ out, const uint32_t* dt, uint32_t smask,
                                                   int32_t hdr_bits) {
    for (; p < p1; ++p) {
        const uint32_t e = dt[s & smask];
        s = dte_ns(e) + br.pop(dte_nb(e));
        br.refill();
        out[p] = (uint8_t)dte_sym(e);
    }
    if (last) out[n - 1u] = (uint8_t)dte_sym(dt[s & smask]);
    return FSE_OK;
}

template <int LMAX, uint32_t PMAX>
struct PreSmem {
    uint32_t pad[4];  // below the image: VAR 6 prefetches may address up to 2 words under it
    uint32_t pay[PMAX / 4];
    uint32_t dt[1u << LMAX];
    int err[16];
};

template <int LMAX, int NW, uint32_t PMAX, int VAR, int NS = 2, bool DUAL = false>
__global__ __launch_bounds__(64 * NW) void decode_pre_kernel(DecParams P) {
    __shared__ PreSmem<LMAX, PMAX> sm;
    constexpr uint32_t NT = 64u * NW;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = P.comp_len[gb];
    const uint64_t ooff = gb * (uint64_t)P.block_size;
    const uint32_t n = (uint32_t)min((uint64_t)P.block_size, P.n_total - ooff);
    uint8_t* out = P.out + ooff;
    const int32_t info = P.dtinfo[gb];
    const uint32_t nwords = (clen + 3u) >> 2;
    constexpr bool PADDED = VAR == 3 || VAR == 5;
    const bool in_lds = PADDED ? (pad_word(nwords) + 2u) * 4u <= PMAX : clen <= PMAX;
    if (P.pass == 2 && P.status[gb] != FSE_DEFERRED) return;  // done by the first pass
    FSE_STAMP(P, 0);
    if (info < 0 || n < 2) {
        if (tid == 0) P.status[gb] = info < 0 ? info : FSE_ERR_LENGTH_MISMATCH;
        return;
    }
    if (P.pass == 1 && !in_lds) {  // too big for this stage: the big-stage pass decodes it
        if (tid == 0) P.status[gb] = FSE_DEFERRED;
        return;
    }
    const int32_t hdr_bits = (info & 0xFFFF) * 8;
    const uint32_t L = (uint32_t)info >> 16;
    {  // stage the block image and the table
        if (in_lds) {
            if (PADDED) {
                // dword LDS-DMA: LDS word d <- source word d - d/33
                const uint32_t nd = pad_word(nwords) + 2u;
                const uint32_t wmax = (uint32_t)min((uint64_t)nwords + 1u, P.slot_bytes / 4u) - 1u;
                const uint32_t* src = reinterpret_cast<const uint32_t*>(in);
                for (uint32_t i = wv * 64u; i < nd; i += NT) {
                    const uint32_t d = i + lane;
                    const uint32_t w = min(d - d / 33u, wmax);
                    if (d < nd) __builtin_amdgcn_global_load_lds(src + w, sm.pay + i, 4, 0, 0);
                }
            } else {
                const uint32_t nvec = (clen + 15u) >> 4;
                const uint4* src4 = reinterpret_cast<const uint4*>(in);
                uint4* dst4 = reinterpret_cast<uint4*>(sm.pay);
                for (uint32_t i = wv * 64u; i < nvec; i += NT)
                    if (i + lane < nvec) __builtin_amdgcn_global_load_lds(src4 + i + lane, dst4 + i, 16, 0, 0);
            }
        }
        const uint32_t dvec = 1u << L >> 2;  // 4 << L bytes
        const uint4* t4 = reinterpret_cast<const uint4*>(P.dt + gb * (uint64_t)(1u << LMAX));
        uint4* d4 = reinterpret_cast<uint4*>(sm.dt);
        for (uint32_t i = wv * 64u; i < dvec; i += NT)
            if (i + lane < dvec) __builtin_amdgcn_global_load_lds(t4 + i + lane, d4 + i, 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    FSE_STAMP(P, 3);
    if (P.debug & 1u) {
        if (tid == 0) P.status[gb] = FSE_OK;
        return;
    }
    const uint32_t smask = (1u << L) - 1u;
    // main-loop steps: pairs (NS = 2) or symbols below the last one (NS = 1)
    const uint32_t Pm = NS == 2 ? ((n & 1u) ? (n - 3u) / 2u : n / 2u - 1u) : n - 1u;
    const uint32_t I = P.ckpt_interval;
    const uint32_t nseg = Pm / I + 1u;
    const uint64_t* sc = P.sidecar + gb * P.ckpt_per_block;
    const uint32_t maxbp = clen * 8u - (uint32_t)hdr_bits;
    const uint8_t* dtb = reinterpret_cast<const uint8_t*>(sm.dt);
    int32_t err = FSE_OK;
    if (NS == 1) {
        for (uint32_t seg = tid; seg < nseg; seg += NT) {
            const uint64_t e = sc[seg];
            const uint32_t p0 = seg * I, p1 = min(p0 + I, Pm);
            const uint32_t bp = (uint32_t)e, s0 = (uint32_t)(e >> 32) & smask;
            const bool lastseg = seg == nseg - 1u;
            int32_t r;
            if (bp > maxbp) {
                r = FSE_ERR_BAD_ARG;
            } else if (in_lds && !PADDED) {
                LdsChain1 c;
                c.init(sm.pay, hdr_bits + (int32_t)bp, s0);
                r = run_chain1(c, sm.pay, dtb, p0, p1, lastseg, n, out, hdr_bits);
            } else {
                GlobalReader br;
                br.init(reinterpret_cast<const uint32_t*>(in), hdr_bits + (int32_t)bp);
                r = decode_segment1(br, s0, p0, p1, lastseg, n, out, sm.dt, smask, hdr_bits);
            }
            if (r != FSE_OK) err = r;
        }
    } else if (DUAL && in_lds) {  // two segments per lane: seg and seg + NT (own instantiation: its
                                  // two chains would otherwise set the kernel's VGPR count)
        for (uint32_t sa = tid; sa < nseg; sa += 2u * NT) {
            const uint32_t sb = sa + NT;
            const uint64_t ea = sc[sa];
            const uint64_t eb = sb < nseg ? sc[sb] : ea;
            if ((uint32_t)ea > maxbp || (uint32_t)eb > maxbp) {
                err = FSE_ERR_BAD_ARG;
                continue;
            }
            LdsChain<VAR> A, Bc;
            A.init(sm.pay, hdr_bits + (int32_t)(uint32_t)ea, (uint32_t)(ea >> 32) & smask, (uint32_t)(ea >> 48) & smask);
            const uint32_t pa = sa * I, pa1 = min(pa + I, Pm);
            int32_t r;
            if (sb < nseg) {
                Bc.init(sm.pay, hdr_bits + (int32_t)(uint32_t)eb, (uint32_t)(eb >> 32) & smask,
                        (uint32_t)(eb >> 48) & smask);
                const uint32_t pb = sb * I, pb1 = min(pb + I, Pm);
                r = decode_dual(sm.pay, dtb, A, pa, pa1, sa == nseg - 1u, Bc, pb, pb1, sb == nseg - 1u, n, Pm, out,
                                hdr_bits);
            } else {
                r = run_chain(A, sm.pay, dtb, pa, pa1, sa == nseg - 1u, n, Pm, out, hdr_bits);
            }
            if (r != FSE_OK) err = r;
        }
    } else
    for (uint32_t base = 0; base < nseg; base += NT) {
        // VAR 6: lane t decodes segment 33t mod NT of each round, so lanes
        // that walk their segments in lockstep read words ~33 segments apart
        // (spread over the banks) instead of ~1 segment (~32 words) apart
        const uint32_t seg = base + ((VAR == 6 || VAR == 0 || VAR == 1 || VAR == 9 || VAR == 12) ? ((tid * 33u) & (NT - 1u)) : tid);
        if (seg >= nseg) continue;
        const uint64_t e = sc[seg];
        const uint32_t p0 = seg * I, p1 = min(p0 + I, Pm);
        const uint32_t bp = (uint32_t)e;
        const uint32_t s0 = (uint32_t)(e >> 32) & smask, s1 = (uint32_t)(e >> 48) & smask;
        const bool lastseg = seg == nseg - 1u;
        int32_t r;
        if (bp > maxbp) {  // corrupt index: never read outside the block
            r = FSE_ERR_BAD_ARG;
        } else if (in_lds) {
            LdsChain<VAR> c;
            c.init(sm.pay, hdr_bits + (int32_t)bp, s0, s1);
            r = run_chain(c, sm.pay, dtb, p0, p1, lastseg, n, Pm, out, hdr_bits);
        } else {
            GlobalReader br;
            br.init(reinterpret_cast<const uint32_t*>(in), hdr_bits + (int32_t)bp);
            r = decode_segment(br, s0, s1, p0, p1, lastseg, n, Pm, out, sm.dt, smask, hdr_bits);
        }
        if (r != FSE_OK) err = r;
    }
    err = -(int32_t)wave_max((uint32_t)(-err));
    if (lane == 0) sm.err[wv] = err;
    __syncthreads();
    FSE_STAMP(P, 4);
    if (tid == 0) {
        int32_t e2 = FSE_OK;
        for (int w = 0; w < NW; ++w)
            if (sm.err[w] != FSE_OK) e2 = sm.err[w];
        P.status[gb] = e2;
        if (P.out_len) P.out_len[gb] = e2 ? 0u : n;
    }
}

// ------------------------------------------------------------------------
// Decode tables for a batch of blocks (C3's "pre-built dtables"; also the
// first kernel of the two-kernel decode): NormHistogram::read on the scalar
// unit + DecodeTable (fse.rs:280-338) by one wave per block, written to HBM
// in the decoder's entry layout.  Small LDS footprint, so many blocks are in
// flight per CU and the serial header parse is overlapped across blocks.
// ------------------------------------------------------------------------
template <int LMAX>
__global__ __launch_bounds__(64) void dtable_blocks_kernel(DtParams P) {
    constexpr uint32_t SIZE = 1u << LMAX;
    __shared__ int32_t norm[256];
    __shared__ __attribute__((aligned(16))) uint8_t sym_at[SIZE];
    // the two-pass rank table (2^L u16) reuses the occurrence owners, the
    // counters and cumul: all three are dead once the spread walk is done
    // (the decoder's visit reads norm only); 7 KB per workgroup at L = 11
    __shared__ __attribute__((aligned(16))) uint16_t rk[SIZE];
    static_assert(SIZE + 256 * 4 + 256 * 2 <= SIZE * 2, "rank table must cover occ, cnt and cumul");
    uint8_t* occ = reinterpret_cast<uint8_t*>(rk);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(rk) + SIZE);
    uint16_t* cumul = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(rk) + SIZE + 1024);
    const uint32_t lane = lane_id();
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = P.comp_len[gb];
    const uint32_t* w = reinterpret_cast<const uint32_t*>(in);
    // The header words are loaded before the length arrives when the slot
    // holds HDR_MAX bytes (always, for encoder slots), so the two loads and
    // the marker byte's load overlap instead of following one another;
    // words past the block are zeroed once the length is known.
    uint32_t r0, r1;
    if (P.slot_bytes >= HDR_MAX) {
        r0 = w[lane];
        r1 = w[lane + 64u];
    }
    const uint32_t last = (clen && clen <= P.slot_bytes) ? in[clen - 1u] : 0u;
    const uint32_t nw = (uint32_t)min((uint64_t)min(clen, HDR_MAX) + 3u, P.slot_bytes) >> 2;
    if (P.slot_bytes < HDR_MAX) {
        r0 = lane < nw ? w[lane] : 0u;
        r1 = lane + 64u < nw ? w[lane + 64u] : 0u;
    }
    r0 = lane < nw ? r0 : 0u;
    r1 = lane + 64u < nw ? r1 : 0u;
    for (uint32_t s = lane; s < 256u; s += WAVE) norm[s] = 0;
    wave_sync();
    uint32_t L = 0, tl = 0;
    const int hl = header_read_wave(r0, r1, clen, (uint32_t)LMAX, norm, &L, &tl);
    int rc = hl < 0 ? hl : FSE_OK;
    if (rc == FSE_OK && ((uint32_t)hl >= clen || last == 0)) rc = FSE_ERR_NO_MARKER;  // lib.rs:222
    wave_sync();
    if (rc == FSE_OK && !(P.debug & 1u)) {
        const uint32_t size = 1u << L;
        uint32_t* dt = P.dt + gb * (uint64_t)SIZE;
        rc = wave_build_spread<SIZE / 64u>(norm, L, tl, sym_at, occ, cumul, cnt, [&](uint32_t i, uint32_t s, uint32_t r) {
            const int32_t v = norm[s];
            const uint32_t nx = (v < 0 ? 1u : (uint32_t)v) + r;
            const uint32_t nb = L - ilog2u(nx);
            if (!(P.debug & 2u)) dt[i] = dte_make(nb, s, (nx << nb) - size);
        }, rk);
    }
    if (lane == 0) P.dtinfo[gb] = rc == FSE_OK ? (int32_t)((uint32_t)hl | (L << 16)) : rc;
}

// ------------------------------------------------------------------------
// fse_decompress (lib.rs:187-211) in reference mode: no sidecar, raw length
// unknown; one lane per block walks the stream with every read checked, on
// tables from dtable_blocks_kernel.  Serial by nature (the host entry point
// and streams produced elsewhere).
// ------------------------------------------------------------------------
template <int LMAX>
__global__ __launch_bounds__(64) void decode1_serial_kernel(DecParams P) {
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks || threadIdx.x != 0) return;
    const int32_t info = P.dtinfo[gb];
    if (info < 0) {
        P.status[gb] = info;
        if (P.out_len) P.out_len[gb] = 0;
        return;
    }
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = P.comp_len[gb];
    const int32_t hdr_bits = (info & 0xFFFF) * 8;
    const uint32_t L = (uint32_t)info >> 16;
    const uint32_t* dt = P.dt + gb * (uint64_t)(1u << LMAX);
    uint8_t* out = P.out + gb * (uint64_t)P.block_size;
    const bool known = P.n_total != 0;  // container length, else reference mode with a capacity
    const uint32_t n = known ? (uint32_t)min((uint64_t)P.block_size, P.n_total - gb * (uint64_t)P.block_size) : 0u;
    const uint32_t cap = known ? n : P.out_cap;
    int32_t err = FSE_OK;
    uint32_t o = 0;
    const int32_t top = (int32_t)(clen - 1u) * 8 + (int32_t)ilog2u(in[clen - 1]);  // marker (BitStackReader::new)
    GlobalReader br;
    br.init(reinterpret_cast<const uint32_t*>(in), top);
    if (br.pos - (int32_t)L < hdr_bits) {
        err = FSE_ERR_TOO_SHORT;  // lib.rs:197 unwrap
    } else {
        uint32_t s = br.pop(L);
        br.refill();
        for (;;) {
            const uint32_t e = dt[s];
            const uint32_t nb = dte_nb(e);
            if (br.pos - (int32_t)nb < hdr_bits) break;  // decode_symbol -> None
            if (o >= cap) {  // nb == 0 forever: a probability-1 symbol never ends in the reference
                err = nb == 0 ? FSE_ERR_SINGLE_SYMBOL : FSE_ERR_DST_TOO_SMALL;
                break;
            }
            s = dte_ns(e) + br.pop(nb);
            br.refill();
            out[o++] = (uint8_t)dte_sym(e);
        }
        if (err == FSE_OK) {
            if (o >= cap) err = FSE_ERR_DST_TOO_SMALL;
            else out[o++] = (uint8_t)dte_sym(dt[s]);  // Decoder::finish (lib.rs:208)
        }
        if (known && (err == FSE_ERR_DST_TOO_SMALL || (err == FSE_OK && o != n))) err = FSE_ERR_LENGTH_MISMATCH;
    }
    P.status[gb] = err;
    if (P.out_len) P.out_len[gb] = err ? 0u : o;
}

// ------------------------------------------------------------------------
// Sidecar-less container decode of 2-state blocks (any valid fse_compress2
// stream, e.g. from the CPU crate), optionally recording the sidecar.
// The two interleaved decoders make the stream essentially serial: a
// decoder started mid-block with guessed states practically never falls
// into step with the exact one (oracle/syncsim.py: 35 of 40 random starts in
// a C2 block never did, the rest after 25K-40K symbols), so speculative
// segment decoding cannot replace the sidecar for this
// format.  The serial decode is instead made as short a dependency chain
// as possible and run at high occupancy: the block's prebuilt table sits in
// LDS (8 KiB -> 20 blocks in flight per CU), one lane walks the stream
// (lib.rs:227-244, container mode as the oracle's decompress2 with known
// length) and the bits come through a register window fed from 16-byte
// chunks that are loaded a whole chunk ahead.
// ------------------------------------------------------------------------
struct ChunkReader {
    const uint4* w4;  // the block as 16-byte quads
    uint64_t buf;     // stream bits [base, base + 64)
    int32_t base, pos;
    uint4 cl, ch, nl, nh;  // chunk c (words 8c..8c+7) and chunk c-1, loading
    int32_t c;
    __device__ __forceinline__ void init(const uint8_t* in, int32_t p) {
        w4 = reinterpret_cast<const uint4*>(in);
        const uint32_t* w = reinterpret_cast<const uint32_t*>(in);
        pos = p;
        base = max(((p + 31) & ~31) - 64, 0);
        buf = (uint64_t)w[base >> 5] | ((uint64_t)w[(base >> 5) + 1] << 32);
        c = ((base >> 5) - 1) >> 3;  // chunk of the next word to enter the window
        cl = w4[2 * max(c, 0)];
        ch = w4[2 * max(c, 0) + 1];
        nl = w4[2 * max(c - 1, 0)];
        nh = w4[2 * max(c - 1, 0) + 1];
    }
    __device__ __forceinline__ uint32_t pop(uint32_t nb) {
        pos -= (int32_t)nb;
        return (uint32_t)(buf >> (uint32_t)(pos - base)) & ((1u << nb) - 1u);
    }
    __device__ __forceinline__ void refill() {
        if (pos - base < 32 && base > 0) {
            base -= 32;
            const int32_t wi = base >> 5;
            if ((wi >> 3) != c) {  // every 8th refill: move down a chunk, prefetch the next
                cl = nl;
                ch = nh;
                c -= 1;
                nl = w4[2 * max(c - 1, 0)];
                nh = w4[2 * max(c - 1, 0) + 1];
            }
            const uint32_t j = (uint32_t)wi & 7u;
            const uint4 q = j < 4u ? cl : ch;
            const uint32_t k = j & 3u;
            const uint32_t v = k == 0 ? q.x : k == 1 ? q.y : k == 2 ? q.z : q.w;
            buf = (buf << 32) | v;
        }
    }
};

// One lane per block; the rest of the wave only stages the table.  Measured
// slower and dropped: an LDS ring for the stream and the output, flushed by
// the whole wave every 128 pairs (its 10.7 KB per block allow 14 blocks per
// CU instead of 20, and the chain is latency-bound either way), and a
// scalar-unit walk with all state in SGPRs (26.5 vs 15.9 ms per 256 MiB:
// the CU's one scalar unit is shared by the 20 blocks in flight).
template <int LMAX>
__global__ __launch_bounds__(64) void serial2_decode_kernel(DecParams P) {
    __shared__ uint32_t tab[1u << LMAX];
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    const int32_t info = P.dtinfo[gb];
    const uint32_t lane = threadIdx.x;
    if (info >= 0) {  // stage the table (prebuilt by dtable_blocks_kernel)
        const uint32_t nv = (1u << ((uint32_t)info >> 16)) >> 2;  // 16-byte chunks
        const uint4* t4 = reinterpret_cast<const uint4*>(P.dt + gb * (uint64_t)(1u << LMAX));
        uint4* d4 = reinterpret_cast<uint4*>(tab);
        for (uint32_t i = lane; i < nv; i += 64u) d4[i] = t4[i];
    }
    __syncthreads();
    if (lane != 0) return;
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = P.comp_len[gb];
    const uint64_t ooff = gb * (uint64_t)P.block_size;
    const uint32_t n = (uint32_t)min((uint64_t)P.block_size, P.n_total - ooff);
    uint8_t* out = P.out + ooff;
    int32_t err = info < 0 ? info : (n < 2 ? FSE_ERR_LENGTH_MISMATCH : FSE_OK);
    const int32_t hdr_bits = (info & 0xFFFF) * 8;
    const uint32_t L = (uint32_t)info >> 16;
    uint32_t o = 0;
    if (err == FSE_OK) {
        const int32_t top = (int32_t)(clen - 1u) * 8 + (int32_t)ilog2u(in[clen - 1]);
        if (top - 2 * (int32_t)L < hdr_bits) err = FSE_ERR_TOO_SHORT;  // lib.rs:224-225
    }
    if (err == FSE_OK) {
        ChunkReader br;
        br.init(in, (int32_t)(clen - 1u) * 8 + (int32_t)ilog2u(in[clen - 1]));
        uint32_t s0 = br.pop(L);
        br.refill();
        uint32_t s1 = br.pop(L);
        br.refill();
        const uint32_t I = P.ckpt_interval;
        uint64_t* rec = (P.sidecar_out && I) ? P.sidecar_out + gb * P.ckpt_per_block : nullptr;
        const uint32_t ckmask = I ? I - 1u : 0u;
        uint32_t pidx = 0;
        auto record = [&]() {
            if (rec && (pidx & ckmask) == 0u && pidx / I < P.ckpt_per_block)
                rec[pidx / I] = (uint64_t)(uint32_t)(br.pos - hdr_bits) | ((uint64_t)s0 << 32) | ((uint64_t)s1 << 48);
        };
        // bulk: groups of 8 pairs that can neither reach the raw length nor
        // run out of bits (<= 2 x 12 bits a pair): no end checks, and the
        // 16 output bytes leave as one dwordx4 store, so few stores are in
        // flight when the next chunk's load is waited on
        while (o + 18u < n && br.pos - hdr_bits >= 8 * 24) {
            uint32_t w[4];
#pragma unroll
            for (uint32_t j = 0; j < 8u; ++j, ++pidx) {
                record();
                const uint32_t e0 = tab[s0];
                s0 = dte_ns(e0) + br.pop(dte_nb(e0));
                br.refill();
                const uint32_t e1 = tab[s1];
                s1 = dte_ns(e1) + br.pop(dte_nb(e1));
                br.refill();
                const uint32_t v = dte_sym(e0) | (dte_sym(e1) << 8);
                if (j & 1u) w[j >> 1] |= v << 16; else w[j >> 1] = v;
            }
            if (!(P.debug & 2u)) *reinterpret_cast<uint4*>(out + o) = make_uint4(w[0], w[1], w[2], w[3]);  // 2: ablation
            o += 16;
        }
        // tail: pair by pair with the reference's end checks
        for (;; ++pidx) {
            record();
            if (o + 2u >= n) {  // the raw length ends the block (o is even here)
                if (o < n) out[o++] = (uint8_t)dte_sym(tab[s0]);
                if (o < n) out[o++] = (uint8_t)dte_sym(tab[s1]);
                break;
            }
            const uint32_t e0 = tab[s0];
            uint32_t nb = dte_nb(e0);
            if (br.pos - (int32_t)nb < hdr_bits) {  // decoder 0 cannot read: lib.rs:242-243
                out[o++] = (uint8_t)dte_sym(e0);
                out[o++] = (uint8_t)dte_sym(tab[s1]);
                break;
            }
            s0 = dte_ns(e0) + br.pop(nb);
            br.refill();
            const uint32_t e1 = tab[s1];
            nb = dte_nb(e1);
            if (br.pos - (int32_t)nb < hdr_bits) {  // decoder 1 cannot read: lib.rs:235-239
                out[o++] = (uint8_t)dte_sym(e0);
                out[o++] = (uint8_t)dte_sym(e1);
                if (o < n) out[o++] = (uint8_t)dte_sym(tab[s0]);
                break;
            }
            s1 = dte_ns(e1) + br.pop(nb);
            br.refill();
            out[o] = (uint8_t)dte_sym(e0);
            out[o + 1] = (uint8_t)dte_sym(e1);
            o += 2;
        }
        if (o != n) err = FSE_ERR_LENGTH_MISMATCH;
    }
    P.status[gb] = err;
    if (P.out_len) P.out_len[gb] = err ? 0u : o;
}

// ------------------------------------------------------------------------
// Histogram::new per block (histogram::count), one wave per block.
// ------------------------------------------------------------------------
__global__ __launch_bounds__(64) void histogram_blocks_kernel(const uint8_t* src, uint64_t n_total,
                                                              uint32_t block_size, uint32_t n_blocks,
                                                              uint32_t* counts, uint32_t* table_len) {
    __shared__ uint32_t h4[HIST_WORDS];
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
// Pack / unpack between the per-block slot layout and one contiguous
// stream (blocks back to back, byte offsets from an exclusive scan of the
// compressed lengths).  One 256-thread workgroup per block; offsets are
// arbitrary, so the copy is done in bytes with 16-byte source reads.
// ------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_blocks_kernel(const uint8_t* __restrict__ slots, uint64_t slot_bytes,
                                                          const uint32_t* __restrict__ comp_len,
                                                          const uint64_t* __restrict__ offsets, uint32_t n_blocks,
                                                          uint8_t* __restrict__ stream, int unpack) {
    const uint64_t b = blockIdx.x;
    if (b >= n_blocks) return;
    const uint32_t len = comp_len[b];
    uint8_t* slot = const_cast<uint8_t*>(slots) + b * slot_bytes;
    const uint64_t o = offsets[b];
    if (!unpack) {
        // dword-aligned stream writes; each from two aligned slot dwords
        // (v_alignbyte); the partial dwords at both ends (shared with the
        // neighbouring blocks) are written bytewise
        const uint64_t d0 = (o + 3u) >> 2, d1 = (o + len) >> 2;  // full stream dwords [d0, d1)
        const uint32_t* src = reinterpret_cast<const uint32_t*>(slot);
        uint32_t* dst = reinterpret_cast<uint32_t*>(stream);
        if (d1 > d0) {
            const uint32_t head = (uint32_t)(4u * d0 - o);  // slot byte feeding stream dword d0
            for (uint64_t d = d0 + threadIdx.x; d < d1; d += 256u) {
                const uint32_t sb = head + 4u * (uint32_t)(d - d0);  // slot byte offset
                const uint32_t q = sb >> 2, sh = sb & 3u;
                const uint32_t lo = src[q], hi = src[q + 1u];  // slot slack covers q + 1
                dst[d] = __builtin_amdgcn_alignbyte(hi, lo, sh);
            }
        }
        const uint64_t hb = min((uint64_t)len, 4u * d0 - o);  // head bytes before dword d0
        if (threadIdx.x < hb) stream[o + threadIdx.x] = slot[threadIdx.x];
        const uint64_t tb0 = d1 > d0 ? 4u * d1 - o : hb;  // tail bytes from here
        for (uint64_t i = tb0 + threadIdx.x; i < len; i += 256u) stream[o + i] = slot[i];
    } else {
        const uint8_t* s = stream + o;
        for (uint32_t i = threadIdx.x; i < len; i += 256u) slot[i] = s[i];
    }
}

// ------------------------------------------------------------------------
// Byte-range gather between two packed streams: block b's len[b] bytes move
// from src + src_off[b] to dst + dst_off[b] (both arbitrary byte offsets).
// Selects a rank's blocks out of a packed stream for the distributed
// scatter (round-robin shards are not contiguous in the global stream).
// Destination dwords come from two aligned source dwords (v_alignbyte); the
// partial dwords at either end, shared with neighbouring blocks, bytewise.
// ------------------------------------------------------------------------
__global__ __launch_bounds__(256) void copy_blocks_kernel(const uint8_t* __restrict__ src,
                                                          const uint64_t* __restrict__ src_off,
                                                          const uint32_t* __restrict__ lens, uint32_t n_blocks,
                                                          uint8_t* __restrict__ dst,
                                                          const uint64_t* __restrict__ dst_off) {
    const uint64_t b = blockIdx.x;
    if (b >= n_blocks) return;
    const uint32_t len = lens[b];
    const uint64_t so = src_off[b], o = dst_off[b];
    const uint64_t d0 = (o + 3u) >> 2, d1 = (o + len) >> 2;  // whole destination dwords [d0, d1)
    uint32_t* dw = reinterpret_cast<uint32_t*>(dst);
    if (d1 > d0) {
        const uint64_t s0 = so + (4u * d0 - o);  // source byte feeding dword d0
        const uint32_t sh = (uint32_t)(s0 & 3u);
        const uint32_t* sw = reinterpret_cast<const uint32_t*>(src) + (s0 >> 2);
        for (uint64_t d = threadIdx.x; d < d1 - d0; d += 256u) {
            const uint32_t lo = sw[d];
            // the word above is read only when it carries bytes of this block
            const uint32_t hi = sh ? sw[d + 1u] : 0u;
            dw[d0 + d] = __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
    }
    const uint64_t hb = min((uint64_t)len, 4u * d0 - o);
    if (threadIdx.x < hb) dst[o + threadIdx.x] = src[so + threadIdx.x];
    const uint64_t tb0 = d1 > d0 ? 4u * d1 - o : hb;
    for (uint64_t i = tb0 + threadIdx.x; i < len; i += 256u) dst[o + i] = src[so + i];
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
    const uint32_t T = P.lanes ? P.lanes : 64;
    const uint32_t bpw = 64u / T;
    const dim3 g((P.n_blocks + bpw - 1u) / bpw), b(64);
    if (P.nstates == 1) {  // fse_compress (lib.rs:112-143)
        if (lmax <= 11) hipLaunchKernelGGL((encode_blocks_kernel<11, 64, 1>), g, b, P.xlds, stream, P);
        else hipLaunchKernelGGL((encode_blocks_kernel<12, 64, 1>), g, b, P.xlds, stream, P);
    } else if (T == 64 && P.scratch) {  // scratch path built in (FSEHIP_ENC_PATH=0|2)
        if (lmax <= 11) hipLaunchKernelGGL((encode_blocks_kernel<11, 64, 2, true>), g, b, P.xlds, stream, P);
        else hipLaunchKernelGGL((encode_blocks_kernel<12, 64, 2, true>), g, b, P.xlds, stream, P);
    } else if (T == 64) {
        if (lmax <= 11) hipLaunchKernelGGL((encode_blocks_kernel<11, 64, 2>), g, b, P.xlds, stream, P);
        else hipLaunchKernelGGL((encode_blocks_kernel<12, 64, 2>), g, b, P.xlds, stream, P);
    } else {
        if (lmax <= 11) hipLaunchKernelGGL((encode_blocks_kernel<11, 32, 2>), g, b, P.xlds, stream, P);
        else hipLaunchKernelGGL((encode_blocks_kernel<12, 32, 2>), g, b, P.xlds, stream, P);
    }
    return hipGetLastError();
}

hipError_t launch_decode(const DecParams& P, uint32_t lmax, hipStream_t stream) {
    // LDS stage for the compressed block, sized for 3 workgroups per CU at L <= 11
    constexpr uint32_t PM4 = 39u << 10, PM8 = 35u << 10;
    const dim3 g(P.n_blocks);
    if (P.dt && !P.sidecar && P.nstates != 1 && P.n_total) {  // sidecar-less container blocks
        if (lmax <= 11) hipLaunchKernelGGL((serial2_decode_kernel<11>), g, dim3(64), 0, stream, P);
        else hipLaunchKernelGGL((serial2_decode_kernel<12>), g, dim3(64), 0, stream, P);
        return hipGetLastError();
    }
    if (P.dt) {  // prebuilt tables: lean kernel; LDS = image + table (44 KB image -> 3 WG/CU)
        constexpr uint32_t PP = 44u << 10;
        auto go = [&](auto kern, uint32_t threads) { hipLaunchKernelGGL(kern, g, dim3(threads), 0, stream, P); };
        if (P.nstates == 1) {  // fse_decompress blocks: linear image, per-lane windows
            if (!P.sidecar) {  // reference mode: serial, every read checked
                if (lmax <= 11) go(decode1_serial_kernel<11>, 64);
                else go(decode1_serial_kernel<12>, 64);
            } else {  // two passes, as for 2-state blocks below
                DecParams P1 = P, P2 = P;
                P1.pass = 1;
                P2.pass = 2;
                if (lmax <= 11) {
                    hipLaunchKernelGGL((decode_pre_kernel<11, 4, PP, 2, 1>), g, dim3(256), 0, stream, P1);
                    hipLaunchKernelGGL((decode_pre_kernel<11, 4, (66u << 10), 2, 1>), g, dim3(256), 0, stream, P2);
                } else {
                    hipLaunchKernelGGL((decode_pre_kernel<12, 4, PP - 8192, 2, 1>), g, dim3(256), 0, stream, P1);
                    hipLaunchKernelGGL((decode_pre_kernel<12, 4, (66u << 10), 2, 1>), g, dim3(256), 0, stream, P2);
                }
            }
            return hipGetLastError();
        }
        if (P.waves == 8) {
            if (lmax <= 11) {
                if (P.variant == 3) go(decode_pre_kernel<11, 8, PP, 3>, 512);
                else if (P.variant == 5) go(decode_pre_kernel<11, 8, PP, 5>, 512);
                else if (P.variant == 6) go(decode_pre_kernel<11, 8, PP, 6>, 512);
                else if (P.variant == 2) go(decode_pre_kernel<11, 8, PP, 2>, 512);
                else go(decode_pre_kernel<11, 8, PP, 12>, 512);
            } else {
                if (P.variant == 3) go(decode_pre_kernel<12, 8, PP - 8192, 3>, 512);
                else if (P.variant == 5) go(decode_pre_kernel<12, 8, PP - 8192, 5>, 512);
                else go(decode_pre_kernel<12, 8, PP - 8192, 2>, 512);
            }
        } else {
            if (lmax <= 11) {
                if (P.dual) {
                    if (P.variant == 3) go(decode_pre_kernel<11, 4, PP, 3, 2, true>, 256);
                    else if (P.variant == 5) go(decode_pre_kernel<11, 4, PP, 5, 2, true>, 256);
                    else go(decode_pre_kernel<11, 4, PP, 2, 2, true>, 256);
                } else if (P.variant == 3) go(decode_pre_kernel<11, 4, PP, 3>, 256);
                else if (P.variant == 5) go(decode_pre_kernel<11, 4, PP, 5>, 256);
                else if (P.variant == 6) go(decode_pre_kernel<11, 4, PP, 6>, 256);
                else if (P.variant == 10) go(decode_pre_kernel<11, 4, PP, 0>, 256);
                else if (P.variant == 11) go(decode_pre_kernel<11, 4, PP, 1>, 256);
                else if (P.variant == 2) go(decode_pre_kernel<11, 4, PP, 2>, 256);
                else if (P.variant == 9) go(decode_pre_kernel<11, 4, PP, 9>, 256);
                else if (P.stage_kib == 40) go(decode_pre_kernel<11, 4, (40u << 10), 2>, 256);
                else if (P.stage_kib == 36) go(decode_pre_kernel<11, 4, (36u << 10), 2>, 256);
                else {
                    // blocks above the 44 KiB stage (e.g. near-uniform data, ~65 KB) are
                    // deferred to a second launch with a 66 KiB stage (2 workgroups per CU)
                    // instead of the global-memory reader
                    DecParams P1 = P, P2 = P;
                    P1.pass = 1;
                    P2.pass = 2;
                    hipLaunchKernelGGL((decode_pre_kernel<11, 4, PP, 12>), g, dim3(256), 0, stream, P1);
                    hipLaunchKernelGGL((decode_pre_kernel<11, 4, (66u << 10), 12>), g, dim3(256), 0, stream, P2);
                }
            } else {
                if (P.variant == 3) go(decode_pre_kernel<12, 4, PP - 8192, 3>, 256);
                else if (P.variant == 5) go(decode_pre_kernel<12, 4, PP - 8192, 5>, 256);
                else {
                    DecParams P1 = P, P2 = P;
                    P1.pass = 1;
                    P2.pass = 2;
                    hipLaunchKernelGGL((decode_pre_kernel<12, 4, PP - 8192, 12>), g, dim3(256), 0, stream, P1);
                    hipLaunchKernelGGL((decode_pre_kernel<12, 4, (66u << 10), 12>), g, dim3(256), 0, stream, P2);
                }
            }
        }
        return hipGetLastError();
    }
    if (P.waves == 8) {
        if (lmax <= 11) hipLaunchKernelGGL((decode_blocks_kernel<11, 8, PM8>), g, dim3(512), 0, stream, P);
        else hipLaunchKernelGGL((decode_blocks_kernel<12, 8, PM8>), g, dim3(512), 0, stream, P);
    } else {
        if (lmax <= 11) hipLaunchKernelGGL((decode_blocks_kernel<11, 4, PM4>), g, dim3(256), 0, stream, P);
        else hipLaunchKernelGGL((decode_blocks_kernel<12, 4, PM4>), g, dim3(256), 0, stream, P);
    }
    return hipGetLastError();
}

int occupancy_report(char* buf, int cap) {
    int len = 0;
    auto one = [&](const char* name, const void* k, int threads) {
        int nb = -1;
        hipFuncAttributes fa{};
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, threads, 0);
        (void)hipFuncGetAttributes(&fa, k);
        if (len < cap)
            len += snprintf(buf + len, cap - len, "%s: %d WG/CU (lds %zu B, vgpr %d)\n", name, nb,
                            fa.sharedSizeBytes, fa.numRegs);
    };
    one("encode<11,64,2>", reinterpret_cast<const void*>(encode_blocks_kernel<11, 64, 2>), 64);
    one("dtable<11>", reinterpret_cast<const void*>(dtable_blocks_kernel<11>), 64);
    one("decode_pre<11,4,44K,2>", reinterpret_cast<const void*>(decode_pre_kernel<11, 4, (44u << 10), 2>), 256);
    one("decode_pre<11,4,40K,2>", reinterpret_cast<const void*>(decode_pre_kernel<11, 4, (40u << 10), 2>), 256);
    one("decode_pre<11,4,36K,2>", reinterpret_cast<const void*>(decode_pre_kernel<11, 4, (36u << 10), 2>), 256);
    one("decode_pre<11,4,44K,3>", reinterpret_cast<const void*>(decode_pre_kernel<11, 4, (44u << 10), 3>), 256);
    one("decode_pre<11,8,44K,3>", reinterpret_cast<const void*>(decode_pre_kernel<11, 8, (44u << 10), 3>), 512);
    one("decode_blocks<11,4>", reinterpret_cast<const void*>(decode_blocks_kernel<11, 4, (39u << 10)>), 256);
    return len;
}

hipError_t launch_dtables(const DtParams& P, uint32_t lmax, hipStream_t stream) {
    if (lmax <= 11) hipLaunchKernelGGL((dtable_blocks_kernel<11>), dim3(P.n_blocks), dim3(64), 0, stream, P);
    else hipLaunchKernelGGL((dtable_blocks_kernel<12>), dim3(P.n_blocks), dim3(64), 0, stream, P);
    return hipGetLastError();
}

hipError_t launch_histogram(const uint8_t* src, uint64_t n_total, uint32_t block_size, uint32_t n_blocks,
                            uint32_t* counts, uint32_t* table_len, hipStream_t stream) {
    hipLaunchKernelGGL(histogram_blocks_kernel, dim3(n_blocks), dim3(64), 0, stream, src, n_total, block_size,
                       n_blocks, counts, table_len);
    return hipGetLastError();
}

hipError_t launch_pack(const uint8_t* slots, uint64_t slot_bytes, const uint32_t* comp_len, const uint64_t* offsets,
                       uint32_t n_blocks, uint8_t* stream, int unpack, hipStream_t hs) {
    hipLaunchKernelGGL(pack_blocks_kernel, dim3(n_blocks), dim3(256), 0, hs, slots, slot_bytes, comp_len, offsets,
                       n_blocks, stream, unpack);
    return hipGetLastError();
}

hipError_t launch_copy(const uint8_t* src, const uint64_t* src_off, const uint32_t* lens, uint32_t n_blocks,
                       uint8_t* dst, const uint64_t* dst_off, hipStream_t hs) {
    hipLaunchKernelGGL(copy_blocks_kernel, dim3(n_blocks), dim3(256), 0, hs, src, src_off, lens, n_blocks, dst,
                       dst_off);
    return hipGetLastError();
}

hipError_t launch_generate(const GenParams& G, hipStream_t stream) {
    const uint64_t threads = (G.n_total + 15) / 16;
    const uint32_t grid = (uint32_t)((threads + 255) / 256);
    hipLaunchKernelGGL(generate_kernel, dim3(grid), dim3(256), 0, stream, G);
    return hipGetLastError();
}

}  // namespace fsehip
