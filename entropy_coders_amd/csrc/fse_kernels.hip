// fse_kernels.hip -- batched FSE (tANS) block codec kernels for gfx950.
//
// Wire format: exactly the reference's fse_compress2 block (lib.rs:146-183):
// NCount header || 2-state payload (backward bit stack + marker bit).
//
// Encode (one 64-lane workgroup = BPW blocks x T lanes):
//   1. per block, one wave: histogram -> normalise -> header -> tables (LDS)
//   2. per block, T lanes, each owning S contiguous pairs:
//        count : bit count from a guessed start state, recording the
//                trajectory (state pairs at a few checkpoints)
//        repair: a lane whose start was wrong re-encodes from the right
//                one until it meets its recorded trajectory (exact)
//        scan  : per-lane bit offsets (the stack writes high pairs first)
//        emit  : bits written straight to the output slot; the two partial
//                words at each lane boundary are OR-merged through LDS
//      The encoder also records decode checkpoints (the sidecar index).
// Also the utility kernels: histogram per block, pack/unpack/copy of
// compressed blocks, the synthetic generator.  Decode: fse_decode.hip.

#include "fse_device.hpp"
#include "fse_kernels.h"

namespace fsehip {

// Tables of this file's kernels whose atomic ranks failed their check and
// were rebuilt with the peer-mask ranks (wave_build_spread); per device.
__device__ uint32_t g_rank_fb_enc;
hipError_t rank_fallbacks_enc(uint32_t* out, bool reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rank_fb_enc), 4, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess && reset) {
        const uint32_t z = 0;
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_rank_fb_enc), &z, 4, 0, hipMemcpyHostToDevice);
    }
    return e;
}

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

// Encoder tables in LDS: stateTable (u16 entries, fse.rs:157-162) and the
// symbol transforms {deltaNbBits, LDS byte address of
// stateTable[deltaFindState]} (fse.rs:165-188): the block's table base is
// folded into the transform, so one state step is add, shift, shift-add,
// ds_read_u16 whichever table of the workgroup the lane uses.
constexpr int ENC_PF = 4;  // source chunk registers of a pass (PF - 1 loads in flight; 6 and 8 measured the same)
struct EncTab {
    const uint2* tt;  // {deltaNbBits, LDS address of stateTable + 2 * deltaFindState}
};
typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
__device__ __forceinline__ uint32_t st_at(uint32_t lds_addr) {
    return *(lds_cu16*)(uintptr_t)lds_addr;
}
// LDS byte address of a __shared__ object
template <class P>
__device__ __forceinline__ uint32_t lds_addr_of(P* p) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) P*)p;
}

// Bit writer of one lane's range: BitStackWriter order (writer.rs:140-222),
// LSB-first words through a 24-word LDS ring.  Every 16-word (64-byte)
// group of the slot that lies wholly inside the lane's range leaves as four
// dwordx4 stores once the lane has moved past it: whole aligned 64-byte
// pieces.  (32-byte groups, the round-4 layout, left 64-byte pieces half
// written at a time; as whole pieces the same bytes cost 0.05 ms less per
// GiB, profiles/r05/enc_store/.)  The partial groups at either end of the
// lane leave as dword stores.  The lane's first word, when it shares it with
// the lane above (off % 32 != 0), is never stored: its value (head_val)
// goes to the merge list, like the lane's last partial word, and the merge
// step rewrites each boundary word with the OR of both lanes' bits.  Stores
// stay below wlim (the slot's words).
//
// The ring: a group is stored at the first drain after it completes, and
// drain runs every <= 8 pairs (<= 8 new words even at L = 15), so the ring
// holds the pending group's 16 words plus <= 8 more: 24 slots, word w at
// slot w mod 24 (a group's four 4-word pieces are 4-aligned slots, since
// 16 g mod 24 is a multiple of 8).
constexpr uint32_t RING_WORDS = 24;  // emit ring words per lane
struct Emit {
    uint32_t lo, hi;    // pending bits: lo = the word being filled, hi = bits past it
    uint32_t nacc;
    uint32_t word;      // index of the word being filled
    uint32_t rix;       // its ring slot, word mod RING_WORDS
    uint32_t w0;        // first word index of the lane
    uint32_t head_val;  // lane's bits of word w0 (valid once word > w0 and the head group left)
    uint32_t wlim;      // words in the slot: stores never leave it
    uint32_t gs;        // next 16-word group to store
    bool skip_head;
    uint32_t* gw;
    uint32_t* ring;     // LDS, RING_WORDS words, 16-byte aligned
    __device__ __forceinline__ void start(uint32_t* g, uint32_t off, uint32_t lim = 0xFFFFFFFFu,
                                          uint32_t* r = nullptr) {
        gw = g;
        wlim = lim;
        ring = r;
        lo = hi = 0;
        nacc = off & 31u;
        word = off >> 5;
        rix = word % RING_WORDS;
        w0 = word;
        gs = word >> 4;
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
    // flush before nacc can reach 64 (<= 2 x 15 bits per flush).
    __device__ __forceinline__ void flush() {
        const bool f = nacc >= 32u;
        ring[rix] = lo;
        lo = f ? hi : lo;
        hi = 0;  // nacc < 32 after the flush
        nacc &= 31u;
        word += f ? 1u : 0u;
        rix += f ? 1u : 0u;
        if constexpr ((RING_WORDS & (RING_WORDS - 1u)) == 0u) rix &= RING_WORDS - 1u;
        else rix = rix == RING_WORDS ? 0u : rix;
    }
    __device__ __forceinline__ uint32_t pos() const { return word * 32u + nacc; }
    // Words [a, b) of the lane's range, within one group: dwords up to the
    // next 4-word boundary, whole 4-word pieces as dwordx4, dwords after
    // (pieces never straddle the ring's end: its slots are 4-aligned)
    __device__ __forceinline__ void store_words(uint32_t a, uint32_t b) {
        b = min(b, wlim);
        uint32_t i = a;
        for (; i < b && (i & 3u); ++i) gw[i] = ring[i % RING_WORDS];
        for (; i + 4u <= b; i += 4u)
            *reinterpret_cast<uint4*>(gw + i) = *reinterpret_cast<const uint4*>(ring + i % RING_WORDS);
        for (; i < b; ++i) gw[i] = ring[i % RING_WORDS];
    }
    __device__ __forceinline__ void store_group(uint32_t g) {
        const uint32_t base = g << 4;
        if (g == (w0 >> 4) && ((w0 & 15u) != 0u || skip_head)) {  // the lane's first group: its own words only
            if (skip_head) head_val = ring[w0 % RING_WORDS];
            store_words(skip_head ? w0 + 1u : w0, base + 16u);
        } else if (base + 16u <= wlim) {
            const uint32_t r0 = base % RING_WORDS;
            uint4* o = reinterpret_cast<uint4*>(gw + base);
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                uint32_t rq = r0 + 4u * q;
                rq = rq >= RING_WORDS ? rq - RING_WORDS : rq;
                const uint4 a = *reinterpret_cast<const uint4*>(ring + rq);
                o[q] = a;
            }
        }
    }
    // Store the group the lane has moved past, if any (called every <= 8
    // pairs: <= 8 new words, fewer than a group, so the ring never overruns
    // a pending group and at most one group completes between calls).
    __device__ __forceinline__ void drain() {
        if (word >= (gs + 1u) << 4) {
            store_group(gs);
            ++gs;
        }
    }
    // End of the lane: remaining whole groups, then the whole words of the
    // last group (the partial word stays in acc for the merge list).
    __device__ __forceinline__ void finish() {
        while (word >= (gs + 1u) << 4) {
            store_group(gs);
            ++gs;
        }
        uint32_t lo = gs << 4;
        if (gs == (w0 >> 4)) {
            lo = w0;
            if (skip_head) {
                lo = w0 + 1u;
                if (word > w0) head_val = ring[w0 % RING_WORDS];
            }
        }
        store_words(lo, word);
    }
};

// Words per lane of the emit ring in LDS (16-byte aligned rows).
constexpr uint32_t RING_STRIDE = RING_WORDS;

// A lane's checkpoints (its range holds at most S / interval of them) are
// kept in registers and written together after its emit pass: recorded one
// by one, 8-byte stores from 64 lanes at a 32-byte stride hit every 128-byte
// line of the sidecar at four different times, and the lines left L2 part
// written (sidecar WRITE_SIZE 3.8x its bytes at C2).
constexpr uint32_t CKQ = 8;
struct Ckpt {
    uint64_t* base;  // this block's sidecar entries, or nullptr
    uint32_t mask;   // interval - 1 (interval is a power of two, >= 8)
    uint32_t shift;  // log2(interval)
    uint32_t hdr_bits;
    uint32_t L;
    bool queue;       // buffer this lane's entries (<= CKQ of them)
    uint32_t cnt;     // entries buffered
    uint32_t lo;      // index of q[0]
    uint64_t q[CKQ];  // q[0] = the latest entry (lowest index)
};

enum { PASS_COUNT = 1, PASS_EMIT = 2, PASS_REPAIR = 3 };
template <int MODE>
constexpr bool emits() { return MODE == PASS_EMIT; }
template <int MODE>
constexpr bool counts() { return MODE == PASS_COUNT || MODE == PASS_REPAIR; }

// Trajectory of a count pass, for convergence-based repair: the state pair
// and running bit count after every ckc-th chunk (at most TRACK_SLOTS slots per lane,
// slot 0 = the lane's end).  A repair re-encodes from the corrected start
// state only until it meets the recorded trajectory: from there on states
// and bits are identical, so the lane's total follows from the record and
// its end state (its neighbour's start) is unchanged.
// Slots hold x0 | x1 << 16 (cx) and, per chain, the bits still to come
// after the slot (cb: .x chain 0, .y chain 1): a pass writes its running
// counts there, and track_fixup turns the slots it wrote into remaining
// counts once the pass totals are known, so every slot stays consistent
// with the lane's current trajectory.
// Trajectory slots per lane.  16 (repairs stop sooner) measured slower
// than 8 on C2: the count pass writes twice as many slots.
constexpr uint32_t TRACK_SLOTS = 8;
// L >= 14: 7, so that the L = 14 kernel's LDS fits 4 workgroups per CU
template <int LMAX>
constexpr uint32_t track_slots() { return LMAX >= 14 ? TRACK_SLOTS - 1u : TRACK_SLOTS; }
struct Track {
    uint32_t* cx;     // this lane's slots: state pairs (LDS)
    uint2* cb;        // this lane's slots: per-chain bit counts (LDS)
    uint32_t ckc;     // chunks per slot
    bool done;        // REPAIR: met the recorded trajectory
    uint32_t jstar;   // REPAIR: the slot where it did (slots above it were rewritten)
};

// After a pass with totals t0 / t1: slots above `jlo` (exclusive) hold
// running counts; make them remaining counts.
__device__ __forceinline__ void track_fixup(Track& tr, uint32_t nslot, int32_t jlo, uint32_t t0, uint32_t t1) {
    for (int32_t j = (int32_t)nslot - 1; j > jlo; --j) {
        const uint2 r = tr.cb[j];
        tr.cb[j] = make_uint2(t0 - r.x, t1 - r.y);
    }
}

struct EncState {
    uint32_t x0, x1, b0, b1;  // states; bits of chain 0 / chain 1 (NS = 1: b0 only)
};

// One state step on the dependent chain x -> stateTable[(x >> nb) + dFS],
// nb = (deltaNbBits + x) >> 16: updates x and returns the sum deltaNbBits + x,
// whose upper word is nb.  Callers take nb = sum >> 16, or (counting passes)
// add the sums as packed 16-bit halves, so that nb's only use on the chain
// is the shift and the compiler takes it as the sum's upper word there (SDWA
// src0_sel:WORD_1): add, shift, shift-add, ds_read_u16.
__device__ __forceinline__ uint32_t state_step(uint32_t& x, const uint2 t) {
    const uint32_t sum = t.x + x;
    x = st_at(((x >> (sum >> 16)) << 1) + t.y);
    return sum;
}
// Packed 16-bit add (v_pk_add_u16): the upper halves add without a carry in
// from the lower ones, so adding step sums accumulates their nb.
typedef uint16_t u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2_t, a) + __builtin_bit_cast(u16x2_t, b));
}

// Encoder::encode_raw (fse.rs:227-239): returns nb, updates x.
__device__ __forceinline__ uint32_t enc_step(uint32_t& x, uint32_t s, const EncTab& T) {
    return state_step(x, T.tt[s]) >> 16;
}

// One 16-byte chunk.  NS = 2 (fse_compress2): pairs c8+7 .. c8 (lib.rs:167-176:
// E1 then E0 per pair).  NS = 1 (fse_compress): symbols c8+15 .. c8 with one
// state (lib.rs:127-138).  FULL chunks need no guard; only the topmost chunk
// of the topmost lane can extend past the last main-loop step pb.
template <int MODE, bool FULL, int NS>
__device__ __forceinline__ void enc_chunk(const uint4& q, uint32_t c8, uint32_t pb, uint32_t& x0, uint32_t& x1,
                                          const EncTab& T, uint32_t& b0, uint32_t& b1, Emit& em) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    // counting passes: each chain's nb summed as packed upper halves of its
    // step sums (<= 16 x 16 per chunk), folded in once per chunk
    constexpr bool PKB = counts<MODE>();
    uint32_t bacc0 = 0, bacc1 = 0;
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
            const uint32_t s0 = state_step(x0, t);
            const uint32_t nb0 = s0 >> 16;
            if (PKB) bacc0 = pk_add16(bacc0, s0);
            if (emits<MODE>()) {
                em.put(__builtin_amdgcn_ubfe(v0, 0u, nb0), nb0);
                if (j & 1) em.flush();  // <= 2 x 12 bits between flushes
            }
        }
        if (emits<MODE>()) em.flush();
        if (PKB) b0 += bacc0 >> 16;
        return;
    }
#pragma unroll
    for (int j = 7; j >= 0; --j) {
        if (!FULL && c8 + (uint32_t)j >= pb) continue;
        const uint32_t v1 = x1, v0 = x0;
        const uint32_t s1 = state_step(x1, t1[j]);
        const uint32_t s0 = state_step(x0, t0[j]);
        const uint32_t nb1 = s1 >> 16, nb0 = s0 >> 16;
        if (PKB) {
            bacc1 = pk_add16(bacc1, s1);
            bacc0 = pk_add16(bacc0, s0);
        }
        if (emits<MODE>()) {
            const uint32_t pairbits = (__builtin_amdgcn_ubfe(v0, 0u, nb0) << nb1) | __builtin_amdgcn_ubfe(v1, 0u, nb1);
            em.put(pairbits, nb1 + nb0);
            em.flush();
        }
    }
    if (PKB) {
        b0 += bacc0 >> 16;
        b1 += bacc1 >> 16;
    }
}

// The same chunk with its symbol transforms already in t0 / t1 (loaded one
// chunk ahead): each pair's two transforms are reloaded from the next
// chunk's words qn as soon as the pair has used them, so the next chunk
// starts with its transforms landed instead of waiting for 16 LDS reads
// (the state loop is latency-bound: that wait was one exposed LDS round
// trip per 8 pairs).  Same registers, same instruction count.
__device__ __forceinline__ void tt_load(const uint4& q, uint2 (&t0)[8], uint2 (&t1)[8], const EncTab& T) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t sh = 16u * (uint32_t)(j & 1);
        t0[j] = T.tt[(w[j >> 1] >> sh) & 0xFFu];
        t1[j] = T.tt[(w[j >> 1] >> (sh + 8u)) & 0xFFu];
    }
}
template <int MODE, int NS>
__device__ __forceinline__ void enc_chunk_pl(const uint4& qn, uint2 (&t0)[8], uint2 (&t1)[8], uint32_t& x0,
                                             uint32_t& x1, const EncTab& T, uint32_t& b0, uint32_t& b1, Emit& em) {
    const uint32_t wn[4] = {qn.x, qn.y, qn.z, qn.w};
    constexpr bool PKB = counts<MODE>();
    uint32_t bacc0 = 0, bacc1 = 0;
    auto reload = [&](int j) {
        const uint32_t sh = 16u * (uint32_t)(j & 1);
        t0[j] = T.tt[(wn[j >> 1] >> sh) & 0xFFu];
        t1[j] = T.tt[(wn[j >> 1] >> (sh + 8u)) & 0xFFu];
    };
    if (NS == 1) {
#pragma unroll
        for (int j = 15; j >= 0; --j) {
            const uint2 t = (j & 1) ? t1[j >> 1] : t0[j >> 1];
            const uint32_t v0 = x0;
            const uint32_t s0 = state_step(x0, t);
            const uint32_t nb0 = s0 >> 16;
            if (PKB) bacc0 = pk_add16(bacc0, s0);
            if (emits<MODE>()) {
                em.put(__builtin_amdgcn_ubfe(v0, 0u, nb0), nb0);
                if (j & 1) em.flush();  // <= 2 x 12 bits between flushes
            }
            if ((j & 1) == 0) reload(j >> 1);
        }
        if (emits<MODE>()) em.flush();
        if (PKB) b0 += bacc0 >> 16;
        return;
    }
#pragma unroll
    for (int j = 7; j >= 0; --j) {
        const uint32_t v1 = x1, v0 = x0;
        const uint32_t s1 = state_step(x1, t1[j]);
        const uint32_t s0 = state_step(x0, t0[j]);
        reload(j);
        const uint32_t nb1 = s1 >> 16, nb0 = s0 >> 16;
        if (PKB) {
            bacc1 = pk_add16(bacc1, s1);
            bacc0 = pk_add16(bacc0, s0);
        }
        if (emits<MODE>()) {
            const uint32_t pairbits = (__builtin_amdgcn_ubfe(v0, 0u, nb0) << nb1) | __builtin_amdgcn_ubfe(v1, 0u, nb1);
            em.put(pairbits, nb1 + nb0);
            em.flush();
        }
    }
    if (PKB) {
        b0 += bacc0 >> 16;
        b1 += bacc1 >> 16;
    }
}

// Sidecar entry for the decoder state before pair p (= encoder state after
// encoding pair p): bit position (payload-relative) and both states.
// (NS = 1: one state, s1 = 0.)
template <int NS>
__device__ __forceinline__ uint64_t ckpt_entry(const Ckpt& ck, uint32_t pos, uint32_t x0, uint32_t x1) {
    return (uint64_t)(pos - ck.hdr_bits) | ((uint64_t)(x0 - (1u << ck.L)) << 32) |
           (NS == 2 ? ((uint64_t)(x1 - (1u << ck.L)) << 48) : 0ull);
}
template <int NS>
__device__ __forceinline__ void ckpt_record(Ckpt& ck, uint32_t p, uint32_t pos, uint32_t x0, uint32_t x1) {
    const uint64_t e = ckpt_entry<NS>(ck, pos, x0, x1);
    if (ck.queue) {  // block-uniform
#pragma unroll
        for (int i = (int)CKQ - 1; i > 0; --i) ck.q[i] = ck.q[i - 1];
        ck.q[0] = e;
        ck.lo = p >> ck.shift;
        ++ck.cnt;
    } else {
        ck.base[p >> ck.shift] = e;
    }
}
// The buffered entries, lowest index first: lane after lane, contiguous.
__device__ __forceinline__ void ckpt_flush(const Ckpt& ck) {
    if (!ck.queue) return;
#pragma unroll
    for (uint32_t i = 0; i < CKQ; ++i)
        if (i < ck.cnt) ck.base[ck.lo + i] = ck.q[i];
}

// Encode pairs pb-1 down to pa.  Source chunks (16 B = 8 pairs) stream
// through four fixed registers, each reloaded right after it is consumed,
// so three loads stay in flight and no register copy forces an early
// s_waitcnt.  Loads are unconditional (the index is clamped to the
// segment); the partial topmost chunk is peeled and loaded byte-wise.
template <int MODE, int NS>
__device__ __forceinline__ EncState enc_range(const uint8_t* __restrict__ blk, uint32_t n, uint32_t pa, uint32_t pb,
                                              EncState st, const EncTab& T, Emit& em, Ckpt& ck, Track& tr) {
    constexpr bool TRACK = counts<MODE>();
    constexpr bool RP = MODE == PASS_REPAIR;
    uint32_t x0 = st.x0, x1 = st.x1, b0 = st.b0, b1 = st.b1;
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
            if (RP) {
                if (tr.cx[slot] == sv) {
                    const uint2 r = tr.cb[slot];
                    tr.done = true;
                    tr.jstar = slot;
                    b0 += r.x;  // the rest of the trajectory is the recorded one
                    b1 += r.y;
                } else {
                    tr.cx[slot] = sv;
                    tr.cb[slot] = make_uint2(b0, b1);
                }
            } else {
                tr.cx[slot] = sv;
                tr.cb[slot] = make_uint2(b0, b1);
            }
            slot -= 1u;
            rem = tr.ckc - 1u;
        } else {
            rem -= 1u;
        }
    };
    if (pb & ((1u << CS) - 1u)) {  // partial topmost chunk
        const uint4 q = load_chunk(blk, n, (uint32_t)c_hi);
        enc_chunk<MODE, false, NS>(q, (uint32_t)c_hi << CS, pb, x0, x1, T, b0, b1, em);
        if (emits<MODE>()) em.drain();
        if (MODE == PASS_EMIT && ck.base && (((uint32_t)c_hi << CS) & ck.mask) == 0u)
            ckpt_record<NS>(ck, (uint32_t)c_hi << CS, em.pos(), x0, x1);
        if (TRACK) track();
        c_hi -= 1;
    }
    if (c_hi < c_lo || (RP && tr.done)) return EncState{x0, x1, b0, b1};
    auto ld = [&](int32_t c) { return v[c < c_lo ? c_lo : c]; };
    // source chunks in flight: PF - 1 ahead of the one being encoded
    constexpr int PF = ENC_PF;
    uint4 q[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) q[k] = ld(c_hi - k);
    uint2 t0[8], t1[8];  // the transforms of the chunk being encoded (tt_load / enc_chunk_pl)
    tt_load(q[0], t0, t1, T);
    // qn: the next chunk's words (already loaded: PF - 1 chunks ahead)
    auto body = [&](const uint4& q, const uint4& qn, int32_t c) {
        (void)q;
        enc_chunk_pl<MODE, NS>(qn, t0, t1, x0, x1, T, b0, b1, em);
        if (emits<MODE>()) em.drain();
        if (MODE == PASS_EMIT && ck.base && (((uint32_t)c << CS) & ck.mask) == 0u)
            ckpt_record<NS>(ck, (uint32_t)c << CS, em.pos(), x0, x1);
        if (TRACK) track();
    };
    auto stop = [&](int32_t cn) { return cn < c_lo || (RP && tr.done); };
    for (int32_t c = c_hi;; c -= PF) {
        bool done = false;
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            body(q[k], q[(k + 1) % PF], c - k);
            if (stop(c - k - 1)) {
                done = true;
                break;
            }
            q[k] = ld(c - k - PF);
        }
        if (done) break;
    }
    return EncState{x0, x1, b0, b1};
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
    e.b0 = e.b1 = 0;
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
        if (MODE == PASS_COUNT) e.b0 = nb;
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
// A block's phase-1 results read by phase 2, and phase 1's small scratch.
template <int BPW>
struct EncTail {
    int32_t status[BPW];
    uint32_t L[BPW];
    uint32_t hl[BPW];
    uint32_t hv[BPW];  // the header's last partial word (merged with the payload's first bits)
    int scratch[4];
};

template <int LMAX, int T>
struct EncSmem {
    static constexpr int BPW = 64 / T;
    static constexpr uint32_t SIZE = 1u << LMAX;
    // L >= 14 (one block per wave): the tail lives in phase 2's trajectory
    // struct, beside its 7 slots and under the ring: 32 bytes that take the
    // L = 14 kernel to 40,960 B and 4 workgroups per CU.  Phase 2 reads it
    // into registers before the emit ring overwrites it.
    static constexpr bool TAIL_IN_P2 = LMAX >= 14;
    static_assert(!TAIL_IN_P2 || BPW == 1, "one block per wave");
    // A block's stateTable and symbol transforms are built last in phase 1,
    // so until then they hold its scratch: the sub-histograms (16 copies,
    // 8 KiB, over st and tt when one block has the wave; 8 copies, 4 KiB,
    // in st[b] when two blocks share it), the spread's occurrence owners
    // (2^L bytes) in st[b], the rank loop's peer masks (512 B) in tt[b]
    static constexpr uint32_t HS = BPW == 1 ? HSUB : 8u;
    static_assert(BPW == 1 || 2u * SIZE >= hist_words<8>() * 4u, "sub-histograms fit the stateTable");
    union {
        struct {
            __attribute__((aligned(16))) uint16_t st[BPW][SIZE];
            uint2 tt[BPW][256];
        };
        __attribute__((aligned(16))) uint32_t hist[BPW == 1 ? hist_words<HS>() : 4];
    };
    // phase-1 scratch (statistics, header, spread) and phase-2 scratch
    // (trajectories, end states, merge list) share the same LDS
    union {
        struct {
            union {
                uint32_t hdrw[HDR_MAX / 4];  // NCount header, stored to the slot before the spread
                // (L >= 13: the spread's symbols are in global memory, EncParams::spread)
                __attribute__((aligned(16))) uint8_t sym_at[enc_gsym(LMAX) ? 16u : SIZE];
            } u;
            int32_t norm[256];
            uint16_t cumul[256];
            uint32_t cnt[256];
        } p1;
        // phase 2, three lifetimes over the same bytes: the count / repair
        // rounds (trajectories, end states), the emit pass (its ring), and
        // the boundary-word merge after it
        union {
            struct {
                uint2 cb[64 * track_slots<LMAX>()];     // trajectories (Track): per-chain bit counts
                uint32_t cx[64 * track_slots<LMAX>()];  // and state pairs
                uint32_t cntF[BPW][T + 1];      // each lane's end state
                EncTail<BPW> tail[TAIL_IN_P2 ? 1 : 0];
            } u;
            __attribute__((aligned(16))) uint32_t ring[64 * RING_STRIDE];  // emit: output ring per lane (Emit)
            struct {
                uint32_t mword[BPW][2 * (T + 1)];
                uint32_t mval[BPW][2 * (T + 1)];
            } mg;
        } p2;
    } ph;
    EncTail<BPW> tail_out[TAIL_IN_P2 ? 0 : 1];
    __device__ __forceinline__ EncTail<BPW>& tail() {
        if constexpr (TAIL_IN_P2) return ph.p2.u.tail[0];
        else return tail_out[0];
    }
};

template <int LMAX, int T, int NS>
__global__ __launch_bounds__(64) void encode_blocks_kernel(EncParams P) {
    constexpr int BPW = 64 / T;
    __shared__ EncSmem<LMAX, T> sm;
    // the tail in phase 2's trajectory struct must sit above every phase-1 byte
    static_assert(!EncSmem<LMAX, T>::TAIL_IN_P2 ||
                      64u * track_slots<LMAX>() * 12u + 4u * (T + 1u) >= sizeof(sm.ph.p1),
                  "tail overlaps phase-1 scratch");
#define ENC_WGID ((uint64_t)blockIdx.x)
#define ENC_SYNC() __syncthreads()
    const uint32_t lane = lane_id();

    FSE_STAMP(P, 0);
    // ---- phase 1: statistics, header and tables, one block at a time
    for (int b = 0; b < BPW; ++b) {
        const uint64_t gb = ENC_WGID * BPW + b;
        if (gb >= P.n_blocks) {
            if (lane == 0) sm.tail().status[b] = 1;  // no block
            continue;
        }
        const uint64_t off = gb * P.block_size;
        const uint32_t n = (uint32_t)min((uint64_t)P.block_size, P.n_total - off);
        const uint8_t* blk = P.src + off;
        uint32_t* counts = sm.ph.p1.cnt;  // the spread reuses cnt[] after normalize
        using Sm = EncSmem<LMAX, T>;
        const uint32_t tl = wave_histogram<Sm::HS>(
            blk, n, BPW == 1 ? sm.hist : reinterpret_cast<uint32_t*>(sm.st[b]), counts);
        FSE_STAMP(P, 1);
        if (FSE_ABLATE(P, 8u)) {  // ablation: histogram only
            if (lane == 0) P.status[gb] = (int32_t)tl;
            continue;
        }
        int rc = FSE_OK;
        uint32_t Lreq = P.table_log, L = 0, slow = 0;
        if (n == 0) rc = FSE_ERR_EMPTY;
        if (rc == FSE_OK && P.table_log == 0) rc = optimal_log2(n, tl, &Lreq);  // histogram.rs:301
        if (rc == FSE_OK) rc = wave_normalize(counts, n, tl, Lreq, sm.ph.p1.norm, &L, &slow, sm.tail().scratch);
        if (rc == FSE_OK && n < 2) rc = FSE_ERR_TOO_SHORT;  // lib.rs:154/156 unwrap
        if (rc == FSE_OK && L > (uint32_t)LMAX) rc = FSE_ERR_UNSUPPORTED;
        FSE_STAMP(P, 2);
        if (rc == FSE_OK) {
            const int hl = wave_header_write(sm.ph.p1.norm, L, tl, sm.ph.p1.u.hdrw);
            if (lane == 0) sm.tail().scratch[1] = hl;
            if (hl < 0) {
                rc = hl;
            } else {
                // whole header words go to the slot now (no payload store
                // touches them); the last partial word is merged at the end
                const uint32_t* h = sm.ph.p1.u.hdrw;
                uint32_t* gw = reinterpret_cast<uint32_t*>(P.out + gb * P.slot_bytes);
                for (uint32_t w = lane; w < (uint32_t)hl / 4u; w += WAVE) gw[w] = h[w];
                if (lane == 0) sm.tail().hv[b] = (hl & 3) ? h[hl / 4] & ((1u << (8u * (hl & 3))) - 1u) : 0u;
            }
            wave_sync();  // the spread reuses the header's LDS
        }
        FSE_STAMP(P, 3);
        if (rc == FSE_OK) {
            const uint32_t size = 1u << L;
            uint16_t* st = sm.st[b];
            const uint16_t* cumul = sm.ph.p1.cumul;
            constexpr bool GSYM = enc_gsym(LMAX);
            uint8_t* const sym_at = !GSYM ? sm.ph.p1.u.sym_at
                                    : P.spread ? P.spread + gb * (uint64_t)(1u << LMAX)
                                               : P.out + gb * P.slot_bytes + ENC_SPREAD_OFF;
            static_assert(ENC_SPREAD_OFF >= HDR_MAX && ENC_SPREAD_OFF % 16u == 0u, "in-slot spread array");
            rc = wave_build_spread<64, false, GSYM>(sm.ph.p1.norm, L, tl, sym_at, reinterpret_cast<uint8_t*>(st), sm.ph.p1.cumul,
                                   sm.ph.p1.cnt,
                                   [&](uint32_t i, uint32_t, uint32_t r) {
                                       st[r] = (uint16_t)(size + i);  // fse.rs:157-162 (r = cumul[s] + rank)
                                   },
                                   [&](uint32_t s) { return (uint32_t)cumul[s]; },
                                   RankAtomic{P.peer_ranks == 0u, nullptr, st, size, &g_rank_fb_enc, P.rank_inject}, nullptr,
                                   reinterpret_cast<uint64_t*>(&sm.tt[b][0]));
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
            // Encoder::new_first_symbol (fse.rs:210-218) forms its table
            // index with wrapping u32/i32 arithmetic and a bounds-checked
            // read: at L = 15 the index of a seed of norm >= 2 usually falls
            // outside the table and the reference panics.  (Inside it, the
            // enc_init state is the reference's, even when it is another
            // symbol's.)
            wave_sync();
            if (lane == 0) {
                auto init_ok = [&](uint32_t s) {
                    const uint2 t = sm.tt[b][s];
                    const uint32_t bo = (t.x + (1u << 15)) >> 16;
                    const uint32_t v = (bo << 16) - t.x;
                    const int32_t idx = (int32_t)((v >> bo) + (uint32_t)((int32_t)(t.y - stb) >> 1));
                    return idx >= 0 && idx < (int32_t)size;
                };
                const bool ok = init_ok(blk[n - 1u]) && (NS == 1 || init_ok(blk[n - 2u]));
                sm.tail().scratch[2] = ok ? FSE_OK : FSE_ERR_ENCODER_INIT;
            }
            wave_sync();
            if (rc == FSE_OK) rc = sm.tail().scratch[2];
        }
        if (lane == 0) {
            const uint32_t hl = (rc == FSE_OK) ? (uint32_t)sm.tail().scratch[1] : 0u;
            sm.tail().status[b] = rc;
            sm.tail().L[b] = L;
            sm.tail().hl[b] = hl;
            if (rc != FSE_OK) {
                P.status[gb] = rc;
                P.comp_len[gb] = 0;
                if (P.payload_bits) P.payload_bits[gb] = 0;
            }
        }
        ENC_SYNC();
    }

    FSE_STAMP(P, 4);
    if (FSE_ABLATE(P, 9u)) return;  // ablation: statistics + tables only (1), histogram only (8)
    // ---- phase 2: T lanes per block
    const int b = BPW == 1 ? 0 : (int)(lane / T);
    const uint32_t k = BPW == 1 ? lane : lane % T;
    const uint64_t gb = ENC_WGID * BPW + b;
    const bool live = sm.tail().status[b] == FSE_OK;
    // (TAIL_IN_P2: read now, the emit ring overwrites the tail)
    using Sm2 = EncSmem<LMAX, T>;
    const uint32_t hl_early = Sm2::TAIL_IN_P2 ? sm.tail().hl[b] : 0u;
    const uint32_t hv_early = Sm2::TAIL_IN_P2 ? sm.tail().hv[b] : 0u;
    const uint64_t boff = gb * P.block_size;
    const uint32_t n = live ? (uint32_t)min((uint64_t)P.block_size, P.n_total - boff) : 0u;
    const uint8_t* blk = P.src + boff;
    const uint32_t L = sm.tail().L[b];
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
    Ckpt ck{nullptr, 0, 0, 0, L, false, 0, 0, {}};

    // Exact start state of every lane (the lane above's end state) and
    // exact bit offset of every lane: count pass from guessed starts with
    // trajectories, then convergence repair (re-encode from the corrected
    // start until the recorded trajectory is met) until the fixed point, then
    // the emit pass writes straight to the final offsets.  A repair round
    // costs the slowest lane's convergence distance.
    constexpr uint32_t TS = track_slots<LMAX>();
    Track tr{&sm.ph.p2.u.cx[lane * TS], &sm.ph.p2.u.cb[lane * TS], max(1u, (S / SPC + TS - 1u) / TS), false, 0u};
    const uint32_t nslot = pb > pa ? (((pb - 1u) / SPC) - (pa / SPC)) / tr.ckc + 1u : 0u;
    uint32_t start = (1u << L) | (NS == 2 ? (1u << L) << 16 : 0u);
    uint32_t bits = 0;
    uint32_t tot0 = 0, tot1 = 0;  // the lane's bits per chain
    uint32_t myF = 0;             // the lane's end state (cntF)
    uint32_t n_iter = 0, n_rerun = 0;  // diagnostics (stamps counters)
    {
        // count pass: the top lane from its exact start (init states + the
        // odd-length extra step), every other lane from a guessed start state,
        // recording its trajectory.  Then verify against the neighbour's end
        // state and repair by convergence (Track) until the fixed point.
        constexpr int MC = PASS_COUNT, MR = PASS_REPAIR;
        if (act) {
            EncState e0 = (k == ktop) ? top_start<PASS_COUNT, NS>(blk, n, tab, em)
                                      : EncState{start & 0xFFFFu, start >> 16, 0u, 0u};
            e0 = enc_range<MC, NS>(blk, n, pa, pb, e0, tab, em, ck, tr);
            tot0 = e0.b0;
            tot1 = e0.b1;
            myF = e0.x0 | (e0.x1 << 16);
            sm.ph.p2.u.cntF[b][k] = myF;
            track_fixup(tr, nslot, -1, tot0, tot1);
        }
        FSE_STAMP(P, 5);
        for (;;) {
            if (FSE_ABLATE(P, 16u)) break;  // ablation: no repair (wrong output)
            ENC_SYNC();
            bool bad0 = false, bad1 = false;
            uint32_t nbF = 0;
            if (act && k < ktop) {
                nbF = sm.ph.p2.u.cntF[b][k + 1];
                bad0 = ((nbF ^ start) & 0xFFFFu) != 0u;
                bad1 = ((nbF ^ start) >> 16) != 0u;
            }
            const bool bad = bad0 || bad1;
            ENC_SYNC();
            if (__ballot(bad) == 0) break;
            ++n_iter;
            n_rerun += (uint32_t)__popcll(__ballot(bad));
            if (bad) {
                start = nbF;
                tr.done = false;
                const EncState e0 = enc_range<MR, NS>(blk, n, pa, pb,
                                                      EncState{start & 0xFFFFu, start >> 16, 0u, 0u}, tab, em, ck, tr);
                tot0 = e0.b0;
                tot1 = e0.b1;
                if (!tr.done) {  // did not converge: new end state
                    myF = e0.x0 | (e0.x1 << 16);
                    sm.ph.p2.u.cntF[b][k] = myF;
                }
                track_fixup(tr, nslot, tr.done ? (int32_t)tr.jstar : -1, tot0, tot1);
            }
        }
        bits = tot0 + tot1;
        if (k == 0) bits += (uint32_t)NS * L + 1u;  // finals + marker (lib.rs:178-181 / 139-141)
    }

    FSE_STAMP(P, 6);
    if (kDiag && P.stamps && lane == 0)
        P.stamps[(uint64_t)blockIdx.x * kStamps + kStamps - 1] = (uint64_t)n_iter | ((uint64_t)n_rerun << 32);
    // offsets: lane k writes after every lane j > k (stack order)
    const uint32_t hl = Sm2::TAIL_IN_P2 ? hl_early : sm.tail().hl[b];
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
    const bool fits = (uint64_t)total_bits <= P.slot_bytes * 8ull && !FSE_ABLATE(P, 2u);
    uint32_t* gw = reinterpret_cast<uint32_t*>(P.out + gb * P.slot_bytes);

    // emit pass (its ring overlays the trajectories and end states: every
    // lane is past the repair rounds here)
    ENC_SYNC();
    if (act && fits) {
        em.start(gw, off, FSE_ABLATE(P, 4u) ? 0u : (uint32_t)(P.slot_bytes >> 2),  // debug bit 2: no payload stores (ablation)
                 &sm.ph.p2.ring[lane * RING_STRIDE]);
        {
            if (P.sidecar && P.ckpt_interval) {
                ck.base = P.sidecar + gb * P.ckpt_per_block;
                ck.mask = P.ckpt_interval - 1u;
                ck.shift = 31u - __clz(P.ckpt_interval);
                ck.hdr_bits = hdr_bits;
                ck.queue = ((S + ck.mask) >> ck.shift) <= CKQ;  // entries in [pa, pa + S)
            }
            EncState e0;
            if (k == ktop) {
                e0 = top_start<PASS_EMIT, NS>(blk, n, tab, em);
                if (ck.base && (Pm & ck.mask) == 0u)  // checkpoint "before step Pm" (outside [pa, pb))
                    ck.base[Pm >> ck.shift] = ckpt_entry<NS>(ck, em.pos(), e0.x0, e0.x1);
            } else {
                e0 = EncState{start & 0xFFFFu, start >> 16, 0u};
            }
            e0 = enc_range<PASS_EMIT, NS>(blk, n, pa, pb, e0, tab, em, ck, tr);
            ckpt_flush(ck);
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
    }
    // boundary words -> merge list (entry order = stream order); the list
    // overlays the ring, so every lane's ring reads are done first
    ENC_SYNC();
    for (uint32_t e = k; e < 2u * (T + 1u); e += T) {
        if (b < BPW) sm.ph.p2.mg.mword[b][e] = 0xFFFFFFFFu;
    }
    ENC_SYNC();
    if (act && fits) {
        const uint32_t slot = 2u * (T - k);
        if ((off & 31u) != 0u && em.word > em.w0) {  // first word stored with the low bits empty
            sm.ph.p2.mg.mword[b][slot] = em.w0;
            sm.ph.p2.mg.mval[b][slot] = em.head_val;
        }
        if (em.nacc) {  // last word never stored
            sm.ph.p2.mg.mword[b][slot + 1] = em.word;
            sm.ph.p2.mg.mval[b][slot + 1] = em.lo;
        }
    }
    // header: whole words were stored in phase 1; the last partial word is merged
    if (live && fits && k == 0 && (hl & 3u)) {
        sm.ph.p2.mg.mword[b][0] = hl / 4u;
        sm.ph.p2.mg.mval[b][0] = Sm2::TAIL_IN_P2 ? hv_early : sm.tail().hv[b];
    }
    FSE_STAMP(P, 7);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stores above land before the merge rewrites
    ENC_SYNC();
    // merge: each run of equal word indices is OR-ed by its first entry
    if (live && fits) {
        constexpr uint32_t NE = 2u * (T + 1u);
        for (uint32_t e = k; e < NE; e += T) {
            const uint32_t w = sm.ph.p2.mg.mword[b][e];
            if (w == 0xFFFFFFFFu) continue;
            bool first = true;
            for (int q = (int)e - 1; q >= 0; --q) {
                const uint32_t wq = sm.ph.p2.mg.mword[b][q];
                if (wq == 0xFFFFFFFFu) continue;
                first = (wq != w);
                break;
            }
            if (!first) continue;
            uint32_t v = sm.ph.p2.mg.mval[b][e];
            for (uint32_t q = e + 1; q < NE; ++q) {
                const uint32_t wq = sm.ph.p2.mg.mword[b][q];
                if (wq == 0xFFFFFFFFu) continue;
                if (wq != w) break;
                v |= sm.ph.p2.mg.mval[b][q];
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

#undef ENC_SYNC
#undef ENC_WGID

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
constexpr uint32_t ENC_WGS = 11u;  // resident encode workgroups per CU at L <= 11 (LDS-padded)
hipError_t launch_encode(const EncParams& P0, uint32_t lmax, hipStream_t stream) {
    EncParams P = P0;
    P.peer_ranks = atomic_ranks_on() ? 0u : 1u;
    // 32 lanes per block (two blocks per wave) for L <= 12 when asked for;
    // L 13..15 tables (64 KiB stateTable) run one block per workgroup
    const uint32_t T = (P.lanes == 32 && lmax <= 12) ? 32u : 64u;
    const uint32_t bpw = 64u / T;
    const dim3 g((P.n_blocks + bpw - 1u) / bpw), b(64);
    auto go = [&](auto kern, uint32_t pad = 0) { hipLaunchKernelGGL(kern, g, b, P.xlds ? P.xlds : pad, stream, P); };
    if (P.nstates == 1) {  // fse_compress (lib.rs:112-143)
        if (lmax <= 11) go(encode_blocks_kernel<11, 64, 1>);
        else if (lmax <= 12) go(encode_blocks_kernel<12, 64, 1>);
        else if (lmax <= 13) go(encode_blocks_kernel<13, 64, 1>);
        else if (lmax <= 14) go(encode_blocks_kernel<14, 64, 1>);
        else go(encode_blocks_kernel<15, 64, 1>);
    } else if (T == 64) {
        // 11 workgroups per CU rather than the 12 its 12.6 KB allowed in
        // round 3: same time on C2, 5% less on near-uniform data
        // (tools/occ_enc.py, one process: 12 -> 2.00 ms, 11 -> 1.90, 10 ->
        // 1.88; C2 1.58 / 1.57 / 1.61), where the twelfth workgroup only adds
        // contention.  (At 14.6 KB, round 5, 11 is also the most that fit.)
        static const uint32_t pad11 = [] {
            hipFuncAttributes fa{};
            if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(encode_blocks_kernel<11, 64, 2>)) != hipSuccess)
                return 0u;
            const size_t per = (160u << 10) / ENC_WGS - 64u;  // LDS per workgroup for 11, less allocation slack
            return fa.sharedSizeBytes < per ? (uint32_t)(per - fa.sharedSizeBytes) : 0u;
        }();
        if (lmax <= 11) go(encode_blocks_kernel<11, 64, 2>, pad11);
        else if (lmax <= 12) go(encode_blocks_kernel<12, 64, 2>);
        else if (lmax <= 13) go(encode_blocks_kernel<13, 64, 2>);
        else if (lmax <= 14) go(encode_blocks_kernel<14, 64, 2>);
        else go(encode_blocks_kernel<15, 64, 2>);
    } else {
        if (lmax <= 11) go(encode_blocks_kernel<11, 32, 2>);
        else go(encode_blocks_kernel<12, 32, 2>);
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
    one("encode<15,64,2>", reinterpret_cast<const void*>(encode_blocks_kernel<15, 64, 2>), 64);
    return len;
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
