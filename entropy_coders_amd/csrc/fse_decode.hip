// fse_decode.hip -- decode side of the batched FSE (tANS) block codec, gfx950.
//
// Wire format: the reference's fse_compress2 / fse_compress blocks
// (lib.rs:112-183): NCount header || backward bit stack + marker bit.
//
//   dtable_blocks_kernel   NormHistogram::read + DecodeTable (histogram.rs:436-505,
//                          fse.rs:280-338), one wave per block, table to HBM
//   decode_pre_kernel      segment-parallel decode on prebuilt tables: one
//                          workgroup per block, the compressed block and its
//                          table staged in LDS, every lane decodes one
//                          sidecar segment (checkpoint to checkpoint)
//   serial2_decode_kernel  sidecar-less 2-state decode (container mode with
//                          the raw length, or the reference's own termination
//                          for host streams of unknown length), one lane per
//                          block with its table in LDS; can record the sidecar
//   decode1_serial_kernel  the same for 1-state blocks (fse_decompress)
//
// Table logs: kernels are instantiated at LMAX = 11, 12, 13, 14 and 15.  Up
// to L = 14 the segment decoder stages the block image beside the table (32
// and 64 KiB tables at 13 and 14: 2 and 1 workgroups per CU); at LMAX = 15
// the table (128 KiB) leaves no LDS for the image, so those blocks are read
// through a register window from global memory.
#include <type_traits>
#include <utility>

#include "fse_device.hpp"
#include "fse_kernels.h"


namespace fsehip {

// Tables of this file's kernels whose atomic ranks failed their check and
// were rebuilt with the peer-mask ranks (wave_build_spread); per device.
__device__ uint32_t g_rank_fb_dec;
hipError_t rank_fallbacks_dec(uint32_t* out, bool reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rank_fb_dec), 4, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess && reset) {
        const uint32_t z = 0;
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_rank_fb_dec), &z, 4, 0, hipMemcpyHostToDevice);
    }
    return e;
}

// cache policy of the segment decoder's LDS-DMA staging loads: nt (2), as the image and table
// are read once (C3 0.96 -> 0.91-0.96 ms, C2 decode 0.558 -> 0.552-0.554 ms, same box)
constexpr int STAGE_AUX = 2;

// ------------------------------------------------------------------------
// Decode table entry (fse.rs:260-265 DecodeTransform, repacked for the
// decode loop): nb | symbol << 8 | new_state << SH.  With SH = 18 (L <= 14)
// the high half is the LDS byte offset of the next state's base entry
// (4 * new_state), nb in bits 0-4 serves directly as a v_bfe width/offset
// operand, and the byte sum of two entries' low bytes is nb0 + nb1.  L = 15
// needs the 15-bit new_state at SH = 17 (global-window kernels only).
// ------------------------------------------------------------------------
template <int LMAX>
struct Dte {
    static constexpr uint32_t SH = LMAX > 14 ? 17u : 18u;
    __device__ static __forceinline__ uint32_t make(uint32_t nb, uint32_t sym, uint32_t ns) {
        return nb | (sym << 8) | (ns << SH);
    }
    __device__ static __forceinline__ uint32_t ns(uint32_t e) { return e >> SH; }
};
__device__ __forceinline__ uint32_t dte_nb(uint32_t e) { return e & 0xFFu; }
__device__ __forceinline__ uint32_t dte_sym(uint32_t e) { return (e >> 8) & 0xFFu; }

// Output group: pairs per lane between stores (32 pairs = 64 B, one HBM
// burst).  Segment starts are multiples of ckpt_interval, so groups are 64 B
// aligned whenever ckpt_interval >= 32.
constexpr uint32_t DEC_GROUP = 32;

// ------------------------------------------------------------------------
// Backward bit reader over global memory (BitStackReader semantics,
// stack_reader.rs:17-215): `pos` = bits remaining above the block start,
// buf holds stream bits [base, base+64); refills pull the next lower word.
// ------------------------------------------------------------------------
struct WindowReader {
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

// Sidecar cross-check: a segment that is not the block's last must end
// exactly where the next checkpoint says the decoder is (bit position and
// both states, a = 4 * state); a mismatch means the index does not belong to
// this stream (corrupt, or built with another checkpoint interval).
__device__ __forceinline__ bool ckpt_match(uint64_t e, int32_t hdr_bits, uint32_t smask, int32_t pos, uint32_t a0,
                                           uint32_t a1) {
    return (int32_t)(uint32_t)e + hdr_bits == pos && ((((uint32_t)(e >> 32) & smask) << 2) == a0) &&
           ((((uint32_t)(e >> 48) & smask) << 2) == a1);
}

// Container-mode end of a 2-state block after its main loop (the oracle's
// decompress2_impl with the raw length; lib.rs:227-244): the last one or two
// symbols come from the final states, and a valid block has then read every
// payload bit.  `ent(s)` is the table entry of state s; the reader pops.
template <int LMAX, class Ent, class Pop>
__device__ __forceinline__ int32_t finish2(uint32_t o, uint32_t n, uint32_t& s0, uint32_t& s1, int32_t& pos,
                                           int32_t hdr_bits, uint8_t* __restrict__ out, Ent ent, Pop pop) {
    for (;;) {
        if (o + 2u == n) {
            out[o++] = (uint8_t)dte_sym(ent(s0));
            out[o++] = (uint8_t)dte_sym(ent(s1));
            break;
        }
        if (o + 1u == n) {
            out[o++] = (uint8_t)dte_sym(ent(s0));
            break;
        }
        const uint32_t e0 = ent(s0);
        uint32_t nb = dte_nb(e0);
        if (pos - (int32_t)nb < hdr_bits) {
            out[o++] = (uint8_t)dte_sym(e0);
            if (o < n) out[o++] = (uint8_t)dte_sym(ent(s1));
            break;
        }
        s0 = Dte<LMAX>::ns(e0) + pop(nb);
        out[o++] = (uint8_t)dte_sym(e0);
        const uint32_t e1 = ent(s1);
        nb = dte_nb(e1);
        if (pos - (int32_t)nb < hdr_bits) {
            out[o++] = (uint8_t)dte_sym(e1);
            if (o < n) out[o++] = (uint8_t)dte_sym(ent(s0));
            break;
        }
        s1 = Dte<LMAX>::ns(e1) + pop(nb);
        out[o++] = (uint8_t)dte_sym(e1);
    }
    return o != n ? FSE_ERR_LENGTH_MISMATCH : pos == hdr_bits ? FSE_OK : FSE_ERR_BAD_SIDECAR;
}

// Main-loop pairs [p0, p1) of one segment read through a global-memory
// window (blocks the LDS stage cannot hold, and every block at LMAX = 15);
// the sidecar guarantees the bits, so no read checks.  `dt` may be LDS.
template <int LMAX>
__device__ __forceinline__ int32_t decode_segment(WindowReader& br, uint32_t& s0, uint32_t& s1, uint32_t p0,
                                                  uint32_t p1, bool last, uint32_t n, uint32_t Pm,
                                                  uint8_t* __restrict__ out, const uint32_t* dt, int32_t hdr_bits) {
    uint32_t p = p0;
    for (; p + 8u <= p1; p += 8u) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t e0 = dt[s0], e1 = dt[s1];
            const uint32_t v0 = br.pop(dte_nb(e0));
            const uint32_t v1 = br.pop(dte_nb(e1));
            s0 = Dte<LMAX>::ns(e0) + v0;
            s1 = Dte<LMAX>::ns(e1) + v1;
            const uint32_t pr = __builtin_amdgcn_perm(e1, e0, 0x0c0c0501u);
            if (j & 1) w[j >> 1] |= pr << 16; else w[j >> 1] = pr;
            br.refill();
        }
        *reinterpret_cast<uint4*>(out + 2u * p) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    for (; p < p1; ++p) {
        const uint32_t e0 = dt[s0], e1 = dt[s1];
        const uint32_t v0 = br.pop(dte_nb(e0));
        const uint32_t v1 = br.pop(dte_nb(e1));
        s0 = Dte<LMAX>::ns(e0) + v0;
        s1 = Dte<LMAX>::ns(e1) + v1;
        out[2u * p] = (uint8_t)dte_sym(e0);
        out[2u * p + 1u] = (uint8_t)dte_sym(e1);
        br.refill();
    }
    if (!last) return FSE_OK;
    return finish2<LMAX>(2u * Pm, n, s0, s1, br.pos, hdr_bits, out, [&](uint32_t s) { return dt[s]; },
                         [&](uint32_t nb) {
                             const uint32_t v = br.pop(nb);
                             br.refill();
                             return v;
                         });
}

// 1-state segment (fse_decompress, lib.rs:187-211) through the window.
template <int LMAX>
__device__ __forceinline__ int32_t decode_segment1(WindowReader& br, uint32_t& s, uint32_t p, uint32_t p1, bool last,
                                                   uint32_t n, uint8_t* __restrict__ out, const uint32_t* dt,
                                                   int32_t hdr_bits) {
    for (; p < p1; ++p) {
        const uint32_t e = dt[s];
        s = Dte<LMAX>::ns(e) + br.pop(dte_nb(e));
        br.refill();
        out[p] = (uint8_t)dte_sym(e);
    }
    if (!last) return FSE_OK;
    out[n - 1u] = (uint8_t)dte_sym(dt[s]);  // Decoder::finish (lib.rs:208)
    return br.pos == hdr_bits ? FSE_OK : FSE_ERR_BAD_SIDECAR;
}

// ------------------------------------------------------------------------
// Segment decode of a block staged in LDS (L <= 14, SH = 18).  One LdsChain
// is one segment's decoder pair: two tANS states as LDS byte offsets
// a0/a1 (4 * state) and the shared bit position.  Per pair the lane reads
// both table entries and ONE payload dword, all three issued together:
// a pair consumes <= 2L <= 28 < 32 bits, so the window base
// lo = (pos - 28) & ~31 (pos - lo in [28, 59]: the pair's bits and the
// 64-bit window both fit) moves down by at most one word per pair and the
// window's upper word is one of the previous pair's two words.  (It was
// pos - 24 while only L <= 12 ran here: at L = 13 and 14 a pair of rare
// symbols takes 26 or 28 bits and then read below the window; the wide
// randomized sweep found one.)  Then pos -= nb0 + nb1 (byte sum of
// the entries), v1 = the low nb1 bits at pos, v0 = the nb0 bits above
// (stack order: decoder 0 pops first), and the next offsets.  ~13 VALU and
// 3 LDS reads per pair, no branch.  The image has a 16-byte pad below it,
// so the window may start at word -1.
// ------------------------------------------------------------------------
constexpr int32_t PAIR_MAX_BITS = 28;  // 2 x 14: the largest pair at the LDS-staged table logs
struct LdsChain {
    int32_t pos, B;
    uint32_t whi, wlo, a0, a1;
    __device__ __forceinline__ void init(const uint32_t* pay, int32_t p, uint32_t s0, uint32_t s1) {
        pos = p;
        a0 = s0 << 2;
        a1 = s1 << 2;
        // the first pair reads word lo/32 and takes word lo/32 + 1 from here
        B = (p - PAIR_MAX_BITS) & ~31;
        wlo = 0;
        whi = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(pay) + (B >> 3) + 4);
    }
    __device__ __forceinline__ uint32_t pair(const uint32_t* pay, const uint8_t* dtb) {
        const int32_t lo = (pos - PAIR_MAX_BITS) & ~31;
        const uint32_t w0 = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(pay) + (lo >> 3));
        const uint32_t e0 = *reinterpret_cast<const uint32_t*>(dtb + a0);
        const uint32_t e1 = *reinterpret_cast<const uint32_t*>(dtb + a1);
        const uint32_t w1 = lo == B ? whi : wlo;
        pos -= (int32_t)((e0 + e1) & 0xFFu);
        const uint32_t x = (uint32_t)((((uint64_t)w1 << 32) | w0) >> (uint32_t)(pos - lo));
        B = lo;
        whi = w1;
        wlo = w0;
        const uint32_t v1 = __builtin_amdgcn_ubfe(x, 0u, e1);
        const uint32_t v0 = __builtin_amdgcn_ubfe(x, e1, e0);
        a0 = (e0 >> 16) + (v0 << 2);
        a1 = (e1 >> 16) + (v1 << 2);
        return __builtin_amdgcn_perm(e1, e0, 0x0c0c0501u);  // sym0 | sym1 << 8
    }
    __device__ __forceinline__ uint32_t s0() const { return a0 >> 2; }
    __device__ __forceinline__ uint32_t s1() const { return a1 >> 2; }
    // decode-table entry of state s (Dte layout)
    __device__ static __forceinline__ uint32_t entry(const uint8_t* dtb, uint32_t s) {
        return *reinterpret_cast<const uint32_t*>(dtb + 4u * s);
    }
};
// Two pairs -> four output bytes (lo.b0 lo.b1 hi.b0 hi.b1).
template <class Chain, class Tab>
__device__ __forceinline__ uint32_t two_pairs(Chain& c, const uint32_t* pay, const Tab& dtb) {
    const uint32_t lo = c.pair(pay, dtb);
    const uint32_t hi = c.pair(pay, dtb);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);  // lo.b0 lo.b1 hi.b0 hi.b1
}
// Bits [pos, pos + 32) of an LDS-staged block (pos >= 0): one ds_read2 of
// the two words holding them and a v_alignbit (the end-of-block steps).
__device__ __forceinline__ uint32_t lds_bits32(const uint32_t* pay, int32_t pos) {
    const uint32_t* wp = pay + ((uint32_t)pos >> 5);
    return __builtin_amdgcn_alignbit(wp[1], wp[0], (uint32_t)pos);
}

// 32 pairs = one whole 64-byte piece of output per lane, stored back to
// back (full HBM write bursts instead of masked partial ones).
__device__ __forceinline__ void store_group(uint8_t* __restrict__ dst, const uint32_t* w) {
    uint4* o4 = reinterpret_cast<uint4*>(dst);
#pragma unroll
    for (uint32_t q = 0; q < DEC_GROUP / 8u; ++q) o4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// Output pieces through the wave's rows.  Lane (row r, column i) = lane
// 16r + i holds a 64-byte piece = chunks C[0..3] of 16 bytes (w[4c..4c+3]).
// A 4x4 transpose of (row, chunk) per column -- permlane32_swap on chunk
// pairs (0,2), (1,3), then permlane16_swap on (0,1), (2,3) -- leaves in lane
// (r, i), slot k, chunk r of lane (k, i)'s piece.  Store k then writes 16
// whole pieces (4 lanes x 16 contiguous bytes each) instead of 64 lanes'
// separate 16-byte pieces of 64 lines: 16 VALU per 32 pairs.
__device__ __forceinline__ void rows_transpose(uint32_t* w) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const auto r = __builtin_amdgcn_permlane32_swap(w[4 * c + d], w[4 * (c + 2) + d], false, false);
            w[4 * c + d] = r[0];
            w[4 * (c + 2) + d] = r[1];
        }
#pragma unroll
    for (int c = 0; c < 4; c += 2)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const auto r = __builtin_amdgcn_permlane16_swap(w[4 * c + d], w[4 * (c + 1) + d], false, false);
            w[4 * c + d] = r[0];
            w[4 * (c + 1) + d] = r[1];
        }
}

// Whole output groups of one chain per lane, wave-synchronous (every lane of
// the wave runs ng_max iterations; a lane decodes only its first my_ng),
// stored through rows_transpose: obase[k] / ong[k] are the piece base and
// group count of lane (k, column) -- the owner of this lane's slot k.
template <class Chain, class Tab>
__device__ __forceinline__ void run_groups_tx(Chain& c, uint32_t my_ng, uint32_t ng_max, const uint32_t* pay,
                                              const Tab& dtb, uint8_t* const* obase, const uint32_t* ong,
                                              uint32_t row) {
    for (uint32_t g = 0; g < ng_max; ++g) {
        uint32_t w[DEC_GROUP / 2u];
        if (g < my_ng) {
#pragma unroll
            for (uint32_t j = 0; j < DEC_GROUP; j += 2u) w[j >> 1] = two_pairs(c, pay, dtb);
        } else {
#pragma unroll
            for (uint32_t j = 0; j < DEC_GROUP / 2u; ++j) w[j] = 0;
        }
        rows_transpose(w);
        // non-temporal: the output is written once and not read back here, so
        // it should not displace the images, tables and sidecars in L2
        // (C3 0.95 -> 0.91 ms, C2 decode 0.60 -> 0.57 ms, same box)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (g < ong[k])
                __builtin_nontemporal_store(u32x4{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]},
                                            reinterpret_cast<u32x4*>(obase[k] + g * 2u * DEC_GROUP + 16u * row));
    }
}

// `ng` whole output groups of two independent chains, their pairs
// interleaved (one lane, two segments: while one chain waits on its LDS
// reads the other's arithmetic issues).
template <class Chain, class Tab>
__device__ __forceinline__ void run_chains2(Chain& a, Chain& b, const uint32_t* pay, const Tab& dtb, uint32_t pa,
                                            uint32_t pb, uint32_t ng, uint8_t* __restrict__ out) {
    for (uint32_t g = 0; g < ng; ++g) {
        uint32_t wa[DEC_GROUP / 2u], wb[DEC_GROUP / 2u];
#pragma unroll
        for (uint32_t j = 0; j < DEC_GROUP; j += 2u) {
            const uint32_t la = a.pair(pay, dtb);
            const uint32_t lb = b.pair(pay, dtb);
            const uint32_t ha = a.pair(pay, dtb);
            const uint32_t hb = b.pair(pay, dtb);
            wa[j >> 1] = __builtin_amdgcn_perm(ha, la, 0x05040100u);
            wb[j >> 1] = __builtin_amdgcn_perm(hb, lb, 0x05040100u);
        }
        store_group(out + 2u * (pa + g * DEC_GROUP), wa);
        store_group(out + 2u * (pb + g * DEC_GROUP), wb);
    }
}

// Pairs [p, p1) of one chain, then (when `last`) the container-mode end.
template <class Chain, class Tab>
__device__ __forceinline__ int32_t run_chain(Chain& c, const uint32_t* pay, const Tab& dtb, uint32_t p, uint32_t p1,
                                             bool last, uint32_t n, uint32_t Pm, uint8_t* __restrict__ out,
                                             int32_t hdr_bits) {
    for (; p + DEC_GROUP <= p1; p += DEC_GROUP) {
        uint32_t w[DEC_GROUP / 2u];
#pragma unroll
        for (uint32_t j = 0; j < DEC_GROUP; j += 2u) w[j >> 1] = two_pairs(c, pay, dtb);
        store_group(out + 2u * p, w);
    }
    for (; p < p1; ++p) {
        const uint32_t pr = c.pair(pay, dtb);
        out[2u * p] = (uint8_t)pr;
        out[2u * p + 1u] = (uint8_t)(pr >> 8);
    }
    if (!last) return FSE_OK;
    // states as indices for the shared end; the chain keeps byte offsets
    uint32_t s0 = c.s0(), s1 = c.s1();
    return finish2<11>(2u * Pm, n, s0, s1, c.pos, hdr_bits, out, [&](uint32_t s) { return Chain::entry(dtb, s); },
                       [&](uint32_t nb) {
                           c.pos -= (int32_t)nb;
                           return __builtin_amdgcn_ubfe(lds_bits32(pay, c.pos), 0u, nb);
                       });
}

// 1-state chain (fse_decompress blocks) without a refill branch (round 6;
// the register window it replaced refilled under a divergent branch every
// few symbols and needed 110 VGPRs, 2 workgroups per CU at 512 threads:
// C2 1-state decode 0.75-0.78 -> 0.57 ms per GiB, profiles/r06/w1/): each call
// cuts x = the 32 bits just below pos from the word pair around pos - 32
// (word pos / 32 carried from the previous call, the word below it read:
// one ds_read, a compare, a select and a v_alignbit), then takes one symbol's
// field (step) or two symbols' fields (pair: <= 2 x 14 bits) from the top
// of x.  The image has 16 pad bytes below it (the word below word 0).
struct LdsChain1 {
    int32_t pos;
    uint32_t Q, whi, wlo, a;
    __device__ __forceinline__ void init(const uint32_t* pay, int32_t p, uint32_t s) {
        pos = p;
        a = s << 2;
        Q = ((uint32_t)p >> 3) & ~3u;
        wlo = 0;
        whi = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(pay) + Q);
    }
    __device__ __forceinline__ uint32_t window(const uint32_t* pay) {
        const uint32_t q = ((uint32_t)pos >> 3) & ~3u;
        const uint32_t wq = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(pay) + q - 4u);
        const uint32_t hi = q == Q ? whi : wlo;
        Q = q;
        whi = hi;
        wlo = wq;
        return __builtin_amdgcn_alignbit(hi, wq, (uint32_t)pos);
    }
    // one symbol; returns the table entry (symbol in bits 8-15)
    __device__ __forceinline__ uint32_t step(const uint32_t* pay, const uint8_t* dtb) {
        const uint32_t e = *reinterpret_cast<const uint32_t*>(dtb + a);
        const uint32_t x = window(pay);
        pos -= (int32_t)(e & 0xFFu);
        a = (e >> 16) + (__builtin_amdgcn_ubfe(x, 0u - e, e) << 2);
        return e;
    }
    // two symbols from one window; returns sym0 | sym1 << 8
    __device__ __forceinline__ uint32_t pair(const uint32_t* pay, const uint8_t* dtb) {
        const uint32_t e0 = *reinterpret_cast<const uint32_t*>(dtb + a);
        const uint32_t x = window(pay);
        const uint32_t o0 = 0u - e0;  // low 5 bits: 32 - nb0
        const uint32_t a1 = (e0 >> 16) + (__builtin_amdgcn_ubfe(x, o0, e0) << 2);
        const uint32_t e1 = *reinterpret_cast<const uint32_t*>(dtb + a1);
        a = (e1 >> 16) + (__builtin_amdgcn_ubfe(x, o0 - e1, e1) << 2);
        pos -= (int32_t)((e0 + e1) & 0xFFu);
        return __builtin_amdgcn_perm(e1, e0, 0x0c0c0501u);
    }
};
struct Chain1x2 {
    LdsChain1 c;
    __device__ __forceinline__ uint32_t pair(const uint32_t* pay, const uint8_t* dtb) { return c.pair(pay, dtb); }
};

// Steps [p, p1) of one 1-state segment; the last segment then emits the
// final state's symbol (container mode: the raw length ends the block, as
// the reference's next read fails right there for a valid stream).
__device__ __forceinline__ int32_t run_chain1(LdsChain1& c, const uint32_t* pay, const uint8_t* dtb, uint32_t p,
                                              uint32_t p1, bool last, uint32_t n, uint8_t* __restrict__ out,
                                              int32_t hdr_bits) {
    constexpr uint32_t G = 2u * DEC_GROUP;  // 64 symbols = one 64-byte piece of output
    for (; p + G <= p1; p += G) {
        uint32_t w[G / 4u];
#pragma unroll
        for (uint32_t j = 0; j < G; j += 4u) {
            const uint32_t lo = c.pair(pay, dtb), hi = c.pair(pay, dtb);
            w[j >> 2] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
        }
        uint4* o4 = reinterpret_cast<uint4*>(out + p);
#pragma unroll
        for (uint32_t q = 0; q < G / 16u; ++q) o4[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    }
    for (; p < p1; ++p) out[p] = (uint8_t)dte_sym(c.step(pay, dtb));
    if (!last) return FSE_OK;
    out[n - 1u] = (uint8_t)dte_sym(*reinterpret_cast<const uint32_t*>(dtb + c.a));  // finish (lib.rs:208)
    return c.pos == hdr_bits ? FSE_OK : FSE_ERR_BAD_SIDECAR;
}

// ------------------------------------------------------------------------
// Segment-parallel decode with prebuilt tables (fsehip_decompress_blocks_dt,
// the second kernel of fsehip_decompress_blocks; C3 times it alone).  One
// 256-thread workgroup per block:
//   1. DMA (global_load_lds) the compressed block and its table into LDS;
//   2. lane t decodes sidecar segment 33t mod 256 of each round (lanes that
//      walk their segments in lockstep then read payload words ~33 segments
//      apart, spread over the banks, instead of ~1 segment apart), storing
//      32 pairs (64 B) at a time;
//   3. every segment's end is checked against the next checkpoint.
// Blocks above the PMAX-byte stage are deferred (pass 1: status
// FSE_DEFERRED) to a second launch with a 66 KiB stage (pass 2); at
// LMAX = 15 the table alone fills the LDS and every block reads its payload
// through a global-memory window (pass 0).
// ------------------------------------------------------------------------
// Segment of thread tid in a round of 256.
template <uint32_t NT = 256u>
__device__ __forceinline__ uint32_t seg_of(uint32_t tid) {
    return (tid * 33u) & (NT - 1u);  // a bijection of [0, NT): 33 is odd
}

template <int LMAX, uint32_t PMAX, uint32_t NW = 4u>
struct PreSmem {
    uint32_t pad[4];  // below the image: the window may start at word -1
    uint32_t pay[PMAX / 4];
    uint32_t dt[1u << LMAX];
    int err[NW];
};

// One block (gb) by the whole workgroup; LDS reuse across calls is safe:
// every reader of the image and table has passed the final barrier before
// the next call's staging writes them.
template <int LMAX, uint32_t PMAX, int NS, uint32_t NT, class Smem>
__device__ __forceinline__ void decode_pre_block(const DecParams& P, Smem& sm, const uint64_t gb) {
    constexpr bool BIG = LMAX > 14;  // no LDS image
    constexpr uint32_t NW = NT / 64u;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    if (gb >= P.n_blocks) return;
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = P.comp_len[gb];
    const uint64_t ooff = gb * (uint64_t)P.block_size;
    const uint32_t n = (uint32_t)min((uint64_t)P.block_size, P.n_total - ooff);
    uint8_t* out = P.out + ooff;
    const int32_t info = P.dtinfo[gb];
    const bool in_lds = !BIG && clen <= PMAX;
    if (P.pass >= 2 && P.status[gb] != FSE_DEFERRED) return;  // done by an earlier pass
    FSE_STAMP(P, 0);
    if (info < 0 || n < (NS == 2 ? 2u : 1u)) {
        if (tid == 0) P.status[gb] = info < 0 ? info : FSE_ERR_LENGTH_MISMATCH;
        return;
    }
    // too big for this stage: a later list pass decodes it (pass 3: a list
    // pass that defers its own oversized blocks again)
    if ((P.pass == 1 || P.pass == 3) && !in_lds) {
        if (tid == 0) P.status[gb] = FSE_DEFERRED;
        return;
    }
    const int32_t hdr_bits = (info & 0xFFFF) * 8;
    const uint32_t L = (uint32_t)info >> 16;
    {  // stage the block image and the table
        if (in_lds) {
            const uint32_t nvec = (clen + 15u) >> 4;
            const uint4* src4 = reinterpret_cast<const uint4*>(in);
            uint4* dst4 = reinterpret_cast<uint4*>(sm.pay);
            for (uint32_t i = wv * 64u; i < nvec; i += NT)
                if (i + lane < nvec) __builtin_amdgcn_global_load_lds(src4 + i + lane, dst4 + i, 16, 0, STAGE_AUX);
        }
        {
            const uint32_t dvec = 1u << L >> 2;  // 4 << L bytes
            const uint4* t4 = reinterpret_cast<const uint4*>(P.dt + gb * (uint64_t)(1u << LMAX));
            uint4* d4 = reinterpret_cast<uint4*>(sm.dt);
            for (uint32_t i = wv * 64u; i < dvec; i += NT)
                if (i + lane < dvec) __builtin_amdgcn_global_load_lds(t4 + i + lane, d4 + i, 16, 0, STAGE_AUX);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    FSE_STAMP(P, 3);
    const uint32_t smask = (1u << L) - 1u;
    // main-loop steps: pairs (NS = 2) or symbols below the last one (NS = 1)
    const uint32_t Pm = NS == 2 ? ((n & 1u) ? (n - 3u) / 2u : n / 2u - 1u) : n - 1u;
    const uint32_t I = P.ckpt_interval;
    const uint32_t nseg = Pm / I + 1u;
    const uint64_t* sc = P.sidecar + gb * P.ckpt_per_block;
    const uint32_t maxbp = clen * 8u - (uint32_t)hdr_bits;
    using Chain = LdsChain;
    const uint8_t* dtb = reinterpret_cast<const uint8_t*>(sm.dt);
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(in);
    int32_t err = FSE_OK;
    uint32_t base0 = 0;
    if (NS == 2 && !BIG && in_lds && NT <= 256u) {  // (512 lanes: one segment each per round, 64 VGPRs)
        // Two segments per lane while a round has more segments than lanes
        // (checkpoints every <= 64 pairs at 64 KiB): segments s and s + NT
        // decoded interleaved, two independent chains per lane.
        for (; base0 + NT < nseg; base0 += 2u * NT) {
            const uint32_t sa = base0 + seg_of<NT>(tid), sb = sa + NT;
            bool act[2] = {sa < nseg, sb < nseg};
            const uint32_t sg[2] = {sa, sb};
            Chain c[2];
            uint32_t pp[2], pe[2];
            uint64_t en[2];
            int32_t r[2] = {FSE_OK, FSE_OK};
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                pp[k] = sg[k] * I;
                pe[k] = min(pp[k] + I, Pm);
                en[k] = 0;
                if (!act[k]) continue;
                const uint64_t e = sc[sg[k]];
                en[k] = sg[k] == nseg - 1u ? 0ull : sc[sg[k] + 1u];
                if ((uint32_t)e > maxbp) {  // corrupt index: never read outside the block
                    r[k] = FSE_ERR_BAD_SIDECAR;
                    act[k] = false;
                    continue;
                }
                c[k].init(sm.pay, hdr_bits + (int32_t)(uint32_t)e, (uint32_t)(e >> 32) & smask,
                          (uint32_t)(e >> 48) & smask);
            }
            const uint32_t ng = (act[0] && act[1]) ? min(pe[0] - pp[0], pe[1] - pp[1]) / DEC_GROUP : 0u;
            run_chains2(c[0], c[1], sm.pay, dtb, pp[0], pp[1], ng, out);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (!act[k]) continue;
                const bool last = sg[k] == nseg - 1u;
                r[k] = run_chain(c[k], sm.pay, dtb, pp[k] + ng * DEC_GROUP, pe[k], last, n, Pm, out, hdr_bits);
                if (r[k] == FSE_OK && !last &&
                    !ckpt_match(en[k], hdr_bits, smask, c[k].pos, c[k].s0() << 2, c[k].s1() << 2))
                    r[k] = FSE_ERR_BAD_SIDECAR;
            }
            if (r[0] != FSE_OK) err = r[0];
            if (r[1] != FSE_OK) err = r[1];
        }
    }
    if (NS == 2 && !BIG && in_lds) {
        // One segment per lane, every lane of a wave in step, output pieces
        // stored through the row transpose (run_groups_tx); then each lane's
        // tail pairs and, for the last segment, the block's end.
        for (; base0 < nseg; base0 += NT) {
            const uint32_t seg = base0 + seg_of<NT>(tid);
            bool act = seg < nseg;
            const uint32_t p0 = seg * I, p1 = act ? min(p0 + I, Pm) : p0;
            const bool lastseg = seg == nseg - 1u;
            int32_t r = FSE_OK;
            Chain c;
            uint64_t en = 0;
            if (act) {
                const uint64_t e = sc[seg];
                en = lastseg ? 0ull : sc[seg + 1u];
                if ((uint32_t)e > maxbp) {  // corrupt index: never read outside the block
                    r = FSE_ERR_BAD_SIDECAR;
                    act = false;
                } else {
                    c.init(sm.pay, hdr_bits + (int32_t)(uint32_t)e, (uint32_t)(e >> 32) & smask,
                           (uint32_t)(e >> 48) & smask);
                }
            }
            const uint32_t my_ng = act ? (p1 - p0) / DEC_GROUP : 0u;
            const uint32_t ng_max = wave_max(my_ng);
            if (ng_max) {
                uint8_t* obase[4];
                uint32_t ong[4];
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) {
                    const uint32_t os = base0 + seg_of<NT>((tid & ~63u) + 16u * k + (tid & 15u));
                    const uint32_t oq = os * I;
                    ong[k] = os < nseg ? (min(oq + I, Pm) - oq) / DEC_GROUP : 0u;
                    obase[k] = out + 2u * oq;
                }
                run_groups_tx(c, my_ng, ng_max, sm.pay, dtb, obase, ong, (tid >> 4) & 3u);
            }
            if (act) {
                r = run_chain(c, sm.pay, dtb, p0 + my_ng * DEC_GROUP, p1, lastseg, n, Pm, out, hdr_bits);
                if (r == FSE_OK && !lastseg && !ckpt_match(en, hdr_bits, smask, c.pos, c.s0() << 2, c.s1() << 2))
                    r = FSE_ERR_BAD_SIDECAR;
            }
            if (r != FSE_OK) err = r;
        }
    }
    if (NS == 1 && !BIG && in_lds) {
        // 1-state: the same transposed stores, 64 symbols (one 64-byte piece)
        // per group, two chain steps per packed pair
        constexpr uint32_t G1 = 2u * DEC_GROUP;
        for (; base0 < nseg; base0 += NT) {
            const uint32_t seg = base0 + seg_of<NT>(tid);
            bool act = seg < nseg;
            const uint32_t p0 = seg * I, p1 = act ? min(p0 + I, Pm) : p0;
            const bool lastseg = seg == nseg - 1u;
            int32_t r = FSE_OK;
            Chain1x2 c;
            uint64_t en = 0;
            if (act) {
                const uint64_t e = sc[seg];
                en = lastseg ? 0ull : sc[seg + 1u];
                if ((uint32_t)e > maxbp) {  // corrupt index: never read outside the block
                    r = FSE_ERR_BAD_SIDECAR;
                    act = false;
                } else {
                    c.c.init(sm.pay, hdr_bits + (int32_t)(uint32_t)e, (uint32_t)(e >> 32) & smask);
                }
            }
            const uint32_t my_ng = act ? (p1 - p0) / G1 : 0u;
            const uint32_t ng_max = wave_max(my_ng);
            if (ng_max) {
                uint8_t* obase[4];
                uint32_t ong[4];
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) {
                    const uint32_t os = base0 + seg_of<NT>((tid & ~63u) + 16u * k + (tid & 15u));
                    const uint32_t oq = os * I;
                    ong[k] = os < nseg ? (min(oq + I, Pm) - oq) / G1 : 0u;
                    obase[k] = out + oq;
                }
                run_groups_tx(c, my_ng, ng_max, sm.pay, dtb, obase, ong, (tid >> 4) & 3u);
            }
            if (act) {
                r = run_chain1(c.c, sm.pay, dtb, p0 + my_ng * G1, p1, lastseg, n, out, hdr_bits);
                if (r == FSE_OK && !lastseg && !ckpt_match(en, hdr_bits, smask, c.c.pos, c.c.a, 0u))
                    r = FSE_ERR_BAD_SIDECAR;
            }
            if (r != FSE_OK) err = r;
        }
    }
    for (uint32_t base = base0; base < nseg; base += NT) {
        const uint32_t seg = base + (NS == 2 ? seg_of<NT>(tid) : tid);
        if (seg >= nseg) continue;
        const uint64_t e = sc[seg];
        const uint32_t p0 = seg * I, p1 = min(p0 + I, Pm);
        const uint32_t bp = (uint32_t)e;
        uint32_t s0 = (uint32_t)(e >> 32) & smask, s1 = NS == 2 ? (uint32_t)(e >> 48) & smask : 0u;
        const bool lastseg = seg == nseg - 1u;
        const uint64_t en = lastseg ? 0ull : sc[seg + 1u];
        int32_t r;
        if (bp > maxbp) {  // corrupt index: never read outside the block
            r = FSE_ERR_BAD_SIDECAR;
        } else if (NS == 1) {
            if (!BIG && in_lds) {
                LdsChain1 c;
                c.init(sm.pay, hdr_bits + (int32_t)bp, s0);
                r = run_chain1(c, sm.pay, dtb, p0, p1, lastseg, n, out, hdr_bits);
                if (r == FSE_OK && !lastseg && !ckpt_match(en, hdr_bits, smask, c.pos, c.a, 0u)) r = FSE_ERR_BAD_SIDECAR;
            } else {
                WindowReader br;
                br.init(gw, hdr_bits + (int32_t)bp);
                r = decode_segment1<LMAX>(br, s0, p0, p1, lastseg, n, out, sm.dt, hdr_bits);
                if (r == FSE_OK && !lastseg && !ckpt_match(en, hdr_bits, smask, br.pos, s0 << 2, 0u))
                    r = FSE_ERR_BAD_SIDECAR;
            }
        } else if (!BIG && in_lds) {
            Chain c;
            c.init(sm.pay, hdr_bits + (int32_t)bp, s0, s1);
            r = run_chain(c, sm.pay, dtb, p0, p1, lastseg, n, Pm, out, hdr_bits);
            if (r == FSE_OK && !lastseg && !ckpt_match(en, hdr_bits, smask, c.pos, c.a0, c.a1)) r = FSE_ERR_BAD_SIDECAR;
        } else {
            WindowReader br;
            br.init(gw, hdr_bits + (int32_t)bp);
            r = decode_segment<LMAX>(br, s0, s1, p0, p1, lastseg, n, Pm, out, sm.dt, hdr_bits);
            if (r == FSE_OK && !lastseg && !ckpt_match(en, hdr_bits, smask, br.pos, s0 << 2, s1 << 2))
                r = FSE_ERR_BAD_SIDECAR;
        }
        if (r != FSE_OK) err = r;
    }
    err = -(int32_t)wave_max((uint32_t)(-err));
    if (lane == 0) sm.err[wv] = err;
    __syncthreads();
    FSE_STAMP(P, 4);
    if (tid == 0) {
        int32_t e2 = FSE_OK;
        for (uint32_t w = 0; w < NW; ++w)
            if (sm.err[w] != FSE_OK) e2 = sm.err[w];
        P.status[gb] = e2;
        if (P.out_len) P.out_len[gb] = e2 ? 0u : n;
    }
}

// PASS 0 (every block) / 1 (blocks the stage holds; the others are marked
// FSE_DEFERRED): one block per workgroup, grid = blocks.  PASS 2 (the
// 66 KiB stage, 2 workgroups per CU): a grid of about one workgroup per slot
// on the chip; workgroup w collects the deferred blocks among w, w + G,
// w + 2G, ... (256 status reads at once, compacted in LDS) and decodes them
// one after the other, so a batch with few or no deferred blocks costs a few
// microseconds instead of a full-grid launch of empty workgroups (~0.03 ms
// per GiB).
template <int LMAX, uint32_t PMAX, int NS, int PASS, uint32_t NT = 256u>
__global__ __launch_bounds__(NT) void decode_pre_kernel(DecParams P) {
    constexpr bool BIG = LMAX > 14;
    constexpr uint32_t NW = NT / 64u;
    __shared__ PreSmem<LMAX, BIG ? 16u : PMAX, NW> sm;
    if constexpr (PASS <= 1) {
        decode_pre_block<LMAX, PMAX, NS, NT>(P, sm, blockIdx.x);
    } else {
        // the deferred blocks among this workgroup's NT candidates, as one
        // ballot mask per wave (64 B of LDS instead of an NT-entry list: the
        // L = 12 list pass fits 2 workgroups per CU with a 65,392-byte stage)
        __shared__ uint64_t dmask[NW];
        const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
        const uint64_t G = gridDim.x;
        for (uint64_t r0 = blockIdx.x; r0 < P.n_blocks; r0 += G * NT) {
            const uint64_t gb = r0 + G * tid;
            const bool d = gb < P.n_blocks && P.status[gb] == FSE_DEFERRED;
            const uint64_t m = __ballot(d);
            if (lane == 0) dmask[wv] = m;
            __syncthreads();
            for (uint32_t w = 0; w < NW; ++w) {
                for (uint64_t mw = dmask[w]; mw; mw &= mw - 1u)  // workgroup-uniform
                    decode_pre_block<LMAX, PMAX, NS, NT>(P, sm, r0 + G * (64u * w + (uint32_t)__builtin_ctzll(mw)));
            }
            __syncthreads();  // dmask is rewritten by the next round
        }
    }
}

// ------------------------------------------------------------------------
// NormHistogram::read (histogram.rs:436-505) for 16 blocks per wave, one lane
// per block.  Parsed on the scalar unit inside dtable_blocks_kernel a header
// costs ~2,200 scalar instructions, and at full occupancy the CU's one scalar
// unit is shared by all its waves (the parse took 29.8K of the kernel's 68.4K
// cycles per block, profiles/r04/probe1/stamps_T64.log).  Here the headers
// are staged into LDS rows (the same 512 bytes the wave parse holds, coalesced
// per block, 16 blocks' loads in flight at once) and each lane runs the same
// parse (header_read_core) on its own row; the counts and the header length /
// L / table_len go to the scratch that dtable_blocks_kernel then reads.
// ------------------------------------------------------------------------
constexpr uint32_t HP_BLOCKS = 16;  // headers per workgroup: 1,024 workgroups at C2 (8 measured no faster: the parse latency is the floor)
template <int LMAX>
__global__ __launch_bounds__(64) void hdr_parse_kernel(DtParams P) {
    static_assert(LMAX <= 12, "headers of L <= 12 fit the 512 staged bytes");
    constexpr uint32_t NB = HP_BLOCKS;
    // block j's header words and counts, rotated by j words (row j, word i at
    // (i + j) % 128): lanes at the same word index hit different banks
    __shared__ uint32_t rows[NB][128];
    __shared__ uint32_t nrm[NB][128];  // 256 x int16 per block
    const uint32_t lane = threadIdx.x;
    const uint64_t gb0 = (uint64_t)blockIdx.x * NB;
    const uint64_t gl = gb0 + lane;
    const bool mine = lane < NB && gl < P.n_blocks;
    const uint32_t clen_l = mine ? P.comp_len[gl] : 0u;
    // the words header_read_wave holds: min(clen, 512) bytes, within the slot
    const uint32_t nw_l = (uint32_t)min((uint64_t)min(clen_l, HDR_MAX) + 3u, P.slot_bytes) >> 2;
    for (uint32_t i = lane; i < NB * 128u; i += 64u) (&nrm[0][0])[i] = 0u;
    // stage: block j's words across the lanes, every block's loads in flight at once
    uint32_t a[NB], b[NB];
#pragma unroll
    for (uint32_t j = 0; j < NB; ++j) {
        const uint32_t nw = (uint32_t)__builtin_amdgcn_readlane((int)nw_l, (int)j);  // 0 past the batch
        const uint32_t* w = reinterpret_cast<const uint32_t*>(P.in + (gb0 + j) * P.slot_bytes);
        a[j] = lane < nw ? w[lane] : 0u;
        b[j] = lane + 64u < nw ? w[lane + 64u] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < NB; ++j) {
        rows[j][(lane + j) & 127u] = a[j];
        rows[j][(lane + 64u + j) & 127u] = b[j];
    }
    __syncthreads();
    if (mine) {
        uint32_t L = 0, tl = 0;
        typedef __attribute__((address_space(3))) int16_t lds_i16;
        const int hl = header_read_row((const lds_u32*)&rows[lane][0], lane, nw_l, clen_l, (uint32_t)LMAX,
                                       (lds_i16*)&nrm[lane][0], &L, &tl);
        P.hdr_meta[gl] = make_int2(hl, (int)(L | (tl << 8)));
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < NB; ++j) {  // counts out, unrotated: word k of block j
        const uint64_t g = gb0 + j;
        if (g >= P.n_blocks) break;
        P.hdr_norm[g * 128u + lane] = nrm[j][(lane + j) & 127u];
        P.hdr_norm[g * 128u + 64u + lane] = nrm[j][(lane + 64u + j) & 127u];
    }
}

// ------------------------------------------------------------------------
// Decode tables for a batch of blocks (C3's "pre-built dtables"; also the
// first kernel of the two-kernel decode): NormHistogram::read on the scalar
// unit + DecodeTable (fse.rs:280-338) by one wave per block, written to HBM
// in the decoder's entry layout.  Small LDS footprint at L <= 12, so many
// blocks are in flight per CU and the serial header parse is overlapped
// across blocks.
// ------------------------------------------------------------------------
template <int LMAX>
__global__ __launch_bounds__(64) void dtable_blocks_kernel(DtParams P) {
    constexpr uint32_t SIZE = 1u << LMAX;
    __shared__ int32_t norm[256];
    __shared__ __attribute__((aligned(16))) uint8_t sym_at[SIZE];
    // the two-pass rank table (2^L u16) reuses the occurrence owners, the
    // counters and cumul: all three are dead once the spread walk is done
    // (the decoder's visit reads norm only); 7 KB per workgroup at L = 11.
    // L >= 13 never takes the two-pass ranks, so the array only has to hold
    // occ, cnt and cumul: 2^L + 1.5 KiB instead of 2^(L+1) bytes (L = 15: 2
    // workgroups per CU instead of 1)
    constexpr uint32_t RKN = LMAX <= 12 ? SIZE : SIZE / 2u + 768u;
    __shared__ __attribute__((aligned(16))) uint16_t rk[RKN];
    static_assert(SIZE + 256 * 4 + 256 * 2 <= RKN * 2, "rank table must cover occ, cnt and cumul");
    // (no LDS peer masks: the peer-mask ranks run only when an atomic-rank
    // table fails its check, and then match keys by ballot; the 512 B they
    // took kept the kernel at 21 workgroups per CU instead of 22)
    uint8_t* occ = reinterpret_cast<uint8_t*>(rk);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(rk) + SIZE);
    uint16_t* cumul = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(rk) + SIZE + 1024);
    const uint32_t lane = lane_id();
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    FSE_STAMP(P, 0);
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = P.comp_len[gb];
    const uint32_t last = (clen && clen <= P.slot_bytes) ? in[clen - 1u] : 0u;
    uint32_t L = 0, tl = 0;
    int hl;
    if (LMAX <= 12 && P.hdr_meta) {  // parsed by hdr_parse_kernel: counts from the scratch
        const int2 m = P.hdr_meta[gb];
        const uint32_t q0 = P.hdr_norm[gb * 128u + lane], q1 = P.hdr_norm[gb * 128u + 64u + lane];
        norm[2u * lane] = (int32_t)(int16_t)(q0 & 0xFFFFu);
        norm[2u * lane + 1u] = (int32_t)(int16_t)(q0 >> 16);
        norm[128u + 2u * lane] = (int32_t)(int16_t)(q1 & 0xFFFFu);
        norm[128u + 2u * lane + 1u] = (int32_t)(int16_t)(q1 >> 16);
        hl = m.x;
        L = (uint32_t)m.y & 0xFFu;
        tl = (uint32_t)m.y >> 8;
        wave_sync();
        FSE_STAMP(P, 1);
        FSE_STAMP(P, 2);
    } else {
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
        const uint32_t nw = (uint32_t)min((uint64_t)min(clen, HDR_MAX) + 3u, P.slot_bytes) >> 2;
        if (P.slot_bytes < HDR_MAX) {
            r0 = lane < nw ? w[lane] : 0u;
            r1 = lane + 64u < nw ? w[lane + 64u] : 0u;
        }
        r0 = lane < nw ? r0 : 0u;
        r1 = lane + 64u < nw ? r1 : 0u;
        for (uint32_t s = lane; s < 256u; s += WAVE) norm[s] = 0;
        wave_sync();
        FSE_STAMP(P, 1);
        hl = header_read_wave(r0, r1, clen, (uint32_t)LMAX, norm, &L, &tl);
        FSE_STAMP(P, 2);
    }
    int rc = hl < 0 ? hl : FSE_OK;
    if (rc == FSE_OK && ((uint32_t)hl >= clen || last == 0)) rc = FSE_ERR_NO_MARKER;  // lib.rs:222
    if (rc == FSE_OK && clen > (1u << 28)) rc = FSE_ERR_UNSUPPORTED;  // bit positions are 32-bit in the decoders
    wave_sync();
    if (rc == FSE_OK) {
        const uint32_t size = 1u << L;
        uint32_t* dt = P.dt + gb * (uint64_t)SIZE;
        auto visit = [&](uint32_t i, uint32_t s, uint32_t nx) {  // nx = the symbol's first x + rank
            const uint32_t nb = L - ilog2u(nx);
            dt[i] = Dte<LMAX>::make(nb, s, (nx << nb) - size);
        };
        auto first_x = [&](uint32_t s) {  // symbol_next (fse.rs:296-308): 1 for a -1 count
            const int32_t v = norm[s];
            return v < 0 ? 1u : (uint32_t)v;
        };
        // two-pass ranks need 2^L / 64 per-chunk registers: up to L = 12
        const RankAtomic ra{P.peer_ranks == 0u, occ, nullptr, 0u, &g_rank_fb_dec, P.rank_inject};
        if (LMAX <= 12)
            rc = wave_build_spread<SIZE / 64u, true>(norm, L, tl, sym_at, occ, cumul, cnt, visit, first_x, ra, rk,
                                                     nullptr, &P);
        else rc = wave_build_spread<64, true>(norm, L, tl, sym_at, occ, cumul, cnt, visit, first_x, ra);
    }
    FSE_STAMP(P, 8);
    if (lane == 0) P.dtinfo[gb] = rc == FSE_OK ? (int32_t)((uint32_t)hl | (L << 16)) : rc;
}


// ------------------------------------------------------------------------
// fse_decompress (lib.rs:187-211) without a sidecar: one lane per block
// walks the stream with every read checked, on tables from
// dtable_blocks_kernel.  Container mode (raw length known) or the
// reference's own termination with a capacity (host streams).
// ------------------------------------------------------------------------
template <int LMAX>
__global__ __launch_bounds__(64) void decode1_serial_kernel(DecParams P) {
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    const int32_t info = P.dtinfo[gb];
    // single-symbol table (every nb 0): the whole wave scans it
    uint32_t nbor = 0;
    if (info >= 0) {
        const uint32_t* t = P.dt + gb * (uint64_t)(1u << LMAX);
        for (uint32_t i = threadIdx.x; i < (1u << ((uint32_t)info >> 16)); i += 64u) nbor |= t[i] & 0xFFu;
    }
    const bool single = __ballot(nbor != 0u) == 0ull;
    if (threadIdx.x != 0) return;
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
    WindowReader br;
    br.init(reinterpret_cast<const uint32_t*>(in), top);
    if (br.pos - (int32_t)L < hdr_bits) {
        err = FSE_ERR_TOO_SHORT;  // lib.rs:197 unwrap
    } else {
        uint32_t s = br.pop(L);
        br.refill();
        for (;;) {
            if (known && single && o + 1u >= n) break;  // raw length ends a single-symbol block
            const uint32_t e = dt[s];
            const uint32_t nb = dte_nb(e);
            if (br.pos - (int32_t)nb < hdr_bits) break;  // decode_symbol -> None
            if (o >= cap) {  // a single-symbol table never ends in the reference (the oracle refuses
                             // it up front); any other stream simply needs more room
                err = single ? FSE_ERR_SINGLE_SYMBOL : FSE_ERR_DST_TOO_SMALL;
                break;
            }
            s = Dte<LMAX>::ns(e) + br.pop(nb);
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
// Sidecar-less decode of 2-state blocks (any valid fse_compress2 stream,
// e.g. from the CPU crate), optionally recording the sidecar.  The two
// interleaved decoders make the stream essentially serial: a decoder
// started mid-block with guessed states practically never falls into step
// with the exact one (oracle/syncsim.py: 35 of 40 random starts in a C2
// block never did, the rest after 25K-40K symbols), so speculative segment
// decoding cannot replace the sidecar for this format.  The
// serial decode is instead made as short a dependency chain as possible and
// run at high occupancy.  This kernel serves tables above L = 12 (128 KiB
// at L = 15): the block's prebuilt table sits in LDS, one lane walks the
// stream (lib.rs:227-244) and the bits come through a register window fed
// from 16-byte chunks loaded a chunk ahead.  At L <= 12 serial_ring_kernel
// below replaces it (3x faster at C2).
//   Container mode (n_total > 0): the raw length ends the block, as the
//   oracle's decompress2 with a known length.
//   Reference mode (n_total == 0, the host fse_decompress2): the block ends
//   where a decoder's read fails (lib.rs:228-243), within out_cap bytes; a
//   single-symbol table never ends in the reference and is refused.
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

template <int LMAX>
__global__ __launch_bounds__(64) void serial2_decode_kernel(DecParams P) {
    __shared__ uint32_t tab[1u << LMAX];
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    const int32_t info = P.dtinfo[gb];
    const uint32_t lane = threadIdx.x;
    uint32_t nbor = 0;  // OR of the staged entries' nb: 0 = single-symbol table
    if (info >= 0) {  // stage the table (prebuilt by dtable_blocks_kernel)
        const uint32_t nv = (1u << ((uint32_t)info >> 16)) >> 2;  // 16-byte chunks
        const uint4* t4 = reinterpret_cast<const uint4*>(P.dt + gb * (uint64_t)(1u << LMAX));
        uint4* d4 = reinterpret_cast<uint4*>(tab);
        for (uint32_t i = lane; i < nv; i += 64u) {
            const uint4 q = t4[i];
            d4[i] = q;
            nbor |= (q.x | q.y | q.z | q.w) & 0xFFu;
        }
    }
    const bool single = __ballot(nbor != 0u) == 0ull;
    __syncthreads();
    if (lane != 0) return;
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = P.comp_len[gb];
    const bool known = P.n_total != 0;
    const uint64_t ooff = gb * (uint64_t)P.block_size;
    const uint32_t n = known ? (uint32_t)min((uint64_t)P.block_size, P.n_total - ooff) : 0u;
    const uint32_t lim = known ? n : P.out_cap;  // bytes the block may produce
    uint8_t* out = P.out + ooff;
    int32_t err = info < 0 ? info : FSE_OK;
    if (err == FSE_OK && known && n < 2) err = FSE_ERR_LENGTH_MISMATCH;
    if (err == FSE_OK && !known && single) err = FSE_ERR_SINGLE_SYMBOL;  // the reference loops forever
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
        // bulk: groups of 8 pairs that can neither reach the raw length (or
        // the capacity) nor run out of bits (<= 2L bits a pair): no end
        // checks, and the 16 output bytes leave as one dwordx4 store, so few
        // stores are in flight when the next chunk's load is waited on
        while (o + 18u < lim && br.pos - hdr_bits >= 16 * (int32_t)L) {
            uint32_t w[4];
#pragma unroll
            for (uint32_t j = 0; j < 8u; ++j, ++pidx) {
                record();
                const uint32_t e0 = tab[s0];
                s0 = Dte<LMAX>::ns(e0) + br.pop(dte_nb(e0));
                br.refill();
                const uint32_t e1 = tab[s1];
                s1 = Dte<LMAX>::ns(e1) + br.pop(dte_nb(e1));
                br.refill();
                const uint32_t v = dte_sym(e0) | (dte_sym(e1) << 8);
                if (j & 1u) w[j >> 1] |= v << 16; else w[j >> 1] = v;
            }
            *reinterpret_cast<uint4*>(out + o) = make_uint4(w[0], w[1], w[2], w[3]);
            o += 16;
        }
        // tail: pair by pair with the reference's end checks
        const int32_t full = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL;
        for (;; ++pidx) {
            record();
            if (known && o + 2u >= n) {  // the raw length ends the block (o is even here)
                if (o < n) out[o++] = (uint8_t)dte_sym(tab[s0]);
                if (o < n) out[o++] = (uint8_t)dte_sym(tab[s1]);
                break;
            }
            const uint32_t e0 = tab[s0];
            uint32_t nb = dte_nb(e0);
            if (br.pos - (int32_t)nb < hdr_bits) {  // decoder 0 cannot read: lib.rs:242-243
                if (o + 2u > lim) { err = full; break; }
                out[o++] = (uint8_t)dte_sym(e0);
                out[o++] = (uint8_t)dte_sym(tab[s1]);
                break;
            }
            s0 = Dte<LMAX>::ns(e0) + br.pop(nb);
            br.refill();
            if (o >= lim) { err = full; break; }
            out[o++] = (uint8_t)dte_sym(e0);
            const uint32_t e1 = tab[s1];
            nb = dte_nb(e1);
            if (br.pos - (int32_t)nb < hdr_bits) {  // decoder 1 cannot read: lib.rs:235-239
                if (o + 2u > lim) { err = full; break; }
                out[o++] = (uint8_t)dte_sym(e1);
                out[o++] = (uint8_t)dte_sym(tab[s0]);
                break;
            }
            s1 = Dte<LMAX>::ns(e1) + br.pop(nb);
            br.refill();
            if (o >= lim) { err = full; break; }
            out[o++] = (uint8_t)dte_sym(e1);
        }
        if (err == FSE_OK && known && o != n) err = FSE_ERR_LENGTH_MISMATCH;
    }
    P.status[gb] = err;
    if (P.out_len) P.out_len[gb] = err ? 0u : o;
}

// ------------------------------------------------------------------------
// Sidecar-less 2-state decode at L <= 12 (the serial decode above, made
// 3x faster at C2).  Two things bound that kernel: its single lane is
// provably lane 0, so the compiler runs the chain as wave-uniform SALU+VALU
// code (~30 issue slots per pair for one chain), and its register window
// waits on the global prefetch at every refill (the compiler merges the
// prefetched registers at each refill branch, so it waits for the load,
// and for any output store issued after it).  Here:
//   - K blocks per workgroup, lane j of wave 0 walking block j: one VALU
//     instruction advances K chains, and LDS caps the chains per CU (K = 6
//     at L <= 11: 6 x (6 KiB table + 512 B ring) = 40.0 KB, 4 workgroups =
//     24 chains per CU; K = 3 at L = 12: 3 x 12.5 KiB, 12 chains per CU);
//   - wave 1 streams each block's payload top down into its 128-word LDS
//     ring in 256-byte chunks (one dword per lane), one chunk ahead of the
//     one being decoded (a chunk lasts ~170 pairs, ~17 us: far longer than a
//     load), and publishes the lowest word landed (ctl[0]);
//   - the decode lanes read only LDS (one payload word and the two table
//     entries per pair, issued together, as the segment decoder's
//     LdsChain), publish the highest word they may still read every 8 pairs
//     (ctl[1]) and store their output without ever waiting on memory.
// Same end checks, statuses and sidecar recording as serial2.
// ------------------------------------------------------------------------
constexpr uint32_t RING_WORDS = 128u, RING_MASK = RING_WORDS - 1u, RING_CHUNK = 64u;
#ifndef FSE_RING_GROUP
#define FSE_RING_GROUP 32
#endif
// state words (pairs, or two 1-state symbols) per bulk iteration with the
// symbols deferred; a multiple of 8 (whole 16-byte groups for sym_map_kernel).
// The loop's control (~45 instructions an iteration: the ring wait, the
// stores, the published position) is paid once per group: C2 sidecar-less
// decode 8.07 ms at 8, 7.31 at 16, 7.01 at 32, 7.20 at 64 (profiles/r06/rg/)
constexpr uint32_t RING_GROUP = FSE_RING_GROUP;
#ifndef FSE_RING_GROUP_SYM
#define FSE_RING_GROUP_SYM 32
#endif
// the same for the kernels that write the symbols themselves (L = 12, the
// fallback without the state workspace, sidecar rebuilds): 32 against 8,
// skewed L = 12 sidecar-less 17.5 -> 16.3 ms per GiB, C2 sidecar rebuild
// 11.7 -> 10.7 ms (profiles/r06/rg/)
constexpr uint32_t RING_GROUP_SYM = FSE_RING_GROUP_SYM;
static_assert(RING_GROUP_SYM % 8u == 0u && RING_GROUP_SYM <= 64u, "ring group");
static_assert(RING_GROUP % 8u == 0u && RING_GROUP <= 64u, "ring group: the tail waits for (2 RING_GROUP + 4) L bits, 45 words at 64");

// Relaxed workgroup-scope atomics keep these as plain ds_read/ds_write (a
// volatile access through a generic pointer becomes a FLAT access that
// waits on vmcnt, i.e. on the output stores); the asm barriers pin their
// place among the ring reads and writes, and LDS runs one wave's accesses
// in order.
__device__ __forceinline__ int32_t lds_load_volatile(int32_t* p) {
    const int32_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __asm__ __volatile__("" ::: "memory");
    return v;
}
__device__ __forceinline__ void lds_store_volatile(int32_t* p, int32_t v) {
    __asm__ __volatile__("" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The ring handoff proper: the loader publishes "landed" with release
// semantics after its ring writes, the decoder reads it with acquire (only
// on its slow path, when the cached value is not low enough).  The
// decoder's "still needed" hints stay relaxed: a stale value is a higher
// one, which only makes the loader wait.
__device__ __forceinline__ int32_t lds_load_acquire(int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_release(int32_t* p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
typedef __attribute__((address_space(3))) const uint8_t lds_cu8;
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
__device__ __forceinline__ uint32_t lds_u16_at(uint32_t a) { return *(lds_cu16*)(uintptr_t)a; }
__device__ __forceinline__ uint32_t lds_u8_at(uint32_t a) { return *(lds_cu8*)(uintptr_t)a; }
__device__ __forceinline__ uint32_t lds_u32_at(uint32_t a) { return *(lds_cu32*)(uintptr_t)a; }
template <class T>
__device__ __forceinline__ uint32_t lds_addr(T* p) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)p;
}

// The sidecar-less decoder's tables in LDS: for the K blocks of a
// workgroup, u16 entries nb | newState << NBW (ent[K][2^LMAX]) followed by
// u8 symbols (sym[K][2^LMAX]), 3 bytes per state (6 KiB at L = 11, 12 KiB
// at L = 12, against 8 / 16 KiB of dtable_blocks_kernel's u32 entries), so
// with 528-byte rings 6 blocks fit a 40 KB workgroup at L <= 11 and 3 at
// L = 12 (4 workgroups per CU).  A chain's state is its entry's LDS byte
// address halved, B = H + state (H = its entry table / 2): the entry is at
// 2B and the symbol at B + SO, SO = sym - ent / 2 being the same for every
// chain (the ds_read's immediate offset), and the next state is
// H + newState + bits (one add3).
// NBW = 5 (L <= 11): nb < 16 leaves bit 4 clear, so the entry is the v_bfe
// width as it is and -e its offset below the top.  NBW = 4 (L = 12,
// newState needs 12 bits): nb = e & 15.  newState = e >> NBW.
template <uint32_t NBW>
struct RingTab {
    static_assert(NBW == 4 || NBW == 5, "nb field width");
    uint32_t H;   // this chain's entry table (LDS byte address) / 2
    uint32_t SO;  // symbol of state B: LDS byte B + SO
    __device__ __forceinline__ uint32_t entry_at(uint32_t B) const { return lds_u16_at(B << 1); }
    __device__ __forceinline__ uint32_t sym_at(uint32_t B) const { return ((lds_cu8*)(uintptr_t)B)[SO]; }
    // nb as a bit-field operand (v_bfe reads its low five bits)
    __device__ __forceinline__ uint32_t nbf(uint32_t e) const { return NBW == 5 ? e : e & 15u; }
    __device__ __forceinline__ uint32_t ns(uint32_t e) const { return e >> NBW; }
    // by state index (end-of-block steps)
    __device__ __forceinline__ uint32_t nb(uint32_t s) const { return entry_at(H + s) & ((1u << NBW) - 1u); }
    __device__ __forceinline__ uint32_t symbol(uint32_t s) const { return sym_at(H + s); }
    __device__ __forceinline__ uint32_t next_base(uint32_t s) const { return ns(entry_at(H + s)); }
};

// Ring of one chain: RING_WORDS words of the payload by word index mod
// RING_WORDS, plus a mirror of slot 0 in slot RING_WORDS, so that words
// (q, q + 1) are always two adjacent slots (one ds_read2_b32).
constexpr uint32_t RING_STRIDE = RING_WORDS + 4u;

// A serial chain over its ring.  NS = 2: a pair (<= 24 bits) per step;
// NS = 1: one symbol.  Each step reads x = the 32 payload bits just below
// pos (words (pos - 32) / 32 and the one above, issued together with the
// table reads: they depend only on pos), then takes decoder 0's nb0 bits
// from the top of x and decoder 1's nb1 bits below them (stack order,
// lib.rs:227-234) as bit fields at 32 - nb0 and 32 - nb0 - nb1: from a
// table read back to the next one is four VALU (negate, bfe, add3, shift)
// and no 64-bit shift or window bookkeeping.
template <int NS, uint32_t NBW>
struct RingChain {
    using Tab = RingTab<NBW>;
    int32_t p32;      // bit position - 32
    uint32_t B0, B1;  // states as halved entry addresses
    uint32_t R;       // this chain's ring (LDS byte address)
    __device__ __forceinline__ void init(uint32_t ring, const Tab& T, int32_t p, uint32_t s0, uint32_t s1) {
        p32 = p - 32;
        R = ring;
        B0 = T.H + s0;
        B1 = T.H + s1;
    }
    __device__ __forceinline__ int32_t pos() const { return p32 + 32; }
    __device__ __forceinline__ uint32_t s0(const Tab& T) const { return B0 - T.H; }
    __device__ __forceinline__ uint32_t s1(const Tab& T) const { return B1 - T.H; }
    // the 32 bits [pos - 32, pos); below bit 0 (pos < 32) the low bits are
    // stale ring contents that no step uses
    __device__ __forceinline__ uint32_t window() const {
        // one v_bfe and one v_lshl_add (from ubfe << 2 the compiler makes a
        // shift, a mask and an add: one VALU more per pair, 1.7 % of the
        // sidecar-less decode, profiles/r06/rg/)
        uint32_t wi;
        asm("v_bfe_u32 %0, %1, 5, 7" : "=v"(wi) : "v"(p32));
        const uint32_t a = R + (wi << 2);
        return __builtin_amdgcn_alignbit(lds_u32_at(a + 4u), lds_u32_at(a), (uint32_t)p32);
    }
    // one pair; returns sym0 | sym1 << 8
    __device__ __forceinline__ uint32_t pair(const Tab& T) {
        const uint32_t e0 = T.entry_at(B0), e1 = T.entry_at(B1);
        const uint32_t y0 = T.sym_at(B0), y1 = T.sym_at(B1);
        const uint32_t x = window();
        const uint32_t n0 = T.nbf(e0), n1 = T.nbf(e1);
        const uint32_t o0 = 0u - n0;
        const uint32_t v0 = __builtin_amdgcn_ubfe(x, o0, n0);
        const uint32_t v1 = __builtin_amdgcn_ubfe(x, o0 - n1, n1);
        p32 -= (int32_t)((n0 + n1) & 31u);
        B0 = T.H + T.ns(e0) + v0;
        B1 = T.H + T.ns(e1) + v1;
        return y0 | (y1 << 8);
    }
    // one pair with the symbols deferred: returns the two states (low 16
    // bits of each halved entry address) for sym_map_kernel
    __device__ __forceinline__ uint32_t pair_states(const Tab& T) {
        const uint32_t e0 = T.entry_at(B0), e1 = T.entry_at(B1);
        const uint32_t v = __builtin_amdgcn_perm(B1, B0, 0x05040100u);
        const uint32_t x = window();
        const uint32_t n0 = T.nbf(e0), n1 = T.nbf(e1);
        const uint32_t o0 = 0u - n0;
        const uint32_t v0 = __builtin_amdgcn_ubfe(x, o0, n0);
        const uint32_t v1 = __builtin_amdgcn_ubfe(x, o0 - n1, n1);
        p32 -= (int32_t)((n0 + n1) & 31u);
        B0 = T.H + T.ns(e0) + v0;
        B1 = T.H + T.ns(e1) + v1;
        return v;
    }
    // NS = 1, symbol deferred: advances; returns the state it left (halved address)
    __device__ __forceinline__ uint32_t step_state(const Tab& T) {
        const uint32_t e = T.entry_at(B0);
        const uint32_t b = B0;
        const uint32_t x = window();
        const uint32_t n0 = T.nbf(e);
        p32 -= (int32_t)(n0 & 31u);
        B0 = T.H + T.ns(e) + __builtin_amdgcn_ubfe(x, 0u - n0, n0);
        return b;
    }
    // NS = 1: one symbol; returns it
    __device__ __forceinline__ uint32_t step(const Tab& T) {
        const uint32_t e = T.entry_at(B0);
        const uint32_t y = T.sym_at(B0);
        const uint32_t x = window();
        const uint32_t n0 = T.nbf(e);
        p32 -= (int32_t)(n0 & 31u);
        B0 = T.H + T.ns(e) + __builtin_amdgcn_ubfe(x, 0u - n0, n0);
        return y;
    }
};

template <int LMAX, uint32_t K, int NS, bool DEF = false, uint32_t DW = 1>
__global__ __launch_bounds__(64 * (DW + 1)) void serial_ring_kernel(DecParams P) {
    static_assert(LMAX <= 12, "entry layout ns << 18: e >> 16 is the next entry's byte offset");
    static_assert(K >= 1 && K <= 64, "one decode lane per block");
    static_assert(!DEF || LMAX <= 11, "deferred symbols: L <= 11");
    static_assert(K % DW == 0, "DW decode waves of K / DW lanes each");
    constexpr uint32_t NT = 64u * (DW + 1u), KW = K / DW;
    constexpr uint32_t NBW = LMAX <= 11 ? 5u : 4u;  // nb | newState << NBW fits 16 bits
    constexpr uint32_t TW = 1u << LMAX;
    // u16 entries of the K blocks, then their u8 symbols (DEF: entries only;
    // the symbols are looked up by sym_map_kernel and, for the few end-of-block
    // steps, in the prebuilt u32 table in HBM)
    __shared__ __attribute__((aligned(16))) uint8_t tab_all[K * (DEF ? 2u : 3u) * TW];
    __shared__ uint32_t ring_all[K * RING_STRIDE];
    __shared__ int32_t ctl_all[K][2];  // [0] lowest word landed, [1] highest word the decoder may still read; INT32_MIN = stop
    __shared__ uint32_t any_nb[K];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint64_t gb0 = (uint64_t)blockIdx.x * K;
    if (tid < K) {
        const uint64_t gb = gb0 + tid;
        int32_t nw = 0;
        if (gb < P.n_blocks && P.dtinfo[gb] >= 0) nw = (int32_t)((P.comp_len[gb] + 3u) >> 2);
        ctl_all[tid][0] = nw;  // nothing landed yet
        ctl_all[tid][1] = nw;
        any_nb[tid] = 0;
    }
    __syncthreads();
    for (uint32_t j = 0; j < K; ++j) {  // stage the prebuilt tables (dtable_blocks_kernel)
        const uint64_t gb = gb0 + j;
        if (gb >= P.n_blocks) break;
        const int32_t info = P.dtinfo[gb];
        if (info < 0) continue;
        const uint32_t nv = (1u << ((uint32_t)info >> 16)) >> 2;
        const uint4* t4 = reinterpret_cast<const uint4*>(P.dt + gb * (uint64_t)TW);
        uint8_t* tb = tab_all + j * 2u * TW;         // entries
        uint8_t* sb = tab_all + K * 2u * TW + j * TW;  // symbols
        uint32_t nbor = 0;
        for (uint32_t i = tid; i < nv; i += NT) {
            const uint4 q = t4[i];
            // nb | ns << NBW (ns = e >> 18; bits 16, 17 of e are clear) and the
            // symbols, 4 entries at a time
            auto c16 = [](uint32_t e) { return (e & 0xFu) | ((e >> (18u - NBW)) & ~((1u << NBW) - 1u)); };
            reinterpret_cast<uint2*>(tb)[i] =
                make_uint2(c16(q.x) | (c16(q.y) << 16), c16(q.z) | (c16(q.w) << 16));
            if (!DEF)
                reinterpret_cast<uint32_t*>(sb)[i] =
                    __builtin_amdgcn_perm(__builtin_amdgcn_perm(q.w, q.z, 0x0c0c0501u),
                                          __builtin_amdgcn_perm(q.y, q.x, 0x0c0c0501u), 0x05040100u);
            nbor |= (q.x | q.y | q.z | q.w) & 0xFFu;
        }
        if (nbor) atomicOr(&any_nb[j], 1u);
    }
    __syncthreads();

    if (tid >= 64u * DW) {  // the last wave: the loader, for all K rings (wave-uniform control)
        int32_t k[K], nwj[K];
        const uint32_t* wj[K];
        uint32_t act = 0;
#pragma unroll
        for (uint32_t j = 0; j < K; ++j) {
            nwj[j] = ctl_all[j][1];
            k[j] = (nwj[j] - 1) / (int32_t)RING_CHUNK;
            wj[j] = reinterpret_cast<const uint32_t*>(P.in + (gb0 + j) * P.slot_bytes);
            if (nwj[j] > 0) act |= 1u << j;
        }
        // one sweep: every ring's chunk loads are issued before the first
        // ring write waits on them (a sweep that waited ring by ring took
        // ~K load latencies, near a chunk's decode time at K = 8)
        constexpr uint32_t NQ = RING_WORDS / RING_CHUNK;
        while (act) {
            uint32_t v[K][NQ];
            int32_t k1s[K];
            uint32_t mv = 0;
#pragma unroll
            for (uint32_t j = 0; j < K; ++j) {
                k1s[j] = k[j];
                if (!(act & (1u << j))) continue;
                const int32_t need = lds_load_volatile(&ctl_all[j][1]);
                if (need == INT32_MIN) {  // the decoder is done (or failed)
                    act &= ~(1u << j);
                    continue;
                }
                // chunk c may overwrite the slots of words 64c + RING_WORDS..: dead once above `need`
                int32_t k1 = k[j];
                while (k1 >= 0 && k1 > k[j] - (int32_t)NQ && k1 * (int32_t)RING_CHUNK + (int32_t)RING_WORDS > need)
                    --k1;
                if (k1 == k[j]) continue;
                k1s[j] = k1;
#pragma unroll
                for (int32_t q = 0; q < (int32_t)NQ; ++q) {
                    const int32_t wi = (k[j] - q) * (int32_t)RING_CHUNK + (int32_t)lane;
                    v[j][q] = (k[j] - q > k1 && wi < nwj[j]) ? wj[j][wi] : 0u;
                }
                mv |= 1u << j;
            }
#pragma unroll
            for (uint32_t j = 0; j < K; ++j) {
                if (!(mv & (1u << j))) continue;
                const int32_t k1 = k1s[j];
#pragma unroll
                for (int32_t q = 0; q < (int32_t)NQ; ++q)
                    if (k[j] - q > k1) {
                        const uint32_t slot = (uint32_t)((k[j] - q) * (int32_t)RING_CHUNK + (int32_t)lane) & RING_MASK;
                        ring_all[j * RING_STRIDE + slot] = v[j][q];
                        if (slot == 0u) ring_all[j * RING_STRIDE + RING_WORDS] = v[j][q];  // the mirror
                    }
                k[j] = k1;
                if (lane == 0) lds_store_release(&ctl_all[j][0], (k1 + 1) * (int32_t)RING_CHUNK);
                if (k1 < 0) act &= ~(1u << j);
            }
            if (!mv) __builtin_amdgcn_s_sleep(2);
        }
        return;
    }
    const uint32_t jc = (tid >> 6) * KW + lane;  // this lane's chain
    const uint64_t gb = gb0 + jc;
    if (lane >= KW || gb >= P.n_blocks) return;

    // wave 0, lane j < K: the decoder of block gb0 + j
    const uint32_t tab0 = lds_addr(tab_all);  // even (16-byte aligned)
    const RingTab<NBW> T{(tab0 >> 1) + jc * TW, K * 2u * TW + (tab0 >> 1)};
    const uint32_t* const ring = ring_all + jc * RING_STRIDE;
    int32_t* const ctl = ctl_all[jc];
    const int32_t info = P.dtinfo[gb];
    const uint32_t* const dtg = P.dt + gb * (uint64_t)TW;
    auto sym = [&](uint32_t s) -> uint32_t {  // symbol of state s (end-of-block steps)
        if constexpr (DEF) return dte_sym(dtg[s]);
        else return T.symbol(s);
    };
    const uint8_t* in = P.in + gb * P.slot_bytes;
    const uint32_t clen = info >= 0 ? P.comp_len[gb] : 0u;
    const int32_t nw = (int32_t)((clen + 3u) >> 2);
    const bool single = any_nb[jc] == 0u;
    const bool known = P.n_total != 0;
    const uint64_t ooff = gb * (uint64_t)P.block_size;
    const uint32_t n = known ? (uint32_t)min((uint64_t)P.block_size, P.n_total - ooff) : 0u;
    const uint32_t lim = known ? n : P.out_cap;
    uint8_t* out = P.out + ooff;
    int32_t err = info < 0 ? info : FSE_OK;
    if (NS == 2 && err == FSE_OK && known && n < 2) err = FSE_ERR_LENGTH_MISMATCH;
    // 2-state: a single-symbol table never ends in the reference (refused up
    // front); 1-state: as decode1_serial_kernel, at the capacity
    if (NS == 2 && err == FSE_OK && !known && single) err = FSE_ERR_SINGLE_SYMBOL;
    const int32_t hdr_bits = (info & 0xFFFF) * 8;
    const uint32_t L = (uint32_t)info >> 16;
    uint32_t o = 0, o_bulk = 0;
    // DEF: pair p's states at st_out[p], i.e. 2 bytes per output byte
    uint32_t* const st_out = DEF ? P.states + gb * (uint64_t)P.block_size / 2u : nullptr;
    int32_t top = 0;
    if (err == FSE_OK) {
        top = (int32_t)(clen - 1u) * 8 + (int32_t)ilog2u(in[clen - 1]);  // marker (BitStackReader::new)
        if (top - NS * (int32_t)L < hdr_bits) err = FSE_ERR_TOO_SHORT;  // lib.rs:197 / 224-225 unwrap
    }
    if (err == FSE_OK) {
        int32_t avail = nw;
        auto wait_words = [&](int32_t wlow) {  // words >= max(wlow, 0) have landed
            wlow = max(wlow, 0);
            while (avail > wlow) {
                avail = lds_load_acquire(&ctl[0]);
                if (avail > wlow) __builtin_amdgcn_s_sleep(1);
            }
        };
        // bits [p, p + 32) via the ring (end-of-block steps)
        auto bits_at = [&](int32_t p) -> uint32_t {
            const uint32_t wi = (uint32_t)p >> 5;
            return __builtin_amdgcn_alignbit(ring[(wi + 1u) & RING_MASK], ring[wi & RING_MASK], (uint32_t)p);
        };
        wait_words((top - NS * (int32_t)L) >> 5);
        const uint32_t s0i = bits_at(top - (int32_t)L) & ((1u << L) - 1u);
        const uint32_t s1i = NS == 2 ? bits_at(top - 2 * (int32_t)L) & ((1u << L) - 1u) : 0u;
        RingChain<NS, NBW> c;
        c.init(lds_addr(ring), T, top - NS * (int32_t)L, s0i, s1i);
        const uint32_t I = P.ckpt_interval;
        uint64_t* rec = (P.sidecar_out && I) ? P.sidecar_out + gb * P.ckpt_per_block : nullptr;
        // checkpoint before pair (NS = 2) / symbol (NS = 1) pidx: bit position
        // and the states, as the encoder records them
        uint32_t pidx = 0, next_ck = rec && P.ckpt_per_block ? 0u : 0xFFFFFFFFu, ck = 0;
        auto record_at = [&](int32_t p, uint32_t s0, uint32_t s1) {  // one compare per step when idle
            if (pidx == next_ck) {
                rec[ck++] = (uint64_t)(uint32_t)(p - hdr_bits) | ((uint64_t)s0 << 32) |
                            (NS == 2 ? (uint64_t)s1 << 48 : 0ull);
                next_ck = ck < P.ckpt_per_block ? next_ck + I : 0xFFFFFFFFu;
            }
        };
        // bulk: 2GS output bytes (GS pairs / 2GS symbols, <= 2GS L bits) without
        // end checks; the checkpoint compare is compiled in only when recording.
        // GS = RING_GROUP with the symbols deferred, RING_GROUP_SYM otherwise
        // (both 32: the loop's control is paid once per 32 pairs)
        constexpr uint32_t GS = DEF ? RING_GROUP : RING_GROUP_SYM;
        auto bulk = [&](auto rec_on) {
            constexpr bool REC = decltype(rec_on)::value;
            auto record = [&]() {
                if (REC) record_at(c.pos(), c.s0(T), c.s1(T));
            };
            while (o + 2u * GS + 2u < lim && c.pos() - hdr_bits >= 2 * (int32_t)GS * (int32_t)L) {
                wait_words((c.pos() - 32 - 2 * (int32_t)GS * (int32_t)L) >> 5);
                // DEF: the states of 2GS symbols, 2 bytes per output byte; else
                // the 2GS symbols themselves
                uint32_t v[DEF ? GS : GS / 2u];
                if constexpr (DEF) {
#pragma unroll
                    for (uint32_t j = 0; j < GS; ++j) {
                        if constexpr (NS == 2) {
                            v[j] = c.pair_states(T);
                        } else {
                            const uint32_t a = c.step_state(T);
                            v[j] = __builtin_amdgcn_perm(c.step_state(T), a, 0x05040100u);
                        }
                    }
                } else if constexpr (NS == 2) {
#pragma unroll
                    for (uint32_t j = 0; j < GS; j += 2u) {
                        record();
                        const uint32_t lo = c.pair(T);
                        ++pidx;
                        record();
                        const uint32_t hi = c.pair(T);
                        ++pidx;
                        v[j >> 1] = lo | (hi << 16);
                    }
                } else {
#pragma unroll
                    for (uint32_t j = 0; j < GS / 2u; ++j) {
                        uint32_t y = 0;
#pragma unroll
                        for (uint32_t q = 0; q < 4u; ++q) {
                            record();
                            y |= c.step(T) << (8u * q);
                            ++pidx;
                        }
                        v[j] = y;
                    }
                }
                uint4* sp = DEF ? reinterpret_cast<uint4*>(st_out + (o >> 1)) : reinterpret_cast<uint4*>(out + o);
#pragma unroll
                for (uint32_t q = 0; q < (DEF ? GS : GS / 2u) / 4u; ++q)
                    sp[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
                o += 2u * GS;
                lds_store_volatile(&ctl[1], c.pos() >> 5);  // the highest word a later step reads
            }
        };
        if (DEF) bulk(std::false_type{});  // (never with a sidecar to record)
        else if (rec) bulk(std::true_type{});
        else bulk(std::false_type{});
        o_bulk = o;
        // the tail reads words <= pos/32 + 1, and it ends within 2GS L bits
        // (bulk stopped by the position) or within 2GS + 2 symbols (stopped by
        // the output limit): wait for just those words, the loader cannot pass
        // the ring's words above what the decoder still reads
        lds_store_volatile(&ctl[1], (c.pos() >> 5) + 1);
        wait_words(max(hdr_bits, c.pos() - (2 * (int32_t)GS + 4) * (int32_t)L) >> 5);
        uint32_t s0 = c.s0(T), s1 = c.s1(T);
        int32_t pos = c.pos();
        auto pop = [&](uint32_t nb) -> uint32_t {
            pos -= (int32_t)nb;
            return bits_at(pos) & ((1u << nb) - 1u);
        };
        if constexpr (NS == 2) {
            // tail: pair by pair with the reference's end checks (lib.rs:227-244)
            const int32_t full = known ? FSE_ERR_LENGTH_MISMATCH : FSE_ERR_DST_TOO_SMALL;
            for (;; ++pidx) {
                record_at(pos, s0, s1);
                if (known && o + 2u >= n) {
                    if (o < n) out[o++] = (uint8_t)sym(s0);
                    if (o < n) out[o++] = (uint8_t)sym(s1);
                    break;
                }
                uint32_t nb = T.nb(s0);
                if (pos - (int32_t)nb < hdr_bits) {  // decoder 0 cannot read: lib.rs:242-243
                    if (o + 2u > lim) { err = full; break; }
                    out[o++] = (uint8_t)sym(s0);
                    out[o++] = (uint8_t)sym(s1);
                    break;
                }
                const uint32_t y0 = sym(s0);
                s0 = T.next_base(s0) + pop(nb);
                if (o >= lim) { err = full; break; }
                out[o++] = (uint8_t)y0;
                nb = T.nb(s1);
                if (pos - (int32_t)nb < hdr_bits) {  // decoder 1 cannot read: lib.rs:235-239
                    if (o + 2u > lim) { err = full; break; }
                    out[o++] = (uint8_t)sym(s1);
                    out[o++] = (uint8_t)sym(s0);
                    break;
                }
                const uint32_t y1 = sym(s1);
                s1 = T.next_base(s1) + pop(nb);
                if (o >= lim) { err = full; break; }
                out[o++] = (uint8_t)y1;
            }
            if (err == FSE_OK && known && o != n) err = FSE_ERR_LENGTH_MISMATCH;
        } else {
            // tail: symbol by symbol (lib.rs:198-208), then Decoder::finish.  A
            // single-symbol table never fails a read (the reference loops
            // forever); with the raw length known it ends at n - 1 symbols.
            for (;; ++pidx) {
                if (known && single && o + 1u >= n) break;
                record_at(pos, s0, 0u);
                const uint32_t nb = T.nb(s0);
                if (pos - (int32_t)nb < hdr_bits) break;  // decode_symbol -> None
                if (o >= lim) {  // a single-symbol table never ends in the reference (the oracle
                                 // refuses it up front); any other stream simply needs more room
                    err = single ? FSE_ERR_SINGLE_SYMBOL : FSE_ERR_DST_TOO_SMALL;
                    break;
                }
                const uint32_t y = sym(s0);
                s0 = T.next_base(s0) + pop(nb);
                out[o++] = (uint8_t)y;
            }
            if (err == FSE_OK) {
                if (o >= lim) err = FSE_ERR_DST_TOO_SMALL;
                else out[o++] = (uint8_t)sym(s0);  // Decoder::finish (lib.rs:208)
            }
            if (known && (err == FSE_ERR_DST_TOO_SMALL || (err == FSE_OK && o != n))) err = FSE_ERR_LENGTH_MISMATCH;
        }
    }
    lds_store_volatile(&ctl[1], INT32_MIN);  // release the loader
    if (DEF)  // every block, so sym_map_kernel never reads a stale length
        reinterpret_cast<uint2*>(P.bulk)[gb] = make_uint2(err == FSE_OK ? o_bulk : 0u, T.H & (TW - 1u));
    P.status[gb] = err;
    if (P.out_len) P.out_len[gb] = err ? 0u : o;
}

// ------------------------------------------------------------------------
// Deferred symbols (serial_ring_kernel<..., DEF = true>): the chains wrote the
// state pair of each pair (low 16 bits of the halved entry addresses) instead
// of its two symbols, so their LDS holds u16 entries only (4 KiB per chain at
// L <= 11: 8 chains per 37 KB workgroup, 32 per CU instead of 24).  Here one
// workgroup per block stages the block's symbol column (dte_sym of the
// prebuilt u32 table) in LDS and maps the bulk's states to bytes: 2 bytes
// read and 1 written per output byte, fully parallel.  The chains' end-of-
// block steps wrote their bytes directly, above the bulk length.
// ------------------------------------------------------------------------
template <int LMAX>
__global__ __launch_bounds__(256) void sym_map_kernel(DecParams P) {
    constexpr uint32_t TW = 1u << LMAX, M = TW - 1u;
    __shared__ uint8_t sy[TW];
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    const uint2 bk = reinterpret_cast<const uint2*>(P.bulk)[gb];
    const int32_t info = P.dtinfo[gb];
    const uint64_t ooff = gb * (uint64_t)P.block_size;
    const uint32_t lim = P.n_total ? (uint32_t)min((uint64_t)P.block_size, P.n_total - ooff) : P.out_cap;
    const uint32_t ob = min(bk.x, lim) & ~15u;  // the bulk is whole 16-byte groups
    if (info < 0 || ob == 0) return;
    const uint32_t tid = threadIdx.x;
    const uint32_t nst = 1u << min((uint32_t)info >> 16, (uint32_t)LMAX);
    const uint32_t* dtg = P.dt + gb * (uint64_t)TW;
    for (uint32_t i = tid; i < nst; i += 256u) sy[i] = (uint8_t)dte_sym(dtg[i]);
    __syncthreads();
    const uint32_t h = bk.y;
    auto two = [&](uint32_t w) { return (uint32_t)sy[(w - h) & M] | ((uint32_t)sy[((w >> 16) - h) & M] << 8); };
    const uint4* src = reinterpret_cast<const uint4*>(P.states + ooff / 2u);
    uint4* dst = reinterpret_cast<uint4*>(P.out + ooff);
    const uint32_t ng = ob >> 4;  // 16 output bytes = 8 pairs = 2 x uint4 of states
#pragma unroll 2
    for (uint32_t i = tid; i < ng; i += 256u) {
        const uint4 a = src[2u * i], b = src[2u * i + 1u];
        dst[i] = make_uint4(two(a.x) | (two(a.y) << 16), two(a.z) | (two(a.w) << 16), two(b.x) | (two(b.y) << 16),
                            two(b.z) | (two(b.w) << 16));
    }
}

// ------------------------------------------------------------------------
// One stream, as fast as one serial chain goes: the host fse_decompress2 /
// fse_decompress (lib.rs:187-248) in the reference's own termination.  A
// lone 2-state stream is a single dependency chain (no
// speculative split), so this kernel minimises the latency of one step
// instead of running many chains per CU:
//   - one wave; the chain is wave-uniform, so it runs on the scalar unit
//     (SGPRs) and never waits on a VGPR round trip;
//   - the bulk reads the table through the scalar cache: fused 64-bit
//     entries (single_ftab_kernel) whose low word is at once the s_bfe_u64
//     operand of the state's bits and the window update, both entries of a
//     pair loaded at an SGPR byte offset and awaited together;
//   - the payload is read from global memory 64 words at a time (one per
//     lane), the next chunk in flight while the current one is consumed; the
//     64-bit window refills from a word taken (v_readlane) one refill ahead,
//     so neither an LDS nor a memory latency is on the chain, and there is no
//     staging phase and no size limit;
//   - the bulk runs 32 pairs (64 symbols) between end checks; each step's
//     entry is parked in a VGPR lane (v_writelane at a constant lane) while
//     the next pair's loads are in flight, and the 64 lanes then store their
//     symbols at once;
//   - the checked tail and the single-symbol test read the table from VGPRs
//     (32 registers: entry s is lane s & 63 of register s >> 6).
// Measured per 64 KiB call (tools/host_latency.py): 3.0-3.6 ms with the
// table in VGPRs (a dependent v_readlane lookup, ~41 cycles) and the payload
// staged in LDS; 2.8 ms with plain scalar loads of the u32 entries; 2.1 ms
// with the fused entries (profiles/r04/single_stream/).
// ------------------------------------------------------------------------

// The table in registers: entry of state s (wave-uniform s)
template <uint32_t NV>
__device__ __forceinline__ uint32_t vtab_at(const uint32_t (&vt)[NV], uint32_t s) {
    return (uint32_t)__builtin_amdgcn_readlane((int)vt[(s >> 6) & (NV - 1u)], (int)(s & 63u));
}
// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>)
template <class F, int... I>
__device__ __forceinline__ void unroll_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void unroll(F&& f) {
    unroll_impl(f, std::make_integer_sequence<int, N>{});
}
// v = lane J of `buf` (a constant lane: no index register)
template <int J>
__device__ __forceinline__ void park(uint32_t& buf, uint32_t v) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(buf) : "s"(v), "i"(J));
}
// lanes J and J + 1 (one asm block: no wait state between the two)
template <int J>
__device__ __forceinline__ void park2(uint32_t& buf, uint32_t a, uint32_t b) {
    asm volatile(
        "v_writelane_b32 %0, %1, %3\n\t"
        "v_writelane_b32 %0, %2, %4"
        : "+v"(buf)
        : "s"(a), "s"(b), "i"(J), "i"(J + 1));
}

// Fused entry of one state, shaped for the scalar unit:
//   lo = nb * 0xFFFF | sym << 24, hi = new_state * 8 (the byte offset of the
//   next entry before its bits: offset = bits * 8 + hi, one s_lshl3_add).
// With `av` the window bits below pos, op = av + lo = (nb << 16) | (av - nb)
// (av >= nb) is at once the s_bfe_u64 operand of the state's bits (offset
// av - nb, width nb; bits 23.. are ignored) and, masked to 16 bits, the new
// av.  Built per call into DecParams::states (2 words per entry).
__global__ __launch_bounds__(256) void single_ftab_kernel(const uint32_t* __restrict__ dt, uint32_t* __restrict__ ft,
                                                           uint32_t tw) {
    dt += (uint64_t)blockIdx.x * tw;  // one workgroup per stream
    ft += (uint64_t)blockIdx.x * 2u * tw;
    for (uint32_t i = threadIdx.x; i < tw; i += blockDim.x) {
        const uint32_t e = dt[i];
        ft[2u * i] = dte_nb(e) * 0xFFFFu | dte_sym(e) << 24;
        ft[2u * i + 1u] = Dte<11>::ns(e) << 3;
    }
}
// One fused step's next offset: bfe(W, op) * 8 + hi (W >> (op & 63) masked
// to (op >> 16) & 127 bits), as two scalar instructions in one asm block
// (the bits go through a fixed register pair: separate asm statements get a
// wait state between them, and the compiler emits a shift and an add for
// the second).  s_bfe and s_lshl3_add write SCC.
__device__ __forceinline__ uint32_t fstep(uint64_t W, uint32_t op, uint32_t hi) {
    uint32_t r;
    asm("s_bfe_u64 s[98:99], %1, %2\n\t"
        "s_lshl3_add_u32 %0, s98, %3"
        : "=s"(r)
        : "s"(W), "s"(op), "s"(hi)
        : "s98", "s99", "scc");
    return r;
}
// The bulk's software pipeline: a step computes its pair's next offsets,
// issues the scalar loads of those entries (fent_issue*: SGPR byte offsets
// into ft, no 64-bit address arithmetic) and parks its own entries in VGPR
// lanes in the same asm block, then refills the window while the loads are
// in flight; the next step starts with fent_wait*.  The compiler does not
// track these loads: the registers they write stay live until the wait that
// names them (so nothing else is put there meanwhile), and `av` is tied to
// the issue and `W`, `av` to the wait so that the refill stays between them.
template <int J>
__device__ __forceinline__ void fent_issue2(uint64_t ft, uint32_t o0, uint32_t o1, uint64_t& f0, uint64_t& f1,
                                            uint32_t& buf, uint32_t a, uint32_t b, uint32_t& av) {
    asm volatile(
        "s_load_dwordx2 %0, %4, %5\n\t"
        "s_load_dwordx2 %1, %4, %6\n\t"
        "v_writelane_b32 %2, %7, %9\n\t"
        "v_writelane_b32 %2, %8, %10"
        : "=&s"(f0), "=&s"(f1), "+v"(buf), "+s"(av)
        : "s"(ft), "s"(o0), "s"(o1), "s"(a), "s"(b), "i"(J), "i"(J + 1));
}
__device__ __forceinline__ void fent_issue2n(uint64_t ft, uint32_t o0, uint32_t o1, uint64_t& f0, uint64_t& f1,
                                             uint32_t& av) {  // no entries to park (the bulk's first pair)
    asm volatile(
        "s_load_dwordx2 %0, %3, %4\n\t"
        "s_load_dwordx2 %1, %3, %5"
        : "=&s"(f0), "=&s"(f1), "+s"(av)
        : "s"(ft), "s"(o0), "s"(o1));
}
__device__ __forceinline__ void fent_wait2(uint64_t& f0, uint64_t& f1, uint64_t& W, uint32_t& av) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(f0), "+s"(f1), "+s"(W), "+s"(av));
}
template <int J>
__device__ __forceinline__ void fent_issue1(uint64_t ft, uint32_t o, uint64_t& f, uint32_t& buf, uint32_t a,
                                            uint32_t& av) {
    asm volatile(
        "s_load_dwordx2 %0, %3, %4\n\t"
        "v_writelane_b32 %1, %5, %6"
        : "=&s"(f), "+v"(buf), "+s"(av)
        : "s"(ft), "s"(o), "s"(a), "i"(J));
}
__device__ __forceinline__ void fent_issue1n(uint64_t ft, uint32_t o, uint64_t& f, uint32_t& av) {
    asm volatile("s_load_dwordx2 %0, %2, %3" : "=&s"(f), "+s"(av) : "s"(ft), "s"(o));
}
__device__ __forceinline__ void fent_wait1(uint64_t& f, uint64_t& W, uint32_t& av) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(f), "+s"(W), "+s"(av));
}

template <int NS>
__global__ __launch_bounds__(64) void single_decode_kernel(DecParams P) {
    constexpr uint32_t LMAX = 11, TW = 1u << LMAX, NV = TW / 64u;
    const uint32_t lane = threadIdx.x;
    // one wave per stream: stream gb at P.in + gb * slot_bytes, its table at
    // P.dt + gb * 2^11 words, fused at P.states + gb * 2^12 words, its output
    // at P.out + gb * block_size
    const uint64_t gb = blockIdx.x;
    if (gb >= P.n_blocks) return;
    const int32_t info = P.dtinfo[gb];
    const uint32_t clen = P.comp_len[gb];
    int32_t err = info < 0 ? info : FSE_OK;
    const uint32_t L = err == FSE_OK ? (uint32_t)info >> 16 : 0u;
    // table into VGPRs; OR of the valid entries' nb: 0 = single-symbol table
    uint32_t vt[NV];
    uint32_t nbor = 0;
    {
        const uint32_t size = 1u << L;
#pragma unroll
        for (uint32_t k = 0; k < NV; ++k) {
            vt[k] = P.dt[gb * TW + k * 64u + lane];
            if (k * 64u + lane < size) nbor |= vt[k] & 0xFFu;
        }
    }
    const bool single = __ballot(nbor != 0u) == 0ull;
    uint8_t* out = P.out + gb * P.block_size;
    const uint32_t cap = P.out_cap;
    if (err == FSE_OK && single) err = FSE_ERR_SINGLE_SYMBOL;  // the reference never ends such a stream
    if (err != FSE_OK) {
        if (lane == 0) {
            P.status[gb] = err;
            if (P.out_len) P.out_len[gb] = 0;
        }
        return;
    }
    const uint32_t* in32 = reinterpret_cast<const uint32_t*>(P.in + gb * P.slot_bytes);
    const int32_t last = (int32_t)((clen - 1u) >> 2);  // the payload's last word
    // 64 payload words from word c on, one per lane.  Words below word 0 are
    // never consumed (bits below the header are not read), so the index is
    // only clamped into the buffer: an unconditional load straight into its
    // register, awaited only when the chunk is used.
    auto chunk = [&](int32_t c) -> uint32_t { return in32[min(max(c + (int32_t)lane, 0), last)]; };
    const int32_t hdr_bits = (info & 0xFFFF) * 8;
    const uint32_t lastw = (uint32_t)__builtin_amdgcn_readfirstlane((int)in32[last]);
    const uint32_t lastb = (lastw >> (8u * ((clen - 1u) & 3u))) & 0xFFu;  // non-zero: checked by the table build
    const int32_t pos0 = (int32_t)(clen - 1u) * 8 + (int32_t)(31u - (uint32_t)__builtin_clz(lastb));  // the marker
    // window W: bits [base, base + 64) of the stream, base = 32 * (cb + li + 1);
    // av = pos - base bits below pos.  cur holds words [cb, cb + 64), pre the
    // 64 below (in flight); nxt = word cb + li, the next one into the window.
    const int32_t wb = (((pos0 + 31) & ~31) - 64) >> 5;  // the window's low word (>= -2)
    int32_t cb = wb + 1 - 63;
    uint32_t cur = chunk(cb);
    uint32_t pre = chunk(cb - 64);
    int32_t li = wb - 1 - cb;
    auto lane_word = [&](int32_t l) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)cur, l); };
    uint64_t W = (uint64_t)lane_word(wb - cb) | ((uint64_t)lane_word(wb + 1 - cb) << 32);
    uint32_t nxt = lane_word(li);
    uint32_t av = (uint32_t)(pos0 - 32 * wb);
    auto bitpos = [&]() -> int32_t { return 32 * (cb + li + 1) + (int32_t)av; };
    auto shift_in = [&]() {  // one word into the window (av < 32 before)
        W = (W << 32) | nxt;
        av += 32u;
        if (li == 0) {  // the chunk below becomes current; the next one is requested
            // the copy first, then the load into the register pre frees (a load
            // into a temporary would be copied, and awaited, at once)
            asm volatile("v_mov_b32 %0, %1" : "=&v"(cur) : "v"(pre) : "memory");
            cb -= 64;
            pre = chunk(cb - 64);
            li = 64;
        }
        --li;
        nxt = lane_word(li);
    };
    auto refill = [&]() {  // keep >= 32 bits below pos in the window
        if (av < 32u) shift_in();
    };
    auto pop = [&](uint32_t nb) -> uint32_t {
        av -= nb;
        return (uint32_t)(W >> av) & ((1u << nb) - 1u);
    };
    const uint64_t ft = (uint64_t)(P.states + gb * 2u * TW);
    uint32_t o = 0;  // bytes decoded
    uint32_t eb = 0;  // the round's 64 entries, one per lane
    auto put64 = [&]() {  // the round's symbols (fused entries: sym in bits 24..31)
        out[o + lane] = (uint8_t)(eb >> 24);
        o += 64u;
    };
    auto put1 = [&](uint32_t sym) {  // one byte (the checked tail)
        if (lane == 0) out[o] = (uint8_t)sym;
        ++o;
    };
    const int32_t full = FSE_ERR_DST_TOO_SMALL;
    if (NS == 2) {
        if (bitpos() - 2 * (int32_t)L < hdr_bits) {
            err = FSE_ERR_TOO_SHORT;  // lib.rs:224-225 unwrap
        } else {
            uint32_t s0 = pop(L);
            refill();
            uint32_t s1 = pop(L);
            refill();
            // bulk: rounds of 32 pairs that can neither run out of bits (<= 2L
            // a pair) nor reach the capacity: no end checks
            for (;;) {
                const uint32_t by_bits = (uint32_t)(bitpos() - hdr_bits) / (64u * L);
                const uint32_t by_cap = cap > o + 66u ? (cap - o - 2u) / 64u : 0u;
                uint32_t g = min(by_bits, by_cap);
                if (g == 0u) break;
                uint32_t x0 = s0 << 3, x1 = s1 << 3;  // the states as byte offsets into ft
                uint64_t fa0, fa1, fb0, fb1;  // entries of even / odd steps
                fent_issue2n(ft, x0, x1, fa0, fa1, av);
                for (; g; --g) {
                    auto step = [&](auto J) {
                        constexpr int j = decltype(J)::value;
                        uint64_t& c0 = (j & 1) ? fb0 : fa0;
                        uint64_t& c1 = (j & 1) ? fb1 : fa1;
                        uint64_t& n0 = (j & 1) ? fa0 : fb0;
                        uint64_t& n1 = (j & 1) ? fa1 : fb1;
                        fent_wait2(c0, c1, W, av);
                        uint32_t op = av + (uint32_t)c0;
                        x0 = fstep(W, op, (uint32_t)(c0 >> 32));
                        op = (op & 0xFFFFu) + (uint32_t)c1;
                        x1 = fstep(W, op, (uint32_t)(c1 >> 32));
                        av = op & 0xFFFFu;
                        fent_issue2<2 * j>(ft, x0, x1, n0, n1, eb, (uint32_t)c0, (uint32_t)c1, av);
                        refill();  // a pair takes <= 2L = 22 bits, a refill leaves >= 32
                    };
                    unroll<32>(step);
                    put64();
                }
                fent_wait2(fa0, fa1, W, av);  // the loads issued after the last pair
                s0 = x0 >> 3;
                s1 = x1 >> 3;
            }
            // tail: pair by pair with the reference's end checks (lib.rs:227-243)
            for (;;) {
                const uint32_t e0 = vtab_at(vt, s0);
                uint32_t nb = dte_nb(e0);
                if (bitpos() - (int32_t)nb < hdr_bits) {  // decoder 0 cannot read
                    if (o + 2u > cap) { err = full; break; }
                    put1(dte_sym(e0));
                    put1(dte_sym(vtab_at(vt, s1)));
                    break;
                }
                s0 = Dte<LMAX>::ns(e0) + pop(nb);
                refill();
                if (o >= cap) { err = full; break; }
                put1(dte_sym(e0));
                const uint32_t e1 = vtab_at(vt, s1);
                nb = dte_nb(e1);
                if (bitpos() - (int32_t)nb < hdr_bits) {  // decoder 1 cannot read
                    if (o + 2u > cap) { err = full; break; }
                    put1(dte_sym(e1));
                    put1(dte_sym(vtab_at(vt, s0)));
                    break;
                }
                s1 = Dte<LMAX>::ns(e1) + pop(nb);
                refill();
                if (o >= cap) { err = full; break; }
                put1(dte_sym(e1));
            }
        }
    } else {
        if (bitpos() - (int32_t)L < hdr_bits) {
            err = FSE_ERR_TOO_SHORT;  // lib.rs:197 unwrap
        } else {
            uint32_t s = pop(L);
            refill();
            for (;;) {  // bulk: rounds of 64 symbols, no end checks
                const uint32_t by_bits = (uint32_t)(bitpos() - hdr_bits) / (64u * L);
                const uint32_t by_cap = cap > o + 65u ? (cap - o - 1u) / 64u : 0u;
                uint32_t g = min(by_bits, by_cap);
                if (g == 0u) break;
                uint32_t x = s << 3;
                uint64_t fa, fb;  // entries of even / odd steps
                fent_issue1n(ft, x, fa, av);
                for (; g; --g) {
                    auto step = [&](auto J) {
                        constexpr int j = decltype(J)::value;
                        uint64_t& c = (j & 1) ? fb : fa;
                        uint64_t& nx = (j & 1) ? fa : fb;
                        fent_wait1(c, W, av);
                        const uint32_t op = av + (uint32_t)c;
                        x = fstep(W, op, (uint32_t)(c >> 32));
                        av = op & 0xFFFFu;
                        fent_issue1<j>(ft, x, nx, eb, (uint32_t)c, av);
                        if (j & 1) refill();  // two symbols take <= 2L = 22 bits
                    };
                    unroll<64>(step);
                    put64();
                }
                fent_wait1(fa, W, av);
                s = x >> 3;
            }
            for (;;) {  // lib.rs:198-207 with the read check, then finish (208)
                const uint32_t e = vtab_at(vt, s);
                const uint32_t nb = dte_nb(e);
                if (bitpos() - (int32_t)nb < hdr_bits) break;
                if (o >= cap) { err = full; break; }
                s = Dte<LMAX>::ns(e) + pop(nb);
                refill();
                put1(dte_sym(e));
            }
            if (err == FSE_OK) {
                if (o >= cap) err = full;
                else put1(dte_sym(vtab_at(vt, s)));
            }
        }
    }
    if (lane == 0) {
        P.status[gb] = err;
        if (P.out_len) P.out_len[gb] = err ? 0u : o;
    }
}

// P.n_blocks streams, one wave each (P.states: 2^12 words of fused table per stream)
hipError_t launch_single(const DecParams& P, uint32_t lmax, hipStream_t stream) {
    if (!P.dt || !P.dtinfo || !P.states || P.n_total || P.sidecar || P.sidecar_out || P.n_blocks == 0 || lmax > 11)
        return hipErrorInvalidValue;
    const dim3 g(P.n_blocks);
    hipLaunchKernelGGL(single_ftab_kernel, g, dim3(256), 0, stream, P.dt, P.states, 2048u);
    if (P.nstates == 1) hipLaunchKernelGGL((single_decode_kernel<1>), g, dim3(64), 0, stream, P);
    else hipLaunchKernelGGL((single_decode_kernel<2>), g, dim3(64), 0, stream, P);
    return hipGetLastError();
}

// ------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------
hipError_t launch_decode(const DecParams& P, uint32_t lmax, hipStream_t stream) {
    const dim3 g(P.n_blocks);
    if (!P.dt || !P.dtinfo) return hipErrorInvalidValue;
    if (!P.sidecar) {  // serial: sidecar-less blocks, reference-mode host streams, sidecar recording
        if (P.nstates == 1) {
            if (lmax <= 11 && P.states && P.bulk && !P.sidecar_out) {  // symbols deferred, as below
                hipLaunchKernelGGL((serial_ring_kernel<11, 8, 1, true>), dim3((P.n_blocks + 7u) / 8u), dim3(128), 0, stream, P);
                hipLaunchKernelGGL((sym_map_kernel<11>), dim3(P.n_blocks), dim3(256), 0, stream, P);
            } else if (lmax <= 11) hipLaunchKernelGGL((serial_ring_kernel<11, 6, 1>), dim3((P.n_blocks + 5u) / 6u), dim3(128), 0, stream, P);
            else if (lmax <= 12) hipLaunchKernelGGL((serial_ring_kernel<12, 3, 1>), dim3((P.n_blocks + 2u) / 3u), dim3(128), 0, stream, P);
            else if (lmax <= 13) hipLaunchKernelGGL((decode1_serial_kernel<13>), g, dim3(64), 0, stream, P);
            else if (lmax <= 14) hipLaunchKernelGGL((decode1_serial_kernel<14>), g, dim3(64), 0, stream, P);
            else hipLaunchKernelGGL((decode1_serial_kernel<15>), g, dim3(64), 0, stream, P);
        } else if (lmax <= 11 && P.states && P.bulk && !P.sidecar_out) {
            // symbols deferred: 8 blocks per workgroup, 32 chains per CU, then the map
            hipLaunchKernelGGL((serial_ring_kernel<11, 8, 2, true>), dim3((P.n_blocks + 7u) / 8u), dim3(128), 0, stream, P);
            hipLaunchKernelGGL((sym_map_kernel<11>), dim3(P.n_blocks), dim3(256), 0, stream, P);
        } else {
            // 6 (L <= 11) or 3 (L = 12) blocks per workgroup: 24 / 12 chains per CU (LDS-bound)
            if (lmax <= 11) hipLaunchKernelGGL((serial_ring_kernel<11, 6, 2>), dim3((P.n_blocks + 5u) / 6u), dim3(128), 0, stream, P);
            else if (lmax <= 12) hipLaunchKernelGGL((serial_ring_kernel<12, 3, 2>), dim3((P.n_blocks + 2u) / 3u), dim3(128), 0, stream, P);
            else if (lmax <= 13) hipLaunchKernelGGL((serial2_decode_kernel<13>), g, dim3(64), 0, stream, P);
            else if (lmax <= 14) hipLaunchKernelGGL((serial2_decode_kernel<14>), g, dim3(64), 0, stream, P);
            else hipLaunchKernelGGL((serial2_decode_kernel<15>), g, dim3(64), 0, stream, P);
        }
        return hipGetLastError();
    }
    // segment-parallel, in two passes: the 44 KiB stage (36 KiB at L = 12;
    // 3 workgroups per CU) for the blocks it holds, then a list pass with a
    // 66 KiB stage (2 per CU) for the deferred ones (near-uniform data,
    // ~65 KB).  Blocks above that use the windowed global-memory reader; at
    // L 13..15 (table 128 KiB) every block does.
    // PB12: the L = 12 list pass's stage, the most that keeps 2 workgroups per
    // CU beside its 16 KiB table (near-uniform blocks at L = 12, ~65.3 KB,
    // fit; 1 per CU with a 66 KiB stage)
#ifndef FSE_DEC_PP
#define FSE_DEC_PP (44u << 10)  // a variant build may lower it (occupancy probes)
#endif
    constexpr uint32_t PP = FSE_DEC_PP, PB = 66u << 10, PB12 = 65392u;
    // PS14: the small first stage at L = 14 (2 workgroups per CU beside the
    // 64 KiB table)
    constexpr uint32_t PS14 = 12u << 10;
    static const uint32_t cus = [] {
        int dev = 0, n = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        return (uint32_t)n;
    }();
    // per_cu: workgroups per CU of a list pass (grid = one per slot on the chip)
    auto run = [&](auto kern, uint32_t pass, uint32_t per_cu, uint32_t nt = 256u) {
        DecParams Q = P;
        Q.pass = pass;
        const dim3 gq(pass <= 1 ? P.n_blocks : std::min<uint32_t>(P.n_blocks, per_cu * cus));
        hipLaunchKernelGGL(kern, gq, dim3(nt), 0, stream, Q);
    };
    // blocks with more than 256 segments (checkpoints every <= 64 pairs or
    // 128 symbols at 64 KiB): 512-thread workgroups, one segment per thread --
    // the same LDS per block, more waves per CU
    const uint32_t bs = P.block_size;
    // main-loop steps of a full block: pairs (2-state) or symbols (1-state)
    const uint32_t pm = bs < 2u ? 0u : P.nstates == 1 ? bs - 1u : (bs & 1u) ? (bs - 3u) / 2u : bs / 2u - 1u;
    const uint32_t nseg = pm / std::max(P.ckpt_interval, 1u) + 1u;
    const bool wide = nseg > 256u;
    if (P.nstates == 1) {
        if (lmax <= 11 && wide) {  // 1-state checkpoints every <= 128 symbols: one segment per thread of 512
            run(decode_pre_kernel<11, PP, 1, 1, 512>, 1, 0, 512);
            run(decode_pre_kernel<11, PB, 1, 2, 512>, 2, 2, 512);
        } else if (lmax <= 11) {
            run(decode_pre_kernel<11, PP, 1, 1>, 1, 0);
            run(decode_pre_kernel<11, PB, 1, 2>, 2, 2);
        } else if (lmax <= 12) {
            run(decode_pre_kernel<12, PP - 8192, 1, 1>, 1, 0);
            run(decode_pre_kernel<12, PB12, 1, 2>, 2, 2);
        } else if (lmax <= 13) {
            run(decode_pre_kernel<13, PP, 1, 1>, 1, 0);
            run(decode_pre_kernel<13, PB, 1, 2>, 2, 1);
        } else if (lmax <= 14) {
            run(decode_pre_kernel<14, PP, 1, 1>, 1, 0);
            run(decode_pre_kernel<14, PB, 1, 2>, 2, 1);
        } else {
            run(decode_pre_kernel<15, 16, 1, 0>, 0, 0);
        }
    } else {
        if (lmax <= 11 && wide) {
            run(decode_pre_kernel<11, PP, 2, 1, 512>, 1, 0, 512);
            run(decode_pre_kernel<11, PB, 2, 2, 512>, 2, 2, 512);
        } else if (lmax <= 11) {
            run(decode_pre_kernel<11, PP, 2, 1>, 1, 0);
            run(decode_pre_kernel<11, PB, 2, 2>, 2, 2);
        } else if (lmax <= 12 && wide) {
            run(decode_pre_kernel<12, PP - 8192, 2, 1, 512>, 1, 0, 512);
            run(decode_pre_kernel<12, PB12, 2, 2, 512>, 2, 2, 512);
        } else if (lmax <= 12) {
            run(decode_pre_kernel<12, PP - 8192, 2, 1>, 1, 0);
            run(decode_pre_kernel<12, PB12, 2, 2>, 2, 2);
        } else if (lmax <= 13 && wide) {  // 32 KiB table: 2 workgroups per CU, the list pass 1
            // (a 16 KiB first stage, 3 per CU, measured a wash: skewed +2.5 %,
            // near-uniform -1 %, profiles/r06/sd/)
            run(decode_pre_kernel<13, PP, 2, 1, 512>, 1, 0, 512);
            run(decode_pre_kernel<13, PB, 2, 2, 512>, 2, 1, 512);
        } else if (lmax <= 13) {
            run(decode_pre_kernel<13, PP, 2, 1>, 1, 0);
            run(decode_pre_kernel<13, PB, 2, 2>, 2, 1);
        } else if (lmax <= 14 && wide) {  // 64 KiB table
            // a 12 KiB stage first (2 workgroups per CU: skewed blocks fit),
            // then the 44 and 66 KiB stages as list passes (1 per CU): C5
            // skewed L = 14 decode 342 -> 368 GiB/s, near-uniform unchanged
            // (profiles/r06/sd/)
            run(decode_pre_kernel<14, PS14, 2, 1, 512>, 1, 0, 512);
            run(decode_pre_kernel<14, PP, 2, 3, 512>, 3, 1, 512);
            run(decode_pre_kernel<14, PB, 2, 2, 512>, 2, 1, 512);
        } else if (lmax <= 14) {
            run(decode_pre_kernel<14, PP, 2, 1>, 1, 0);
            run(decode_pre_kernel<14, PB, 2, 2>, 2, 1);
        } else if (wide) {  // 128 KiB table: 1 workgroup per CU, 8 waves instead of 4
            // (near-uniform C5 L = 15 decode 72.7 -> 77.2 GiB/s, profiles/r06/w15/)
            run(decode_pre_kernel<15, 16, 2, 0, 512>, 0, 0, 512);
        } else {
            run(decode_pre_kernel<15, 16, 2, 0>, 0, 0);
        }
    }
    return hipGetLastError();
}

int occupancy_report_dec(char* buf, int cap) {
    int len = 0;
    auto one = [&](const char* name, const void* k, int threads = 256) {
        int nb = -1;
        hipFuncAttributes fa{};
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, threads, 0);
        (void)hipFuncGetAttributes(&fa, k);
        if (len < cap)
            len += snprintf(buf + len, cap - len, "%s: %d WG/CU (lds %zu B, vgpr %d)\n", name, nb, fa.sharedSizeBytes,
                            fa.numRegs);
    };
    one("decode_pre<11,45056,2,1>", reinterpret_cast<const void*>(decode_pre_kernel<11, 45056u, 2, 1>));
    one("decode_pre<11,45056,2,1,512>", reinterpret_cast<const void*>(decode_pre_kernel<11, 45056u, 2, 1, 512>));
    one("decode_pre<11,67584,2,2>", reinterpret_cast<const void*>(decode_pre_kernel<11, 67584u, 2, 2>));
    one("serial_ring<11,6,2>", reinterpret_cast<const void*>(serial_ring_kernel<11, 6, 2>), 128);
    one("serial_ring<11,8,2,defer>", reinterpret_cast<const void*>(serial_ring_kernel<11, 8, 2, true>), 128);
    one("sym_map<11>", reinterpret_cast<const void*>(sym_map_kernel<11>));
    return len;
}

hipError_t launch_dtables(const DtParams& P0, uint32_t lmax, hipStream_t stream) {
    DtParams P = P0;
    P.peer_ranks = atomic_ranks_on() ? 0u : 1u;
    if (lmax > 12) P.hdr_meta = nullptr;  // the staged rows hold headers up to L = 12
    if (P.hdr_meta && P.hdr_norm) {
        const dim3 gp((P.n_blocks + HP_BLOCKS - 1u) / HP_BLOCKS);
        if (lmax <= 11) hipLaunchKernelGGL((hdr_parse_kernel<11>), gp, dim3(64), 0, stream, P);
        else hipLaunchKernelGGL((hdr_parse_kernel<12>), gp, dim3(64), 0, stream, P);
    } else {
        P.hdr_meta = nullptr;
    }
    const dim3 g(P.n_blocks), b(64);
    if (lmax <= 11) hipLaunchKernelGGL((dtable_blocks_kernel<11>), g, b, P.xlds, stream, P);
    else if (lmax <= 12) hipLaunchKernelGGL((dtable_blocks_kernel<12>), g, b, P.xlds, stream, P);
    else if (lmax <= 13) hipLaunchKernelGGL((dtable_blocks_kernel<13>), g, b, P.xlds, stream, P);
    else if (lmax <= 14) hipLaunchKernelGGL((dtable_blocks_kernel<14>), g, b, P.xlds, stream, P);
    else hipLaunchKernelGGL((dtable_blocks_kernel<15>), g, b, P.xlds, stream, P);
    return hipGetLastError();
}

}  // namespace fsehip
