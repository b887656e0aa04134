// fse_blocks.hip -- the crate's building blocks as gfx950 kernels.
//
//   norm_kernel       Histogram::normalize / normalize_optimal /
//                     NormHistogram::new (histogram.rs:95-155, 264-303)
//   hdr_write_kernel  NormHistogram::write (histogram.rs:376-431)
//   hdr_read_kernel   NormHistogram::read (histogram.rs:436-505)
//   table_kernel      EncodeTable::new / DecodeTable::new (fse.rs:88-189,
//                     269-338) as plain-data tables
//   bits_*            the bitstream (bitstream/*.rs) as batched device
//                     primitives: a device-wide prefix scan of the field
//                     widths gives every field's bit offset, then each thread
//                     packs (BitStackWriter) or extracts (BitStackReader from
//                     the top, BitStreamReader from the bottom) 16 fields.
//
// The table kernels run one wave on one item (the reference's per-call
// granularity); the bitstream kernels are HBM-bound streaming passes.
#include <atomic>
#include <mutex>

#include "fse_device.hpp"
#include "fse_kernels.h"

namespace fsehip {

// Tables of this file's kernels whose atomic ranks failed their check and
// were rebuilt with the peer-mask ranks (wave_build_spread); per device.
__device__ uint32_t g_rank_fb_tab;
hipError_t rank_fallbacks_tab(uint32_t* out, bool reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rank_fb_tab), 4, 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess && reset) {
        const uint32_t z = 0;
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_rank_fb_tab), &z, 4, 0, hipMemcpyHostToDevice);
    }
    return e;
}

// ------------------------------------------------------------------------
// Normalisation: mode 0 = Histogram::normalize(log2), 1 = normalize_optimal
// (optimal_log2 first), 2 = NormHistogram::new from raw bytes.
// ------------------------------------------------------------------------
__global__ __launch_bounds__(64) void norm_kernel(NormArgs A) {
    __shared__ uint32_t hs[HIST_WORDS];
    __shared__ uint32_t counts[256];
    __shared__ int32_t norm[256];
    __shared__ int scratch[4];
    const uint32_t lane = lane_id();
    uint32_t size = A.size, tl = A.table_len;
    if (A.mode == 2) {
        tl = wave_histogram(A.src, (uint32_t)A.n, hs, counts);
        size = (uint32_t)A.n;
    } else {
        for (uint32_t s = lane; s < 256u; s += WAVE) counts[s] = A.counts[s];
        wave_sync();
    }
    int rc = FSE_OK;
    uint32_t Lreq = A.log2, L = 0, slow = 0;
    if (A.mode != 0) {
        if (size == 0) rc = FSE_ERR_EMPTY;  // size.ilog2() (histogram.rs:266)
        else rc = optimal_log2(size, tl, &Lreq);
    }
    if (rc == FSE_OK) rc = wave_normalize(counts, size, tl, Lreq, norm, &L, &slow, scratch);
    wave_sync();
    for (uint32_t s = lane; s < 256u; s += WAVE) A.out->norm[s] = (s < tl && rc == FSE_OK) ? norm[s] : 0;
    if (lane == 0) {
        A.out->log2 = L;
        A.out->table_len = tl;
        if (A.counts_out) {
            A.counts_out[256] = size;
            A.counts_out[257] = tl;
        }
        *A.status = rc;
    }
    if (A.counts_out)
        for (uint32_t s = lane; s < 256u; s += WAVE) A.counts_out[s] = counts[s];
}

// ------------------------------------------------------------------------
// NormHistogram::write: the reference's field loop on one lane (its panic
// on an inconsistent table becomes BAD_TABLE), bytes and the bit count out.
// ------------------------------------------------------------------------
__global__ __launch_bounds__(64) void hdr_write_kernel(const fse_norm_histogram* nh, uint8_t* out, uint32_t* bits,
                                                       int32_t* status) {
    __shared__ uint8_t hdr[HDR_MAX];
    __shared__ int32_t norm[256];
    __shared__ int res[1];
    const uint32_t lane = lane_id();
    for (uint32_t s = lane; s < 256u; s += WAVE) norm[s] = nh->norm[s];
    wave_sync();
    const uint32_t L = nh->log2, tl = nh->table_len;
    if (lane == 0) {
        uint32_t b = 0;
        int r;
        if (L < LOG_MIN || L > LOG_MAX_REF) r = FSE_ERR_TABLELOG_RANGE;  // u32 underflow of log2 - 5
        else if (tl > 256u) r = FSE_ERR_BAD_ARG;
        else r = header_write_lane(norm, L, tl, hdr, &b);
        res[0] = r;
        *bits = r < 0 ? 0u : b;
        *status = r < 0 ? r : FSE_OK;
    }
    wave_sync();
    const int r = res[0];
    for (int i = (int)lane; i < r; i += (int)WAVE) out[i] = hdr[i];
}

// ------------------------------------------------------------------------
// NormHistogram::read of n bytes (the rest of the slice follows the header):
// the wave-uniform scalar parse of the decode tables.  `src` must be
// readable up to HDR_MAX bytes (the host stage pads it).
// ------------------------------------------------------------------------
__global__ __launch_bounds__(64) void hdr_read_kernel(const uint8_t* src, uint32_t n, fse_norm_histogram* out, uint32_t* used,
                                                      int32_t* status) {
    __shared__ int32_t norm[256];
    const uint32_t lane = lane_id();
    const uint32_t* w = reinterpret_cast<const uint32_t*>(src);
    const uint32_t nw = (min(n, HDR_MAX) + 3u) >> 2;
    uint32_t r0 = lane < nw ? w[lane] : 0u, r1 = lane + 64u < nw ? w[lane + 64u] : 0u;
    // bytes past the slice read as nothing: mask the partial last word
    const uint32_t tail = n & 3u;
    if (tail && n <= HDR_MAX) {
        const uint32_t lw = n >> 2, m = (1u << (8u * tail)) - 1u;
        if (lane == lw) r0 &= m;
        if (lane + 64u == lw) r1 &= m;
    }
    for (uint32_t s = lane; s < 256u; s += WAVE) norm[s] = 0;
    wave_sync();
    uint32_t L = 0, tl = 0;
    const int hl = header_read_wave(r0, r1, n, LOG_MAX_REF, norm, &L, &tl);
    wave_sync();
    for (uint32_t s = lane; s < 256u; s += WAVE) out->norm[s] = hl < 0 ? 0 : norm[s];
    if (lane == 0) {
        out->log2 = hl < 0 ? 0u : L;
        out->table_len = hl < 0 ? 0u : tl;
        *used = hl < 0 ? 0u : (uint32_t)hl;
        *status = hl < 0 ? hl : FSE_OK;
    }
}

// ------------------------------------------------------------------------
// EncodeTable::new (enc != 0) / DecodeTable::new as plain data, any L in
// 5..15: the wave spread of the codec kernels with the reference's entry
// formulas (fse.rs:157-188, 329-337).
// ------------------------------------------------------------------------
__global__ __launch_bounds__(64) void table_kernel(const fse_norm_histogram* nh, int enc, fse_encode_table* et, fse_decode_table* dt,
                                                   int32_t* status, uint32_t peer_ranks) {
    constexpr uint32_t SMAX = 1u << LOG_MAX_REF;
    __shared__ __attribute__((aligned(16))) uint8_t sym_at[SMAX];
    __shared__ __attribute__((aligned(16))) uint8_t occ[SMAX];
    __shared__ int32_t norm[256];
    __shared__ uint16_t cumul[256];
    __shared__ uint32_t cnt[256];
    const uint32_t lane = lane_id();
    const uint32_t L = nh->log2, tl = nh->table_len;
    for (uint32_t s = lane; s < 256u; s += WAVE) norm[s] = nh->norm[s];
    wave_sync();
    if (L < LOG_MIN || L > LOG_MAX_REF || tl == 0 || tl > 256u) {  // TABLE_LOG_RANGE assert (fse.rs:103-106)
        if (lane == 0) *status = (tl == 0 || tl > 256u) ? FSE_ERR_BAD_ARG : FSE_ERR_TABLELOG_RANGE;
        return;
    }
    const uint32_t size = 1u << L;
    int rc;
    if (enc) {
        rc = wave_build_spread<64, true>(
            norm, L, tl, sym_at, occ, cumul, cnt,
            [&](uint32_t i, uint32_t s, uint32_t r) {
                et->table[r] = (uint16_t)(size + i);  // fse.rs:157-162 (r = cumul[s] + rank)
                et->symbols[i] = (uint8_t)s;
            },
            [&](uint32_t s) { return (uint32_t)cumul[s]; }, RankAtomic{peer_ranks == 0u, occ, nullptr, 0u, &g_rank_fb_tab, 0u});
        // symbol transforms (fse.rs:165-188); total before symbol s = cumul[s]
        for (uint32_t s = lane; s < 256u; s += WAVE) {
            uint32_t bits = 0;
            int32_t fs = 0;
            const int32_t x = s < tl ? norm[s] : 0;
            if (s < tl) {
                if (x == 0) {
                    bits = ((L + 1u) << 16) - (1u << L);
                } else if (x == -1 || x == 1) {
                    bits = (L << 16) - (1u << L);
                    fs = (int32_t)cumul[s] - 1;
                } else {
                    const uint32_t mb = L - ilog2u((uint32_t)(x - 1));
                    bits = (mb << 16) - ((uint32_t)x << mb);
                    fs = (int32_t)cumul[s] - x;
                }
            }
            et->symbol_tt[s].bits = bits;
            et->symbol_tt[s].find_state = fs;
        }
        if (lane == 0) et->table_log = L;
    } else {
        rc = wave_build_spread<64, true>(norm, L, tl, sym_at, occ, cumul, cnt, [&](uint32_t i, uint32_t s, uint32_t r) {
            const uint32_t nx = r;  // symbol_next + rank (fse.rs:296-308, 329-331)
            const uint32_t nb = L - ilog2u(nx);
            fse_decode_transform e;
            e.new_state = (uint16_t)((nx << nb) - size);
            e.symbol = (uint8_t)s;
            e.num_bits = (uint8_t)nb;
            dt->table[i] = e;
        },
        [&](uint32_t s) {
            const int32_t v = norm[s];
            return v < 0 ? 1u : (uint32_t)v;
        },
        RankAtomic{peer_ranks == 0u, occ, nullptr, 0u, &g_rank_fb_tab, 0u});
        uint32_t big = 0;  // fast_mode: no norm >= 2^(L-1) (fse.rs:302-305)
        for (uint32_t s = lane; s < tl; s += WAVE)
            if (norm[s] > 0 && (uint32_t)norm[s] >= (1u << (L - 1u))) big = 1;
        big = wave_max(big);
        if (lane == 0) {
            dt->table_log = L;
            dt->fast_mode = big ? 0u : 1u;
        }
    }
    if (lane == 0) *status = rc;
}

// ------------------------------------------------------------------------
// Bitstream primitives.  Fields are (value, width) with width <= 32; a
// tile is 256 threads x 16 fields.
//   bits_tile_sum   widths -> per-tile bit sums
//   bits_tile_scan  one workgroup: exclusive scan of the tile sums -> tile
//                   bit offsets (u64) and the total
//   bits_pack       BitStackWriter::write_bits_unmasked x count + finish
//                   (writer.rs:140-222): fields LSB-first from bit 0; words
//                   wholly inside a thread's range are stored, the two at
//                   its ends OR-ed atomically (zeroed by bits_zero first)
//   bits_unpack     BitStackReader (stack_reader.rs:17-215: field i ends at
//                   top - S_i, read downwards from the marker) or
//                   BitStreamReader (stream_reader.rs:16-135: field i starts
//                   at S_i, and may be a read, a peek or an advance_by);
//                   steps past the available bits fail, and result[0] = the
//                   index of the first failing step
// ------------------------------------------------------------------------
constexpr uint32_t BT_THREADS = 256, BT_PER = 16, BT_TILE = BT_THREADS * BT_PER;

// Bits field i moves the position: its width, or 0 for a peek (ops[i] ==
// FSE_BITS_PEEK; `ops` may be null: all reads / writes).
__device__ __forceinline__ uint32_t field_advance(const uint8_t* nbits, const uint8_t* ops, uint64_t i) {
    return ops && ops[i] == FSE_BITS_PEEK ? 0u : min((uint32_t)nbits[i], 32u);
}
__device__ __forceinline__ uint32_t thread_bits(const uint8_t* nbits, const uint8_t* ops, uint64_t count, uint64_t i0) {
    uint32_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < BT_PER; ++k) s += i0 + k < count ? field_advance(nbits, ops, i0 + k) : 0u;
    return s;
}

// Workgroup exclusive scan of one value per thread (256 threads); returns
// the thread's exclusive prefix and the total in *tot.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* tot) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t incl = wave_incl_sum(v);
    if (lane == 63u) sh[wv] = incl;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < BT_THREADS / 64u; ++w) {
        base += w < wv ? sh[w] : 0u;
        all += sh[w];
    }
    __syncthreads();
    *tot = all;
    return base + incl - v;
}

__global__ __launch_bounds__(256) void bits_tile_sum(const uint8_t* __restrict__ nbits, const uint8_t* __restrict__ ops,
                                                     uint64_t count, uint32_t* __restrict__ tile_sum) {
    __shared__ uint32_t sh[BT_THREADS / 64u];
    const uint64_t i0 = (uint64_t)blockIdx.x * BT_TILE + (uint64_t)threadIdx.x * BT_PER;
    uint32_t tot;
    (void)block_excl_scan(thread_bits(nbits, ops, count, i0), sh, &tot);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void bits_tile_scan(const uint32_t* __restrict__ tile_sum, uint64_t ntiles,
                                                       uint64_t* __restrict__ tile_off, uint64_t* __restrict__ total) {
    __shared__ uint64_t sh[16];
    __shared__ uint64_t carry;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint64_t b = 0; b < ntiles; b += 1024u) {
        const uint64_t i = b + tid;
        const uint64_t v = i < ntiles ? tile_sum[i] : 0u;
        // 64-bit inclusive wave scan (sums may exceed 2^32 over many tiles)
        uint64_t incl = v;
#pragma unroll
        for (uint32_t d = 1; d < 64u; d <<= 1) {
            const uint64_t o = (uint64_t)__shfl_up((unsigned long long)incl, d, 64);
            if (lane >= d) incl += o;
        }
        if (lane == 63u) sh[wv] = incl;
        __syncthreads();
        uint64_t base = carry, all = 0;
        for (uint32_t w = 0; w < 16u; ++w) {
            base += w < wv ? sh[w] : 0u;
            all += sh[w];
        }
        if (i < ntiles) tile_off[i] = base + incl - v;
        __syncthreads();
        if (tid == 0) carry += all;
        __syncthreads();
    }
    if (tid == 0) *total = carry;
}

// Zero the bytes [0, ceil(total / 32) * 4) of the output (the packed bits
// and the rest of their last word); `lim` bounds it by the capacity.
__global__ __launch_bounds__(256) void bits_zero(uint32_t* out, const uint64_t* total, uint64_t lim_words) {
    const uint64_t nw = min((*total + 31u) >> 5, lim_words);
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * 256u) out[i] = 0;
}

__global__ __launch_bounds__(256) void bits_pack(const uint32_t* __restrict__ vals, const uint8_t* __restrict__ nbits,
                                                 uint64_t count, const uint64_t* __restrict__ tile_off,
                                                 const uint64_t* __restrict__ total, uint32_t* __restrict__ out,
                                                 uint64_t lim_words) {
    __shared__ uint32_t sh[BT_THREADS / 64u];
    const uint64_t i0 = (uint64_t)blockIdx.x * BT_TILE + (uint64_t)threadIdx.x * BT_PER;
    uint32_t tot;
    const uint64_t start = tile_off[blockIdx.x] + block_excl_scan(thread_bits(nbits, nullptr, count, i0), sh, &tot);
    if ((*total + 31u) >> 5 > lim_words) return;  // the host checked the capacity; never write past it
    // the thread's fields as one bit run from `start`: a 64-bit accumulator,
    // each completed word stored as it completes; the first word (shared
    // with the thread below when start is not word aligned) and the last
    // partial one are OR-ed atomically into the zeroed output
    uint64_t acc = 0;
    uint32_t nacc = (uint32_t)(start & 31u);
    uint64_t wi = start >> 5;
    bool head = nacc != 0u;
    for (uint32_t k = 0; k < BT_PER; ++k) {
        if (i0 + k >= count) break;
        const uint32_t nb = min((uint32_t)nbits[i0 + k], 32u);
        const uint32_t v = nb == 32u ? vals[i0 + k] : vals[i0 + k] & ((1u << nb) - 1u);  // masked (writer.rs:147)
        acc |= (uint64_t)v << nacc;
        nacc += nb;
        if (nacc >= 32u) {
            if (head) atomicOr(&out[wi], (uint32_t)acc);
            else out[wi] = (uint32_t)acc;
            head = false;
            acc >>= 32;
            nacc -= 32u;
            ++wi;
        }
    }
    if (nacc) atomicOr(&out[wi], (uint32_t)acc);
}

// Bits available to the reader: BitStreamReader = total_bits (the caller's);
// BitStackReader = the bits below the marker (the highest set bit, which must
// lie in the last byte: stack_reader.rs:77-83), or none (-1) without one.
__device__ __forceinline__ int64_t bits_avail(const uint8_t* in, uint64_t n_bytes, uint64_t total_bits, int stack) {
    if (!stack) return (int64_t)total_bits;
    const uint32_t last = n_bytes ? in[n_bytes - 1u] : 0u;
    if (last == 0u) return -1;
    return (int64_t)(8u * (n_bytes - 1u) + ilog2u(last));
}

__global__ __launch_bounds__(256) void bits_unpack(const uint8_t* __restrict__ in, uint64_t n_bytes,
                                                   uint64_t total_bits, int stack, const uint8_t* __restrict__ nbits,
                                                   const uint8_t* __restrict__ ops, uint64_t count,
                                                   const uint64_t* __restrict__ tile_off,
                                                   uint32_t* __restrict__ vals, uint64_t* __restrict__ result) {
    __shared__ uint32_t sh[BT_THREADS / 64u];
    const uint64_t i0 = (uint64_t)blockIdx.x * BT_TILE + (uint64_t)threadIdx.x * BT_PER;
    uint32_t tot;
    uint64_t s = tile_off[blockIdx.x] + block_excl_scan(thread_bits(nbits, ops, count, i0), sh, &tot);
    const int64_t av = bits_avail(in, n_bytes, total_bits, stack);
    const uint64_t avail = av < 0 ? 0u : (uint64_t)av;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(in);
    for (uint32_t k = 0; k < BT_PER; ++k) {
        const uint64_t i = i0 + k;
        if (i >= count) break;
        const uint32_t nb = min((uint32_t)nbits[i], 32u);
        const uint32_t op = ops ? ops[i] : FSE_BITS_READ;
        uint32_t v = 0;
        // read, peek and advance_by all fail past the available bits
        // (stream_reader.rs:70-72, 85-87); advance_by returns no value
        if (av < 0 || s + nb > avail) {  // None / Err(UnexpectedEof)
            atomicMin(reinterpret_cast<unsigned long long*>(result), (unsigned long long)i);
        } else if (nb && op != FSE_BITS_ADVANCE) {
            const uint64_t lo = stack ? avail - s - nb : s;  // first bit of the field
            const uint64_t wi = lo >> 5;
            const uint32_t sh5 = (uint32_t)(lo & 31u);
            const uint64_t x = (uint64_t)w[wi] | (sh5 + nb > 32u ? (uint64_t)w[wi + 1u] << 32 : 0ull);
            v = (uint32_t)(x >> sh5) & (nb == 32u ? 0xFFFFFFFFu : (1u << nb) - 1u);
        }
        vals[i] = v;
        s += op == FSE_BITS_PEEK ? 0u : nb;
    }
}

// After the scan: result = {reads that succeed (lowered by bits_unpack to
// the first failing read), finished (every available bit read), status}.
__global__ void bits_read_init(const uint8_t* in, uint64_t n_bytes, uint64_t total_bits, int stack, uint64_t count,
                               const uint64_t* total, uint64_t* result) {
    const int64_t av = bits_avail(in, n_bytes, total_bits, stack);
    result[0] = count;
    result[1] = av >= 0 && *total == (uint64_t)av ? 1u : 0u;
    result[2] = av < 0 ? (uint64_t)(int64_t)FSE_ERR_NO_MARKER : 0u;
    if (av < 0) result[0] = 0;
}

// Host-call return (fse_compress2 / fse_decompress2 etc.): the call's 16-byte
// result record and min(*len, max) bytes of its output into pinned host
// memory, in the call's stream, so the host waits once and reads both (no
// device-to-host copy of the record first to learn the length).
__global__ __launch_bounds__(256) void host_return_kernel(const uint4* __restrict__ meta, const uint8_t* __restrict__ src,
                                                          const uint32_t* __restrict__ len, uint4* hmeta,
                                                          uint8_t* hdst, uint32_t max) {
    const uint32_t n = min(*len, max);
    if (threadIdx.x == 0) *hmeta = *meta;
    const uint32_t nv = n >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(hdst);
    for (uint32_t i = threadIdx.x; i < nv; i += blockDim.x) d4[i] = s4[i];
    for (uint32_t i = (nv << 4) + threadIdx.x; i < n; i += blockDim.x) hdst[i] = src[i];
}

// ------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------
hipError_t launch_norm(const NormArgs& A, hipStream_t s) {
    hipLaunchKernelGGL(norm_kernel, dim3(1), dim3(64), 0, s, A);
    return hipGetLastError();
}
hipError_t launch_hdr_write(const fse_norm_histogram* nh, uint8_t* out, uint32_t* bits, int32_t* status, hipStream_t s) {
    hipLaunchKernelGGL(hdr_write_kernel, dim3(1), dim3(64), 0, s, nh, out, bits, status);
    return hipGetLastError();
}
hipError_t launch_hdr_read(const uint8_t* src, uint32_t n, fse_norm_histogram* out, uint32_t* used, int32_t* status,
                           hipStream_t s) {
    hipLaunchKernelGGL(hdr_read_kernel, dim3(1), dim3(64), 0, s, src, n, out, used, status);
    return hipGetLastError();
}
hipError_t launch_table(const fse_norm_histogram* nh, int enc, fse_encode_table* et, fse_decode_table* dt, int32_t* status,
                        hipStream_t s) {
    hipLaunchKernelGGL(table_kernel, dim3(1), dim3(64), 0, s, nh, enc, et, dt, status, atomic_ranks_on() ? 0u : 1u);
    return hipGetLastError();
}

// ------------------------------------------------------------------------
// The lane-order check behind the atomic ranks (wave_build_spread): every
// lane of every wave draws a key (1..64 distinct keys, uniform or skewed)
// and an activity bit, reads its key's LDS counter, does ds_add_rtn_u32 on
// it, and compares the old value returned with counter-before + the active
// lanes below it with the same key (ballot peers).  Counts the mismatches.
// ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rc_mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__global__ __launch_bounds__(256) void rank_order_check_kernel(uint32_t* bad, unsigned long long* total) {
    __shared__ uint32_t cnt[4][64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    cnt[w][lane] = 0;
    __syncthreads();
    const uint32_t nkeys = 1u + (blockIdx.x % 64u), skew = (blockIdx.x >> 6) & 1u;
    uint32_t nbad = 0, nops = 0;
    for (uint32_t it = 0; it < 64u; ++it) {
        const uint32_t h = rc_mix(it * 0x9E3779B9u ^ (blockIdx.x * 256u + threadIdx.x) * 0x85EBCA6Bu);
        const uint32_t key = skew ? min((uint32_t)__builtin_ctz((h >> 8) | 0x80000000u), nkeys - 1u) : h % nkeys;
        const bool act = (it & 1u) == 0u || ((h >> 5) & 7u) != 0u;  // every lane, then ~7/8 of them
        const uint32_t before = cnt[w][key];
        __builtin_amdgcn_wave_barrier();
        uint32_t r = 0;
        if (act)
            r = __hip_atomic_fetch_add((__attribute__((address_space(3))) uint32_t*)&cnt[w][key], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
        uint64_t peers = 0;
        for (uint32_t k = 0; k < nkeys; ++k) {
            const uint64_t m = __ballot(act && key == k);
            if (key == k) peers = m;
        }
        const uint32_t below = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (act) {
            nops += 1u;
            nbad += r != before + below ? 1u : 0u;
        }
        __builtin_amdgcn_wave_barrier();
    }
    atomicAdd(bad, nbad);
    atomicAdd(total, (unsigned long long)nops);
}

hipError_t rank_order_check(uint32_t* violations, uint64_t* atomics) {
    uint32_t* d = nullptr;
    if (hipError_t e = hipMalloc(&d, 16)) return e;
    hipError_t e = hipMemsetAsync(d, 0, 16, nullptr);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(rank_order_check_kernel, dim3(256), dim3(256), 0, nullptr, d,
                           reinterpret_cast<unsigned long long*>(d + 2));
        e = hipGetLastError();
    }
    uint32_t h[4] = {0, 0, 0, 0};
    if (e == hipSuccess) e = hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);  // waits for the kernel
    (void)hipFree(d);
    if (e != hipSuccess) return e;
    *violations = h[0];
    *atomics = (uint64_t)h[2] | ((uint64_t)h[3] << 32);
    return hipSuccess;
}

static std::atomic<int> g_rank_mode{-1};  // fsehipx_rank_mode: -1 / 0 atomic (checked per table), 1 peer-mask
int rank_mode(int mode) { return g_rank_mode.exchange(mode); }

bool atomic_ranks_on() { return g_rank_mode.load(std::memory_order_relaxed) != 1; }

hipError_t launch_host_return(const void* meta, const uint8_t* src, const uint32_t* len, void* hmeta, uint8_t* hdst,
                              uint32_t max, hipStream_t s) {
    hipLaunchKernelGGL(host_return_kernel, dim3(1), dim3(256), 0, s, static_cast<const uint4*>(meta), src, len,
                       static_cast<uint4*>(hmeta), hdst, max);
    return hipGetLastError();
}

uint64_t bits_tiles(uint64_t count) { return (count + BT_TILE - 1u) / BT_TILE; }

hipError_t launch_bits_scan(const uint8_t* nbits, const uint8_t* ops, uint64_t count, uint32_t* tile_sum,
                            uint64_t* tile_off, uint64_t* total, hipStream_t s) {
    const uint64_t nt = bits_tiles(count);
    if (nt) hipLaunchKernelGGL(bits_tile_sum, dim3((uint32_t)nt), dim3(BT_THREADS), 0, s, nbits, ops, count, tile_sum);
    hipLaunchKernelGGL(bits_tile_scan, dim3(1), dim3(1024), 0, s, tile_sum, nt, tile_off, total);
    return hipGetLastError();
}

hipError_t launch_bits_pack(const uint32_t* vals, const uint8_t* nbits, uint64_t count, const uint64_t* tile_off,
                            const uint64_t* total, uint32_t* out, uint64_t lim_words, hipStream_t s) {
    const uint64_t nt = bits_tiles(count);
    const uint64_t zb = (lim_words + 255u) / 256u;
    const uint32_t zg = (uint32_t)(zb < 4096u ? zb : 4096u);
    if (zg) hipLaunchKernelGGL(bits_zero, dim3(zg), dim3(256), 0, s, out, total, lim_words);
    if (nt)
        hipLaunchKernelGGL(bits_pack, dim3((uint32_t)nt), dim3(BT_THREADS), 0, s, vals, nbits, count, tile_off, total,
                           out, lim_words);
    return hipGetLastError();
}

hipError_t launch_bits_unpack(const uint8_t* in, uint64_t n_bytes, uint64_t total_bits, int stack,
                              const uint8_t* nbits, const uint8_t* ops, uint64_t count, const uint64_t* tile_off,
                              const uint64_t* total, uint32_t* vals, uint64_t* result, hipStream_t s) {
    hipLaunchKernelGGL(bits_read_init, dim3(1), dim3(1), 0, s, in, n_bytes, total_bits, stack, count, total, result);
    const uint64_t nt = bits_tiles(count);
    if (nt)
        hipLaunchKernelGGL(bits_unpack, dim3((uint32_t)nt), dim3(BT_THREADS), 0, s, in, n_bytes, total_bits, stack,
                           nbits, ops, count, tile_off, vals, result);
    return hipGetLastError();
}

}  // namespace fsehip
