// fse_kernels.h -- internal launch interface between the C ABI (fse_capi.cpp)
// and the gfx950 kernels (fse_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fsehip.h"

namespace fsehip {

struct EncParams {
    const uint8_t* src;
    uint64_t n_total;
    uint32_t block_size;
    uint32_t n_blocks;
    uint32_t table_log;      // 0 = NormHistogram::new (optimal_log2)
    uint32_t ckpt_interval;  // pairs between sidecar checkpoints (power of 2) or 0
    uint32_t ckpt_per_block; // sidecar entries reserved per block
    uint8_t* out;            // n_blocks * slot_bytes
    uint64_t slot_bytes;
    uint32_t* comp_len;
    uint32_t* payload_bits;
    uint64_t* sidecar;
    int32_t* status;
    uint32_t lanes;  // encoder lanes per block (32 or 64; 0 = default)
    uint32_t nstates;  // 2 = fse_compress2 (default), 1 = fse_compress
    uint32_t debug;  // ablation: bit0 = tables only, bit1 = no emit pass, bit2 = no payload stores,
                     // bit3 = histogram only, bit4 = no repair rounds
    uint64_t* stamps;  // diagnostics: per-workgroup s_memtime at phase ends
    uint32_t xlds;            // diagnostics: extra dynamic LDS bytes per workgroup (occupancy probe)
    uint32_t peer_ranks;      // set by launch_encode: 1 = peer-mask ranks (forced by rank_mode)
    uint32_t rank_inject;     // diagnostics build only: fault injection into the atomic ranks (FSEHIP_RANK_INJECT)
    // kernels at L >= 13 (enc_gsym): the spread's 2^LMAX-byte symbol array of
    // block b at spread + b * 2^LMAX, or (nullptr) in the block's own output
    // slot after its header words, when slot_bytes >= HDR_MAX + 2^LMAX
    uint8_t* spread;
};
// Encoder kernels whose spread symbol array lives in global memory (L >= 13):
// their LDS then fits 7 / 4 / 2 workgroups per CU at L = 13 / 14 / 15
// instead of 5 / 3 / 1.
constexpr bool enc_gsym(uint32_t lmax) { return lmax >= 13u; }
// byte offset of the in-slot spread array (after the header words, <= 512 B)
constexpr uint32_t ENC_SPREAD_OFF = 512;

struct DecParams {
    const uint8_t* in;
    uint64_t slot_bytes;
    const uint32_t* comp_len;
    const uint64_t* sidecar;  // nullptr -> serial reference-mode decode
    uint32_t ckpt_interval;
    uint32_t ckpt_per_block;
    uint8_t* out;
    uint64_t n_total;  // 0 -> raw length unknown (reference mode, out_cap bytes)
    uint32_t block_size;
    uint32_t n_blocks;
    uint32_t out_cap;
    int32_t* status;
    uint32_t* out_len;
    uint64_t* sidecar_out;  // serial mode: record checkpoints here
    uint64_t* stamps;       // diagnostics: per-workgroup s_memtime at phase ends
    const uint32_t* dt;     // prebuilt decode tables [n_blocks][1 << lmax] (dtable_blocks_kernel)
    const int32_t* dtinfo;  // per block: header bytes | L << 16, or < 0 = status
    uint32_t pass;          // segment decode: 0 = all blocks, 1 = defer blocks the LDS stage cannot
                            // hold (status FSE_DEFERRED), 2 = only the deferred blocks (list pass)
    uint32_t nstates;       // 2 = fse_compress2 blocks (default), 1 = fse_compress blocks
    // Sidecar-less 2-state decode at L <= 11 with symbols deferred (optional
    // workspace; nullptr -> the single-kernel serial decode): the chains write
    // their state pairs here ([n_blocks][block_size / 2] u32, 2 bytes per
    // output byte) and the bulk length | table base per block (uint2), and a
    // map kernel turns the states into symbols.
    uint32_t* states;
    uint32_t* bulk;
};

// Decode-table build (header parse + DecodeTable) for a batch of blocks.
struct DtParams {
    const uint8_t* in;
    uint64_t slot_bytes;
    const uint32_t* comp_len;
    uint32_t n_blocks;
    uint32_t* dt;      // [n_blocks][1 << lmax] entries (dte_make layout)
    int32_t* dtinfo;   // header bytes | L << 16, or < 0 = status
    uint32_t xlds;     // diagnostics: extra dynamic LDS bytes per workgroup (occupancy probe)
    uint64_t* stamps;  // diagnostics: per-workgroup phase stamps (FSEHIP_STAMPS), or nullptr
    // Optional scratch (lmax <= 12): the headers are parsed first, one lane
    // per block (hdr_parse_kernel), and the table kernel reads the result
    // instead of parsing on the scalar unit.  hdr_meta[b] = {header bytes or
    // status, L | table_len << 8}; hdr_norm[b] = 256 x int16 counts (128 words).
    int2* hdr_meta;
    uint32_t* hdr_norm;
    uint32_t peer_ranks;  // set by launch_dtables: 1 = peer-mask ranks (forced by rank_mode)
    uint32_t rank_inject; // diagnostics build only: fault injection into the atomic ranks (FSEHIP_RANK_INJECT)
};
constexpr uint64_t hdr_scratch_bytes(uint64_t n_blocks) { return n_blocks * (512u + 8u); }

struct GenParams {
    uint8_t* out;
    uint64_t n_total;
    uint64_t block_size;
    uint64_t seed;
    int32_t kind;
    uint32_t nsym;
    uint16_t bound[1024];
};

// Building blocks (fse_blocks.hip): normalisation of one histogram.
struct NormArgs {
    int mode;                // 0 = Histogram::normalize(log2), 1 = normalize_optimal, 2 = NormHistogram::new(src)
    const uint8_t* src;      // mode 2: raw bytes
    uint64_t n;
    const uint32_t* counts;  // modes 0/1: counts[256]
    uint32_t size, table_len, log2;
    fse_norm_histogram* out;
    uint32_t* counts_out;    // optional: counts[256], size, table_len (mode 2's histogram)
    int32_t* status;
};
hipError_t launch_norm(const NormArgs& A, hipStream_t s);
hipError_t launch_hdr_write(const fse_norm_histogram* nh, uint8_t* out, uint32_t* bits, int32_t* status, hipStream_t s);
hipError_t launch_hdr_read(const uint8_t* src, uint32_t n, fse_norm_histogram* out, uint32_t* used, int32_t* status,
                           hipStream_t s);
hipError_t launch_table(const fse_norm_histogram* nh, int enc, fse_encode_table* et, fse_decode_table* dt,
                        int32_t* status, hipStream_t s);
// The table builds rank positions with one LDS atomic per 64 positions,
// which needs same-address ds_add_rtn_u32 results in ascending lane order
// (fse_device.hpp wave_build_spread).  Every table checks its own ranks and
// is rebuilt with the peer-mask ranks when the check fails; the per-device
// counts of such rebuilds: rank_fallbacks_enc (encode_blocks_kernel),
// _dec (dtable_blocks_kernel), _tab (table_kernel), read and optionally reset.
// rank_order_check runs a stand-alone probe of the lane order (synchronous;
// counts the violations among `atomics` checked), for tests and tools only.
hipError_t rank_order_check(uint32_t* violations, uint64_t* atomics);
hipError_t rank_fallbacks_enc(uint32_t* out, bool reset);
hipError_t rank_fallbacks_dec(uint32_t* out, bool reset);
hipError_t rank_fallbacks_tab(uint32_t* out, bool reset);
// false only when rank_mode forces the peer-mask ranks
bool atomic_ranks_on();
// Tests: -1 = default (atomic ranks, checked per table), 0 = the same, 1 = peer-mask ranks; returns the previous mode.
int rank_mode(int mode);
// Host-call return: the 16-byte record at meta and min(*len, max) bytes of
// src into pinned host memory (hmeta, hdst; 16-byte aligned).
hipError_t launch_host_return(const void* meta, const uint8_t* src, const uint32_t* len, void* hmeta, uint8_t* hdst,
                              uint32_t max, hipStream_t s);
// Bitstream primitives: a tile scan of the field widths (tile_sum: u32 per
// tile, tile_off: u64 per tile, total: u64), then pack or unpack.
uint64_t bits_tiles(uint64_t count);
hipError_t launch_bits_scan(const uint8_t* nbits, const uint8_t* ops, uint64_t count, uint32_t* tile_sum,
                            uint64_t* tile_off, uint64_t* total, hipStream_t s);
hipError_t launch_bits_pack(const uint32_t* vals, const uint8_t* nbits, uint64_t count, const uint64_t* tile_off,
                            const uint64_t* total, uint32_t* out, uint64_t lim_words, hipStream_t s);
hipError_t launch_bits_unpack(const uint8_t* in, uint64_t n_bytes, uint64_t total_bits, int stack,
                              const uint8_t* nbits, const uint8_t* ops, uint64_t count, const uint64_t* tile_off,
                              const uint64_t* total, uint32_t* vals, uint64_t* result, hipStream_t s);

#ifndef FSEHIP_KSTAMPS
#define FSEHIP_KSTAMPS
constexpr int kStamps = 10;  // stamp slots per workgroup (also declared in fse_device.hpp)
#endif
constexpr int32_t FSE_DEFERRED = 1;  // internal block status between the decode passes

hipError_t launch_encode(const EncParams& P, uint32_t lmax, hipStream_t stream);
hipError_t launch_dtables(const DtParams& P, uint32_t lmax, hipStream_t stream);
// lmax: 11 (blocks of L <= 11), 12 or 15 (L 13..15); decode tables are laid
// out at that stride (4 << lmax bytes per block).
hipError_t launch_decode(const DecParams& P, uint32_t lmax, hipStream_t stream);
// One stream, latency-first (the host fse_decompress2 / fse_decompress):
// reference mode only (n_total = 0, no sidecar, n_blocks = 1), table logs
// <= 11, any payload length.  P.states: single_ftab_bytes() of device
// scratch (the fused bulk table).
hipError_t launch_single(const DecParams& P, uint32_t lmax, hipStream_t stream);
constexpr uint32_t single_ftab_bytes() { return 2048u * 8u; }
// Diagnostics: resident workgroups per CU of the main kernels, as text.
int occupancy_report(char* buf, int cap);
int occupancy_report_dec(char* buf, int cap);
hipError_t launch_histogram(const uint8_t* src, uint64_t n_total, uint32_t block_size, uint32_t n_blocks,
                            uint32_t* counts, uint32_t* table_len, hipStream_t stream);
hipError_t launch_generate(const GenParams& G, hipStream_t stream);
hipError_t launch_pack(const uint8_t* slots, uint64_t slot_bytes, const uint32_t* comp_len, const uint64_t* offsets,
                       uint32_t n_blocks, uint8_t* stream, int unpack, hipStream_t hs);
hipError_t launch_copy(const uint8_t* src, const uint64_t* src_off, const uint32_t* lens, uint32_t n_blocks,
                       uint8_t* dst, const uint64_t* dst_off, hipStream_t hs);

}  // namespace fsehip
