// fse_kernels.h -- internal launch interface between the C ABI (fse_capi.cpp)
// and the gfx950 kernels (fse_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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
    // Scratch-emit path (see encode_blocks_kernel): each lane writes its
    // bits to a lane-private scratch stream from the start state the count
    // pass gives it, and a copy pass moves the streams to their final bit
    // offsets once the exact lengths are known.  nullptr = repair path only.
    uint32_t* scratch;        // [n_blocks][lanes][scr_lane_words]
    uint32_t scr_lane_words;  // words per lane stream (worst case, multiple of 32)
    uint32_t warm;            // count-pass warm-up pairs above the lane's range (scratch path)
    uint32_t path;            // 0 = by distribution, 1 = repair path, 2 = scratch path
    uint32_t pmax256;         // auto: scratch path when max norm <= pmax256/256 of the table
    uint32_t xlds;            // diagnostics: extra dynamic LDS bytes per workgroup (occupancy probe)
};

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
    uint32_t debug;         // ablation: bit0 = header + table only
    uint64_t* stamps;       // diagnostics: per-workgroup s_memtime at phase ends
    uint32_t waves;         // waves per block workgroup: 4 (default) or 8
    const uint32_t* dt;     // prebuilt decode tables [n_blocks][1 << lmax], or nullptr
    const int32_t* dtinfo;  // per block: header bytes | L << 16, or < 0 = status
    uint32_t variant;       // LDS layout / reader: 3/5 = padded image (prebuilt tables), else linear window
    uint32_t dual;          // two segments per lane, interleaved (prebuilt-table kernel)
    uint32_t stage_kib;     // LDS image size of the prebuilt-table kernel: 44 (default), 40 or 36 KiB
    uint32_t pass;          // prebuilt-table kernel: 0 = all blocks, 1 = defer blocks the stage cannot
                            // hold (status FSE_DEFERRED), 2 = only the deferred blocks (big stage)
    uint32_t nstates;       // 2 = fse_compress2 blocks (default), 1 = fse_compress blocks
};

// Decode-table build (header parse + DecodeTable) for a batch of blocks.
struct DtParams {
    const uint8_t* in;
    uint64_t slot_bytes;
    const uint32_t* comp_len;
    uint32_t n_blocks;
    uint32_t* dt;      // [n_blocks][1 << lmax] entries (dte_make layout)
    int32_t* dtinfo;   // header bytes | L << 16, or < 0 = status
    uint32_t debug;    // ablation: bit0 = header parse only, bit1 = no table stores
};

struct GenParams {
    uint8_t* out;
    uint64_t n_total;
    uint64_t block_size;
    uint64_t seed;
    int32_t kind;
    uint32_t nsym;
    uint16_t bound[1024];
};

constexpr int kStamps = 10;  // stamp slots per workgroup
constexpr int32_t FSE_DEFERRED = 1;  // internal block status between the two decode passes

hipError_t launch_encode(const EncParams& P, uint32_t lmax, hipStream_t stream);
hipError_t launch_dtables(const DtParams& P, uint32_t lmax, hipStream_t stream);
hipError_t launch_decode(const DecParams& P, uint32_t lmax, hipStream_t stream);
// Diagnostics: resident workgroups per CU of the main kernels, as text.
int occupancy_report(char* buf, int cap);
hipError_t launch_histogram(const uint8_t* src, uint64_t n_total, uint32_t block_size, uint32_t n_blocks,
                            uint32_t* counts, uint32_t* table_len, hipStream_t stream);
hipError_t launch_generate(const GenParams& G, hipStream_t stream);
hipError_t launch_pack(const uint8_t* slots, uint64_t slot_bytes, const uint32_t* comp_len, const uint64_t* offsets,
                       uint32_t n_blocks, uint8_t* stream, int unpack, hipStream_t hs);
hipError_t launch_copy(const uint8_t* src, const uint64_t* src_off, const uint32_t* lens, uint32_t n_blocks,
                       uint8_t* dst, const uint64_t* dst_off, hipStream_t hs);

}  // namespace fsehip
