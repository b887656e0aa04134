/*
 * fse_oracle.h -- CPU restatement of the reference FSE (tANS) coder.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle and the CPU baseline
 * ("kind": "port") for bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker.  The
 * product library (entropy_coders_amd/libfsehip.so) never links or calls it.
 *
 * Reference: Cognoscan/entropy_coders (Rust crate), read-only at
 * /root/reference.  Every function cites the file:line it restates.  The
 * crate cannot be built here (no cargo/rustc), so parity is pinned by
 *   (1) the reference's own known-answer tests (histogram.rs:595-656),
 *   (2) the reference's round-trip/bitstream properties (bitstream/mod.rs,
 *       lib.rs:280-302, histogram.rs:553-587),
 *   (3) byte-for-byte agreement with an independent pure-Python restatement
 *       (oracle/spec.py) on the committed golden vectors (tests/golden/).
 * Exact compressed bytes are therefore pinned by two independent
 * restatements, not by reference-produced fixtures (the reference ships none).
 *
 * Integer semantics follow a Rust *release* build (wrapping u32 arithmetic,
 * no overflow panics) because that is what the crate's benchmark runs.  Every
 * reference panic is mapped to a negative status code (see fse_status.h).
 */
#ifndef FSE_ORACLE_H
#define FSE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/fse_status.h"

#ifdef __cplusplus
extern "C" {
#endif

#define FO_LOG_MIN 5u      /* lib.rs:9  TABLE_LOG_MIN */
#define FO_LOG_MAX 15u     /* lib.rs:10 TABLE_LOG_MAX */
#define FO_LOG_DEFAULT 11u /* lib.rs:12 TABLE_LOG_DEFAULT */

/* histogram.rs:10-14 */
typedef struct {
    uint32_t counts[256];
    uint32_t size;
    uint32_t table_len;
} fo_hist;

/* histogram.rs:290-294 */
typedef struct {
    int32_t norm[256];
    uint32_t log2;
    uint32_t table_len;
} fo_norm;

/* fse.rs:72-84: stateTable, symbol transforms, spread symbols. */
typedef struct {
    uint32_t log2;
    uint16_t st[1u << FO_LOG_MAX];
    uint32_t dnb[256]; /* SymbolTransform.bits (deltaNbBits) */
    int32_t dfs[256];  /* SymbolTransform.find_state (deltaFindState) */
    uint8_t spread[1u << FO_LOG_MAX];
} fo_ctable;

/* fse.rs:254-265 */
typedef struct {
    uint32_t log2;
    uint16_t new_state[1u << FO_LOG_MAX];
    uint8_t sym[1u << FO_LOG_MAX];
    uint8_t nb[1u << FO_LOG_MAX];
} fo_dtable;

/* ---- statistics (histogram.rs) ---- */
int fo_hist_count(const uint8_t* src, size_t n, fo_hist* h);
int fo_optimal_log2(const fo_hist* h, uint32_t* log2_out);
/* normalize(L); *used_slow = 1 when normalize_slow ran (it prints in the ref). */
int fo_normalize(const fo_hist* h, uint32_t log2, fo_norm* out, int* used_slow);
int fo_norm_new(const uint8_t* src, size_t n, fo_norm* out);
size_t fo_header_write_bound(const fo_norm* nh);
/* Appends the NCount header at dst; returns bytes written via *len. */
int fo_header_write(const fo_norm* nh, uint8_t* dst, size_t cap, size_t* len);
/* Parses a header; *consumed = bytes up to the next byte boundary. */
int fo_header_read(const uint8_t* src, size_t n, fo_norm* out, size_t* consumed);

/* ---- tables (fse.rs) ---- */
int fo_build_ctable(const fo_norm* nh, fo_ctable* ct);
int fo_build_dtable(const fo_norm* nh, fo_dtable* dt);

/* ---- block codecs (lib.rs) ----
 * dst receives header||payload starting at dst[0]; *out_len = bytes written.
 * *payload_bits = the Rust return value (payload bits incl. marker).      */
int fo_compress2(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                 size_t* out_len, uint64_t* payload_bits);
/* compress2 with an explicit table log: Histogram::new(src).normalize(L)
 * then the fse_compress2 body (public pieces, histogram.rs:95).           */
int fo_compress2_log(const uint8_t* src, size_t n, uint32_t log2, uint8_t* dst,
                     size_t cap, size_t* out_len, uint64_t* payload_bits);
int fo_decompress2(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                   size_t* out_len);
/* Same as fo_decompress2 but the raw length is known (container): decoding
 * stops after exactly raw_len symbols; required for single-symbol blocks,
 * on which the reference decoder never terminates (SURVEY TL;DR 10).       */
int fo_decompress2_n(const uint8_t* src, size_t n, uint8_t* dst, size_t raw_len);
int fo_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                size_t* out_len, uint64_t* payload_bits);
int fo_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                  size_t* out_len);

/* Decode checkpoints of a compress2 stream (the GPU container's sidecar):
 * for every pair index p multiple of `interval` (p < n_pairs_main), the bit
 * position (relative to payload start) and both decoder states just before
 * the decoder processes pair p.  Returns the number of checkpoints.        */
int fo_checkpoints2(const uint8_t* src, size_t n, uint32_t interval,
                    uint32_t* bitpos, uint16_t* s0, uint16_t* s1, size_t cap,
                    size_t* count);
/* The same for a 1-state stream: the state before symbol p.              */
int fo_checkpoints1(const uint8_t* src, size_t n, uint32_t interval, uint32_t* bitpos, uint16_t* s0o,
                    size_t cap, size_t* count);

/* ---- bitstream primitives (bitstream/ files), for property tests ---- */
/* Write (val,bits) pairs LSB-first after `offset` pre-existing bytes, then
 * optionally the 1-bit marker; returns total bytes.  writer.rs:140-222     */
size_t fo_bits_write(const uint64_t* vals, const uint8_t* bits, size_t count,
                     int mark, uint8_t* dst, size_t cap, uint64_t* written_bits);
/* Pop `count` values of widths bits[count-1..0] (stack order).  Returns
 * 0 on success; stack_reader.rs:17-215                                     */
int fo_bits_read_stack(const uint8_t* src, size_t n, const uint8_t* bits,
                       size_t count, uint64_t* vals_out, size_t* bits_left);

/* ---- synthetic generators (bench/test inputs) ---- */
uint64_t fo_splitmix64_mix(uint64_t z);
/* benches/fse_benchmark.rs:5-20: LUT of 4096 symbols for probability p. */
int fo_build_lut(double prob, uint8_t lut[4096]);
/* byte i of block b = lut[mix(seed_b + (i+1)*GOLDEN) & 4095],
 * seed_b = seed ^ (b * GOLDEN).  kind: 0=LUT, 1=geometric p=0.5,
 * 2=uniform 0..239.                                                         */
void fo_generate(int kind, double prob, uint64_t seed, uint64_t block_index,
                 uint8_t* out, size_t n);

/* multi-threaded CPU baseline: compress2/decompress2 over independent blocks */
int fo_compress2_blocks(const uint8_t* src, size_t n_total, size_t block,
                        uint8_t* dst, size_t slot, uint32_t* lens, int threads);
int fo_decompress2_blocks(const uint8_t* src, size_t slot, const uint32_t* lens,
                          size_t n_blocks, uint8_t* dst, size_t block,
                          size_t n_total, int threads);

#ifdef __cplusplus
}
#endif
#endif
