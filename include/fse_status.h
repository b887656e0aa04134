/*
 * fse_status.h -- status codes shared by the C ABI (fsehip.h).
 *
 * The reference crate reports failures three ways: Option::None, Result::Err
 * and panics.  Each is mapped to one negative code here so a C caller (or the
 * Rust FFI shim in INTEGRATION.md) can reproduce the reference's behaviour.
 */
#ifndef FSE_STATUS_H
#define FSE_STATUS_H

#define FSE_OK 0
/* Empty input: Histogram size.ilog2() panics (histogram.rs:266) on compress;
 * BitStreamReader::new asserts non-empty (stream_reader.rs:17) on decompress. */
#define FSE_ERR_EMPTY (-1)
/* Input too short: compress of 1 byte panics at (size-1).ilog2()
 * (histogram.rs:271) / chunks unwrap (lib.rs:154-156); decompress of a
 * payload too short for the initial states panics at lib.rs:224-225.        */
#define FSE_ERR_TOO_SHORT (-2)
/* Every byte is symbol 0: table_len == 1 -> (table_len-1).ilog2() panics
 * (histogram.rs:98, 267).                                                   */
#define FSE_ERR_ALL_ZERO_SYMBOL0 (-3)
/* Decoding a single-symbol block (one symbol with count 2^L) never
 * terminates in the reference (num_bits = 0, fse.rs:333); without a known
 * raw length we refuse instead of looping.                                  */
#define FSE_ERR_SINGLE_SYMBOL (-4)
/* NormHistogram::read error: TableLogTooLarge / TooManySymbols / Io
 * (histogram.rs:438-505).                                                   */
#define FSE_ERR_BAD_HEADER (-5)
/* BitStackReader::new returned None: empty payload or last byte zero
 * (stack_reader.rs:18-20, 77-83).                                           */
#define FSE_ERR_NO_MARKER (-6)
/* Caller-provided capacity too small (the reference grows a Vec instead). */
#define FSE_ERR_DST_TOO_SMALL (-7)
/* tableLog outside the range this entry point accepts.                     */
#define FSE_ERR_TABLELOG_RANGE (-8)
/* normalize_slow panic "What did you do, to make a distribution so cursed"
 * (histogram.rs:248), or its even-spread loop that cannot terminate.       */
#define FSE_ERR_CURSED (-9)
/* Normalized table inconsistent (header write panic histogram.rs:420, or
 * spread assert fse.rs:151/326).                                            */
#define FSE_ERR_BAD_TABLE (-10)
#define FSE_ERR_BAD_ARG (-11)
/* A HIP runtime call failed (GPU entry points only).                       */
#define FSE_ERR_HIP (-12)
/* Decoded length differs from the container's raw length.                  */
#define FSE_ERR_LENGTH_MISMATCH (-13)
/* Supported by the reference but not (yet) by the GPU kernels (L > 12).   */
#define FSE_ERR_UNSUPPORTED (-14)
/* No HIP device / HIP extension not usable: product paths fail loudly.     */
#define FSE_ERR_NO_DEVICE (-15)
/* A decode checkpoint (sidecar entry) disagrees with the stream: a segment
 * did not end at the next checkpoint's bit position and states, or the last
 * segment did not consume the payload exactly (corrupt index, or one built
 * with a different ckpt_interval).                                          */
#define FSE_ERR_BAD_SIDECAR (-16)
/* Encoder::new_first_symbol indexes outside the state table (fse.rs:212-216):
 * at tableLog 15 its rounding constant 1 << 15 no longer covers the smallest
 * state of a symbol with norm >= 2, the u32 subtraction wraps and the
 * bounds-checked table read panics.                                         */
#define FSE_ERR_ENCODER_INIT (-17)
/* A bit reader ran out of bits: BitStackReader::peek/read returned None
 * (stack_reader.rs:176-215) or BitStreamReader::peek/read/advance_by
 * returned Err(UnexpectedEof) (stream_reader.rs:56-114).  Reported by the
 * cursor readers of fsehip.h section 1c; the reference's callers treat it as
 * end of stream.                                                            */
#define FSE_ERR_EOF (-18)

#endif
