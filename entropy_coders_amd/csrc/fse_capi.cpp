// fse_capi.cpp -- C ABI (include/fsehip.h) over the gfx950 kernels.
//
// The reference-shaped entry points (fse_compress2, fse_decompress2,
// histogram_count) stage host buffers through device memory and run the
// same kernels as the batched API; there is no CPU compute path: without a
// usable HIP device they return FSE_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/fsehip.h"
#include "fse_kernels.h"

namespace {

constexpr uint32_t kDefaultBlock = 65536;

uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// Per-(device, stream, purpose) grow-only device scratch for the two-kernel
// encode and decode: calls on one stream are ordered, so they may share it;
// calls on different streams get different buffers.
struct Scratch {
    int dev;
    void* stream;
    int tag;
    void* ptr;
    uint64_t bytes;
};
std::mutex g_ws_mu;
std::vector<Scratch> g_ws;

void* scratch(void* stream, int tag, uint64_t bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_ws_mu);
    Scratch* w = nullptr;
    for (auto& x : g_ws)
        if (x.dev == dev && x.stream == stream && x.tag == tag) w = &x;
    if (!w) {
        g_ws.push_back(Scratch{dev, stream, tag, nullptr, 0});
        w = &g_ws.back();
    }
    if (w->bytes < bytes) {
        if (w->ptr) {
            (void)hipStreamSynchronize(static_cast<hipStream_t>(stream));
            (void)hipFree(w->ptr);
            w->ptr = nullptr;
        }
        if (hipMalloc(&w->ptr, bytes) != hipSuccess) {
            w->bytes = 0;
            w->ptr = nullptr;
            return nullptr;
        }
        w->bytes = bytes;
    }
    return w->ptr;
}
enum { SCRATCH_DT = 1, SCRATCH_DTINFO = 2, SCRATCH_ENC = 3 };

// Tuning / ablation knobs (not part of the ABI): FSEHIP_ENC_LANES=32|64,
// FSEHIP_DEBUG bit mask (see fse_kernels.h).
uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* v = getenv(name);
    return v && *v ? (uint32_t)strtoul(v, nullptr, 0) : dflt;
}

// FSEHIP_STAMPS=1: per-workgroup phase stamps, averaged and printed to
// stderr after the (synchronised) launch.  Diagnostics only.
struct Stamps {
    uint64_t* d = nullptr;
    size_t n = 0;
    uint64_t* get(size_t groups) {
        if (!env_u32("FSEHIP_STAMPS", 0)) return nullptr;
        size_t need = groups * fsehip::kStamps;
        if (n < need) {
            if (d) (void)hipFree(d);
            if (hipMalloc(&d, need * 8) != hipSuccess) return d = nullptr;
            n = need;
        }
        (void)hipMemset(d, 0, need * 8);
        return d;
    }
    void report(const char* what, size_t groups, hipStream_t s) {
        if (!d) return;
        (void)hipStreamSynchronize(s);
        std::vector<uint64_t> h(groups * fsehip::kStamps);
        (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
        // deltas between consecutive recorded slots (kernels may skip slots);
        // per XCD (workgroups are placed round-robin over the 8 XCDs) the
        // span from the first start to the last stamp, for the mean number
        // of workgroups in flight per CU (32 CUs per XCD)
        double acc[fsehip::kStamps] = {0}, life = 0;
        size_t cnt[fsehip::kStamps] = {0}, nlife = 0;
        uint64_t lo_x[8], hi_x[8];
        for (int x = 0; x < 8; ++x) lo_x[x] = ~0ull, hi_x[x] = 0;
        for (size_t g = 0; g < groups; ++g) {
            const uint64_t* r = &h[g * fsehip::kStamps];
            int prev = -1;
            for (int k = 0; k < fsehip::kStamps - 1; ++k) {
                if (!r[k]) continue;
                if (prev >= 0 && r[k] >= r[prev]) { acc[k] += (double)(r[k] - r[prev]); cnt[k]++; }
                prev = k;
            }
            if (r[0] && prev > 0 && r[prev] >= r[0]) {
                life += (double)(r[prev] - r[0]);
                nlife++;
                lo_x[g % 8] = std::min(lo_x[g % 8], r[0]);
                hi_x[g % 8] = std::max(hi_x[g % 8], r[prev]);
            }
        }
        fprintf(stderr, "[stamps] %s:", what);
        for (int k = 1; k < fsehip::kStamps - 1; ++k)
            if (cnt[k]) fprintf(stderr, " %d:%.0f", k, acc[k] / cnt[k]);
        double span = 0;
        for (int x = 0; x < 8; ++x)
            if (hi_x[x] > lo_x[x]) span += (double)(hi_x[x] - lo_x[x]);
        fprintf(stderr, " (mean cycles per workgroup since the previous stamp)\n");
        if (nlife && span > 0)
            fprintf(stderr, "[stamps] %s: lifetime %.0f cycles, XCD span %.0f cycles, %.2f workgroups in flight per CU\n",
                    what, life / nlife, span / 8, life / (span * 32.0) * ((double)groups / nlife));
        // slot kStamps-1: kernel-defined counters (low / high 32 bits), averaged
        double lo = 0, hi = 0;
        for (size_t g = 0; g < groups; ++g) {
            const uint64_t v = h[g * fsehip::kStamps + fsehip::kStamps - 1];
            lo += (double)(v & 0xFFFFFFFFu);
            hi += (double)(v >> 32);
        }
        fprintf(stderr, "[stamps] %s counters: lo %.3f hi %.3f (mean per workgroup)\n", what, lo / groups, hi / groups);
    }
};
Stamps g_stamps_enc, g_stamps_dec;

bool device_ok() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return false;
    return n > 0;
}

uint32_t lmax_for(const fsehip_params* p) {
    if (p->max_table_log) return p->max_table_log;
    if (p->table_log == 0) return 11;  // optimal_log2 never exceeds 11 (histogram.rs:273-276)
    return p->table_log < 11 ? 11 : p->table_log;
}

// Device staging for the host-pointer entry points (grow-only, per thread).
struct Staging {
    uint8_t* buf[4] = {nullptr, nullptr, nullptr, nullptr};
    size_t cap[4] = {0, 0, 0, 0};
    int device = -1;
    ~Staging() {
        for (int i = 0; i < 4; ++i)
            if (buf[i]) (void)hipFree(buf[i]);
    }
    uint8_t* get(int i, size_t bytes) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (dev != device) {
            for (int j = 0; j < 4; ++j) {
                if (buf[j]) (void)hipFree(buf[j]);
                buf[j] = nullptr;
                cap[j] = 0;
            }
            device = dev;
        }
        if (cap[i] < bytes) {
            if (buf[i]) (void)hipFree(buf[i]);
            buf[i] = nullptr;
            cap[i] = 0;
            void* p = nullptr;
            size_t want = round_up(std::max<size_t>(bytes, 4096), 4096);
            if (hipMalloc(&p, want) != hipSuccess) return nullptr;
            buf[i] = static_cast<uint8_t*>(p);
            cap[i] = want;
        }
        return buf[i];
    }
};
thread_local Staging g_stage;

struct Meta {
    uint32_t comp_len;
    uint32_t payload_bits;
    int32_t status;
    uint32_t pad;
};

int compress_one(const uint8_t* src, size_t n, uint32_t table_log, uint8_t* dst, size_t dst_cap, size_t* dst_len,
                 uint64_t* payload_bits, uint32_t nstates = 2) {
    if (!dst_len) return FSE_ERR_BAD_ARG;
    if (n == 0) return FSE_ERR_EMPTY;  // size.ilog2() panics (histogram.rs:266)
    if (n > (1u << 28)) return FSE_ERR_UNSUPPORTED;
    if (table_log > 12) return FSE_ERR_UNSUPPORTED;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    fsehip_params p{(uint32_t)round_up(n, 16), table_log, 0, table_log ? std::max<uint32_t>(table_log, 11) : 11,
                    nstates};
    const uint64_t slot = fsehip_slot_bytes(p.block_size, p.max_table_log);
    uint8_t* d_src = g_stage.get(0, round_up(n, 16) + 16);
    uint8_t* d_out = g_stage.get(1, slot);
    uint8_t* d_meta = g_stage.get(2, sizeof(Meta));
    if (!d_src || !d_out || !d_meta) return FSE_ERR_HIP;
    if (hipMemcpy(d_src, src, n, hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    Meta* m = reinterpret_cast<Meta*>(d_meta);
    int rc = fsehip_compress_blocks(&p, d_src, n, d_out, slot, &m->comp_len, &m->payload_bits, nullptr,
                                    &m->status, nullptr);
    if (rc) return rc;
    Meta h{};
    if (hipMemcpy(&h, d_meta, sizeof(Meta), hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    if (h.status != FSE_OK) return h.status;
    if (*dst_len > dst_cap || dst_cap - *dst_len < h.comp_len) return FSE_ERR_DST_TOO_SMALL;
    if (hipMemcpy(dst + *dst_len, d_out, h.comp_len, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    *dst_len += h.comp_len;
    if (payload_bits) *payload_bits = h.payload_bits;
    return FSE_OK;
}

}  // namespace

extern "C" {

uint64_t fsehip_slot_bytes(uint32_t block_size, uint32_t max_table_log) {
    const uint64_t L = max_table_log ? max_table_log : 12;
    // header <= 512 bytes; every symbol costs <= L bits (fse.rs:170-186);
    // + both final states and the marker (lib.rs:178-181).
    const uint64_t payload = ((uint64_t)block_size * L + 2 * L + 1 + 7) / 8;
    return round_up(512 + payload + 16, 256);
}

uint32_t fsehip_sidecar_per_block(uint32_t block_size, uint32_t ckpt_interval) {
    if (ckpt_interval == 0) return 0;
    return block_size / 2u / ckpt_interval + 2u;
}

uint32_t fsehip_sidecar_per_block_ns(uint32_t block_size, uint32_t ckpt_interval, uint32_t nstates) {
    if (ckpt_interval == 0) return 0;
    return nstates == 1 ? block_size / ckpt_interval + 2u : block_size / 2u / ckpt_interval + 2u;
}

int fsehip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* fsehip_version(void) { return "fsehip 0.1 (gfx950)"; }

int fsehip_compress_blocks(const fsehip_params* p, const uint8_t* d_src, uint64_t n_total, uint8_t* d_out,
                           uint64_t slot_bytes, uint32_t* d_comp_len, uint32_t* d_payload_bits, uint64_t* d_sidecar,
                           int32_t* d_status, fsehip_stream_t stream) {
    if (!p || !d_src || !d_out || !d_comp_len || !d_status) return FSE_ERR_BAD_ARG;
    if (n_total == 0) return FSE_ERR_EMPTY;
    const uint32_t bs = p->block_size ? p->block_size : kDefaultBlock;
    const uint64_t n_blocks = (n_total + bs - 1) / bs;
    if (n_blocks > 1 && (bs & 15u)) return FSE_ERR_BAD_ARG;
    if (n_blocks > 0xFFFFFFFFull) return FSE_ERR_BAD_ARG;
    if (p->table_log > 15) return FSE_ERR_TABLELOG_RANGE;
    const uint32_t lmax = lmax_for(p);
    if (lmax > 12) return FSE_ERR_UNSUPPORTED;
    if (slot_bytes & 15u) return FSE_ERR_BAD_ARG;
    const uint32_t ns = p->nstates == 1 ? 1u : 2u;
    if (p->nstates > 2) return FSE_ERR_BAD_ARG;
    if (p->ckpt_interval && (p->ckpt_interval < (ns == 1 ? 16u : 8u) || (p->ckpt_interval & (p->ckpt_interval - 1))))
        return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    fsehip::EncParams P{};
    P.nstates = ns;
    P.src = d_src;
    P.n_total = n_total;
    P.block_size = bs;
    P.n_blocks = (uint32_t)n_blocks;
    P.table_log = p->table_log;
    P.ckpt_interval = d_sidecar ? p->ckpt_interval : 0;
    P.ckpt_per_block = fsehip_sidecar_per_block_ns(bs, P.ckpt_interval, ns);
    P.out = d_out;
    P.slot_bytes = slot_bytes;
    P.comp_len = d_comp_len;
    P.payload_bits = d_payload_bits;
    P.sidecar = P.ckpt_interval ? d_sidecar : nullptr;
    P.status = d_status;
    P.lanes = (ns == 2 && env_u32("FSEHIP_ENC_LANES", 64) == 32) ? 32 : 64;
    P.debug = env_u32("FSEHIP_DEBUG", 0);
    // scratch-path lane streams: worst case of a lane's steps at L = lmax,
    // plus the top lane's extra step and lane 0's finals + marker, in whole
    // 128-byte lines so no two lanes share a cache line
    // (measured slower than the repair path on C2, skewed and uniform data:
    // opt-in, FSEHIP_ENC_PATH=2 or 0 = by distribution)
    P.path = env_u32("FSEHIP_ENC_PATH", 1);
    P.warm = env_u32("FSEHIP_ENC_WARM", 64);
    P.pmax256 = env_u32("FSEHIP_ENC_PMAX", 128);
    P.xlds = env_u32("FSEHIP_ENC_XLDS", 0);
    P.scratch = nullptr;
    if (P.path != 1 && P.lanes == 64 && ns == 2) {
        const uint64_t steps = ns == 2 ? (bs >= 2 ? bs / 2 - 1 : 1) : (bs >= 1 ? bs - 1 : 1);
        const uint64_t spc = ns == 2 ? 8 : 16;
        uint64_t S = (steps + P.lanes - 1) / P.lanes;
        S = std::max<uint64_t>(spc, (S + spc - 1) / spc * spc);
        const uint64_t maxbits = S * ns * lmax + 3ull * lmax + 1;
        P.scr_lane_words = (uint32_t)round_up((maxbits + 31) / 32 + 1, 32);
        P.scratch = static_cast<uint32_t*>(
            scratch(stream, SCRATCH_ENC, n_blocks * P.lanes * (uint64_t)P.scr_lane_words * 4u));
        if (!P.scratch) return FSE_ERR_HIP;
    }
    const size_t groups = (n_blocks * P.lanes + 63) / 64;
    P.stamps = g_stamps_enc.get(groups);
    hipError_t e = fsehip::launch_encode(P, lmax, static_cast<hipStream_t>(stream));
    if (P.stamps) g_stamps_enc.report("encode", groups, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

static int decompress_impl(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                           const uint32_t* d_comp_len, const uint64_t* d_sidecar, uint8_t* d_out, uint64_t n_total,
                           uint64_t* d_sidecar_out, int32_t* d_status, uint32_t* d_out_len, uint32_t out_cap,
                           fsehip_stream_t stream, const uint32_t* d_dt = nullptr,
                           const int32_t* d_dtinfo = nullptr) {
    if (!p || !d_in || !d_comp_len || !d_out || !d_status) return FSE_ERR_BAD_ARG;
    const uint32_t bs = p->block_size ? p->block_size : kDefaultBlock;
    const uint64_t n_blocks = n_total ? (n_total + bs - 1) / bs : 1;
    if (n_blocks > 1 && (bs & 15u)) return FSE_ERR_BAD_ARG;
    if (slot_bytes & 3u) return FSE_ERR_BAD_ARG;
    const uint32_t ns = p->nstates == 1 ? 1u : 2u;
    if (p->nstates > 2) return FSE_ERR_BAD_ARG;
    if ((d_sidecar || d_sidecar_out) &&
        (p->ckpt_interval < (ns == 1 ? 16u : 8u) || (p->ckpt_interval & (p->ckpt_interval - 1))))
        return FSE_ERR_BAD_ARG;
    if (ns == 1 && (!d_dt || d_sidecar_out)) return FSE_ERR_UNSUPPORTED;  // 1-state runs on prebuilt tables only
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    fsehip::DecParams P{};
    P.nstates = ns;
    P.in = d_in;
    P.slot_bytes = slot_bytes;
    P.comp_len = d_comp_len;
    P.sidecar = d_sidecar;
    P.ckpt_interval = p->ckpt_interval;
    P.ckpt_per_block = fsehip_sidecar_per_block_ns(bs, p->ckpt_interval, ns);
    P.out = d_out;
    P.n_total = n_total;
    P.block_size = bs;
    P.n_blocks = (uint32_t)n_blocks;
    P.out_cap = out_cap;
    P.status = d_status;
    P.out_len = d_out_len;
    P.sidecar_out = d_sidecar_out;
    P.debug = env_u32("FSEHIP_DEBUG", 0) >> 4;
    P.waves = env_u32("FSEHIP_DEC_WAVES", 4) == 8 ? 8 : 4;
    P.variant = env_u32("FSEHIP_DEC_VAR", 12);
    P.dual = env_u32("FSEHIP_DEC_DUAL", 0);
    P.stage_kib = env_u32("FSEHIP_DEC_PP", 44);
    // the decoder reads L from each header; size its tables for the bound
    uint32_t lmax = p->max_table_log ? p->max_table_log : 12;
    P.dt = d_dt;
    P.dtinfo = d_dtinfo;
    P.stamps = g_stamps_dec.get(n_blocks);
    hipError_t e = fsehip::launch_decode(P, lmax, static_cast<hipStream_t>(stream));
    if (P.stamps) g_stamps_dec.report("decode", n_blocks, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

static uint32_t dt_lmax(const fsehip_params* p) { return (p && p->max_table_log && p->max_table_log <= 11) ? 11 : 12; }

uint64_t fsehip_dtable_bytes(uint32_t max_table_log) {
    return 4ull << ((max_table_log && max_table_log <= 11) ? 11 : 12);
}

int fsehip_build_dtables(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes, const uint32_t* d_comp_len,
                         uint32_t n_blocks, uint32_t* d_dtables, int32_t* d_dtinfo, fsehip_stream_t stream) {
    if (!p || !d_in || !d_comp_len || !d_dtables || !d_dtinfo || (slot_bytes & 255u)) return FSE_ERR_BAD_ARG;
    if (n_blocks == 0) return FSE_OK;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    fsehip::DtParams D{};
    D.debug = env_u32("FSEHIP_DT_DEBUG", 0);
    D.in = d_in;
    D.slot_bytes = slot_bytes;
    D.comp_len = d_comp_len;
    D.n_blocks = n_blocks;
    D.dt = d_dtables;
    D.dtinfo = d_dtinfo;
    hipError_t e = fsehip::launch_dtables(D, dt_lmax(p), static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

int fsehip_decompress_blocks_dt(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                                const uint32_t* d_comp_len, const uint64_t* d_sidecar, const uint32_t* d_dtables,
                                const int32_t* d_dtinfo, uint8_t* d_out, uint64_t n_total, int32_t* d_status,
                                fsehip_stream_t stream) {
    if (n_total == 0) return FSE_ERR_EMPTY;
    if (!p || !d_dtables || !d_dtinfo) return FSE_ERR_BAD_ARG;
    if (d_sidecar && p->ckpt_interval == 0) return FSE_ERR_BAD_ARG;
    // without a sidecar: 2-state blocks take the speculative sync decoder,
    // 1-state blocks the serial one
    fsehip_params q = *p;
    q.max_table_log = dt_lmax(p);  // the table stride the tables were built with
    return decompress_impl(&q, d_in, slot_bytes, d_comp_len, d_sidecar, d_out, n_total, nullptr, d_status, nullptr,
                           0, stream, d_dtables, d_dtinfo);
}


int fsehip_decompress_blocks(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                             const uint32_t* d_comp_len, const uint64_t* d_sidecar, uint8_t* d_out, uint64_t n_total,
                             int32_t* d_status, fsehip_stream_t stream) {
    if (n_total == 0) return FSE_ERR_EMPTY;
    if (d_sidecar && p && p->ckpt_interval == 0) return FSE_ERR_BAD_ARG;
    // FSEHIP_DEC_FUSED=1: the one-kernel path (serial one lane per block without a sidecar)
    if (p && (p->nstates == 1 || !env_u32("FSEHIP_DEC_FUSED", 0))) {
        // two kernels: decode tables for all blocks at high occupancy, then
        // the LDS-heavy segment decode with no serial phase
        const uint32_t bs = p->block_size ? p->block_size : kDefaultBlock;
        const uint64_t n_blocks = (n_total + bs - 1) / bs;
        if (!device_ok()) return FSE_ERR_NO_DEVICE;
        uint32_t* dt = static_cast<uint32_t*>(scratch(stream, SCRATCH_DT, fsehip_dtable_bytes(p->max_table_log) * n_blocks));
        int32_t* info = static_cast<int32_t*>(scratch(stream, SCRATCH_DTINFO, 4ull * n_blocks));
        if (!dt || !info) return FSE_ERR_HIP;
        int rc = fsehip_build_dtables(p, d_in, slot_bytes, d_comp_len, (uint32_t)n_blocks, dt, info, stream);
        if (rc != FSE_OK) return rc;
        return fsehip_decompress_blocks_dt(p, d_in, slot_bytes, d_comp_len, d_sidecar, dt, info, d_out, n_total,
                                           d_status, stream);
    }
    return decompress_impl(p, d_in, slot_bytes, d_comp_len, d_sidecar, d_out, n_total, nullptr, d_status, nullptr,
                           0, stream);
}

int fsehip_build_sidecar(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                         const uint32_t* d_comp_len, uint8_t* d_out, uint64_t n_total, uint64_t* d_sidecar_out,
                         int32_t* d_status, fsehip_stream_t stream) {
    if (n_total == 0) return FSE_ERR_EMPTY;
    if (p && p->nstates != 1 && d_sidecar_out && !env_u32("FSEHIP_DEC_FUSED", 0)) {
        // tables for all blocks, then the serial decoder (table in LDS, 20 blocks per CU) records it
        if (p->ckpt_interval < 8 || (p->ckpt_interval & (p->ckpt_interval - 1))) return FSE_ERR_BAD_ARG;
        const uint32_t bs = p->block_size ? p->block_size : kDefaultBlock;
        const uint64_t n_blocks = (n_total + bs - 1) / bs;
        if (!device_ok()) return FSE_ERR_NO_DEVICE;
        uint32_t* dt = static_cast<uint32_t*>(scratch(stream, SCRATCH_DT, fsehip_dtable_bytes(p->max_table_log) * n_blocks));
        int32_t* info = static_cast<int32_t*>(scratch(stream, SCRATCH_DTINFO, 4ull * n_blocks));
        if (!dt || !info) return FSE_ERR_HIP;
        int rc = fsehip_build_dtables(p, d_in, slot_bytes, d_comp_len, (uint32_t)n_blocks, dt, info, stream);
        if (rc != FSE_OK) return rc;
        fsehip_params q = *p;
        q.max_table_log = dt_lmax(p);
        return decompress_impl(&q, d_in, slot_bytes, d_comp_len, nullptr, d_out, n_total, d_sidecar_out, d_status,
                               nullptr, 0, stream, dt, info);
    }
    return decompress_impl(p, d_in, slot_bytes, d_comp_len, nullptr, d_out, n_total, d_sidecar_out, d_status,
                           nullptr, 0, stream);
}

int fsehip_histogram_blocks(const uint8_t* d_src, uint64_t n_total, uint32_t block_size, uint32_t* d_counts,
                            uint32_t* d_table_len, fsehip_stream_t stream) {
    if (!d_src || !d_counts) return FSE_ERR_BAD_ARG;
    const uint32_t bs = block_size ? block_size : kDefaultBlock;
    const uint64_t n_blocks = n_total ? (n_total + bs - 1) / bs : 1;
    if (n_blocks > 1 && (bs & 15u)) return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    hipError_t e = fsehip::launch_histogram(d_src, n_total, bs, (uint32_t)n_blocks, d_counts, d_table_len,
                                            static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

int fsehip_pack_blocks(const uint8_t* d_slots, uint64_t slot_bytes, const uint32_t* d_comp_len,
                       const uint64_t* d_offsets, uint32_t n_blocks, uint8_t* d_stream, fsehip_stream_t stream) {
    if (!d_slots || !d_comp_len || !d_offsets || !d_stream || (slot_bytes & 15u)) return FSE_ERR_BAD_ARG;
    if (n_blocks == 0) return FSE_OK;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    hipError_t e = fsehip::launch_pack(d_slots, slot_bytes, d_comp_len, d_offsets, n_blocks, d_stream, 0,
                                       static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

int fsehip_unpack_blocks(const uint8_t* d_stream, const uint64_t* d_offsets, const uint32_t* d_comp_len,
                         uint32_t n_blocks, uint8_t* d_slots, uint64_t slot_bytes, fsehip_stream_t stream) {
    if (!d_slots || !d_comp_len || !d_offsets || !d_stream || (slot_bytes & 15u)) return FSE_ERR_BAD_ARG;
    if (n_blocks == 0) return FSE_OK;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    hipError_t e = fsehip::launch_pack(d_slots, slot_bytes, d_comp_len, d_offsets, n_blocks,
                                       const_cast<uint8_t*>(d_stream), 1, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

int fsehip_copy_blocks(const uint8_t* d_src, const uint64_t* d_src_offsets, const uint32_t* d_lens, uint32_t n_blocks,
                       uint8_t* d_dst, const uint64_t* d_dst_offsets, fsehip_stream_t stream) {
    if (n_blocks == 0) return FSE_OK;
    if (!d_src || !d_src_offsets || !d_lens || !d_dst || !d_dst_offsets) return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    hipError_t e = fsehip::launch_copy(d_src, d_src_offsets, d_lens, n_blocks, d_dst, d_dst_offsets,
                                       static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

int fsehip_generate(int kind, double prob, uint64_t seed, uint32_t block_size, uint8_t* d_out, uint64_t n_total,
                    fsehip_stream_t stream) {
    if (!d_out || kind < 0 || kind > 2) return FSE_ERR_BAD_ARG;
    if (n_total == 0) return FSE_OK;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    fsehip::GenParams G{};
    G.out = d_out;
    G.n_total = n_total;
    G.block_size = block_size ? block_size : kDefaultBlock;
    G.seed = seed;
    G.kind = kind;
    if (kind == 0) {
        // LUT of benches/fse_benchmark.rs:5-20 as symbol start indices
        if (prob < 0.005) prob = 0.005;
        if (prob > 0.995) prob = 0.995;
        size_t remaining = 4096, idx = 0;
        uint32_t s = 0;
        while (remaining > 0) {
            size_t cnt = (size_t)((double)remaining * prob);
            if (cnt < 1) cnt = 1;
            if (s >= 1024) return FSE_ERR_BAD_ARG;
            G.bound[s++] = (uint16_t)idx;
            idx += cnt;
            remaining -= cnt;
        }
        G.nsym = s;
    }
    hipError_t e = fsehip::launch_generate(G, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

// ---------------------------------------------------------------- host API

int fse_compress2(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len,
                  uint64_t* payload_bits) {
    return compress_one(src, n, 0, dst, dst_cap, dst_len, payload_bits);
}

int fse_compress2_log(const uint8_t* src, size_t n, uint32_t table_log, uint8_t* dst, size_t dst_cap,
                      size_t* dst_len, uint64_t* payload_bits) {
    if (table_log == 0) return FSE_ERR_TABLELOG_RANGE;
    return compress_one(src, n, table_log, dst, dst_cap, dst_len, payload_bits);
}

int fse_decompress2(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len) {
    if (!dst_len || *dst_len > dst_cap) return FSE_ERR_BAD_ARG;
    if (n == 0) return FSE_ERR_EMPTY;  // BitStreamReader::new asserts (stream_reader.rs:17)
    if (n > (1u << 30)) return FSE_ERR_UNSUPPORTED;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    const uint64_t padded = round_up(n, 16) + 16;
    const uint64_t cap64 = std::min<uint64_t>(dst_cap - *dst_len, 0x7FFFFFFFu);
    uint8_t* d_in = g_stage.get(0, padded);
    uint8_t* d_out = g_stage.get(1, std::max<uint64_t>(cap64, 16));
    uint8_t* d_meta = g_stage.get(2, sizeof(Meta));
    if (!d_in || !d_out || !d_meta) return FSE_ERR_HIP;
    if (hipMemset(d_in, 0, padded) != hipSuccess) return FSE_ERR_HIP;
    if (hipMemcpy(d_in, src, n, hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    Meta* m = reinterpret_cast<Meta*>(d_meta);
    Meta h0{(uint32_t)n, 0, 0, 0};
    if (hipMemcpy(d_meta, &h0, sizeof(Meta), hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    fsehip_params p{0, 0, 0, 12};
    int rc = decompress_impl(&p, d_in, padded, &m->comp_len, nullptr, d_out, 0, nullptr, &m->status,
                             &m->payload_bits, (uint32_t)cap64, nullptr);
    if (rc) return rc;
    Meta h{};
    if (hipMemcpy(&h, d_meta, sizeof(Meta), hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    if (h.status != FSE_OK) return h.status;
    const uint32_t out_len = h.payload_bits;  // decoded byte count
    if (out_len && hipMemcpy(dst + *dst_len, d_out, out_len, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    *dst_len += out_len;
    return FSE_OK;
}

int fse_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len, uint64_t* payload_bits) {
    // lib.rs:112-143; n == 1 is valid here (a lone seed state), unlike fse_compress2
    return compress_one(src, n, 0, dst, dst_cap, dst_len, payload_bits, 1);
}

int fse_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len) {
    if (!dst_len || *dst_len > dst_cap) return FSE_ERR_BAD_ARG;
    if (n == 0) return FSE_ERR_EMPTY;  // BitStreamReader::new asserts (stream_reader.rs:17)
    if (n > (1u << 30)) return FSE_ERR_UNSUPPORTED;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    const uint64_t padded = round_up(n + 16, 256);
    const uint64_t cap64 = std::min<uint64_t>(dst_cap - *dst_len, 0x7FFFFFFFu);
    uint8_t* d_in = g_stage.get(0, padded);
    uint8_t* d_out = g_stage.get(1, std::max<uint64_t>(cap64, 16));
    uint8_t* d_meta = g_stage.get(2, sizeof(Meta));
    uint8_t* d_dt = g_stage.get(3, fsehip_dtable_bytes(12) + 16);
    if (!d_in || !d_out || !d_meta || !d_dt) return FSE_ERR_HIP;
    if (hipMemset(d_in, 0, padded) != hipSuccess) return FSE_ERR_HIP;
    if (hipMemcpy(d_in, src, n, hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    Meta* m = reinterpret_cast<Meta*>(d_meta);
    Meta h0{(uint32_t)n, 0, 0, 0};
    if (hipMemcpy(d_meta, &h0, sizeof(Meta), hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    fsehip_params p{0, 0, 0, 12, 1};
    uint32_t* dt = reinterpret_cast<uint32_t*>(d_dt);
    int32_t* info = reinterpret_cast<int32_t*>(d_dt + fsehip_dtable_bytes(12));
    int rc = fsehip_build_dtables(&p, d_in, padded, &m->comp_len, 1, dt, info, nullptr);
    if (rc) return rc;
    rc = decompress_impl(&p, d_in, padded, &m->comp_len, nullptr, d_out, 0, nullptr, &m->status, &m->payload_bits,
                         (uint32_t)cap64, nullptr, dt, info);
    if (rc) return rc;
    Meta h{};
    if (hipMemcpy(&h, d_meta, sizeof(Meta), hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    if (h.status != FSE_OK) return h.status;
    const uint32_t out_len = h.payload_bits;  // decoded byte count
    if (out_len && hipMemcpy(dst + *dst_len, d_out, out_len, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    *dst_len += out_len;
    return FSE_OK;
}

int histogram_count(const uint8_t* src, size_t n, uint32_t counts[256], uint32_t* table_len) {
    if (!counts) return FSE_ERR_BAD_ARG;
    if (n > 0xFFFFFFFFull) return FSE_ERR_BAD_ARG;  // histogram.rs:19 assert
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    uint8_t* d_src = g_stage.get(0, round_up(n, 16) + 16);
    uint8_t* d_cnt = g_stage.get(2, 257 * 4);
    if (!d_src || !d_cnt) return FSE_ERR_HIP;
    if (n && hipMemcpy(d_src, src, n, hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    uint32_t* c = reinterpret_cast<uint32_t*>(d_cnt);
    hipError_t e = fsehip::launch_histogram(d_src, n, (uint32_t)std::max<size_t>(n, 1), 1, c, c + 256, nullptr);
    if (e != hipSuccess) return FSE_ERR_HIP;
    uint32_t h[257];
    if (hipMemcpy(h, d_cnt, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    memcpy(counts, h, 256 * sizeof(uint32_t));
    if (table_len) *table_len = h[256];
    return FSE_OK;
}

// Diagnostics only (not part of include/fsehip.h): resident workgroups per CU.
int fsehipx_occupancy(char* buf, int cap) {
    if (!buf || cap <= 0 || !device_ok()) return 0;
    return fsehip::occupancy_report(buf, cap);
}

}  // extern "C"
