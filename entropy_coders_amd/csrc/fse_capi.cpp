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
#include <atomic>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/fsehip.h"
#include "fse_kernels.h"

namespace {

constexpr uint32_t kDefaultBlock = 65536;
// Largest block: the kernels count a block's bits in u32 (payload bits,
// sidecar bit positions, suffix sums), and block_size * 15 + header must stay
// below 2^32 bits.
constexpr uint32_t kMaxBlock = 1u << 28;

uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// Per-(device, stream) grow-only device workspace for the two-kernel encode
// and decode.  A caller holds the workspace's lock (a Lease) from taking the
// buffers until its last launch on them is enqueued: calls on one stream then
// use the buffers in stream order, and a call that has to grow a buffer
// synchronises the stream (the work of earlier holders has been enqueued on
// it) before freeing the old one.  Different streams get different
// workspaces.
enum {
    SCRATCH_DT = 0,
    SCRATCH_DTINFO = 1,
    SCRATCH_BITS = 2,
    SCRATCH_STATES = 3,
    SCRATCH_BULK = 4,
    SCRATCH_HDR = 5,  // the lane-parallel header parse's output (optional)
    SCRATCH_SPREAD = 6,  // the L >= 13 encoder's spread symbols when the slots cannot hold them
    SCRATCH_KINDS = 7
};
struct Workspace {
    int dev;
    void* stream;
    std::mutex mu;
    void* ptr[SCRATCH_KINDS] = {};
    uint64_t bytes[SCRATCH_KINDS] = {};
    // smallest size whose allocation failed (optional buffers only): later
    // calls asking for as much or more take their fallback at once instead of
    // retrying a multi-GiB hipMalloc on every call; cleared by
    // fsehip_release_workspace
    uint64_t failed[SCRATCH_KINDS] = {};
};
std::mutex g_ws_mu;
std::vector<std::unique_ptr<Workspace>> g_ws;

struct Lease {
    Workspace* ws = nullptr;
    std::unique_lock<std::mutex> lk;
    explicit Lease(void* stream) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return;
        {
            std::lock_guard<std::mutex> g(g_ws_mu);
            for (auto& x : g_ws)
                if (x->dev == dev && x->stream == stream) ws = x.get();
            if (!ws) {
                g_ws.push_back(std::make_unique<Workspace>());
                ws = g_ws.back().get();
                ws->dev = dev;
                ws->stream = stream;
            }
        }
        lk = std::unique_lock<std::mutex>(ws->mu);
    }
    // `optional`: the caller has a fallback without the buffer (the
    // deferred-symbol decode), so a failed size is remembered
    void* get(int tag, uint64_t bytes, bool optional = false) {
        if (!ws) return nullptr;
        if (ws->bytes[tag] < bytes) {
            if (optional && ws->failed[tag] && bytes >= ws->failed[tag]) return nullptr;
            if (ws->ptr[tag]) {
                (void)hipStreamSynchronize(static_cast<hipStream_t>(ws->stream));
                (void)hipFree(ws->ptr[tag]);
                ws->ptr[tag] = nullptr;
            }
            ws->bytes[tag] = 0;
            if (hipMalloc(&ws->ptr[tag], bytes) != hipSuccess) {
                (void)hipGetLastError();  // an optional buffer's failure must not surface in a later launch check
                ws->ptr[tag] = nullptr;
                if (optional) ws->failed[tag] = ws->failed[tag] ? std::min(ws->failed[tag], bytes) : bytes;
                return nullptr;
            }
            ws->bytes[tag] = bytes;
        }
        return ws->ptr[tag];
    }
};

// Free every buffer of the matching workspaces (device < 0: all devices;
// stream is matched as given) after the work enqueued on their streams.
int release_workspaces(int device, void* stream, bool any_stream) {
    std::vector<Workspace*> hit;
    {
        std::lock_guard<std::mutex> g(g_ws_mu);
        for (auto& x : g_ws)
            if ((device < 0 || x->dev == device) && (any_stream || x->stream == stream)) hit.push_back(x.get());
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    int rc = FSE_OK;
    for (Workspace* w : hit) {
        std::lock_guard<std::mutex> lk(w->mu);
        if (hipSetDevice(w->dev) != hipSuccess) {
            (void)hipGetLastError();
            rc = FSE_ERR_HIP;
            continue;
        }
        bool any = false;
        for (int t = 0; t < SCRATCH_KINDS; ++t) any = any || w->ptr[t];
        if (any && hipStreamSynchronize(static_cast<hipStream_t>(w->stream)) != hipSuccess) rc = FSE_ERR_HIP;
        for (int t = 0; t < SCRATCH_KINDS; ++t) {
            if (w->ptr[t] && hipFree(w->ptr[t]) != hipSuccess) rc = FSE_ERR_HIP;
            w->ptr[t] = nullptr;
            w->bytes[t] = 0;
            w->failed[t] = 0;
        }
    }
    (void)hipSetDevice(prev);
    return rc;
}

// Tuning / ablation / diagnostics knobs (FSEHIP_ENC_LANES, FSEHIP_DEBUG,
// FSEHIP_STAMPS, FSEHIP_SERIAL_*, FSEHIP_*_XLDS; see fse_kernels.h) exist
// only in the diagnostics build libfsehip_diag.so (make diag, -DFSEHIP_DIAG):
// several of them change the output on purpose (ablations).  The product
// libfsehip.so reads no environment variable -- every call's result depends
// on its arguments alone, as the crate's pure functions do.
#ifdef FSEHIP_DIAG
uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* v = getenv(name);
    return v && *v ? (uint32_t)strtoul(v, nullptr, 0) : dflt;
}
#else
uint32_t env_u32(const char*, uint32_t dflt) { return dflt; }
#endif

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
Stamps g_stamps_enc, g_stamps_dec, g_stamps_dt;

bool device_ok() {
    static std::atomic<bool> seen{false};  // devices do not go away: ask the runtime once (~17 us a call)
    if (seen.load(std::memory_order_relaxed)) return true;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return false;
    seen.store(true, std::memory_order_relaxed);
    return true;
}

uint32_t lmax_for(const fsehip_params* p) {
    if (p->max_table_log) return p->max_table_log;
    if (p->table_log == 0) return 11;  // optimal_log2 never exceeds 11 (histogram.rs:273-276)
    return p->table_log < 11 ? 11 : p->table_log;
}

// Kernel table bound for a max_table_log: tables are instantiated at 11
// (L <= 11), 12, 13, 14 and 15 (normalize clamps requests to 15,
// histogram.rs:96); 0 = 12.  Decode tables use this stride.
uint32_t kern_lmax(uint32_t max_table_log) {
    if (max_table_log == 0) return 12;
    return max_table_log <= 11 ? 11 : max_table_log >= 15 ? 15 : max_table_log;
}

// Device staging for the host-pointer entry points (grow-only, per thread).
struct Staging {
    static constexpr int K = 8;
    uint8_t* buf[K] = {};
    size_t cap[K] = {};
    int device = -1;
    ~Staging() { release(); }
    void release() {
        for (int i = 0; i < K; ++i) {
            if (buf[i]) (void)hipFree(buf[i]);
            buf[i] = nullptr;
            cap[i] = 0;
        }
    }
    uint8_t* get(int i, size_t bytes) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (dev != device) {
            for (int j = 0; j < K; ++j) {
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

// Pinned host staging for the host-pointer calls (grow-only, per thread):
// [0] the call's input on its way to the device, [1] its result record and
// output on the way back.  A pageable hipMemcpy costs ~100 us per call here
// (profiles/r04/single_stream/), a copy through pinned memory a few.
constexpr size_t kPinOut = size_t(4) << 20;  // output bytes returned through [1]; the rest by hipMemcpy
struct PinnedStaging {
    uint8_t* buf[2] = {};
    size_t cap[2] = {};
    ~PinnedStaging() { release(); }
    void release() {
        for (int i = 0; i < 2; ++i) {
            if (buf[i]) (void)hipHostFree(buf[i]);
            buf[i] = nullptr;
            cap[i] = 0;
        }
    }
    uint8_t* get(int i, size_t bytes) {
        if (cap[i] < bytes) {
            if (buf[i]) (void)hipHostFree(buf[i]);
            buf[i] = nullptr;
            cap[i] = 0;
            void* p = nullptr;
            const size_t want = round_up(std::max<size_t>(bytes, size_t(64) << 10), 4096);
            if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return nullptr;
            buf[i] = static_cast<uint8_t*>(p);
            cap[i] = want;
        }
        return buf[i];
    }
};
thread_local PinnedStaging g_pin;

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
    if (n > kMaxBlock) return FSE_ERR_UNSUPPORTED;
    if (table_log > 15) table_log = 15;  // Histogram::normalize clamps (histogram.rs:96)
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    fsehip_params p{(uint32_t)round_up(n, 16), table_log, 0, table_log ? std::max<uint32_t>(table_log, 11) : 11,
                    nstates};
    const uint64_t slot = fsehip_slot_bytes(p.block_size, p.max_table_log);
    const size_t in_bytes = round_up(n, 16);
    const size_t pin_out = std::min<size_t>(slot, kPinOut);
    uint8_t* d_src = g_stage.get(0, in_bytes + 16);
    uint8_t* d_out = g_stage.get(1, slot);
    uint8_t* d_meta = g_stage.get(2, sizeof(Meta));
    uint8_t* h_in = g_pin.get(0, in_bytes);
    uint8_t* h_ret = g_pin.get(1, 256 + pin_out);
    if (!d_src || !d_out || !d_meta || !h_in || !h_ret) return FSE_ERR_HIP;
    memcpy(h_in, src, n);
    auto fail = [](int rc) {  // nothing may still read or write the pinned buffers
        (void)hipStreamSynchronize(nullptr);
        return rc;
    };
    if (hipMemcpyAsync(d_src, h_in, in_bytes, hipMemcpyHostToDevice, nullptr) != hipSuccess) return fail(FSE_ERR_HIP);
    Meta* m = reinterpret_cast<Meta*>(d_meta);
    int rc = fsehip_compress_blocks(&p, d_src, n, d_out, slot, &m->comp_len, &m->payload_bits, nullptr,
                                    &m->status, nullptr);
    if (rc) return fail(rc);
    if (fsehip::launch_host_return(d_meta, d_out, &m->comp_len, h_ret, h_ret + 256, (uint32_t)pin_out, nullptr) !=
        hipSuccess)
        return fail(FSE_ERR_HIP);
    if (hipStreamSynchronize(nullptr) != hipSuccess) return FSE_ERR_HIP;
    Meta h;
    memcpy(&h, h_ret, sizeof h);
    if (h.status != FSE_OK) return h.status;
    if (*dst_len > dst_cap || dst_cap - *dst_len < h.comp_len) return FSE_ERR_DST_TOO_SMALL;
    const size_t head = std::min<size_t>(h.comp_len, pin_out);
    memcpy(dst + *dst_len, h_ret + 256, head);
    if (h.comp_len > head &&
        hipMemcpy(dst + *dst_len + head, d_out + head, h.comp_len - head, hipMemcpyDeviceToHost) != hipSuccess)
        return FSE_ERR_HIP;
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

#ifdef FSEHIP_DIAG
const char* fsehip_version(void) { return "fsehip 0.2 (gfx950, diagnostics build: environment knobs live)"; }
#else
const char* fsehip_version(void) { return "fsehip 0.2 (gfx950)"; }
#endif

int fsehip_release_workspace(int device, fsehip_stream_t stream) {
    const int rc = release_workspaces(device, stream, false);
    g_stage.release();
    g_pin.release();
    return rc;
}

int fsehip_compress_blocks(const fsehip_params* p, const uint8_t* d_src, uint64_t n_total, uint8_t* d_out,
                           uint64_t slot_bytes, uint32_t* d_comp_len, uint32_t* d_payload_bits, uint64_t* d_sidecar,
                           int32_t* d_status, fsehip_stream_t stream) {
    if (!p || !d_src || !d_out || !d_comp_len || !d_status) return FSE_ERR_BAD_ARG;
    if (n_total == 0) return FSE_ERR_EMPTY;
    const uint32_t bs = p->block_size ? p->block_size : kDefaultBlock;
    if (bs > kMaxBlock) return FSE_ERR_UNSUPPORTED;
    const uint64_t n_blocks = (n_total + bs - 1) / bs;
    if (n_blocks > 1 && (bs & 15u)) return FSE_ERR_BAD_ARG;
    if (n_blocks > 0xFFFFFFFFull) return FSE_ERR_BAD_ARG;
    const uint32_t lmax = kern_lmax(lmax_for(p));
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
    P.xlds = env_u32("FSEHIP_ENC_XLDS", 0);  // diagnostics: occupancy probe
    P.rank_inject = env_u32("FSEHIP_RANK_INJECT", 0);  // diagnostics: fault injection into the atomic ranks
    const size_t groups = (n_blocks * P.lanes + 63) / 64;
    P.stamps = g_stamps_enc.get(groups);
    // the L >= 13 kernels keep the spread's 2^lmax symbols in global memory:
    // in each block's slot after its header words when the slot has room,
    // else in a workspace buffer (held until the launch is enqueued)
    std::unique_ptr<Lease> lease;
    if (fsehip::enc_gsym(lmax) && slot_bytes < fsehip::ENC_SPREAD_OFF + (1ull << lmax)) {
        lease = std::make_unique<Lease>(stream);
        P.spread = static_cast<uint8_t*>(lease->get(SCRATCH_SPREAD, n_blocks << lmax));
        if (!P.spread) return FSE_ERR_HIP;
    }
    hipError_t e = fsehip::launch_encode(P, lmax, static_cast<hipStream_t>(stream));
    if (P.stamps) g_stamps_enc.report("encode", groups, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

// Sidecar-less decode at L <= 11 (both formats): the chains defer their symbols to
// a map kernel when the stream's workspace can hold the state pairs (2 bytes
// per output byte); without it the single-kernel serial decode runs.
// FSEHIP_SERIAL_DEFER=0 (diagnostics) always takes the latter.
// The map kernel runs one 256-thread workgroup per block, so batches of
// 2^24 blocks or more (grid x threads >= 2^32) take the single-kernel decode.
static void defer_symbols(Lease& lease, fsehip::DecParams& P, uint32_t lmax) {
    if (lmax > 11 || P.block_size < 2u || P.n_blocks >= (1u << 24) || !env_u32("FSEHIP_SERIAL_DEFER", 1)) return;
    // the small buffer first: when it cannot be had, the multi-GiB state
    // buffer is never allocated (and never held by a decode that cannot use it)
    P.bulk = static_cast<uint32_t*>(lease.get(SCRATCH_BULK, 8ull * P.n_blocks, true));
    P.states = P.bulk ? static_cast<uint32_t*>(lease.get(SCRATCH_STATES, 2ull * P.n_blocks * P.block_size, true))
                      : nullptr;
    if (!P.states || !P.bulk) P.states = P.bulk = nullptr;
}

// Decode on prebuilt tables (dtable_blocks_kernel at stride kern_lmax):
// segment-parallel with a sidecar, else serial (container mode when n_total
// is known, the reference's own termination within out_cap otherwise).
static int decompress_impl(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                           const uint32_t* d_comp_len, const uint64_t* d_sidecar, uint8_t* d_out, uint64_t n_total,
                           uint64_t* d_sidecar_out, int32_t* d_status, uint32_t* d_out_len, uint32_t out_cap,
                           fsehip_stream_t stream, const uint32_t* d_dt, const int32_t* d_dtinfo,
                           Lease* lease = nullptr) {
    if (!p || !d_in || !d_comp_len || !d_out || !d_status || !d_dt || !d_dtinfo) return FSE_ERR_BAD_ARG;
    const uint32_t bs = p->block_size ? p->block_size : kDefaultBlock;
    if (bs > kMaxBlock) return FSE_ERR_UNSUPPORTED;
    const uint64_t n_blocks = n_total ? (n_total + bs - 1) / bs : 1;
    if (n_blocks > 1 && (bs & 15u)) return FSE_ERR_BAD_ARG;
    if (n_blocks > 0xFFFFFFFFull) return FSE_ERR_BAD_ARG;
    // the decoders stage / read whole 16- and 32-byte chunks of a slot and
    // store 16-byte output groups: aligned slots and buffers keep every
    // chunk inside its slot and every access aligned
    if ((slot_bytes & 31u) || (reinterpret_cast<uintptr_t>(d_in) & 15u) || (reinterpret_cast<uintptr_t>(d_out) & 15u))
        return FSE_ERR_BAD_ARG;
    const uint32_t ns = p->nstates == 1 ? 1u : 2u;
    if (p->nstates > 2) return FSE_ERR_BAD_ARG;
    if ((d_sidecar || d_sidecar_out) &&
        (p->ckpt_interval < (ns == 1 ? 16u : 8u) || (p->ckpt_interval & (p->ckpt_interval - 1))))
        return FSE_ERR_BAD_ARG;
    if (ns == 1 && d_sidecar_out && kern_lmax(p->max_table_log) > 12) return FSE_ERR_UNSUPPORTED;  // decode1_serial_kernel records nothing
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
    P.dt = d_dt;
    P.dtinfo = d_dtinfo;
    if (lease && !d_sidecar && !d_sidecar_out) defer_symbols(*lease, P, kern_lmax(p->max_table_log));
    P.stamps = g_stamps_dec.get(n_blocks);
    hipError_t e = fsehip::launch_decode(P, kern_lmax(p->max_table_log), static_cast<hipStream_t>(stream));
    if (P.stamps) g_stamps_dec.report("decode", n_blocks, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

uint64_t fsehip_dtable_bytes(uint32_t max_table_log) { return 4ull << kern_lmax(max_table_log); }

// The table build; `lease` (held by the caller) supplies the header-parse
// scratch when the batch is large enough for the lane-parallel parse to pay
// (a workgroup parses 64 headers), else the table kernel parses on its own.
static int build_dtables_impl(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                              const uint32_t* d_comp_len, uint32_t n_blocks, uint32_t* d_dtables, int32_t* d_dtinfo,
                              fsehip_stream_t stream, Lease* lease) {
    if (!p || !d_in || !d_comp_len || !d_dtables || !d_dtinfo || (slot_bytes & 255u)) return FSE_ERR_BAD_ARG;
    if (n_blocks == 0) return FSE_OK;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    fsehip::DtParams D{};
    if (lease && n_blocks >= 256u && kern_lmax(p->max_table_log) <= 12 && !env_u32("FSEHIP_DT_WAVE_PARSE", 0)) {
        uint8_t* h = static_cast<uint8_t*>(lease->get(SCRATCH_HDR, fsehip::hdr_scratch_bytes(n_blocks), true));
        if (h) {
            D.hdr_norm = reinterpret_cast<uint32_t*>(h);
            D.hdr_meta = reinterpret_cast<int2*>(h + 512ull * n_blocks);
        }
    }
    D.in = d_in;
    D.slot_bytes = slot_bytes;
    D.comp_len = d_comp_len;
    D.n_blocks = n_blocks;
    D.dt = d_dtables;
    D.dtinfo = d_dtinfo;
    D.xlds = env_u32("FSEHIP_DT_XLDS", 0);  // diagnostics: occupancy probe
    D.rank_inject = env_u32("FSEHIP_RANK_INJECT", 0);  // diagnostics: fault injection into the atomic ranks
    D.stamps = g_stamps_dt.get(n_blocks);
    hipError_t e = fsehip::launch_dtables(D, kern_lmax(p->max_table_log), static_cast<hipStream_t>(stream));
    if (D.stamps) g_stamps_dt.report("dtables", n_blocks, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

int fsehip_build_dtables(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes, const uint32_t* d_comp_len,
                         uint32_t n_blocks, uint32_t* d_dtables, int32_t* d_dtinfo, fsehip_stream_t stream) {
    if (n_blocks < 256u) return build_dtables_impl(p, d_in, slot_bytes, d_comp_len, n_blocks, d_dtables, d_dtinfo, stream,
                                                   nullptr);
    Lease lease(stream);  // the header-parse scratch
    return build_dtables_impl(p, d_in, slot_bytes, d_comp_len, n_blocks, d_dtables, d_dtinfo, stream, &lease);
}

int fsehip_decompress_blocks_dt(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                                const uint32_t* d_comp_len, const uint64_t* d_sidecar, const uint32_t* d_dtables,
                                const int32_t* d_dtinfo, uint8_t* d_out, uint64_t n_total, int32_t* d_status,
                                fsehip_stream_t stream) {
    if (n_total == 0) return FSE_ERR_EMPTY;
    if (!p || !d_dtables || !d_dtinfo) return FSE_ERR_BAD_ARG;
    if (d_sidecar && p->ckpt_interval == 0) return FSE_ERR_BAD_ARG;
    if (d_sidecar)
        return decompress_impl(p, d_in, slot_bytes, d_comp_len, d_sidecar, d_out, n_total, nullptr, d_status, nullptr,
                               0, stream, d_dtables, d_dtinfo);
    Lease lease(stream);  // the deferred-symbol workspace
    return decompress_impl(p, d_in, slot_bytes, d_comp_len, nullptr, d_out, n_total, nullptr, d_status, nullptr, 0,
                           stream, d_dtables, d_dtinfo, &lease);
}

extern "C++" {
// Decode tables for all blocks at high occupancy into the stream's
// workspace, then `run(dt, info, lease)` enqueues the decode on them; both under
// the workspace lock.
template <class Run>
static int with_dtables_n(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes, const uint32_t* d_comp_len,
                          uint64_t n_blocks, fsehip_stream_t stream, Run run) {
    if (n_blocks > 0xFFFFFFFFull) return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    Lease lease(stream);
    uint32_t* dt = static_cast<uint32_t*>(lease.get(SCRATCH_DT, fsehip_dtable_bytes(p->max_table_log) * n_blocks));
    int32_t* info = static_cast<int32_t*>(lease.get(SCRATCH_DTINFO, 4ull * n_blocks));
    if (!dt || !info) return FSE_ERR_HIP;
    int rc = build_dtables_impl(p, d_in, slot_bytes, d_comp_len, (uint32_t)n_blocks, dt, info, stream, &lease);
    return rc != FSE_OK ? rc : run(dt, info, lease);
}
template <class Run>
static int with_dtables(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes, const uint32_t* d_comp_len,
                        uint64_t n_total, fsehip_stream_t stream, Run run) {
    const uint32_t bs = p->block_size ? p->block_size : kDefaultBlock;
    if (bs > kMaxBlock) return FSE_ERR_UNSUPPORTED;
    return with_dtables_n(p, d_in, slot_bytes, d_comp_len, (n_total + bs - 1) / bs, stream, run);
}
}  // extern "C++"

int fsehip_decompress_blocks(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                             const uint32_t* d_comp_len, const uint64_t* d_sidecar, uint8_t* d_out, uint64_t n_total,
                             int32_t* d_status, fsehip_stream_t stream) {
    if (n_total == 0) return FSE_ERR_EMPTY;
    if (!p) return FSE_ERR_BAD_ARG;
    if (d_sidecar && p->ckpt_interval == 0) return FSE_ERR_BAD_ARG;
    return with_dtables(p, d_in, slot_bytes, d_comp_len, n_total, stream,
                        [&](const uint32_t* dt, const int32_t* info, Lease& lease) {
                            return decompress_impl(p, d_in, slot_bytes, d_comp_len, d_sidecar, d_out, n_total, nullptr,
                                                   d_status, nullptr, 0, stream, dt, info, &lease);
                        });
}

int fsehip_build_sidecar(const fsehip_params* p, const uint8_t* d_in, uint64_t slot_bytes,
                         const uint32_t* d_comp_len, uint8_t* d_out, uint64_t n_total, uint64_t* d_sidecar_out,
                         int32_t* d_status, fsehip_stream_t stream) {
    if (n_total == 0) return FSE_ERR_EMPTY;
    if (!p || !d_sidecar_out) return FSE_ERR_BAD_ARG;
    const uint32_t ns = p->nstates == 1 ? 1u : 2u;
    // 1-state blocks above L = 12 decode on decode1_serial_kernel, which records nothing
    if (ns == 1 && kern_lmax(p->max_table_log) > 12) return FSE_ERR_UNSUPPORTED;
    if (p->ckpt_interval < (ns == 1 ? 16u : 8u) || (p->ckpt_interval & (p->ckpt_interval - 1))) return FSE_ERR_BAD_ARG;
    return with_dtables(p, d_in, slot_bytes, d_comp_len, n_total, stream, [&](const uint32_t* dt, const int32_t* info, Lease&) {
        return decompress_impl(p, d_in, slot_bytes, d_comp_len, nullptr, d_out, n_total, d_sidecar_out, d_status,
                               nullptr, 0, stream, dt, info);
    });
}

int fsehip_decompress_streams(uint32_t nstates, uint32_t max_table_log, const uint8_t* d_in, uint64_t in_stride,
                              const uint32_t* d_comp_len, uint32_t n_streams, uint8_t* d_out, uint32_t out_stride,
                              uint32_t* d_out_len, int32_t* d_status, fsehip_stream_t stream) {
    if (n_streams == 0) return FSE_ERR_EMPTY;
    if (nstates > 2 || !d_in || !d_comp_len || !d_out || !d_out_len || !d_status || out_stride == 0 ||
        (in_stride & 255u) || (reinterpret_cast<uintptr_t>(d_in) & 15u) || (out_stride & 15u) ||
        (reinterpret_cast<uintptr_t>(d_out) & 15u))  // 16-byte input chunks and output groups
        return FSE_ERR_BAD_ARG;
    if (max_table_log > 15) return FSE_ERR_UNSUPPORTED;
    const fsehip_params p{out_stride, 0, 0, max_table_log ? max_table_log : 11u, nstates ? nstates : 2u};
    return with_dtables_n(&p, d_in, in_stride, d_comp_len, n_streams, stream,
                          [&](const uint32_t* dt, const int32_t* info, Lease& lease) {
                              fsehip::DecParams P{};
                              P.nstates = p.nstates;
                              P.in = d_in;
                              P.slot_bytes = in_stride;
                              P.comp_len = d_comp_len;
                              P.out = d_out;
                              P.n_total = 0;  // reference mode: each stream ends where the crate's decoder stops
                              P.block_size = out_stride;
                              P.n_blocks = n_streams;
                              P.out_cap = out_stride;
                              P.status = d_status;
                              P.out_len = d_out_len;
                              P.dt = dt;
                              P.dtinfo = info;
                              defer_symbols(lease, P, kern_lmax(p.max_table_log));
                              return fsehip::launch_decode(P, kern_lmax(p.max_table_log),
                                                           static_cast<hipStream_t>(stream)) == hipSuccess
                                         ? (int)FSE_OK
                                         : (int)FSE_ERR_HIP;
                          });
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
    // Histogram::normalize clamps any request into 5..15 (histogram.rs:96):
    // 0 acts as 5 (table_log 0 in the batched params means NormHistogram::new)
    return compress_one(src, n, std::max<uint32_t>(table_log, 5u), dst, dst_cap, dst_len, payload_bits);
}

// Host block decode (reference mode: the raw length is not in the format):
// the block's table (stride 15, any L) and the serial decoder with the
// reference's own termination within the caller's capacity.
constexpr uint32_t LOG_MIN_HOST = 5;  // TABLE_LOG_MIN (lib.rs:9)

static int decompress_one(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len,
                          uint32_t nstates) {
    if (!dst_len || *dst_len > dst_cap) return FSE_ERR_BAD_ARG;
    if (n == 0) return FSE_ERR_EMPTY;  // BitStreamReader::new asserts (stream_reader.rs:17)
    if (n > (1u << 30)) return FSE_ERR_UNSUPPORTED;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    const uint64_t padded = round_up(n + 16, 256);
    const uint64_t cap64 = std::min<uint64_t>(dst_cap - *dst_len, 0x7FFFFFFFu);
    const size_t pin_out = std::min<size_t>(cap64, kPinOut);
    // one device buffer: the result record (Meta) at 0, the stream at 256
    uint8_t* d_buf = g_stage.get(0, 256 + padded);
    uint8_t* d_out = g_stage.get(1, std::max<uint64_t>(cap64, 16));
    // the header's first field is the table log (histogram.rs:438: read(4) +
    // 5): size the tables and pick the kernels by it (the L <= 11 / 12
    // kernels keep the table in LDS; a bad header fails the parse either way)
    const uint32_t Lh = (uint32_t)(src[0] & 15u) + LOG_MIN_HOST;
    const uint32_t mtl = Lh <= 11u ? 11u : Lh <= 12u ? 12u : 15u;
    uint8_t* d_dt = g_stage.get(3, fsehip_dtable_bytes(mtl) + 16);
    uint8_t* h_in = g_pin.get(0, 256 + padded);
    uint8_t* h_ret = g_pin.get(1, 256 + pin_out);
    if (!d_buf || !d_out || !d_dt || !h_in || !h_ret) return FSE_ERR_HIP;
    // the record and the zero-padded stream go over in one copy
    const Meta h0{(uint32_t)n, 0, 0, 0};
    memcpy(h_in, &h0, sizeof h0);
    memcpy(h_in + 256, src, n);
    memset(h_in + 256 + n, 0, padded - n);
    auto fail = [](int rc) {  // nothing may still read or write the pinned buffers
        (void)hipStreamSynchronize(nullptr);
        return rc;
    };
    if (hipMemcpyAsync(d_buf, h_in, 256 + padded, hipMemcpyHostToDevice, nullptr) != hipSuccess)
        return fail(FSE_ERR_HIP);
    uint8_t* d_in = d_buf + 256;
    Meta* m = reinterpret_cast<Meta*>(d_buf);
    fsehip_params p{0, 0, 0, mtl, nstates};
    uint32_t* dt = reinterpret_cast<uint32_t*>(d_dt);
    int32_t* info = reinterpret_cast<int32_t*>(d_dt + fsehip_dtable_bytes(mtl));
    int rc = fsehip_build_dtables(&p, d_in, padded, &m->comp_len, 1, dt, info, nullptr);
    if (rc) return fail(rc);
    if (mtl == 11) {
        // the latency-first single-stream decoder (chain on the scalar unit,
        // fused table through the scalar cache, payload streamed by chunks)
        fsehip::DecParams P{};
        P.nstates = nstates;
        P.in = d_in;
        P.slot_bytes = padded;
        P.comp_len = &m->comp_len;
        P.out = d_out;
        P.n_total = 0;
        P.block_size = 0;
        P.n_blocks = 1;
        P.out_cap = (uint32_t)cap64;
        P.status = &m->status;
        P.out_len = &m->payload_bits;
        P.dt = dt;
        P.dtinfo = info;
        P.states = reinterpret_cast<uint32_t*>(g_stage.get(6, fsehip::single_ftab_bytes()));  // fused bulk table
        if (!P.states) return fail(FSE_ERR_HIP);
        if (fsehip::launch_single(P, 11, nullptr) != hipSuccess) return fail(FSE_ERR_HIP);
    } else {
        rc = decompress_impl(&p, d_in, padded, &m->comp_len, nullptr, d_out, 0, nullptr, &m->status, &m->payload_bits,
                             (uint32_t)cap64, nullptr, dt, info);
        if (rc) return fail(rc);
    }
    // payload_bits holds the decoded byte count here (0 on error)
    if (fsehip::launch_host_return(d_buf, d_out, &m->payload_bits, h_ret, h_ret + 256, (uint32_t)pin_out, nullptr) !=
        hipSuccess)
        return fail(FSE_ERR_HIP);
    if (hipStreamSynchronize(nullptr) != hipSuccess) return FSE_ERR_HIP;
    Meta h;
    memcpy(&h, h_ret, sizeof h);
    if (h.status != FSE_OK) return h.status;
    const uint32_t out_len = h.payload_bits;  // decoded byte count
    const size_t head = std::min<size_t>(out_len, pin_out);
    memcpy(dst + *dst_len, h_ret + 256, head);
    if (out_len > head &&
        hipMemcpy(dst + *dst_len + head, d_out + head, out_len - head, hipMemcpyDeviceToHost) != hipSuccess)
        return FSE_ERR_HIP;
    *dst_len += out_len;
    return FSE_OK;
}

int fse_decompress2(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len) {
    return decompress_one(src, n, dst, dst_cap, dst_len, 2);
}

int fse_compress(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len, uint64_t* payload_bits) {
    // lib.rs:112-143; n == 1 is valid here (a lone seed state), unlike fse_compress2
    return compress_one(src, n, 0, dst, dst_cap, dst_len, payload_bits, 1);
}

int fse_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len) {
    return decompress_one(src, n, dst, dst_cap, dst_len, 1);
}

// Many host streams in one call: the batching pattern for a caller holding
// many crate streams (lib.rs:187-248 per stream).  One pinned staging copy
// in (lengths + streams at a common stride), the header parse + decode
// tables + serial decoders of fsehip_decompress_streams on the default
// stream (one chain per stream, thousands at once), one copy back of the
// per-stream record (length, status) and output.  One or two streams take
// the single-stream call instead (its chain is ~2x faster than one serial
// ring chain, and the batch kernels' fixed cost buys nothing).
// fn(i) for i in [0, n) on up to 16 host threads (contiguous ranges), one
// thread per ~2 MB of copying: the staging memcpys of a large batch are the
// call's host-side cost (one core copies ~5-10 GB/s).
extern "C++" {
template <class Fn>
static void for_streams(size_t n, uint64_t bytes, Fn fn) {
    const size_t T = (size_t)std::min<uint64_t>({16, (bytes >> 21) + 1, n});
    if (T <= 1) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    std::vector<std::thread> th;
    auto range = [&](size_t t) {
        for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) fn(i);
    };
    size_t started = 1;  // ranges handed to threads (range 0 runs here)
    try {
        th.reserve(T - 1);
        for (; started < T; ++started) th.emplace_back(range, started);
    } catch (...) {  // no thread to be had (resource limits): the rest runs here
    }
    range(0);
    for (size_t t = started; t < T; ++t) range(t);
    for (auto& x : th) x.join();
}
}  // extern "C++"

// Batches of at most this many streams at table log <= 11 decode one stream
// per wave on the scalar unit (single_decode_kernel), larger ones on the
// serial ring kernel (32 lanes of chains per CU).  Measured with 64 KiB C2
// streams, host buffers in and out (tools/many_ab.py, profiles/r06/many/):
// 3 streams 2.13 -> 1.48 ms, 16 streams 2.27 -> 2.08 ms (1-state 3.38 ->
// 2.01), but 64 streams 2.62 -> 2.90: the scalar chains share their CU's
// scalar cache, whose 16 KiB fused tables then evict one another.
#ifndef FSE_SCALAR_MANY
#define FSE_SCALAR_MANY 32
#endif
constexpr size_t kScalarMany = FSE_SCALAR_MANY;

// One batch: the streams idx[0..m) (each 0 < n <= kManyStream, non-null),
// staged at a common stride, decoded as fsehip_decompress_streams does.
static int decompress_batch(const uint8_t* const* srcs, const size_t* src_lens, const std::vector<size_t>& idx,
                            uint8_t* dst, size_t dst_stride, size_t* dst_lens, int32_t* statuses, uint32_t nstates) {
    const size_t m = idx.size();
    size_t maxn = 1;
    uint32_t lmax = 11;
    uint64_t in_total = 0;
    for (size_t i : idx) {
        maxn = std::max(maxn, src_lens[i]);
        in_total += src_lens[i];
        lmax = std::max<uint32_t>(lmax, (uint32_t)(srcs[i][0] & 15u) + LOG_MIN_HOST);  // histogram.rs:438
    }
    const uint32_t mtl = lmax <= 11u ? 11u : lmax <= 12u ? 12u : 15u;
    const uint64_t in_stride = round_up(maxn + 32, 256);
    const uint64_t out_stride = round_up(dst_stride, 16);
    const uint64_t head = round_up(4ull * m, 256);  // the lengths ahead of the streams
    const uint64_t in_bytes = head + in_stride * m;
    const uint64_t rec = round_up(8ull * m, 256);  // (length, status) per stream ahead of the output
    const uint64_t out_bytes = rec + out_stride * m;
    uint8_t* d_in = g_stage.get(4, in_bytes);
    uint8_t* d_out = g_stage.get(5, out_bytes);
    uint8_t* h_in = g_pin.get(0, in_bytes);
    uint8_t* h_out = g_pin.get(1, out_bytes);
    if (!d_in || !d_out || !h_in || !h_out) return FSE_ERR_HIP;
    uint32_t* lens = reinterpret_cast<uint32_t*>(h_in);
    for_streams(m, in_total, [&](size_t k) {
        const size_t n = src_lens[idx[k]];
        uint8_t* s = h_in + head + k * in_stride;
        lens[k] = (uint32_t)n;
        memcpy(s, srcs[idx[k]], n);
        memset(s + n, 0, std::min<uint64_t>(in_stride, round_up(n, 32) + 32) - n);
    });
    auto fail = [](int rc) {  // nothing may still read or write the pinned buffers
        (void)hipStreamSynchronize(nullptr);
        return rc;
    };
    if (hipMemcpyAsync(d_in, h_in, in_bytes, hipMemcpyHostToDevice, nullptr) != hipSuccess) return fail(FSE_ERR_HIP);
    const uint32_t* d_len = reinterpret_cast<const uint32_t*>(d_in);
    uint32_t* d_olen = reinterpret_cast<uint32_t*>(d_out);
    int32_t* d_stat = reinterpret_cast<int32_t*>(d_out + 4ull * m);
    const fsehip_params p{(uint32_t)out_stride, 0, 0, mtl, nstates};
    int rc = with_dtables_n(&p, d_in + head, in_stride, d_len, m, nullptr,
                            [&](const uint32_t* dt, const int32_t* info, Lease& lease) {
                                fsehip::DecParams P{};
                                P.nstates = nstates;
                                P.in = d_in + head;
                                P.slot_bytes = in_stride;
                                P.comp_len = d_len;
                                P.out = d_out + rec;
                                P.n_total = 0;  // reference mode: each stream ends where the crate stops
                                P.block_size = (uint32_t)out_stride;
                                P.n_blocks = (uint32_t)m;
                                P.out_cap = (uint32_t)dst_stride;
                                P.status = d_stat;
                                P.out_len = d_olen;
                                P.dt = dt;
                                P.dtinfo = info;
                                if (mtl == 11u && m <= kScalarMany) {
                                    // few streams: one scalar-unit chain each (the single
                                    // call's kernel), ~2x faster per chain than a ring lane
                                    P.states = static_cast<uint32_t*>(
                                        lease.get(SCRATCH_STATES, fsehip::single_ftab_bytes() * m, true));
                                    if (P.states)
                                        return fsehip::launch_single(P, 11, nullptr) == hipSuccess ? (int)FSE_OK
                                                                                                    : (int)FSE_ERR_HIP;
                                }
                                defer_symbols(lease, P, kern_lmax(mtl));
                                return fsehip::launch_decode(P, kern_lmax(mtl), nullptr) == hipSuccess
                                           ? (int)FSE_OK
                                           : (int)FSE_ERR_HIP;
                            });
    if (rc) return fail(rc);
    if (hipMemcpyAsync(h_out, d_out, out_bytes, hipMemcpyDeviceToHost, nullptr) != hipSuccess) return fail(FSE_ERR_HIP);
    if (hipStreamSynchronize(nullptr) != hipSuccess) return FSE_ERR_HIP;
    const uint32_t* olen = reinterpret_cast<const uint32_t*>(h_out);
    const int32_t* ost = reinterpret_cast<const int32_t*>(h_out + 4ull * m);
    uint64_t out_total = 0;
    for (size_t k = 0; k < m; ++k) out_total += ost[k] == FSE_OK ? olen[k] : 0;
    for_streams(m, out_total, [&](size_t k) {
        const size_t i = idx[k];
        statuses[i] = ost[k];
        dst_lens[i] = ost[k] == FSE_OK ? olen[k] : 0;
        if (ost[k] == FSE_OK) memcpy(dst + i * dst_stride, h_out + rec + k * out_stride, olen[k]);
    });
    return FSE_OK;
}

// Many host streams in one call (lib.rs:187-248 per stream).  Streams the
// batch takes (up to 4 MiB each) go in groups of at most kManyStage bytes
// of staging each way; longer ones, and calls of one or two streams, take
// the single-stream path one by one (its chain is ~2x faster than a serial
// ring chain, and a lone long stream should not set the stride of all).
constexpr size_t kManyStream = size_t(4) << 20;
constexpr uint64_t kManyStage = uint64_t(512) << 20;
static int decompress_many(const uint8_t* const* srcs, const size_t* src_lens, size_t n_streams, uint8_t* dst,
                           size_t dst_stride, size_t* dst_lens, int32_t* statuses, uint32_t nstates) {
    if (n_streams == 0) return FSE_OK;
    if (!srcs || !src_lens || !dst || !dst_lens || !statuses || dst_stride == 0) return FSE_ERR_BAD_ARG;
    if (n_streams > (1u << 24) || dst_stride > 0x7FFFFFFFull) return FSE_ERR_UNSUPPORTED;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    const uint64_t out_stride = round_up(dst_stride, 16);
    // Groups by the header's table log (histogram.rs:438: the first nibble +
    // 5): <= 11, 12 and 13..15 take the kernels and decode-table stride of
    // their class, so one stream with a large (or corrupt) log neither moves
    // the others off the L <= 11 kernels nor multiplies their table scratch;
    // a nibble above 15 can only fail, on the single path.  A group is capped
    // by its staging bytes and by its decode-table + header scratch.
    std::vector<size_t> single, group[3];
    uint64_t gmax[3] = {0, 0, 0};  // each group's largest staged stream
    constexpr uint32_t kClassLog[3] = {11, 12, 15};
    auto run_group = [&](int c) -> int {
        std::vector<size_t>& g = group[c];
        gmax[c] = 0;
        if (g.empty()) return FSE_OK;
        if (g.size() <= 2) {  // not worth the batch kernels' fixed cost
            single.insert(single.end(), g.begin(), g.end());
            g.clear();
            return FSE_OK;
        }
        const int rc = decompress_batch(srcs, src_lens, g, dst, dst_stride, dst_lens, statuses, nstates);
        g.clear();
        return rc;
    };
    for (size_t i = 0; i < n_streams; ++i) {
        const size_t n = src_lens[i];
        if (n == 0 || !srcs[i] || n > kManyStream || n_streams <= 2 || out_stride > kManyStage / 4) {
            single.push_back(i);  // statuses and long streams: the single call's own path
            continue;
        }
        const uint32_t L = (uint32_t)(srcs[i][0] & 15u) + LOG_MIN_HOST;
        if (L > 15u) {
            single.push_back(i);
            continue;
        }
        const int c = L <= 11u ? 0 : L == 12u ? 1 : 2;
        const uint64_t in_s = round_up(n + 32, 256), gm = std::max(gmax[c], in_s);
        const uint64_t per_table = fsehip_dtable_bytes(kClassLog[c]) + fsehip::hdr_scratch_bytes(1) + 8u;
        const uint64_t m1 = group[c].size() + 1;
        if (!group[c].empty() && (m1 * std::max(gm, out_stride) > kManyStage || m1 * per_table > kManyStage)) {
            if (int rc = run_group(c)) return rc;
        }
        group[c].push_back(i);
        gmax[c] = std::max(gmax[c], in_s);
    }
    for (int c = 0; c < 3; ++c)
        if (int rc = run_group(c)) return rc;
    for (size_t i : single) {
        size_t len = 0;
        const int32_t st = src_lens[i] == 0 ? FSE_ERR_EMPTY  // BitStreamReader::new asserts (stream_reader.rs:17)
                           : !srcs[i]      ? FSE_ERR_BAD_ARG
                                           : decompress_one(srcs[i], src_lens[i], dst + i * dst_stride, dst_stride,
                                                            &len, nstates);
        if (st == FSE_ERR_HIP || st == FSE_ERR_NO_DEVICE) return st;
        statuses[i] = st;
        dst_lens[i] = st == FSE_OK ? len : 0;
    }
    return FSE_OK;
}

int fse_decompress2_many(const uint8_t* const* srcs, const size_t* src_lens, size_t n_streams, uint8_t* dst,
                         size_t dst_stride, size_t* dst_lens, int32_t* statuses) {
    return decompress_many(srcs, src_lens, n_streams, dst, dst_stride, dst_lens, statuses, 2);
}

int fse_decompress_many(const uint8_t* const* srcs, const size_t* src_lens, size_t n_streams, uint8_t* dst,
                        size_t dst_stride, size_t* dst_lens, int32_t* statuses) {
    return decompress_many(srcs, src_lens, n_streams, dst, dst_stride, dst_lens, statuses, 1);
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

// ------------------------------------------------------- building blocks

int histogram_new(const uint8_t* src, size_t n, fse_histogram* out) {
    if (!out) return FSE_ERR_BAD_ARG;
    uint32_t tl = 0;
    int rc = histogram_count(src, n, out->counts, &tl);
    if (rc) return rc;
    out->size = (uint32_t)n;
    out->table_len = tl;
    return FSE_OK;
}

// One normalisation on the GPU (fse_blocks.hip norm_kernel).
static int normalize_dev(int mode, const uint8_t* src, size_t n, const fse_histogram* h, uint32_t log2,
                         fse_norm_histogram* out) {
    if (!out) return FSE_ERR_BAD_ARG;
    if (mode == 2 && n > 0xFFFFFFFFull) return FSE_ERR_BAD_ARG;  // histogram.rs:19 assert
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    uint8_t* d_src = mode == 2 ? g_stage.get(0, round_up(n, 16) + 16) : nullptr;
    uint8_t* d_io = g_stage.get(2, sizeof(fse_norm_histogram) + sizeof(fse_histogram) + 16);
    if ((mode == 2 && !d_src) || !d_io) return FSE_ERR_HIP;
    auto* d_nh = reinterpret_cast<fse_norm_histogram*>(d_io);
    auto* d_h = reinterpret_cast<fse_histogram*>(d_io + sizeof(fse_norm_histogram));
    int32_t* d_st = reinterpret_cast<int32_t*>(d_io + sizeof(fse_norm_histogram) + sizeof(fse_histogram));
    if (mode == 2 && n && hipMemcpy(d_src, src, n, hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    if (mode != 2 && hipMemcpy(d_h, h, sizeof(fse_histogram), hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    fsehip::NormArgs A{};
    A.mode = mode;
    A.src = d_src;
    A.n = n;
    A.counts = d_h->counts;
    if (mode != 2) {
        A.size = h->size;
        A.table_len = h->table_len;
    }
    A.log2 = log2;
    A.out = d_nh;
    A.status = d_st;
    if (fsehip::launch_norm(A, nullptr) != hipSuccess) return FSE_ERR_HIP;
    int32_t st = 0;
    if (hipMemcpy(&st, d_st, 4, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    if (st != FSE_OK) return st;
    if (hipMemcpy(out, d_nh, sizeof(fse_norm_histogram), hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    return FSE_OK;
}

int histogram_normalize(const fse_histogram* h, uint32_t log2, fse_norm_histogram* out) {
    if (!h || h->table_len > 256) return FSE_ERR_BAD_ARG;
    return normalize_dev(0, nullptr, 0, h, log2, out);
}

int histogram_normalize_optimal(const fse_histogram* h, fse_norm_histogram* out) {
    if (!h || h->table_len > 256) return FSE_ERR_BAD_ARG;
    return normalize_dev(1, nullptr, 0, h, 0, out);
}

int norm_histogram_new(const uint8_t* src, size_t n, fse_norm_histogram* out) {
    if (!src && n) return FSE_ERR_BAD_ARG;
    return normalize_dev(2, src, n, nullptr, 0, out);
}

int norm_histogram_write(const fse_norm_histogram* nh, uint8_t* dst, size_t dst_cap, size_t* dst_len,
                         uint64_t* bits_written) {
    if (!nh || !dst_len || *dst_len > dst_cap) return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    uint8_t* d = g_stage.get(2, sizeof(fse_norm_histogram) + 16 + 512);
    if (!d) return FSE_ERR_HIP;
    auto* d_nh = reinterpret_cast<fse_norm_histogram*>(d);
    uint32_t* d_meta = reinterpret_cast<uint32_t*>(d + sizeof(fse_norm_histogram));  // bits, status
    uint8_t* d_out = d + sizeof(fse_norm_histogram) + 16;
    if (hipMemcpy(d_nh, nh, sizeof(*nh), hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    if (fsehip::launch_hdr_write(d_nh, d_out, d_meta, reinterpret_cast<int32_t*>(d_meta + 1), nullptr) != hipSuccess)
        return FSE_ERR_HIP;
    uint32_t meta[2];
    if (hipMemcpy(meta, d_meta, 8, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    if ((int32_t)meta[1] != FSE_OK) return (int32_t)meta[1];
    const size_t len = (meta[0] + 7u) / 8u;
    if (dst_cap - *dst_len < len) return FSE_ERR_DST_TOO_SMALL;
    if (len && (!dst || hipMemcpy(dst + *dst_len, d_out, len, hipMemcpyDeviceToHost) != hipSuccess))
        return FSE_ERR_HIP;
    *dst_len += len;
    if (bits_written) *bits_written = meta[0];
    return FSE_OK;
}

int norm_histogram_read(const uint8_t* src, size_t n, fse_norm_histogram* out, size_t* consumed) {
    if (!out || (!src && n)) return FSE_ERR_BAD_ARG;
    if (n == 0) return FSE_ERR_EMPTY;  // BitStreamReader::new asserts a non-empty slice (stream_reader.rs:17)
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    const size_t take = std::min<size_t>(n, 512);  // a header never exceeds 483 bytes (write_bound)
    uint8_t* d = g_stage.get(2, sizeof(fse_norm_histogram) + 16 + 528);
    if (!d) return FSE_ERR_HIP;
    auto* d_nh = reinterpret_cast<fse_norm_histogram*>(d);
    uint32_t* d_meta = reinterpret_cast<uint32_t*>(d + sizeof(fse_norm_histogram));  // used, status
    uint8_t* d_in = d + sizeof(fse_norm_histogram) + 16;
    if (hipMemset(d_in, 0, 528) != hipSuccess || hipMemcpy(d_in, src, take, hipMemcpyHostToDevice) != hipSuccess)
        return FSE_ERR_HIP;
    // the reader sees the whole slice's length (its bounds checks), the
    // header's bits come from the first 512 bytes
    if (fsehip::launch_hdr_read(d_in, (uint32_t)std::min<size_t>(n, 0xFFFFFFFFu), d_nh, d_meta,
                                reinterpret_cast<int32_t*>(d_meta + 1), nullptr) != hipSuccess)
        return FSE_ERR_HIP;
    uint32_t meta[2];
    if (hipMemcpy(meta, d_meta, 8, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    if ((int32_t)meta[1] != FSE_OK) return (int32_t)meta[1];
    if (hipMemcpy(out, d_nh, sizeof(*out), hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    if (consumed) *consumed = meta[0];
    return FSE_OK;
}

static int table_new(const fse_norm_histogram* nh, int enc, void* out, size_t bytes) {
    if (!nh || !out) return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    uint8_t* d = g_stage.get(4, sizeof(fse_norm_histogram) + 16 + bytes);
    if (!d) return FSE_ERR_HIP;
    auto* d_nh = reinterpret_cast<fse_norm_histogram*>(d);
    int32_t* d_st = reinterpret_cast<int32_t*>(d + sizeof(fse_norm_histogram));
    uint8_t* d_tab = d + sizeof(fse_norm_histogram) + 16;
    if (hipMemcpy(d_nh, nh, sizeof(*nh), hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    if (hipMemset(d_tab, 0, bytes) != hipSuccess) return FSE_ERR_HIP;
    if (fsehip::launch_table(d_nh, enc, reinterpret_cast<fse_encode_table*>(d_tab),
                             reinterpret_cast<fse_decode_table*>(d_tab), d_st, nullptr) != hipSuccess)
        return FSE_ERR_HIP;
    int32_t st = 0;
    if (hipMemcpy(&st, d_st, 4, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    if (st != FSE_OK) return st;
    return hipMemcpy(out, d_tab, bytes, hipMemcpyDeviceToHost) == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

int encode_table_new(const fse_norm_histogram* nh, fse_encode_table* out) {
    return table_new(nh, 1, out, sizeof(fse_encode_table));
}

int decode_table_new(const fse_norm_histogram* nh, fse_decode_table* out) {
    return table_new(nh, 0, out, sizeof(fse_decode_table));
}

int fse_compress_nh(const uint8_t* src, size_t n, uint8_t* dst, size_t dst_cap, size_t* dst_len,
                    uint64_t* payload_bits, fse_norm_histogram* nh) {
    const size_t at = dst_len ? *dst_len : 0;
    int rc = fse_compress(src, n, dst, dst_cap, dst_len, payload_bits);
    if (rc || !nh) return rc;
    // the returned NormHistogram is the one the block's header carries
    return norm_histogram_read(dst + at, *dst_len - at, nh, nullptr);
}

// ------------------------------------------------------------- bitstream

// Scan of the widths into the workspace of `stream`; returns the device
// tile offsets and total (valid in stream order).
static int bits_scan(Lease& lease, const uint8_t* d_nbits, const uint8_t* d_ops, uint64_t count, uint64_t** tile_off,
                     uint64_t** total, fsehip_stream_t stream) {
    const uint64_t nt = fsehip::bits_tiles(count);
    uint8_t* w = static_cast<uint8_t*>(lease.get(SCRATCH_BITS, 16 + nt * 12 + 16));
    if (!w) return FSE_ERR_HIP;
    *total = reinterpret_cast<uint64_t*>(w);
    *tile_off = reinterpret_cast<uint64_t*>(w + 16);
    uint32_t* tile_sum = reinterpret_cast<uint32_t*>(w + 16 + nt * 8);
    return fsehip::launch_bits_scan(d_nbits, d_ops, count, tile_sum, *tile_off, *total,
                                    static_cast<hipStream_t>(stream)) ==
                   hipSuccess
               ? FSE_OK
               : FSE_ERR_HIP;
}

int fsehip_bitstack_write(const uint32_t* d_vals, const uint8_t* d_nbits, uint64_t count, uint8_t* d_out,
                          uint64_t out_cap, uint64_t* d_total_bits, fsehip_stream_t stream) {
    if ((count && (!d_vals || !d_nbits)) || !d_out || !d_total_bits || (reinterpret_cast<uintptr_t>(d_out) & 3u))
        return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    Lease lease(stream);
    uint64_t *tile_off = nullptr, *total = nullptr;
    int rc = bits_scan(lease, d_nbits, nullptr, count, &tile_off, &total, stream);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (fsehip::launch_bits_pack(d_vals, d_nbits, count, tile_off, total, reinterpret_cast<uint32_t*>(d_out),
                                 out_cap / 4u, s) != hipSuccess)
        return FSE_ERR_HIP;
    return hipMemcpyAsync(d_total_bits, total, 8, hipMemcpyDeviceToDevice, s) == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

static int bits_read_dev(const uint8_t* d_in, uint64_t n_bytes, uint64_t total_bits, int stack, const uint8_t* d_nbits,
                         const uint8_t* d_ops, uint64_t count, uint32_t* d_vals, uint64_t* d_result,
                         fsehip_stream_t stream) {
    if ((count && (!d_nbits || !d_vals)) || !d_result || (!d_in && n_bytes)) return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    Lease lease(stream);
    uint64_t *tile_off = nullptr, *total = nullptr;
    int rc = bits_scan(lease, d_nbits, d_ops, count, &tile_off, &total, stream);
    if (rc) return rc;
    return fsehip::launch_bits_unpack(d_in, n_bytes, total_bits, stack, d_nbits, d_ops, count, tile_off, total, d_vals,
                                      d_result, static_cast<hipStream_t>(stream)) == hipSuccess
               ? FSE_OK
               : FSE_ERR_HIP;
}

int fsehip_bitstack_read(const uint8_t* d_in, uint64_t n_bytes, const uint8_t* d_nbits, uint64_t count,
                         uint32_t* d_vals, uint64_t* d_result, fsehip_stream_t stream) {
    return bits_read_dev(d_in, n_bytes, 0, 1, d_nbits, nullptr, count, d_vals, d_result, stream);
}

int fsehip_bitstream_read_ops(const uint8_t* d_in, uint64_t n_bytes, uint64_t total_bits, const uint8_t* d_nbits,
                              const uint8_t* d_ops, uint64_t count, uint32_t* d_vals, uint64_t* d_result,
                              fsehip_stream_t stream) {
    if (n_bytes == 0 || (total_bits + 7u) / 8u != n_bytes) return FSE_ERR_BAD_ARG;  // stream_reader.rs:17-21 asserts
    return bits_read_dev(d_in, n_bytes, total_bits, 0, d_nbits, d_ops, count, d_vals, d_result, stream);
}

int fsehip_bitstream_read(const uint8_t* d_in, uint64_t n_bytes, uint64_t total_bits, const uint8_t* d_nbits,
                          uint64_t count, uint32_t* d_vals, uint64_t* d_result, fsehip_stream_t stream) {
    return fsehip_bitstream_read_ops(d_in, n_bytes, total_bits, d_nbits, nullptr, count, d_vals, d_result, stream);
}

int bitstack_write(const uint32_t* vals, const uint8_t* nbits, size_t count, uint8_t* dst, size_t dst_cap,
                   size_t* dst_len, uint64_t* bits_written) {
    if (!dst_len || *dst_len > dst_cap || (count && (!vals || !nbits))) return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    uint8_t* d_v = g_stage.get(0, count * 4 + 16);
    uint8_t* d_nb = g_stage.get(1, count + 16);
    uint8_t* d_out = g_stage.get(5, count * 4 + 16);
    uint8_t* d_tot = g_stage.get(2, 16);
    if (!d_v || !d_nb || !d_out || !d_tot) return FSE_ERR_HIP;
    if (count && (hipMemcpy(d_v, vals, count * 4, hipMemcpyHostToDevice) != hipSuccess ||
                  hipMemcpy(d_nb, nbits, count, hipMemcpyHostToDevice) != hipSuccess))
        return FSE_ERR_HIP;
    uint64_t* tot = reinterpret_cast<uint64_t*>(d_tot);
    int rc = fsehip_bitstack_write(reinterpret_cast<const uint32_t*>(d_v), d_nb, count, d_out, count * 4 + 16, tot,
                                   nullptr);
    if (rc) return rc;
    uint64_t bits = 0;
    if (hipMemcpy(&bits, tot, 8, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    const size_t len = (size_t)((bits + 7u) / 8u);
    if (dst_cap - *dst_len < len) return FSE_ERR_DST_TOO_SMALL;
    if (len && (!dst || hipMemcpy(dst + *dst_len, d_out, len, hipMemcpyDeviceToHost) != hipSuccess))
        return FSE_ERR_HIP;
    *dst_len += len;
    if (bits_written) *bits_written = bits;
    return FSE_OK;
}

static int bits_read_host(const uint8_t* src, size_t n, uint64_t total_bits, int stack, const uint8_t* nbits,
                          const uint8_t* ops, size_t count, uint32_t* vals, uint64_t res[3]) {
    if ((count && (!nbits || !vals)) || (!src && n)) return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    uint8_t* d_in = g_stage.get(0, round_up(n, 4) + 16);
    uint8_t* d_nb = g_stage.get(1, count + 16);
    uint8_t* d_v = g_stage.get(5, count * 4 + 16);
    uint8_t* d_res = g_stage.get(2, 32);
    uint8_t* d_ops = ops ? g_stage.get(3, count + 16) : nullptr;
    if (!d_in || !d_nb || !d_v || !d_res || (ops && !d_ops)) return FSE_ERR_HIP;
    if (hipMemset(d_in, 0, round_up(n, 4) + 16) != hipSuccess) return FSE_ERR_HIP;
    if (n && hipMemcpy(d_in, src, n, hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    if (count && hipMemcpy(d_nb, nbits, count, hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    if (ops && count && hipMemcpy(d_ops, ops, count, hipMemcpyHostToDevice) != hipSuccess) return FSE_ERR_HIP;
    uint64_t* r = reinterpret_cast<uint64_t*>(d_res);
    int rc = stack ? fsehip_bitstack_read(d_in, n, d_nb, count, reinterpret_cast<uint32_t*>(d_v), r, nullptr)
                   : fsehip_bitstream_read_ops(d_in, n, total_bits, d_nb, d_ops, count,
                                               reinterpret_cast<uint32_t*>(d_v), r, nullptr);
    if (rc) return rc;
    if (hipMemcpy(res, r, 24, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    if ((int64_t)res[2] != FSE_OK) return (int)(int64_t)res[2];
    if (res[0] && hipMemcpy(vals, d_v, res[0] * 4, hipMemcpyDeviceToHost) != hipSuccess) return FSE_ERR_HIP;
    return FSE_OK;
}

int bitstack_read(const uint8_t* src, size_t n, const uint8_t* nbits, size_t count, uint32_t* vals, size_t* n_read,
                  int* finished) {
    uint64_t res[3] = {0, 0, 0};
    int rc = bits_read_host(src, n, 0, 1, nbits, nullptr, count, vals, res);
    if (rc) return rc;
    if (n_read) *n_read = (size_t)res[0];
    // finish() after the successful reads: all bits consumed (reads stop at
    // the first None, which consumes nothing)
    if (finished) *finished = res[0] == count ? (int)res[1] : 0;
    return FSE_OK;
}

int bitstream_read_ops(const uint8_t* src, size_t n, uint64_t total_bits, const uint8_t* nbits, const uint8_t* ops,
                       size_t count, uint32_t* vals, size_t* n_done, uint64_t* bits_left) {
    if (ops)
        for (size_t i = 0; i < count; ++i)
            if (ops[i] > FSE_BITS_ADVANCE) return FSE_ERR_BAD_ARG;
    uint64_t res[3] = {0, 0, 0};
    int rc = bits_read_host(src, n, total_bits, 0, nbits, ops, count, vals, res);
    if (rc) return rc;
    if (n_done) *n_done = (size_t)res[0];
    if (bits_left) {
        uint64_t used = 0;
        for (size_t i = 0; i < res[0]; ++i)
            if (!ops || ops[i] != FSE_BITS_PEEK) used += std::min<uint32_t>(nbits[i], 32u);
        *bits_left = total_bits - used;
    }
    return FSE_OK;
}

int bitstream_read(const uint8_t* src, size_t n, uint64_t total_bits, const uint8_t* nbits, size_t count,
                   uint32_t* vals, size_t* n_read, uint64_t* bits_left) {
    return bitstream_read_ops(src, n, total_bits, nbits, nullptr, count, vals, n_read, bits_left);
}

// Diagnostics only (not part of include/fsehip.h): resident workgroups per CU.
int fsehipx_occupancy(char* buf, int cap) {
    if (!buf || cap <= 0 || !device_ok()) return 0;
    const int n = fsehip::occupancy_report(buf, cap);
    return n < cap ? n + fsehip::occupancy_report_dec(buf + n, cap - n) : n;
}

// Diagnostics only: the lane-order check behind the table builds' atomic
// ranks, run now (fse_kernels.h rank_order_check); FSE_OK with the counts.
int fsehipx_rank_order_check(uint32_t* violations, uint64_t* atomics) {
    if (!violations || !atomics) return FSE_ERR_BAD_ARG;
    if (!device_ok()) return FSE_ERR_NO_DEVICE;
    return fsehip::rank_order_check(violations, atomics) == hipSuccess ? FSE_OK : FSE_ERR_HIP;
}

int fsehip_rank_fallbacks(int device, uint32_t counts[3], int reset) {
    if (!counts) return FSE_ERR_BAD_ARG;
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return FSE_ERR_NO_DEVICE;
    const bool r = reset != 0;
    const bool ok = fsehip::rank_fallbacks_enc(&counts[0], r) == hipSuccess &&
                    fsehip::rank_fallbacks_dec(&counts[1], r) == hipSuccess &&
                    fsehip::rank_fallbacks_tab(&counts[2], r) == hipSuccess;
    (void)hipSetDevice(prev);
    return ok ? FSE_OK : FSE_ERR_HIP;
}

// Diagnostics only: force the table builds' rank method (tests of the
// fallback): -1 / 0 = atomic ranks checked per table (the default), 1 =
// peer-mask ranks.  Returns the previous mode.
int fsehipx_rank_mode(int mode) { return fsehip::rank_mode(mode < 0 ? -1 : mode > 0 ? 1 : 0); }

}  // extern "C"
