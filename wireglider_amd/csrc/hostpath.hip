// hostpath.hip — the host-memory path: the batch starts and
// ends in host memory (tun reads, worker/encap.cpp:74-97; UDP GRO recvmsg
// buffers, worker/decap.cpp:16-28,90-156).
//
// Per host thread a pipeline of kSlots device slots on three streams (H2D,
// exec, D2H; PCIe is full duplex, so chunk k+1's upload, chunk k's kernels
// and chunk k-1's download run together).  For chunk k in slot s:
//   H2D  waits for the kernels that last read slot s, uploads, records copied[s];
//   exec waits for copied[s] and for the download that last drained slot s's
//        outputs, runs the step's kernels, records computed[s];
//   D2H  waits for computed[s], downloads, records drained[s].
// Large outputs (messages, plaintext) go straight to the caller's buffers;
// small per-unit results gather in pinned buffers and reach the caller once
// at the end, so no small D2H targets pageable memory mid-pipeline.  Device
// memory is reused across calls and only grows.  The caller's current device
// is the one used, and it is never changed on return.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "wg_internal.hpp"
#include "wireglider_amd.h"

namespace wg {
namespace {

constexpr int kSlots = 3;
constexpr int kRoles = 8;
enum { kH2D = 0, kExec = 1, kD2H = 2 };

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
};

// Sets device d for its scope and restores the caller's current device.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int d) {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        if (d >= 0 && prev != d)
            (void)hipSetDevice(d);
    }
    ~DeviceScope() {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

struct Pipe {
    int device = -1;
    hipStream_t s[3] = {};
    hipEvent_t copied[kSlots] = {}, computed[kSlots] = {}, drained[kSlots] = {};
    DevBuf dev[kSlots][kRoles];  // device slot buffers, by role
    DevBuf stage[kSlots];        // pinned host staging per slot (rebased descriptors)
    DevBuf gather[kRoles];       // pinned host gather buffers for small per-unit results
    DevBuf ctr;                  // device: chained message counters (encap)
    DevBuf hctr;                 // pinned: the final counter
    void release();
    ~Pipe();
};

// Set by an atexit handler (registered when the first pipeline is built):
// thread-exit destructors that run after it must not call into a HIP runtime
// that may already be torn down — the process is ending and the driver
// reclaims the memory anyway.
std::atomic<bool> g_exiting{false};

void free_dev(DevBuf &b) {
    if (b.p) (void)hipFree(b.p);  // teardown: nothing left to report to
    b = DevBuf{};
}
void free_pin(DevBuf &b) {
    if (b.p) (void)hipHostFree(b.p);
    b = DevBuf{};
}

void Pipe::release() {
    if (device < 0)
        return;
    DeviceScope ds(device);
    for (hipStream_t st : s)
        if (st) (void)hipStreamSynchronize(st);
    for (int k = 0; k < kSlots; k++) {
        for (DevBuf &b : dev[k]) free_dev(b);
        free_pin(stage[k]);
        if (copied[k]) (void)hipEventDestroy(copied[k]);
        if (computed[k]) (void)hipEventDestroy(computed[k]);
        if (drained[k]) (void)hipEventDestroy(drained[k]);
        copied[k] = computed[k] = drained[k] = nullptr;
    }
    for (DevBuf &b : gather) free_pin(b);
    free_dev(ctr);
    free_pin(hctr);
    for (hipStream_t &st : s) {
        if (st) (void)hipStreamDestroy(st);
        st = nullptr;
    }
    device = -1;
}

Pipe::~Pipe() {
    if (!g_exiting.load())
        release();
}

thread_local Pipe g_pipe;

// The calling thread's pipeline on its current device.
int pipe_init(Pipe &c) {
    if (wg_device_count() <= 0)
        return WG_ERR_NODEV;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return WG_ERR_NODEV;
    if (c.device == dev)
        return WG_OK;
    c.release();  // first use on this thread, or the thread switched devices (current device kept)
    static std::once_flag once;
    std::call_once(once, [] { std::atexit([] { g_exiting.store(true); }); });
    // Test hook (WG_INTERNAL_TEST_FAULT_INJECT_PIPE=k, read once): the process's first
    // pipeline build fails at its k-th event creation, as under resource
    // exhaustion (tests/test_gpu_hostpath.py::test_pipeline_build_failure).
    static std::atomic<int> fail_at{[] {
        const char *v = std::getenv("WG_INTERNAL_TEST_FAULT_INJECT_PIPE");
        return v && *v ? std::atoi(v) : 0;
    }()};
    int nev = 0;
    auto mk_event = [&](hipEvent_t *e) {
        if (++nev == fail_at.load() && fail_at.exchange(0) != 0) {
            *e = nullptr;
            return false;
        }
        return hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
    };
    // Every handle is created before the pipeline is marked as built for
    // this device: a failure part-way releases what exists, so the next call
    // builds it again instead of finding null streams or events.
    bool ok = true;
    for (hipStream_t &st : c.s)
        ok = ok && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
    for (int k = 0; k < kSlots && ok; k++)
        ok = mk_event(&c.copied[k]) && mk_event(&c.computed[k]) && mk_event(&c.drained[k]);
    c.device = dev;  // release() below, or the built pipeline
    if (!ok) {
        c.release();
        return WG_ERR_RUNTIME;
    }
    return WG_OK;
}

// Grow-only buffers.  Called before a call enqueues anything (every call
// drains its streams before returning), so nothing in flight uses them.
int grow_dev(DevBuf &b, size_t bytes) {
    if (bytes <= b.cap)
        return WG_OK;
    free_dev(b);
    if (hipMalloc(&b.p, bytes) != hipSuccess) {
        b.p = nullptr;
        return WG_ERR_RUNTIME;
    }
    b.cap = bytes;
    return WG_OK;
}
int grow_pin(DevBuf &b, size_t bytes) {
    if (bytes <= b.cap)
        return WG_OK;
    free_pin(b);
    bytes = bytes < 4096 ? 4096 : bytes;
    if (hipHostMalloc(&b.p, bytes, hipHostMallocDefault) != hipSuccess) {
        b.p = nullptr;
        return WG_ERR_RUNTIME;
    }
    b.cap = bytes;
    return WG_OK;
}

template <typename T = uint8_t>
T *dp(Pipe &c, int slot, int role) {
    return static_cast<T *>(c.dev[slot][role].p);
}

// One call's chunk schedule.  If anything was enqueued and the call returns
// early (a failed copy, launch or event call), the destructor drains all
// three streams: no DMA may still read the caller's input or write its
// outputs once the call has returned.
struct Flight {
    Pipe &c;
    uint64_t k = 0;  // chunks begun
    bool armed = false;
    explicit Flight(Pipe &p) : c(p) {}
    ~Flight() {
        if (armed)
            drain();
    }
    int drain() {
        int rc = WG_OK;
        for (hipStream_t st : c.s)
            if (hipStreamSynchronize(st) != hipSuccess)
                rc = WG_ERR_RUNTIME;
        armed = false;
        return rc;
    }
    // Before chunk k's uploads.  staging: the slot's pinned staging is about
    // to be rewritten by the host, so its previous upload — on the exec
    // stream, ahead of that chunk's kernels — must have finished.
    int begin(int slot, bool staging) {
        armed = true;
        if (k >= (uint64_t)kSlots) {
            if (staging && hipEventSynchronize(c.computed[slot]) != hipSuccess)
                return WG_ERR_RUNTIME;
            if (hipStreamWaitEvent(c.s[kH2D], c.computed[slot], 0) != hipSuccess)
                return WG_ERR_RUNTIME;
        }
        return WG_OK;
    }
    // After the uploads, before the kernels.
    int uploaded(int slot) {
        if (hipEventRecord(c.copied[slot], c.s[kH2D]) != hipSuccess ||
            hipStreamWaitEvent(c.s[kExec], c.copied[slot], 0) != hipSuccess)
            return WG_ERR_RUNTIME;
        if (k >= (uint64_t)kSlots && hipStreamWaitEvent(c.s[kExec], c.drained[slot], 0) != hipSuccess)
            return WG_ERR_RUNTIME;
        return WG_OK;
    }
    // After the kernels, before the downloads.
    int computed(int slot) {
        if (hipEventRecord(c.computed[slot], c.s[kExec]) != hipSuccess ||
            hipStreamWaitEvent(c.s[kD2H], c.computed[slot], 0) != hipSuccess)
            return WG_ERR_RUNTIME;
        return WG_OK;
    }
    // After the downloads.
    int end(int slot) {
        k++;
        return hipEventRecord(c.drained[slot], c.s[kD2H]) == hipSuccess ? WG_OK : WG_ERR_RUNTIME;
    }
};

int h2d(Pipe &c, void *dst, const void *src, size_t n) {
    return !n || hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c.s[kH2D]) == hipSuccess ? WG_OK
                                                                                               : WG_ERR_RUNTIME;
}
int d2h(Pipe &c, void *dst, const void *src, size_t n) {
    return !n || hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c.s[kD2H]) == hipSuccess ? WG_OK
                                                                                               : WG_ERR_RUNTIME;
}
// Small per-unit results (a few bytes a message) stored straight into the
// call's pinned gather buffer by a kernel on the exec stream, behind the
// chunk's kernels: a runtime copy costs ~30 us of stream latency each (three
// per chunk idled the D2H stream between plaintext downloads), and a copy
// on the exec stream queued behind the uploads on the copy engine (decap
// 35 -> 101 ms).
__global__ void __launch_bounds__(256) small_store_kernel(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                          uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
        dst[i] = src[i];
}

// dst_alias: the device-visible address of dst (pinned), else nullptr: then
// a runtime copy on the D2H stream.
int xd2h(Pipe &c, void *dst, uint8_t *dst_alias, const void *src, size_t n) {
    if (!n)
        return WG_OK;
    if (!dst_alias)
        return d2h(c, dst, src, n);
    uint64_t blocks = (n + 255) / 256;
    blocks = blocks < 1024 ? blocks : 1024;
    hipLaunchKernelGGL(small_store_kernel, dim3((uint32_t)blocks), dim3(256), 0, c.s[kExec],
                       static_cast<const uint8_t *>(src), dst_alias, (uint64_t)n);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

// Downloads into pinned host memory by a store kernel on the D2H stream
// (knob host_d2h, bit 1: encap messages, bit 2: decap plaintext): 16-B
// loads from the slot, 16-B stores across PCIe, four in flight per lane.
// The runtime's hipMemcpyAsync picks its copy engine per call (an SDMA
// engine or a blit kernel); in the encap pipeline its message downloads ran
// at a fraction of the link while uploads were in flight (2 GiB of tun
// reads: 101 ms a call, 56 ms with the store kernel), while the decap
// pipeline's plaintext downloads are faster by SDMA (35.2 vs 38.5 ms)
// (tools/host_probe.py, profiles/r03_host_d2h_probe.txt).
__global__ void __launch_bounds__(256) d2h_store_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                        uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 1024u;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024u + threadIdx.x; i < n16; i += stride) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (i + k * 256u < n16)
                v[k] = src[i + k * 256u];
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (i + k * 256u < n16)
                dst[i + k * 256u] = v[k];
    }
}

// The device-visible address of a caller's host buffer when it is pinned
// (hipHostMalloc, wg_host_alloc, hipHostRegister), else nullptr: pageable
// memory is left to the runtime's staged copies.
uint8_t *pinned_alias(const void *host) {
    hipPointerAttribute_t a{};
    if (!host || hipPointerGetAttributes(&a, host) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer)
        return nullptr;
    const auto *h = static_cast<const uint8_t *>(host), *hb = static_cast<const uint8_t *>(a.hostPointer);
    return h >= hb ? static_cast<uint8_t *>(a.devicePointer) + (h - hb) : nullptr;
}

// A large download: the store kernel when knob host_d2h has `bit`, the
// destination is pinned (dst_alias: its device-visible address) and both
// ends and the length are 16-B multiples, else hipMemcpyAsync.
// force: the store kernel regardless of the knob (same conditions otherwise).
int d2h_big(Pipe &c, uint32_t bit, void *dst, uint8_t *dst_alias, const void *src, size_t n, bool force = false) {
    if (!n)
        return WG_OK;
    if (!dst_alias || !(force || (tune().host_d2h & bit)) || ((reinterpret_cast<uintptr_t>(dst_alias) | n) & 15) ||
        (reinterpret_cast<uintptr_t>(src) & 15))
        return d2h(c, dst, src, n);
    const uint64_t n16 = n / 16;
    uint64_t blocks = (n16 + 1023) / 1024;
    blocks = blocks < 1024 ? blocks : 1024;
    hipLaunchKernelGGL(d2h_store_kernel, dim3((uint32_t)blocks), dim3(256), 0, c.s[kD2H],
                       static_cast<const uint4 *>(src), reinterpret_cast<uint4 *>(dst_alias), n16);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

uint64_t chunk_bytes() { return (uint64_t)tune().host_chunk_mb << 20; }


#define WG_TRY(x)                 \
    do {                          \
        const int rc_ = (x);      \
        if (rc_ != WG_OK)         \
            return rc_;           \
    } while (0)

}  // namespace
}  // namespace wg

using namespace wg;

extern "C" int wg_l4csum_uniform_host(const uint8_t *host_base, uint64_t total_len, uint32_t segment_size,
                                      uint16_t csum_start, uint32_t flags, uint16_t *host_out) {
    if (!segment_size || (total_len && (!host_base || !host_out)))
        return WG_ERR_INVALID;
    if (!total_len)
        return WG_OK;
    Pipe &c = g_pipe;
    WG_TRY(pipe_init(c));
    const uint64_t nseg_total = (total_len + segment_size - 1) / segment_size;
    // whole segments per chunk, ~host_chunk_mb MiB
    uint64_t per = chunk_bytes() / segment_size;
    per = per ? per : 1;
    const uint64_t chunk = per * segment_size;
    const uint64_t slot_bytes = chunk < total_len ? chunk : total_len;
    const uint64_t slot_res = per < nseg_total ? per : nseg_total;
    for (int s = 0; s < kSlots; s++) {
        WG_TRY(grow_dev(c.dev[s][0], slot_bytes));
        WG_TRY(grow_dev(c.dev[s][1], slot_res * 2));
    }
    WG_TRY(grow_pin(c.gather[0], nseg_total * 2));
    uint16_t *hres = static_cast<uint16_t *>(c.gather[0].p);
    Flight f(c);
    for (uint64_t off = 0; off < total_len; off += chunk) {
        const int slot = (int)(f.k % kSlots);
        const uint64_t len = total_len - off < chunk ? total_len - off : chunk;
        const uint64_t first = off / segment_size, nseg = (len + segment_size - 1) / segment_size;
        WG_TRY(f.begin(slot, false));
        WG_TRY(h2d(c, dp(c, slot, 0), host_base + off, len));
        WG_TRY(f.uploaded(slot));
        WG_TRY(wg_l4csum_uniform(dp(c, slot, 0), len, segment_size, csum_start, flags, dp<uint16_t>(c, slot, 1),
                                 c.s[kExec]));
        WG_TRY(f.computed(slot));
        WG_TRY(d2h(c, hres + first, dp(c, slot, 1), nseg * 2));
        WG_TRY(f.end(slot));
    }
    WG_TRY(f.drain());
    std::memcpy(host_out, hres, nseg_total * sizeof(uint16_t));
    return WG_OK;
}

extern "C" int wg_decap_host(const uint8_t *host_msgs, uint64_t total_len, uint32_t segment_size,
                             const uint8_t key[32], uint8_t *host_plain, int8_t *host_status, uint8_t *host_verdict,
                             uint16_t *host_l4) {
    if (!segment_size || segment_size > 65535u + 32u || !key || (!host_verdict != !host_l4))
        return WG_ERR_INVALID;
    if (!total_len)
        return WG_OK;
    if (!host_msgs || !host_status || (segment_size > 32u && !host_plain))
        return WG_ERR_INVALID;
    Pipe &c = g_pipe;
    WG_TRY(pipe_init(c));
    const bool ver = host_verdict != nullptr;
    const uint64_t n = (total_len + segment_size - 1) / segment_size;
    const uint64_t pstride = segment_size > 32u ? segment_size - 32u : 0u;
    uint64_t per = chunk_bytes() / segment_size;
    per = per ? per : 1;
    per = per < n ? per : n;
    const uint64_t chunk = per * segment_size;
    enum { kIn, kPlain, kSt, kVer, kL4 };
    for (int s = 0; s < kSlots; s++) {
        WG_TRY(grow_dev(c.dev[s][kIn], chunk));
        WG_TRY(grow_dev(c.dev[s][kPlain], per * pstride + 16));
        WG_TRY(grow_dev(c.dev[s][kSt], per));
        WG_TRY(grow_dev(c.dev[s][kVer], per));
        WG_TRY(grow_dev(c.dev[s][kL4], per * 2));
    }
    WG_TRY(grow_pin(c.gather[kSt], n));
    WG_TRY(grow_pin(c.gather[kVer], n));
    WG_TRY(grow_pin(c.gather[kL4], n * 2));
    auto *gst = static_cast<int8_t *>(c.gather[kSt].p);
    auto *gver = static_cast<uint8_t *>(c.gather[kVer].p);
    auto *gl4 = static_cast<uint16_t *>(c.gather[kL4].p);
    uint8_t *const plain_alias = pstride ? pinned_alias(host_plain) : nullptr;
    uint8_t *const ast = pinned_alias(gst), *const aver = pinned_alias(gver), *const al4 = pinned_alias(gl4);
    // uniform chunks: a ramped schedule (short first and last chunks, as the
    // encap step has) made the runtime's plaintext downloads fall to a third
    // of the link at 32-MiB chunks (87.7 vs 34.0 ms,
    // profiles/r05_hostpath/ab_decap_ramp_32mib.txt)
    Flight f(c);
    for (uint64_t off = 0; off < total_len; off += chunk) {
        const int slot = (int)(f.k % kSlots);
        const uint64_t len = total_len - off < chunk ? total_len - off : chunk;
        const uint64_t first = off / segment_size, m = (len + segment_size - 1) / segment_size;
        WG_TRY(f.begin(slot, false));
        WG_TRY(h2d(c, dp(c, slot, kIn), host_msgs + off, len));
        WG_TRY(f.uploaded(slot));
        if (ver)
            WG_TRY(wg_aead_decrypt_verify_batch(dp(c, slot, kIn), len, segment_size, key, dp(c, slot, kPlain),
                                                dp<int8_t>(c, slot, kSt), dp(c, slot, kVer),
                                                dp<uint16_t>(c, slot, kL4), c.s[kExec]));
        else
            WG_TRY(wg_aead_decrypt_batch(dp(c, slot, kIn), len, segment_size, key, dp(c, slot, kPlain),
                                         dp<int8_t>(c, slot, kSt), c.s[kExec]));
        // the small per-message results: stored into the gather buffers by
        // kernels on the exec stream (xd2h), so the D2H stream carries only
        // plaintext, back to back
        WG_TRY(xd2h(c, gst + first, ast ? ast + first : nullptr, dp(c, slot, kSt), m));
        if (ver) {
            WG_TRY(xd2h(c, gver + first, aver ? aver + first : nullptr, dp(c, slot, kVer), m));
            WG_TRY(xd2h(c, gl4 + first, al4 ? al4 + 2 * first : nullptr, dp(c, slot, kL4), m * 2));
        }
        WG_TRY(f.computed(slot));
        // plaintext: the runtime's copy (faster from ~32 MiB up), the store
        // kernel under 24 MiB — the runtime's copies of 16-MiB chunks ran at a
        // third of the link beside the uploads (109 vs 34 ms a call,
        // profiles/r05_hostpath/chunk_sweep.jsonl).  Knob host_d2h: bit 2 the
        // store kernel for every plaintext chunk, bit 4 (default) for chunks
        // under 24 MiB; neither: the runtime's copy always.
        const bool small_chunk = m * pstride < (24ull << 20) && (tune().host_d2h & 4u);
        WG_TRY(d2h_big(c, 2u, host_plain + first * pstride, plain_alias ? plain_alias + first * pstride : nullptr,
                       dp(c, slot, kPlain), m * pstride, small_chunk));
        WG_TRY(f.end(slot));
    }
    WG_TRY(f.drain());
    std::memcpy(host_status, gst, n);
    if (ver) {
        std::memcpy(host_verdict, gver, n);
        std::memcpy(host_l4, gl4, n * 2);
    }
    return WG_OK;
}

extern "C" int wg_encap_host(const uint8_t *host_in, const wg_gso_desc *host_desc, uint64_t n, const uint8_t key[32],
                             uint32_t receiver_index, uint64_t counter0, uint32_t max_segments,
                             uint32_t max_segment_size, uint32_t msg_cap, uint8_t *host_msgs,
                             wg_encap_result *host_res, wg_gso_result *host_gso_res, uint64_t *next_counter) {
    if (!key || !max_segments || !max_segment_size || max_segment_size > 65535u || !msg_cap || (msg_cap & 15u))
        return WG_ERR_INVALID;
    if (!n) {
        if (next_counter)
            *next_counter = counter0;
        return WG_OK;
    }
    if (!host_in || !host_desc || !host_msgs || !host_res)
        return WG_ERR_INVALID;
    // super-buffers in input order, not overlapping: a chunk uploads one span
    for (uint64_t i = 0; i + 1 < n; i++)
        if (host_desc[i].in_offset + host_desc[i].in_len > host_desc[i + 1].in_offset)
            return WG_ERR_INVALID;
    // chunk boundaries: super-buffers until ~host_chunk_mb MiB of input (at
    // least one per chunk), every chunk's message count within the scan's
    // 32-bit index and n <= 2^20 per device call; and the chunk's per-slot
    // OUTPUT buffers (messages at msg_cap each, split headers at out_cap
    // each) within twice that budget, so many small tun reads with a msg_cap
    // sized for 64-KiB TSO reads do not size a slot at tens of GiB
    const uint64_t cb = chunk_bytes();
    const uint64_t ob = 2 * cb;
    const uint64_t max_cnt_call = (((1ull << 32) - 1) / max_segments) < (1ull << 20)
                                      ? (((1ull << 32) - 1) / max_segments)
                                      : (1ull << 20);
    if (!max_cnt_call)
        return WG_ERR_INVALID;
    // The first chunks are 1/8, 1/4 and 1/2 of the budget and the last one is
    // cut into halves the same way, so the pipeline fills and drains behind
    // short transfers (its first upload and last download run alone).
    std::vector<uint64_t> bounds{0};
    uint64_t max_cnt = 0, max_span = 0, max_seg = 0;
    for (uint64_t i = 0; i < n;) {
        const uint64_t i0 = i, s0 = host_desc[i0].in_offset;
        const size_t kb = bounds.size() - 1;
        const uint64_t cbk = kb < 3 ? cb >> (3 - kb) : cb;
        uint64_t segb = 0;
        do {
            segb += host_desc[i].out_cap;
            i++;
        } while (i < n && i - i0 < max_cnt_call && host_desc[i].in_offset + host_desc[i].in_len - s0 <= cbk &&
                 (i - i0 + 1) * (uint64_t)msg_cap <= ob && segb + host_desc[i].out_cap <= ob);
        const uint64_t span = host_desc[i - 1].in_offset + host_desc[i - 1].in_len - s0;
        bounds.push_back(i);
        max_cnt = i - i0 > max_cnt ? i - i0 : max_cnt;
        max_span = span > max_span ? span : max_span;
        max_seg = segb > max_seg ? segb : max_seg;
    }
    if (bounds.size() > 4) {  // the last chunk in pieces of 1/2, 1/4, 1/8, 1/8 (subsets: the slot bounds hold)
        const uint64_t a = bounds[bounds.size() - 2], b = bounds.back();
        if (b - a >= 8) {
            bounds.pop_back();
            const uint64_t m = b - a;
            bounds.push_back(a + m / 2);
            bounds.push_back(a + m / 2 + m / 4);
            bounds.push_back(a + m / 2 + m / 4 + m / 8);
            bounds.push_back(b);
        }
    }
    const uint64_t nchunks = bounds.size() - 1;
    Pipe &c = g_pipe;
    WG_TRY(pipe_init(c));
    enum { kIn, kDesc, kSeg, kGres, kMsgs, kEres, kWork };  // kDesc: rebased descriptors, then message offsets
    const size_t stage_bytes = max_cnt * (sizeof(wg_gso_desc) + sizeof(uint64_t));
    for (int s = 0; s < kSlots; s++) {
        WG_TRY(grow_dev(c.dev[s][kIn], max_span + 64));
        WG_TRY(grow_dev(c.dev[s][kDesc], max_cnt * (sizeof(wg_gso_desc) + sizeof(uint64_t))));  // + message offsets
        WG_TRY(grow_dev(c.dev[s][kSeg], max_seg + 64));
        WG_TRY(grow_dev(c.dev[s][kGres], max_cnt * sizeof(wg_gso_result)));
        WG_TRY(grow_dev(c.dev[s][kMsgs], max_cnt * msg_cap));
        WG_TRY(grow_dev(c.dev[s][kEres], max_cnt * sizeof(wg_encap_result)));
        WG_TRY(grow_dev(c.dev[s][kWork], 4 * (max_cnt + 1024)));
        WG_TRY(grow_pin(c.stage[s], stage_bytes));
    }
    WG_TRY(grow_pin(c.gather[kEres], n * sizeof(wg_encap_result)));
    WG_TRY(grow_pin(c.gather[kGres], n * sizeof(wg_gso_result)));
    WG_TRY(grow_dev(c.ctr, (nchunks + 1) * sizeof(uint64_t)));
    WG_TRY(grow_pin(c.hctr, sizeof(uint64_t)));
    auto *geres = static_cast<wg_encap_result *>(c.gather[kEres].p);
    auto *ggres = static_cast<wg_gso_result *>(c.gather[kGres].p);
    auto *ctr = static_cast<uint64_t *>(c.ctr.p);
    uint8_t *const msgs_alias = pinned_alias(host_msgs);
    Flight f(c);
    f.armed = true;
    if (hipMemsetAsync(ctr, 0, sizeof(uint64_t), c.s[kExec]) != hipSuccess)
        return WG_ERR_RUNTIME;
    for (uint64_t k = 0; k < nchunks; k++) {
        const int slot = (int)(f.k % kSlots);
        const uint64_t i0 = bounds[k], cnt = bounds[k + 1] - i0;
        const uint64_t s0 = host_desc[i0].in_offset;
        const uint64_t span = host_desc[i0 + cnt - 1].in_offset + host_desc[i0 + cnt - 1].in_len - s0;
        WG_TRY(f.begin(slot, true));
        // descriptors rebased to the slot: input relative to the chunk's
        // span, segment-header slots packed by out_cap, messages at i * msg_cap
        auto *sd = static_cast<wg_gso_desc *>(c.stage[slot].p);
        auto *so = reinterpret_cast<uint64_t *>(sd + cnt);
        uint64_t oo = 0;
        for (uint64_t j = 0; j < cnt; j++) {
            sd[j] = host_desc[i0 + j];
            sd[j].in_offset -= s0;
            sd[j].out_offset = oo;
            oo += sd[j].out_cap;
            so[j] = j * msg_cap;
        }
        // the H2D stream carries only the payload spans, back to back; the
        // rebased descriptors and message offsets (contiguous in the staging
        // buffer and in the slot) go up in ONE copy on the exec stream, ahead
        // of the kernels (a small copy costs ~30 us of stream latency: three
        // per chunk on the H2D stream were ~90 us of idle link per chunk)
        WG_TRY(h2d(c, dp(c, slot, kIn), host_in + s0, span));
        WG_TRY(f.uploaded(slot));
        uint8_t *const dd = dp(c, slot, kDesc);
        if (hipMemcpyAsync(dd, sd, cnt * (sizeof(wg_gso_desc) + sizeof(uint64_t)), hipMemcpyHostToDevice,
                           c.s[kExec]) != hipSuccess)
            return WG_ERR_RUNTIME;
        WG_TRY(encap_batch_launch(dp(c, slot, kIn), reinterpret_cast<wg_gso_desc *>(dd), cnt, dp(c, slot, kSeg),
                                  dp<wg_gso_result>(c, slot, kGres), key, receiver_index, counter0,
                                  reinterpret_cast<uint64_t *>(dd + cnt * sizeof(wg_gso_desc)), msg_cap, max_segments,
                                  max_segment_size,
                                  dp(c, slot, kMsgs), dp<wg_encap_result>(c, slot, kEres), dp<uint32_t>(c, slot, kWork),
                                  ctr + k + 1, ctr + k, c.s[kExec]));
        WG_TRY(f.computed(slot));
        WG_TRY(d2h_big(c, 1u, host_msgs + i0 * msg_cap, msgs_alias ? msgs_alias + i0 * msg_cap : nullptr,
                       dp(c, slot, kMsgs), cnt * msg_cap));
        WG_TRY(d2h(c, geres + i0, dp(c, slot, kEres), cnt * sizeof(wg_encap_result)));
        if (host_gso_res)
            WG_TRY(d2h(c, ggres + i0, dp(c, slot, kGres), cnt * sizeof(wg_gso_result)));
        WG_TRY(f.end(slot));
    }
    WG_TRY(d2h(c, c.hctr.p, ctr + nchunks, sizeof(uint64_t)));
    WG_TRY(f.drain());
    std::memcpy(host_res, geres, n * sizeof(wg_encap_result));
    if (host_gso_res)
        std::memcpy(host_gso_res, ggres, n * sizeof(wg_gso_result));
    if (next_counter)
        *next_counter = counter0 + *static_cast<uint64_t *>(c.hctr.p);
    return WG_OK;
}

extern "C" int wg_host_release(void) {
    g_pipe.release();
    return WG_OK;
}

extern "C" int wg_host_alloc(void **ptr, uint64_t bytes) {
    if (!ptr || !bytes)
        return WG_ERR_INVALID;
    *ptr = nullptr;
    if (wg_device_count() <= 0)
        return WG_ERR_NODEV;
    return hipHostMalloc(ptr, bytes, hipHostMallocDefault) == hipSuccess ? WG_OK : WG_ERR_RUNTIME;
}

extern "C" int wg_host_free(void *ptr) {
    if (!ptr)
        return WG_OK;
    return hipHostFree(ptr) == hipSuccess ? WG_OK : WG_ERR_RUNTIME;
}
