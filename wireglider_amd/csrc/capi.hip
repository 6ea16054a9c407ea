// capi.hip — misc C ABI (version, errors, device count), launch tuning and
// the roofline probes.  The host-memory path is hostpath.hip.
#include <hip/hip_runtime.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "wg_device.hpp"
#include "wg_internal.hpp"
#include "wireglider_amd.h"

namespace wg {

// One table of knobs: name, field, and the values it accepts.  Both the
// environment (WG_<NAME>, read once) and wg_tune_set go through it, so a value
// either is accepted by both or ignored / rejected by both.
struct Knob {
    const char *name;
    uint64_t Tune::*f64;
    uint32_t Tune::*f32;
    uint64_t lo, hi;      // accepted range ...
    const uint64_t *set;  // ... or, when non-null, one of these nset values
    size_t nset;
};

static const uint64_t kL4Small[] = {0, 5}, kL4SU[] = {0, 2}, kVSmall[] = {0, 6, 7, 8},
                      kWaves[] = {1, 2, 4, 8}, kAbl[] = {0, 1, 32},
                      kUnroll[] = {4, 8}, kCoopW[] = {2, 4, 8, 16}, kAeadK[] = {0, 2, 3}, kParts[] = {1, 2, 3, 4, 8}, kCoop[] = {0, 1};
#define WG_N(a) (sizeof(a) / sizeof(a[0]))
static const Knob kKnobs[] = {
    {"l4_blocks", &Tune::l4_blocks, nullptr, 1, 1u << 20, nullptr, 0},
    {"l4_nt", nullptr, &Tune::l4_nt, 0, 1, nullptr, 0},
    {"l4_small", nullptr, &Tune::l4_small, 0, 0, kL4Small, WG_N(kL4Small)},
    {"l4_small_uniform", nullptr, &Tune::l4_small_uniform, 0, 0, kL4SU, WG_N(kL4SU)},
    {"gso_blocks", &Tune::gso_blocks, nullptr, 1, 1u << 23, nullptr, 0},
    {"gso_waves", nullptr, &Tune::gso_waves, 0, 0, kWaves, WG_N(kWaves)},
    {"gso_split", nullptr, &Tune::gso_split, 1, 64, nullptr, 0},
    {"gso_groups", nullptr, &Tune::gso_groups, 1, 64, nullptr, 0},
    {"gso_spw", nullptr, &Tune::gso_spw, 0, 4, nullptr, 0},
    {"encap_spw", nullptr, &Tune::encap_spw, 0, 4, nullptr, 0},
    {"verify_small", nullptr, &Tune::verify_small, 0, 0, kVSmall, WG_N(kVSmall)},
    {"verify_auto_t", nullptr, &Tune::verify_auto_t, 1, 64, nullptr, 0},
    {"verify_k2min", nullptr, &Tune::verify_k2min, 8, 65536, nullptr, 0},
    {"gso_ablate", nullptr, &Tune::gso_ablate, 0, 0, kAbl, WG_N(kAbl)},
    {"host_chunk_mb", nullptr, &Tune::host_chunk_mb, 1, 4096, nullptr, 0},
    {"host_d2h", nullptr, &Tune::host_d2h, 0, 7, nullptr, 0},
    {"l4_unroll", nullptr, &Tune::l4_unroll, 0, 0, kUnroll, WG_N(kUnroll)},
    {"l4_coop", &Tune::l4_coop, nullptr, 0, 1u << 20, nullptr, 0},
    {"l4_coop_waves", nullptr, &Tune::l4_coop_waves, 0, 0, kCoopW, WG_N(kCoopW)},
    {"aead_k", nullptr, &Tune::aead_k, 0, 0, kAeadK, WG_N(kAeadK)},
    {"aead_stage", nullptr, &Tune::aead_stage, 0, 1, nullptr, 0},
    {"encap_parts", nullptr, &Tune::encap_parts, 0, 0, kParts, WG_N(kParts)},
    {"encap_synth", nullptr, &Tune::encap_synth, 0, 1, nullptr, 0},
    {"lane_coop", nullptr, &Tune::lane_coop, 0, 0, kCoop, WG_N(kCoop)},
};
#undef WG_N

static const Knob *find_knob(const char *key) {
    for (const Knob &k : kKnobs)
        if (std::strcmp(k.name, key) == 0)
            return &k;
    return nullptr;
}

static bool knob_set(Tune &t, const Knob &k, uint64_t v) {
    bool ok = false;
    if (k.set) {
        for (size_t i = 0; i < k.nset; i++)
            ok = ok || v == k.set[i];
    } else {
        ok = v >= k.lo && v <= k.hi;
    }
    if (!ok)
        return false;
    if (k.f64)
        t.*(k.f64) = v;
    else
        t.*(k.f32) = (uint32_t)v;
    return true;
}

// The knobs' defaults and environment overrides (read once).
static Tune tune_initial() {
    Tune x;
    // Measured on MI355X (tools/tune_l4.py, profiles/): one iteration per
    // wave (grid = n / (4 * ppw), i.e. no grid-stride loop), 4 packets per
    // wave, non-temporal loads: 7.26 TB/s vs 5.6 TB/s for a 2048-block
    // grid-stride launch with default-policy loads.
    x.l4_blocks = 1u << 20;
    x.l4_nt = 1;
    // Descriptor batches: the split-role kernel (l4_small = 5): small
    // packets of all-small groups a lane each, the rest wave-per-packet.
    // Config 4's 64-B sub-batch 0.336 -> 0.061 ms (35 % of the roofline);
    // config 5 and config 4's mixed batch within 0.6 % of the
    // wave-per-packet kernel (interleaved A/B, profiles/r02_small_ab.json).
    x.l4_small = 5;
    x.l4_small_uniform = 2;  // lane per segment: 64-B PacketBatch 0.342 -> 0.043 ms (a lane quad: 0.074)
    x.gso_blocks = 1u << 23;
    // GSO: three 4-wave blocks per super-buffer (3 groups -2.5 % vs 1 on
    // two boxes once the per-wave setup is one scalar round trip), each
    // wave issuing the loads of 4 segments before finishing them (93
    // VGPRs, 5 waves/SIMD: config 3 -1.7 %, the fused encap -1.4 % vs
    // the ping-pong pipeline, profiles/r02_gso_spw_ab.json); the verify
    // kernel at 8 waves/SIMD (64 VGPRs, no spill) (tools/ab.py,
    // profiles/r01_ab_*.json).
    x.gso_waves = 4;
    x.gso_split = 1;
    x.gso_spw = 4;
    // the encap step's headers-only split: 3 segments per wave step,
    // encap 18.37 -> 18.13 ms (profiles/r03_encap_gso_ab.json)
    x.encap_spw = 3;
    x.gso_groups = 3;
    // verify_small 7: per call the walking kernel (first call on a stream,
    // all-small sample), the wave kernel or the compacting path, from a
    // cost model of the previous call's sampled size mix (l4csum.hip
    // wg_verify_desc); auto_t = the fewest small packets among the 64
    // samples that may pick compaction
    x.verify_small = 7;
    x.verify_auto_t = 1;
    x.verify_k2min = 2048;
    x.gso_ablate = 0;
    // descriptor batches' small packets: chunks loaded by the wave together
    // (coop_chunks): config 4's 64-B sub-batch 46.0 -> 45.3 us, config 4 / 5
    // unchanged (profiles/r06_coop_ab.txt)
    x.lane_coop = 1;
    // host pipeline chunk: 128-512 MiB reach 97-98 % of the raw H2D rate
    // (8 MiB: 70 %, per-chunk overheads; profiles/r02_host_path.json);
    // with both directions in flight 64 MiB: decap 35.2 ms vs 37.3 at
    // 256 MiB (shorter fill and drain), encap within 2 %
    // (profiles/r03_host_d2h_probe.txt)
    x.host_chunk_mb = 64;
    // encap message downloads by the store kernel (bit 1), decap plaintext
    // by the runtime's copy except chunks under 24 MiB (bit 4; bit 2: every
    // plaintext chunk) (hostpath.hip d2h_store_kernel)
    x.host_d2h = 5;
    // descriptor batches: 8 loads in flight per lane on a long packet's
    // rest (5 waves/SIMD instead of 6): config 4 -1.4 %, config 1 (64 KiB
    // buffers) -26 %, config 5 (no long packets) unchanged
    // (profiles/r02_unroll_ab.json)
    x.l4_unroll = 8;
    // descriptor batches of <= 16,384 packets: a 4-wave block per packet.
    // The split kernel's grid is sized by descriptor count (n / 16
    // waves), so few long packets starve the HBM pipe: 16,384 x 64 KiB
    // 0.178 -> 0.159 ms, 1,024 x 64 KiB 0.146 -> 0.014 ms; at 16,384
    // packets of 64 / 1,500 / 9,000 B within +1.3 us, past 16 K packets
    // of 1,500 B the split kernel wins 2x (profiles/r02_coop_probe.json)
    x.l4_coop = 16384;
    x.l4_coop_waves = 4;
    // AEAD: K consecutive ChaCha20 blocks per lane, chosen per batch (0:
    // 2 or 3, whichever fills the wave better), each lane's blocks two at
    // a time with interleaved quarter rounds (the kernel waits on
    // dependent VALU issue, not memory), groups of exactly the lanes a
    // packet needs.  1 M x 1500 B: K = 3 in 9-lane groups 1.401 ms vs
    // K = 2 in 16-lane groups 1.506 (profiles/r02_aead_flex_ab.json), the
    // interleave -8 % (profiles/r02_aead_pair_ab.json)
    x.aead_k = 0;
    // encrypt: messages assembled in LDS, written in whole lines: writes
    // 2.53 -> 1.61 GB per 1 M x 1500 B (= the message bytes), encrypt
    // -1.0 %, encap -2.9 % (profiles/r04_aead_stage/)
    x.aead_stage = 1;
    x.encap_parts = 1;
    // wg_encap_batch: the AEAD builds the segment headers, the split only
    // plans: config 3's super-buffers 16.99 -> 14.96 ms
    // (profiles/r04_encap_synth/)
    x.encap_synth = 1;
    // environment overrides: WG_<KNOB> (upper case), same accepted values
    // as wg_tune_set; anything else is ignored
    for (const Knob &k : kKnobs) {
        std::string env = "WG_";
        for (const char *c = k.name; *c; c++) env += (char)std::toupper((unsigned char)*c);
        const char *v = std::getenv(env.c_str());
        if (!v || !*v)
            continue;
        char *end = nullptr;
        const unsigned long long val = std::strtoull(v, &end, 0);
        if (end && *end == 0)
            knob_set(x, k, val);
    }
    return x;
}

// The knob table, published copy-on-write: launches read the current
// immutable snapshot through one acquire load (no lock, no shared line
// written on the launch path — VERDICT r05 weak item 2: the per-launch
// mutex put every worker thread's launches on one contended cache line);
// wg_tune_set copies it under g_tune_mu, changes the copy and publishes
// it.  A replaced snapshot stays allocated (a reader may still be copying
// it) and reachable in g_tune_old: one ~100-B Tune per accepted set.
static std::mutex g_tune_mu;  // writers only
static std::atomic<const Tune *> g_tune_cur{nullptr};
static std::vector<const Tune *> g_tune_old;

static const Tune *tune_current_locked() {  // caller holds g_tune_mu
    const Tune *p = g_tune_cur.load(std::memory_order_relaxed);
    if (!p) {
        p = new Tune(tune_initial());
        g_tune_cur.store(p, std::memory_order_release);
    }
    return p;
}

// One consistent copy of every knob per launch: a concurrent wg_tune_set is
// seen entirely or not at all, never half-applied (and never a data race).
Tune tune() {
    const Tune *p = g_tune_cur.load(std::memory_order_acquire);
    if (__builtin_expect(p == nullptr, 0)) {
        std::lock_guard<std::mutex> lk(g_tune_mu);
        p = tune_current_locked();
    }
    return *p;
}

bool debug_sync(hipStream_t st, const char *kernel) {
    static const bool on = [] {
        const char *v = std::getenv("WG_DEBUG_SYNC");
        return v && *v == '1';
    }();
    if (!on)
        return true;
    const hipError_t e = hipStreamSynchronize(st);
    if (e == hipSuccess)
        return true;
    std::fprintf(stderr, "wireglider_amd: %s failed: %s\n", kernel, hipGetErrorString(e));
    return false;
}

// Read-roofline probe: the checksum kernels' access structure with nothing
// else — one-shot waves (no grid-stride loop), each streaming U contiguous
// KiB with non-temporal global_load_dwordx4 (all U issued before the first
// use), folded into one word per wave.  Its bandwidth is the measured read
// ceiling the checksum kernels are compared against.
template <int U>
__global__ __launch_bounds__(256) void probe_read_kernel(const uint8_t *dev, uint64_t nchunks, uint64_t *out) {
    const uint64_t wave = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t c0 = wave * (uint64_t)U * 64u;
    const uintptr_t base = reinterpret_cast<uintptr_t>(dev);
    const uint32_t lane = lane_id();
    if (c0 >= nchunks)
        return;
    const uint64_t last = nchunks - 1;
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        uint64_t c = c0 + (uint64_t)u * 64u + lane;
        v[u] = ld16_nt(base + 16u * (c < last ? c : last));
    }
    Acc acc;
#pragma unroll
    for (int u = 0; u < U; u++) acc.add4(v[u]);
    const uint32_t s = wave_sum_u32(fold16(acc.value()));
    // Keep the loads live without a contended atomic: a data-dependent store
    // that (for any real data) never fires.
    if (lane == 0 && s == 0xFFFFFFFFu) *out = s;
}

// Read probe with the packet kernels' issue structure: one-shot waves, each
// reading P = 4 runs of `run` bytes (consecutive runs = consecutive
// packets of a uniform batch), every run as two 64-lane 16-B loads (the
// aligned chunks covering it, clamped onto its last chunk — duplicate lanes
// coalesce), all 8 loads issued before the first use, non-temporal.  The
// same bytes and the same load pattern as l4csum_kernel on a PacketBatch of
// run-byte segments, with none of its work: its rate bounds that kernel.
template <int P>
__global__ __launch_bounds__(256) void probe_read_runs_kernel(const uint8_t *dev, uint64_t nruns, uint32_t run,
                                                              uint64_t *out) {
    const uint64_t wave = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t r0 = wave * P;
    if (r0 >= nruns)
        return;
    const uint32_t lane = lane_id();
    v4u v[2 * P];
#pragma unroll
    for (int j = 0; j < P; j++) {
        const uint64_t r = r0 + j < nruns ? r0 + j : nruns - 1;
        const uintptr_t a = reinterpret_cast<uintptr_t>(dev) + r * run;
        const uintptr_t c0 = a & ~(uintptr_t)15;
        const uint32_t last = (uint32_t)(((a + run - 1) & ~(uintptr_t)15) - c0) >> 4;
        v[2 * j] = ld16_nt(c0 + 16u * (lane < last ? lane : last));
        v[2 * j + 1] = ld16_nt(c0 + 16u * (lane + 64 < last ? lane + 64 : last));
    }
    Acc acc;
#pragma unroll
    for (int j = 0; j < 2 * P; j++) acc.add4(v[j]);
    const uint32_t s = wave_sum_u32(fold16(acc.value()));
    if (lane == 0 && s == 0xFFFFFFFFu) *out = s;
}

// Copy-roofline probe: one-shot waves, each copying U contiguous KiB (all
// loads issued first, then the stores; non-temporal loads and stores, or the
// default cache policy when kNT is false).
template <int U, bool kNT = true>
__global__ __launch_bounds__(256) void probe_copy_kernel(const uint8_t *src, uint8_t *dst, uint64_t nchunks) {
    const uint64_t wave = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t c0 = wave * (uint64_t)U * 64u;
    const uint32_t lane = lane_id();
    if (c0 >= nchunks)
        return;
    const uintptr_t s = reinterpret_cast<uintptr_t>(src), d = reinterpret_cast<uintptr_t>(dst);
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t c = c0 + (uint64_t)u * 64u + lane;
        v[u] = ld16x<kNT>(s + 16u * (c < nchunks ? c : nchunks - 1));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t c = c0 + (uint64_t)u * 64u + lane;
        auto *p = reinterpret_cast<__attribute__((address_space(1))) v4u *>(d + 16u * c);
        if (c < nchunks) {
            if constexpr (kNT)
                __builtin_nontemporal_store(v[u], p);
            else
                *p = v[u];
        }
    }
}

}  // namespace wg

using namespace wg;

extern "C" int wg_probe_copy(const uint8_t *src, uint8_t *dst, uint64_t nbytes, uint32_t kib_per_wave, void *stream) {
    if (!src || !dst || ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) || nbytes < 16)
        return WG_ERR_INVALID;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t nch = nbytes >> 4;
    const bool dflt = kib_per_wave & WG_PROBE_DEFAULT_POLICY;  // default cache policy instead of non-temporal
    kib_per_wave &= ~WG_PROBE_DEFAULT_POLICY;
    const uint32_t U = kib_per_wave == 2 || kib_per_wave == 4 ? kib_per_wave : 1;
    uint64_t blocks = (nch + 256ull * U - 1) / (256ull * U);
    if (blocks >= 8) blocks = (blocks + 7) & ~7ull;
    if (blocks > 0x7fffffffull) return WG_ERR_INVALID;
    const dim3 g((unsigned)blocks), b(256);
    switch (U * 2 + (dflt ? 1 : 0)) {
    case 4: hipLaunchKernelGGL((probe_copy_kernel<2, true>), g, b, 0, st, src, dst, nch); break;
    case 5: hipLaunchKernelGGL((probe_copy_kernel<2, false>), g, b, 0, st, src, dst, nch); break;
    case 8: hipLaunchKernelGGL((probe_copy_kernel<4, true>), g, b, 0, st, src, dst, nch); break;
    case 9: hipLaunchKernelGGL((probe_copy_kernel<4, false>), g, b, 0, st, src, dst, nch); break;
    case 3: hipLaunchKernelGGL((probe_copy_kernel<1, false>), g, b, 0, st, src, dst, nch); break;
    default: hipLaunchKernelGGL((probe_copy_kernel<1, true>), g, b, 0, st, src, dst, nch); break;
    }
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_probe_read(const uint8_t *dev, uint64_t nbytes, uint64_t *dev_out, uint32_t kib_per_wave,
                             uint32_t run_bytes, void *stream) {
    if (!dev || !dev_out || (reinterpret_cast<uintptr_t>(dev) & 15) || nbytes < 16) return WG_ERR_INVALID;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (run_bytes) {  // the packet kernels' structure: 4 runs of run_bytes per wave
        if (run_bytes > 2048 || nbytes < run_bytes) return WG_ERR_INVALID;
        const uint64_t nruns = nbytes / run_bytes;
        uint64_t blocks = (nruns + 15) / 16;
        if (blocks >= 8) blocks = (blocks + 7) & ~7ull;
        if (blocks > 0x7fffffffull) return WG_ERR_INVALID;
        hipLaunchKernelGGL(probe_read_runs_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, st, dev, nruns, run_bytes,
                           dev_out);
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    const uint64_t nch = nbytes >> 4;
    const uint32_t U = kib_per_wave == 2 || kib_per_wave == 4 || kib_per_wave == 8 ? kib_per_wave : 1;
    uint64_t blocks = (nch + 256ull * U - 1) / (256ull * U);
    if (blocks >= 8) blocks = (blocks + 7) & ~7ull;
    switch (U) {
    case 2: hipLaunchKernelGGL(probe_read_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, st, dev, nch, dev_out); break;
    case 4: hipLaunchKernelGGL(probe_read_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, st, dev, nch, dev_out); break;
    case 8: hipLaunchKernelGGL(probe_read_kernel<8>, dim3((unsigned)blocks), dim3(256), 0, st, dev, nch, dev_out); break;
    default: hipLaunchKernelGGL(probe_read_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, st, dev, nch, dev_out); break;
    }
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_abi_version(void) { return WG_ABI_VERSION; }

extern "C" const char *wg_strerror(int code) {
    switch (code) {
    case WG_OK: return "ok";
    case WG_ERR_INVALID: return "invalid argument";
    case WG_ERR_NODEV: return "no HIP device";
    case WG_ERR_LAUNCH: return "kernel launch failed";
    case WG_ERR_RUNTIME: return "HIP runtime failure";
    default: return "unknown error";
    }
}

extern "C" int wg_tune_set(const char *key, uint64_t value) {
    const Knob *k = key ? find_knob(key) : nullptr;
    if (!k)
        return WG_ERR_INVALID;
    std::lock_guard<std::mutex> lk(g_tune_mu);
    const Tune *cur = tune_current_locked();
    Tune x = *cur;
    if (!knob_set(x, *k, value))
        return WG_ERR_INVALID;
    g_tune_old.push_back(cur);
    g_tune_cur.store(new Tune(x), std::memory_order_release);
    return WG_OK;
}

extern "C" int wg_tune_get(const char *key, uint64_t *value) {
    const Knob *k = key ? find_knob(key) : nullptr;
    if (!k || !value)
        return WG_ERR_INVALID;
    const Tune t = tune();
    *value = k->f64 ? t.*(k->f64) : (uint64_t)(t.*(k->f32));
    return WG_OK;
}

extern "C" int wg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}
