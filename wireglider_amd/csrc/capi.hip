// capi.hip — misc C ABI (version, errors, device count), launch tuning, and
// the host-memory path (tun / UDP buffers live in host memory).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <string>

#include "wg_device.hpp"
#include "wg_internal.hpp"
#include "wireglider_amd.h"

namespace wg {

static uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *v = std::getenv(name);
    if (!v || !*v)
        return dflt;
    char *end = nullptr;
    unsigned long long x = std::strtoull(v, &end, 0);
    return (end && *end == 0 && x > 0) ? (uint64_t)x : dflt;
}

Tune &tune_mut() {
    static Tune t = [] {
        Tune x;
        // Measured on MI355X (tools/tune_l4.py, profiles/): one iteration per
        // wave (grid = n / (4 * ppw), i.e. no grid-stride loop), 4 packets per
        // wave, non-temporal loads: 7.26 TB/s vs 5.6 TB/s for a 2048-block
        // grid-stride launch with default-policy loads.
        x.l4_blocks = env_u64("WG_L4_BLOCKS", 1u << 20);
        x.l4_ppw = (uint32_t)env_u64("WG_L4_PPW", 4);
        x.l4_nt = (uint32_t)env_u64("WG_L4_NT", 1);
        // Descriptor batches: each wave takes 4 iterations and prefetches the
        // next iteration's descriptors by one vector load during the current
        // one's finish (+3-5 % on config 5, profiles/r01_ab_session2.json).
        x.l4_descv = (uint32_t)env_u64("WG_L4_DESCV", 2);
        x.l4_occ = (uint32_t)env_u64("WG_L4_OCC", 0);
        x.l4_iters = (uint32_t)env_u64("WG_L4_ITERS", 4);
        x.gso_blocks = env_u64("WG_GSO_BLOCKS", 1u << 23);
        // GSO: three 4-wave blocks per super-buffer, each wave a ping-pong
        // pipeline (next segment's loads in flight while this one finishes;
        // 3 groups -2.5 % vs 1 on two boxes once the per-wave setup is one
        // scalar round trip); the verify kernel at 8 waves/SIMD (64 VGPRs,
        // no spill) (tools/ab.py, profiles/r01_ab_*.json).
        x.gso_waves = (uint32_t)env_u64("WG_GSO_WAVES", 4);
        x.gso_split = (uint32_t)env_u64("WG_GSO_SPLIT", 1);
        x.gso_spw = (uint32_t)env_u64("WG_GSO_SPW", 1);
        x.gso_groups = (uint32_t)env_u64("WG_GSO_GROUPS", 3);
        x.verify_occ = (uint32_t)env_u64("WG_VERIFY_OCC", 8);
        x.verify_dm = (uint32_t)env_u64("WG_VERIFY_DM", 0);
        x.gro_lds = (uint32_t)env_u64("WG_GRO_LDS", 1);
        x.gro_wide = (uint32_t)env_u64("WG_GRO_WIDE", 1);
        x.gso_ablate = 0;
        return x;
    }();
    return t;
}

const Tune &tune() { return tune_mut(); }

// Per-host-thread device workspace for the host-memory path.  Grows to the
// largest batch seen; freed at thread exit.
struct HostCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t *dbuf = nullptr;
    size_t dcap = 0;
    uint16_t *dout = nullptr;
    size_t ocap = 0;
    ~HostCtx() {
        if (device < 0)
            return;
        hipSetDevice(device);
        if (dbuf) hipFree(dbuf);
        if (dout) hipFree(dout);
        if (stream) hipStreamDestroy(stream);
    }
};

static thread_local HostCtx g_host;

static int host_ctx_reserve(size_t bytes, size_t outs) {
    HostCtx &c = g_host;
    if (c.device < 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess)
            return WG_ERR_NODEV;
        if (hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess)
            return WG_ERR_RUNTIME;
        c.device = dev;
    }
    if (bytes > c.dcap) {
        if (c.dbuf) hipFree(c.dbuf);
        c.dbuf = nullptr;
        size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes;
        if (hipMalloc(&c.dbuf, cap) != hipSuccess) {
            c.dcap = 0;
            return WG_ERR_RUNTIME;
        }
        c.dcap = cap;
    }
    if (outs > c.ocap) {
        if (c.dout) hipFree(c.dout);
        c.dout = nullptr;
        size_t cap = outs < 4096 ? 4096 : outs;
        if (hipMalloc(&c.dout, cap * sizeof(uint16_t)) != hipSuccess) {
            c.ocap = 0;
            return WG_ERR_RUNTIME;
        }
        c.ocap = cap;
    }
    return WG_OK;
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

// Copy-roofline probe: one-shot waves, each copying U contiguous KiB
// (non-temporal loads, all issued first, then non-temporal stores).
template <int U>
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
        v[u] = ld16_nt(s + 16u * (c < nchunks ? c : nchunks - 1));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t c = c0 + (uint64_t)u * 64u + lane;
        if (c < nchunks)
            __builtin_nontemporal_store(v[u], reinterpret_cast<__attribute__((address_space(1))) v4u *>(d + 16u * c));
    }
}

}  // namespace wg

using namespace wg;

extern "C" int wg_probe_copy(const uint8_t *src, uint8_t *dst, uint64_t nbytes, uint32_t kib_per_wave, void *stream) {
    if (!src || !dst || ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) || nbytes < 16)
        return WG_ERR_INVALID;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t nch = nbytes >> 4;
    const uint32_t U = kib_per_wave == 2 || kib_per_wave == 4 ? kib_per_wave : 1;
    uint64_t blocks = (nch + 256ull * U - 1) / (256ull * U);
    if (blocks >= 8) blocks = (blocks + 7) & ~7ull;
    switch (U) {
    case 2: hipLaunchKernelGGL(probe_copy_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, nch); break;
    case 4: hipLaunchKernelGGL(probe_copy_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, nch); break;
    default: hipLaunchKernelGGL(probe_copy_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, nch); break;
    }
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_probe_read(const uint8_t *dev, uint64_t nbytes, uint64_t *dev_out, uint32_t kib_per_wave,
                             uint32_t unused, void *stream) {
    (void)unused;
    if (!dev || !dev_out || (reinterpret_cast<uintptr_t>(dev) & 15) || nbytes < 16) return WG_ERR_INVALID;
    hipStream_t st = static_cast<hipStream_t>(stream);
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
    if (!key)
        return WG_ERR_INVALID;
    Tune &t = tune_mut();
    const std::string k(key);
    if (k == "l4_blocks" && value >= 1 && value <= (1u << 20))
        t.l4_blocks = value;
    else if (k == "l4_ppw" && (value == 1 || value == 2 || value == 4 || value == 8))
        t.l4_ppw = (uint32_t)value;
    else if (k == "l4_nt" && value <= 1)
        t.l4_nt = (uint32_t)value;
    else if (k == "l4_iters" && value >= 1 && value <= 64)
        t.l4_iters = (uint32_t)value;
    else if (k == "l4_descv" && value <= 2)
        t.l4_descv = (uint32_t)value;
    else if (k == "l4_occ" && (value == 0 || value == 7 || value == 8))
        t.l4_occ = (uint32_t)value;
    else if (k == "gso_blocks" && value >= 1 && value <= (1u << 23))
        t.gso_blocks = value;
    else if (k == "gro_lds" && value <= 1)
        t.gro_lds = (uint32_t)value;
    else if (k == "gro_wide" && value <= 1)
        t.gro_wide = (uint32_t)value;
    else if (k == "verify_dm" && (value == 0 || value == 2))
        t.verify_dm = (uint32_t)value;
    else if (k == "verify_occ" && (value == 0 || value == 6 || value == 8))
        t.verify_occ = (uint32_t)value;
    else if (k == "gso_groups" && value >= 1 && value <= 64)
        t.gso_groups = (uint32_t)value;
    else if (k == "gso_waves" && (value == 1 || value == 2 || value == 4 || value == 8))
        t.gso_waves = (uint32_t)value;
    else if (k == "gso_split" && value >= 1 && value <= 64)
        t.gso_split = (uint32_t)value;
    else if (k == "gso_spw" && value <= 2)
        t.gso_spw = (uint32_t)value;
    else if (k == "gso_ablate" && (value <= 2 || value == 32))
        t.gso_ablate = (uint32_t)value;
    else
        return WG_ERR_INVALID;
    return WG_OK;
}

extern "C" int wg_tune_get(const char *key, uint64_t *value) {
    if (!key || !value)
        return WG_ERR_INVALID;
    const Tune &t = tune();
    const std::string k(key);
    if (k == "l4_blocks") *value = t.l4_blocks;
    else if (k == "l4_ppw") *value = t.l4_ppw;
    else if (k == "l4_nt") *value = t.l4_nt;
    else if (k == "l4_descv") *value = t.l4_descv;
    else if (k == "l4_occ") *value = t.l4_occ;
    else if (k == "l4_iters") *value = t.l4_iters;
    else if (k == "gso_blocks") *value = t.gso_blocks;
    else if (k == "gso_waves") *value = t.gso_waves;
    else if (k == "gso_split") *value = t.gso_split;
    else if (k == "gso_spw") *value = t.gso_spw;
    else if (k == "gso_groups") *value = t.gso_groups;
    else if (k == "verify_occ") *value = t.verify_occ;
    else if (k == "verify_dm") *value = t.verify_dm;
    else if (k == "gro_lds") *value = t.gro_lds;
    else if (k == "gro_wide") *value = t.gro_wide;
    else if (k == "gso_ablate") *value = t.gso_ablate;
    else return WG_ERR_INVALID;
    return WG_OK;
}

extern "C" int wg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

extern "C" int wg_l4csum_uniform_host(const uint8_t *host_base, uint64_t total_len, uint32_t segment_size,
                                      uint16_t csum_start, uint32_t flags, uint16_t *host_out) {
    if (!segment_size || (total_len && (!host_base || !host_out)))
        return WG_ERR_INVALID;
    if (!total_len)
        return WG_OK;
    if (wg_device_count() <= 0)
        return WG_ERR_NODEV;
    const uint64_t n = (total_len + segment_size - 1) / segment_size;
    int rc = host_ctx_reserve((size_t)total_len, (size_t)n);
    if (rc != WG_OK)
        return rc;
    HostCtx &c = g_host;
    if (hipMemcpyAsync(c.dbuf, host_base, total_len, hipMemcpyHostToDevice, c.stream) != hipSuccess)
        return WG_ERR_RUNTIME;
    rc = wg_l4csum_uniform(c.dbuf, total_len, segment_size, csum_start, flags, c.dout, c.stream);
    if (rc != WG_OK)
        return rc;
    if (hipMemcpyAsync(host_out, c.dout, n * sizeof(uint16_t), hipMemcpyDeviceToHost, c.stream) != hipSuccess)
        return WG_ERR_RUNTIME;
    return hipStreamSynchronize(c.stream) == hipSuccess ? WG_OK : WG_ERR_RUNTIME;
}
