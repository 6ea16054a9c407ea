// capi.hip — misc C ABI (version, errors, device count), launch tuning, and
// the host-memory path (tun / UDP buffers live in host memory).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>

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

const Tune &tune() {
    static Tune t = [] {
        Tune x;
        // 256 CUs x 8 four-wave blocks = 32 waves/CU resident at <= 64 VGPRs.
        x.l4_blocks = env_u64("WG_L4_BLOCKS", 2048);
        x.gso_blocks = env_u64("WG_GSO_BLOCKS", 2048);
        return x;
    }();
    return t;
}

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

}  // namespace wg

using namespace wg;

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
