// checksum.cpp — drop-in for the reference's checksum.cpp (dinhngtu/wireglider
// @ 2024-11-01, checksum.cpp:8-36): the one out-of-line symbol
//   uint16_t wireglider::calc_l4_checksum(std::span<const uint8_t>, bool, bool, uint16_t)
// with the same C++ mangled name, so objects compiled against the reference
// header (or wireglider/checksum.hpp) link against libwireglider_amd.so.
//
// Placement (SURVEY §7 "Hard parts", §8b): the reference's callers use the
// result of each call immediately, one packet at a time
// (worker/offload.cpp:202-204), so the call is answered on the calling CPU by
// the header's host::calc_l4_checksum.  WG_PERCALL=gpu routes every call
// through the host-memory GPU path (one H2D / kernel / D2H round trip); a
// failure there (no device, runtime error) falls back to the host answer,
// which is the same checksum by construction (tests/test_dropin_host.py).
// wg_percall_stats counts which placement answered, so a test can tell a GPU
// answer from a fallback although both give the same checksum.
#include <atomic>
#include <cstdlib>
#include <cstring>

#include "wireglider/checksum.hpp"

namespace wireglider {

namespace {

// Who answered each call (wg_percall_stats): the GPU round trip, the host
// after a failed GPU round trip, or the host by placement.
std::atomic<uint64_t> g_gpu{0}, g_fallback{0}, g_host{0};

bool percall_gpu() {
    static const bool on = [] {
        const char *v = std::getenv("WG_PERCALL");
        return v && std::strcmp(v, "gpu") == 0;
    }();
    return on;
}

}  // namespace

uint16_t calc_l4_checksum(std::span<const uint8_t> ippkt, bool isv6, bool istcp, uint16_t csum_start) {
    if (percall_gpu() && !ippkt.empty()) {
        uint16_t out = 0;
        const int rc = wg_l4csum_uniform_host(ippkt.data(), ippkt.size(), static_cast<uint32_t>(ippkt.size()),
                                              csum_start, (isv6 ? WG_PKT_V6 : 0u) | (istcp ? WG_PKT_TCP : 0u), &out);
        if (rc == WG_OK) {
            g_gpu.fetch_add(1, std::memory_order_relaxed);
            return out;
        }
        g_fallback.fetch_add(1, std::memory_order_relaxed);
    } else {
        g_host.fetch_add(1, std::memory_order_relaxed);
    }
    return host::calc_l4_checksum(ippkt, isv6, istcp, csum_start);
}

}  // namespace wireglider

extern "C" int wg_percall_stats(uint64_t *gpu_answered, uint64_t *host_fallback, uint64_t *host_answered) {
    if (gpu_answered) *gpu_answered = wireglider::g_gpu.load();
    if (host_fallback) *host_fallback = wireglider::g_fallback.load();
    if (host_answered) *host_answered = wireglider::g_host.load();
    return WG_OK;
}
