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
//
// The counts are per thread: the reference calls this from one worker thread
// per tun queue (wireglider.cpp:117-151), and a process-wide atomic would
// move one cache line between those cores on every call.  Each thread owns a
// cache-line-sized slot (written only by that thread, plain relaxed stores);
// wg_percall_stats sums the live slots plus what exited threads left behind.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "wireglider/checksum.hpp"

namespace wireglider {

namespace {

struct alignas(64) Slot {
    // who answered: the GPU round trip, the host after a failed GPU round
    // trip, the host by placement
    std::atomic<uint64_t> gpu{0}, fallback{0}, host{0};
};

struct Registry {
    std::mutex mu;
    std::vector<Slot *> live;
    uint64_t gone[3] = {0, 0, 0};  // exited threads' counts
};

Registry &registry() {
    static Registry *r = new Registry;  // never destroyed: threads may exit after static destruction
    return *r;
}

// The calling thread's slot: a trivially initialised thread-local pointer
// (initial-exec TLS: one load, no guard, no __tls_get_addr call per call),
// set on the thread's first call by registering a slot whose owner folds it
// into `gone` when the thread exits.
struct SlotOwner;
__attribute__((tls_model("initial-exec"))) thread_local Slot *t_slot = nullptr;

struct SlotOwner {
    Slot slot;
    SlotOwner() {
        Registry &r = registry();
        std::lock_guard<std::mutex> g(r.mu);
        r.live.push_back(&slot);
    }
    ~SlotOwner() {
        t_slot = nullptr;
        Registry &r = registry();
        std::lock_guard<std::mutex> g(r.mu);
        r.gone[0] += slot.gpu.load(std::memory_order_relaxed);
        r.gone[1] += slot.fallback.load(std::memory_order_relaxed);
        r.gone[2] += slot.host.load(std::memory_order_relaxed);
        for (auto it = r.live.begin(); it != r.live.end(); ++it)
            if (*it == &slot) {
                r.live.erase(it);
                break;
            }
    }
};

__attribute__((noinline)) Slot *register_slot() {
    thread_local SlotOwner owner;
    t_slot = &owner.slot;
    return t_slot;
}

inline Slot &my_slot() {
    Slot *s = t_slot;
    if (__builtin_expect(s == nullptr, 0))
        s = register_slot();
    return *s;
}

// Owner-only increment: a load and a store, no locked read-modify-write.
inline void bump(std::atomic<uint64_t> &c) {
    c.store(c.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
}

bool percall_gpu() {
    static const bool on = [] {
        const char *v = std::getenv("WG_PERCALL");
        return v && std::strcmp(v, "gpu") == 0;
    }();
    return on;
}

}  // namespace

uint16_t calc_l4_checksum(std::span<const uint8_t> ippkt, bool isv6, bool istcp, uint16_t csum_start) {
    Slot &s = my_slot();
    if (percall_gpu() && !ippkt.empty()) {
        uint16_t out = 0;
        const int rc = wg_l4csum_uniform_host(ippkt.data(), ippkt.size(), static_cast<uint32_t>(ippkt.size()),
                                              csum_start, (isv6 ? WG_PKT_V6 : 0u) | (istcp ? WG_PKT_TCP : 0u), &out);
        if (rc == WG_OK) {
            bump(s.gpu);
            return out;
        }
        bump(s.fallback);
    } else {
        bump(s.host);
    }
    return host::calc_l4_checksum(ippkt, isv6, istcp, csum_start);
}

}  // namespace wireglider

extern "C" int wg_percall_stats(uint64_t *gpu_answered, uint64_t *host_fallback, uint64_t *host_answered) {
    using namespace wireglider;
    Registry &r = registry();
    uint64_t t[3];
    {
        std::lock_guard<std::mutex> g(r.mu);
        t[0] = r.gone[0];
        t[1] = r.gone[1];
        t[2] = r.gone[2];
        for (const Slot *s : r.live) {
            t[0] += s->gpu.load(std::memory_order_relaxed);
            t[1] += s->fallback.load(std::memory_order_relaxed);
            t[2] += s->host.load(std::memory_order_relaxed);
        }
    }
    if (gpu_answered) *gpu_answered = t[0];
    if (host_fallback) *host_fallback = t[1];
    if (host_answered) *host_answered = t[2];
    return WG_OK;
}
