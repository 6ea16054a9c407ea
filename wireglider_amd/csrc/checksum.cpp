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

// The calling thread's slot: a trivially initialised thread-local pointer,
// set on the thread's first call by registering a slot whose owner folds it
// into `gone` when the thread exits.  Default TLS model (the
// initial-exec model draws on glibc's static-TLS surplus, which a library
// loaded by dlopen — ctypes after torch — can find used up); the compiler
// makes these local-dynamic accesses.
struct SlotOwner;
thread_local Slot *t_slot = nullptr;
// Set by ~SlotOwner: a call made later in the thread's exit (from another
// thread_local's destructor) must not re-register through the destroyed
// owner; it is counted straight into `gone` instead.  Trivially destructible,
// so it stays readable through every TLS destructor.
thread_local bool t_exited = false;

struct SlotOwner {
    Slot slot;
    SlotOwner() {
        Registry &r = registry();
        std::lock_guard<std::mutex> g(r.mu);
        r.live.push_back(&slot);
    }
    ~SlotOwner() {
        t_slot = nullptr;
        t_exited = true;
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
    if (t_exited)
        return nullptr;  // the thread's owner is gone: the caller counts into `gone`
    thread_local SlotOwner owner;
    t_slot = &owner.slot;
    return t_slot;
}

enum Placement { kGpu = 0, kFallback = 1, kHost = 2 };

__attribute__((noinline)) void count_exited(Placement which) {
    Registry &r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    r.gone[which]++;
}

// Owner-only increment: a load and a store, no locked read-modify-write.
inline void bump(std::atomic<uint64_t> &c) {
    c.store(c.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
}

inline void count(Placement which) {
    Slot *s = t_slot;
    if (__builtin_expect(s == nullptr, 0)) {
        s = register_slot();
        if (!s) {
            count_exited(which);
            return;
        }
    }
    bump(which == kGpu ? s->gpu : which == kFallback ? s->fallback : s->host);
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
    if (percall_gpu() && !ippkt.empty()) {
        uint16_t out = 0;
        const int rc = wg_l4csum_uniform_host(ippkt.data(), ippkt.size(), static_cast<uint32_t>(ippkt.size()),
                                              csum_start, (isv6 ? WG_PKT_V6 : 0u) | (istcp ? WG_PKT_TCP : 0u), &out);
        if (rc == WG_OK) {
            count(kGpu);
            return out;
        }
        count(kFallback);
    } else {
        count(kHost);
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
