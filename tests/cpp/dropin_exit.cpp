// dropin_exit.cpp — TEST HARNESS: wireglider::calc_l4_checksum called from a
// thread_local destructor that runs after the library's per-thread slot owner
// is gone (such a call re-registered through the destroyed owner
// and its count was lost).  Each worker thread: construct a thread_local
// object FIRST (destroyed last), make K calls (the library's owner is then
// constructed, destroyed before ours), and at thread exit our destructor makes
// E more calls.  Prints the library's placement counts; every call must be
// counted once: threads * (K + E) host answers.
#include <cstdio>
#include <cstdlib>
#include <span>
#include <thread>
#include <vector>

#include "wireglider/checksum.hpp"
#include "wireglider_amd.h"

namespace {
int g_exit_calls = 0;
unsigned g_sink = 0;

struct AtExit {
    bool armed = false;
    ~AtExit() {
        if (!armed)
            return;
        std::vector<uint8_t> p(60, 0x5a);
        for (int i = 0; i < g_exit_calls; i++)
            g_sink += wireglider::calc_l4_checksum(std::span<const uint8_t>(p), false, true, 20);
    }
};
thread_local AtExit t_exit;
}  // namespace

int main(int argc, char **argv) {
    const int threads = argc > 1 ? std::atoi(argv[1]) : 4;
    const int k = argc > 2 ? std::atoi(argv[2]) : 100;
    g_exit_calls = argc > 3 ? std::atoi(argv[3]) : 7;
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
        th.emplace_back([k] {
            t_exit.armed = true;  // constructed before the library's slot owner
            std::vector<uint8_t> p(1500, 0x33);
            for (int i = 0; i < k; i++)
                g_sink += wireglider::calc_l4_checksum(std::span<const uint8_t>(p), false, false, 20);
        });
    for (auto &x : th) x.join();
    uint64_t g = 0, f = 0, h = 0;
    wg_percall_stats(&g, &f, &h);
    std::printf("{\"threads\": %d, \"calls\": %d, \"exit_calls\": %d, \"gpu\": %llu, \"fallback\": %llu, \"host\": %llu}\n",
                threads, k, g_exit_calls, (unsigned long long)g, (unsigned long long)f, (unsigned long long)h);
    return g_sink == 0xffffffffu;  // keep the results live
}
