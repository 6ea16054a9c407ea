// Per-call latency of the drop-in wireglider::calc_l4_checksum (checksum.cpp:8,
// called once per segment by worker/offload.cpp:202 and per packet by
// include/worker/evaluator.hpp:64,93).  Linked against libwireglider_amd.so;
// the placement comes from the environment (WG_PERCALL unset: host, =gpu:
// host-memory GPU path).
//
// usage: percall_latency [reps] [threads ...]
// With no thread counts: one thread, the single-threaded object below.  With
// thread counts (e.g. `1 16`): for each count T, T threads — one per tun
// queue worker, as wireglider.cpp:117-151 runs them — each call the function
// `reps` times per size on their own packet copy, started together; the
// object per T holds the mean ns per call over the threads.
// Prints one JSON object: ns per call for packet sizes 64 / 1500 / 9000 B, one
// result per size, and the XOR of all results (keeps the timed calls live).
#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "wireglider/checksum.hpp"

namespace {

const size_t kSizes[] = {64, 1500, 9000};

std::vector<uint8_t> make_packet() {
    std::vector<uint8_t> pkt(9000);
    uint64_t x = 0x5EED;
    for (auto &b : pkt) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        b = static_cast<uint8_t>(x >> 56);
    }
    pkt[0] = 0x45;
    return pkt;
}

// One thread's timed loops: ns per call for each size.
void run_sizes(int reps, const std::vector<uint8_t> &pkt, double ns[3], unsigned res[3], unsigned &acc_out,
               std::atomic<int> *gate, int nthreads) {
    unsigned acc = 0;  // thread-private: the threads' acc_out slots share a cache line
    for (size_t k = 0; k < 3; k++) {
        const std::span<const uint8_t> p(pkt.data(), kSizes[k]);
        res[k] = wireglider::calc_l4_checksum(p, false, false, 20);
        for (int i = 0; i < reps / 10; i++)  // warm up (first GPU call creates the stream / workspace)
            acc ^= wireglider::calc_l4_checksum(p, false, false, 20);
        if (gate) {  // every thread starts each size's timed loop together
            gate->fetch_add(1);
            while (gate->load() < nthreads * (int)(k + 1)) std::this_thread::yield();
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; i++)
            acc ^= wireglider::calc_l4_checksum(p, false, false, 20);
        const auto t1 = std::chrono::steady_clock::now();
        ns[k] = std::chrono::duration<double, std::nano>(t1 - t0).count() / reps;
    }
    acc_out ^= acc;
}

}  // namespace

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20000;
    const std::vector<uint8_t> pkt = make_packet();
    if (argc <= 2) {
        double ns[3];
        unsigned res[3] = {0, 0, 0}, acc = 0;
        run_sizes(reps, pkt, ns, res, acc, nullptr, 1);
        std::printf("{\"ns_per_call_64B\": %.1f, \"ns_per_call_1500B\": %.1f, \"ns_per_call_9000B\": %.1f, "
                    "\"reps\": %d, \"results\": [%u, %u, %u], \"xor\": %u}\n",
                    ns[0], ns[1], ns[2], reps, res[0], res[1], res[2], acc);
        return 0;
    }
    std::string out = "{";
    for (int a = 2; a < argc; a++) {
        const int T = std::atoi(argv[a]);
        if (T < 1)
            return 2;
        std::vector<std::thread> th;
        std::vector<std::array<double, 3>> ns(T);
        std::vector<std::array<unsigned, 3>> res(T);
        std::vector<unsigned> acc(T, 0);
        std::vector<std::vector<uint8_t>> pk(T, pkt);  // own copy per thread, as each worker has its buffers
        std::atomic<int> gate{0};
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] { run_sizes(reps, pk[t], ns[t].data(), res[t].data(), acc[t], &gate, T); });
        for (auto &x : th) x.join();
        double mean[3] = {0, 0, 0}, worst[3] = {0, 0, 0};
        unsigned x = 0;
        bool same = true;
        for (int t = 0; t < T; t++) {
            for (int k = 0; k < 3; k++) {
                mean[k] += ns[t][k] / T;
                worst[k] = ns[t][k] > worst[k] ? ns[t][k] : worst[k];
                same = same && res[t][k] == res[0][k];
            }
            x ^= acc[t];
        }
        char buf[512];
        std::snprintf(buf, sizeof buf,
                      "%s\"threads_%d\": {\"ns_per_call_64B\": %.1f, \"ns_per_call_1500B\": %.1f, "
                      "\"ns_per_call_9000B\": %.1f, \"worst_thread_ns\": [%.1f, %.1f, %.1f], \"reps\": %d, "
                      "\"results\": [%u, %u, %u], \"results_agree\": %s, \"xor\": %u}",
                      a > 2 ? ", " : "", T, mean[0], mean[1], mean[2], worst[0], worst[1], worst[2], reps,
                      res[0][0], res[0][1], res[0][2], same ? "true" : "false", x);
        out += buf;
    }
    uint64_t g = 0, f = 0, h = 0;
    wg_percall_stats(&g, &f, &h);  // summed over every thread's slot, exited threads included
    char tail[160];
    std::snprintf(tail, sizeof tail, ", \"percall_stats\": {\"gpu\": %llu, \"fallback\": %llu, \"host\": %llu}}",
                  (unsigned long long)g, (unsigned long long)f, (unsigned long long)h);
    out += tail;
    std::printf("%s\n", out.c_str());
    return 0;
}
