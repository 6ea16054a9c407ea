// Per-call latency of the drop-in wireglider::calc_l4_checksum (checksum.cpp:8,
// called once per segment by worker/offload.cpp:202 and per packet by
// include/worker/evaluator.hpp:64,93).  Linked against libwireglider_amd.so;
// the placement comes from the environment (WG_PERCALL unset: host, =gpu:
// host-memory GPU path).  Prints one JSON object: ns per call for packet
// sizes 64 / 1500 / 9000 B, one result per size, and the XOR of all
// results (keeps the timed calls live).
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "wireglider/checksum.hpp"

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20000;
    std::vector<uint8_t> pkt(9000);
    uint64_t x = 0x5EED;
    for (auto &b : pkt) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        b = static_cast<uint8_t>(x >> 56);
    }
    pkt[0] = 0x45;
    unsigned acc = 0;
    unsigned res[3] = {0, 0, 0};
    std::printf("{");
    const size_t sizes[] = {64, 1500, 9000};
    for (size_t k = 0; k < 3; k++) {
        const std::span<const uint8_t> p(pkt.data(), sizes[k]);
        res[k] = wireglider::calc_l4_checksum(p, false, false, 20);
        for (int i = 0; i < reps / 10; i++)  // warm up (first GPU call creates the stream / workspace)
            acc ^= wireglider::calc_l4_checksum(p, false, false, 20);
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; i++)
            acc ^= wireglider::calc_l4_checksum(p, false, false, 20);
        const auto t1 = std::chrono::steady_clock::now();
        const double ns = std::chrono::duration<double, std::nano>(t1 - t0).count() / reps;
        std::printf("%s\"ns_per_call_%zuB\": %.1f", k ? ", " : "", sizes[k], ns);
    }
    std::printf(", \"reps\": %d, \"results\": [%u, %u, %u], \"xor\": %u}\n", reps, res[0], res[1], res[2], acc);
    return 0;
}
