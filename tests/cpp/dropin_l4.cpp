// Drop-in check: a caller compiled against wireglider/checksum.hpp exactly
// like the reference's callers (worker/offload.cpp:202,
// include/worker/evaluator.hpp:64,93), linked against libwireglider_amd.so
// through the reference's C++ symbol wireglider::calc_l4_checksum.
//
// stdin: records {u32 len, u8 isv6, u8 istcp, u16 csum_start, len bytes}
// stdout: one hex result per record; stderr: the library's per-call
// placement counters (wg_percall_stats) at the end.
#include <cstdint>
#include <cstdio>
#include <vector>

#include "wireglider/checksum.hpp"

int main() {
    for (;;) {
        uint32_t len;
        uint8_t v6, tcp;
        uint16_t cs;
        if (fread(&len, 4, 1, stdin) != 1)
            break;
        if (fread(&v6, 1, 1, stdin) != 1 || fread(&tcp, 1, 1, stdin) != 1 || fread(&cs, 2, 1, stdin) != 1)
            return 2;
        std::vector<uint8_t> pkt(len);
        if (len && fread(pkt.data(), 1, len, stdin) != len)
            return 2;
        uint16_t r = wireglider::calc_l4_checksum(std::span<const uint8_t>(pkt), v6 != 0, tcp != 0, cs);
        printf("%04x\n", r);
    }
    uint64_t gpu = 0, fallback = 0, host = 0;
    wg_percall_stats(&gpu, &fallback, &host);
    fprintf(stderr, "percall gpu=%llu fallback=%llu host=%llu\n", (unsigned long long)gpu,
            (unsigned long long)fallback, (unsigned long long)host);
    return 0;
}
