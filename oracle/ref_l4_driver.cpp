// oracle/ref_l4_driver.cpp — TEST INFRASTRUCTURE ONLY.
//
// Drives the reference's OWN calc_l4_checksum (/root/reference/checksum.cpp:8-36,
// compiled UNCHANGED by oracle/Makefile `ref-l4` with this repository's drop-in
// header, include/wireglider/checksum.hpp, found as "checksum.hpp") over a
// fixture batch, and writes the results: the golden vectors of SURVEY §8(c)
// item (2) (tests/golden/gen_l4_golden.py).  This file only declares the
// function (through the same header) and calls it; the definition linked in is
// the reference's object file, oracle/_ref/ref_checksum.o.
//
// usage: ref_l4 <packets.bin> <desc.bin> <out.u16>
//   desc.bin: wg_pkt_desc records {u64 offset, u32 len, u16 csum_start, u8 flags, u8 reserved}
#include <cstdint>
#include <cstring>
#include <span>
#include <cstdio>
#include <vector>

#include "checksum.hpp"

static std::vector<uint8_t> slurp(const char *path) {
    std::vector<uint8_t> v;
    FILE *f = std::fopen(path, "rb");
    if (!f)
        return v;
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0)
        v.insert(v.end(), buf, buf + k);
    std::fclose(f);
    return v;
}

int main(int argc, char **argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s packets.bin desc.bin out.u16\n", argv[0]);
        return 2;
    }
    const std::vector<uint8_t> pk = slurp(argv[1]);
    const std::vector<uint8_t> dr = slurp(argv[2]);
    if (dr.size() % sizeof(wg_pkt_desc)) {
        std::fprintf(stderr, "desc.bin: %zu bytes is not a whole number of 16-B records\n", dr.size());
        return 2;
    }
    const size_t n = dr.size() / sizeof(wg_pkt_desc);
    std::vector<uint16_t> out(n);
    for (size_t i = 0; i < n; i++) {
        wg_pkt_desc d;
        std::memcpy(&d, dr.data() + i * sizeof d, sizeof d);
        const size_t amin = (d.flags & WG_PKT_V6) ? 40 : 20;
        // the reference's contract (checksum.cpp:17-18,27-28,35): the
        // addresses inside the packet, csum_start <= size
        if (d.offset + d.len > pk.size() || d.len < amin || d.csum_start > d.len) {
            std::fprintf(stderr, "record %zu is outside the reference's contract\n", i);
            return 3;
        }
        out[i] = wireglider::calc_l4_checksum(std::span<const uint8_t>(pk.data() + d.offset, d.len),
                                              (d.flags & WG_PKT_V6) != 0, (d.flags & WG_PKT_TCP) != 0, d.csum_start);
    }
    FILE *f = std::fopen(argv[3], "wb");
    if (!f || std::fwrite(out.data(), 2, n, f) != n)
        return 4;
    std::fclose(f);
    return 0;
}
