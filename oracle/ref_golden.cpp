// ref_golden.cpp — golden-vector driver around the reference's OWN test oracle.
//
// TEST INFRASTRUCTURE ONLY.  Compiled by oracle/Makefile against the
// reference header where it lies (-I $(REF)/tests), output to oracle/_ref/.
// It includes tests/checksum_tests.hpp (checksum_ref1 :11-34, create_packet
// :36-42, create_packet_carry :44-48) unchanged; this file only drives it and
// writes the results as raw little-endian binary fixtures:
//
//   <outdir>/create_packet_65536.bin   create_packet(65536) bytes
//   <outdir>/ref1_random_1_1500.u16    checksum_ref1(create_packet(n)), n=1..1500
//   <outdir>/ref1_carry_1_63.u16       checksum_ref1(create_packet_carry(n)), n=1..63
//   <outdir>/ref1_random_65536.u16     checksum_ref1(create_packet(65536))
//
// These are the inputs/expected outputs of tests/test-checksum.cpp:11-25.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "checksum_tests.hpp"

static void write_file(const std::string &path, const void *data, size_t n) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f || std::fwrite(data, 1, n, f) != n) {
        std::fprintf(stderr, "write failed: %s\n", path.c_str());
        std::exit(1);
    }
    std::fclose(f);
}

int main(int argc, char **argv) {
    if (argc != 2) {
        std::fprintf(stderr, "usage: %s <outdir>\n", argv[0]);
        return 2;
    }
    std::string out = argv[1];

    auto big = create_packet(65536);
    write_file(out + "/create_packet_65536.bin", big.data(), big.size());

    std::vector<uint16_t> r;
    for (size_t n = 1; n <= 1500; n++) {
        auto p = create_packet(n);
        r.push_back(checksum_ref1(p.data(), p.size()));
    }
    write_file(out + "/ref1_random_1_1500.u16", r.data(), r.size() * 2);

    r.clear();
    for (size_t n = 1; n <= 63; n++) {
        auto p = create_packet_carry(n);
        r.push_back(checksum_ref1(p.data(), p.size()));
    }
    write_file(out + "/ref1_carry_1_63.u16", r.data(), r.size() * 2);

    uint16_t c = checksum_ref1(big.data(), big.size());
    write_file(out + "/ref1_random_65536.u16", &c, 2);
    std::printf("ok\n");
    return 0;
}
