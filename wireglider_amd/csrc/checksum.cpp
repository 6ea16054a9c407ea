// checksum.cpp — drop-in for the reference's checksum.cpp (dinhngtu/wireglider
// @ 2024-11-01, checksum.cpp:8-36): the one out-of-line symbol
//   uint16_t wireglider::calc_l4_checksum(std::span<const uint8_t>, bool, bool, uint16_t)
// with the same C++ mangled name, so objects compiled against the reference
// header (or wireglider/checksum.hpp) link against libwireglider_amd.so.
//
// The packet is a one-segment PacketBatch sent through the C ABI's
// host-memory path (H2D, gfx950 kernel, D2H).  This is correct but
// latency-bound (one round trip per call); batch callers use
// wireglider::gpu::calc_l4_checksum_batch instead.
#include <cstdio>
#include <cstdlib>

#include "wireglider/checksum.hpp"

namespace wireglider {

uint16_t calc_l4_checksum(std::span<const uint8_t> ippkt, bool isv6, bool istcp, uint16_t csum_start) {
    uint16_t out = 0;
    if (ippkt.empty()) {
        // Zero-length segment: nothing to transfer; same closed form as the
        // kernel (pseudo-header only, l4Len = (uint16_t)(0 - csum_start)).
        const std::array<uint8_t, 16> zero{};
        const uint16_t l4len = static_cast<uint16_t>(0u - csum_start);
        const size_t alen = isv6 ? 16 : 4;
        const std::span<const uint8_t> a(zero.data(), alen);
        return checksum_impl::fold_complement(
            checksum_impl::pseudo_header_checksum_nofold(istcp ? 6 : 17, a, a, l4len));
    }
    const int rc = wg_l4csum_uniform_host(ippkt.data(), ippkt.size(), static_cast<uint32_t>(ippkt.size()),
                                          csum_start, (isv6 ? WG_PKT_V6 : 0u) | (istcp ? WG_PKT_TCP : 0u), &out);
    if (rc != WG_OK) {
        std::fprintf(stderr, "wireglider_amd: calc_l4_checksum failed: %s\n", wg_strerror(rc));
        std::abort();
    }
    return out;
}

}  // namespace wireglider
