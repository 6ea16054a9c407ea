// gro.hip — batched GRO finalize on MI355X (gfx950).
//
// Per coalesced flow: PacketRefBatch::finalize (reference
// include/worker/flowkey_ref.hpp:82-117; OwnedPacketBatch::finalize,
// include/worker/flowkey_own.hpp:83-115) on the flow's header buffer, in
// place: UDP length / IPv6 payload length / IPv4 total length, IPv4 header
// checksum, and the VIRTIO_NET_HDR_F_NEEDS_CSUM seed = pseudo_header_checksum
// (complemented fold, as the reference stores it) over the header's
// source/destination addresses.  The reference's own call binds the TAddress
// overload and sums the std::span objects (pointer + size) instead —
// pointer-dependent, not reproduced.
//
// Header-only work (<= a few hundred bytes per flow): one thread per flow.
#include <hip/hip_runtime.h>

#include "wg_device.hpp"
#include "wireglider_amd.h"

namespace wg {

__device__ __forceinline__ void stb(uint8_t *p, uint32_t v) { *p = (uint8_t)v; }
__device__ __forceinline__ void st_be16(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

__global__ __launch_bounds__(256) void gro_finalize_kernel(uint8_t *hdrs, wg_gro_desc *desc, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        wg_gro_desc d = desc[i];
        uint8_t *h = hdrs + d.hdr_offset;
        const uint32_t H = d.hdr_len, cs = d.csum_start, l4off = (uint32_t)d.csum_start + d.csum_offset;
        const bool v6 = d.flags & WG_PKT_V6, tcp = d.flags & WG_PKT_TCP;
        const uint32_t iph = v6 ? 40u : 20u;
        if (cs < iph || cs > H || l4off < cs || l4off + 2 > H || (!tcp && cs + 8 > H)) {
            desc[i].status = -3;
            continue;
        }
        const uint64_t l4len = (uint64_t)(H - cs) + d.payload_bytes;  // :84
        if (!tcp)
            st_be16(h + cs + 4, (uint32_t)l4len);  // udp->len (uint16), :85-86
        uint32_t proto, ao, al;
        if (v6) {
            proto = h[6];
            ao = 8;
            al = 32;
            st_be16(h + 4, (uint32_t)l4len);  // ip6_plen, :95
        } else {
            proto = h[9];
            ao = 12;
            al = 8;
            st_be16(h + 2, (uint32_t)((uint64_t)H + d.payload_bytes));  // ip_len, :103
            uint32_t s = 0;  // checksum(hdrbuf[0:cs]) with ip_sum = 0, :104-106
            for (uint32_t j = 0; j < cs; j++)
                s += (j == 10 || j == 11) ? 0u : (uint32_t)h[j] << (8u * (j & 1u));
            const uint32_t c = ~fold16_32(s) & 0xffffu;
            stb(h + 10, c & 0xffu);  // native order
            stb(h + 11, c >> 8);
        }
        uint32_t ps = 0;  // pseudo-header: addresses + {0, proto} + l4len (uint16), :108-112
        for (uint32_t j = 0; j < al; j++)
            ps += (uint32_t)h[ao + j] << (8u * (j & 1u));
        ps += (proto << 8) + bswap16((uint32_t)l4len & 0xffffu);
        const uint32_t seed = ~fold16_32(ps) & 0xffffu;
        stb(h + l4off, seed & 0xffu);  // native order, :114
        stb(h + l4off + 1, seed >> 8);
        desc[i].status = 0;
    }
}

}  // namespace wg

using namespace wg;

extern "C" int wg_gro_finalize(uint8_t *dev_hdrs, wg_gro_desc *dev_desc, uint64_t n, void *stream) {
    if (!n)
        return WG_OK;
    if (!dev_hdrs || !dev_desc || (reinterpret_cast<uintptr_t>(dev_desc) & 7))
        return WG_ERR_INVALID;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 8192)
        blocks = 8192;
    hipLaunchKernelGGL(gro_finalize_kernel, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       dev_hdrs, dev_desc, n);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}
