// l4csum.hip — batched L4 / plain Internet checksum on MI355X (gfx950).
//
// Replaces, at batch granularity, wireglider::calc_l4_checksum
// (reference checksum.cpp:8-36) and wireglider::checksum
// (include/netio/checksum.hpp:146-149).  One wavefront per packet: the
// 16-byte-aligned interior of the summed region streams through
// global_load_dwordx4 (64 lanes x 16 B = 1 KiB per instruction, coalesced),
// the <=15-byte unaligned head and tail plus the pseudo-header addresses come
// in through ONE byte-gather instruction (one lane per byte), and the
// wave's partial sums meet in a DPP butterfly.  No LDS: every byte is used
// exactly once, so staging it would only add LDS traffic.
#include <hip/hip_runtime.h>

#include "wg_device.hpp"
#include "wg_internal.hpp"
#include "wireglider_amd.h"

namespace wg {

// This lane's share of one packet's one's-complement sum, in TRUE pairing
// (relative to the packet's csum_start / address start).  kL4 adds the
// pseudo-header source/destination address bytes; the constant
// proto/length words are added by the caller once per packet.
template <bool kL4>
__device__ __forceinline__ uint32_t packet_partial(const uint8_t *pkt, uint32_t len, uint32_t cs,
                                                   bool v6, uint32_t lane) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(pkt);
    const uintptr_t r1 = a + len;
    const uintptr_t r0 = cs < len ? a + cs : r1;  // summed region [r0, r1)
    const uintptr_t c0 = (r0 + 15) & ~(uintptr_t)15;
    const uintptr_t c1 = r1 & ~(uintptr_t)15;

    // Interior: whole aligned 16-B chunks, 4 in flight per lane per round.
    uint64_t acc = 0;
    if (c1 > c0) {
        const uint32_t nint = (uint32_t)((c1 - c0) >> 4);
        const uintptr_t q = c0;
        uint32_t k = lane;
        for (; k + 192 < nint; k += 256) {
            v4u v0 = ld16(q + 16ull * k);
            v4u v1 = ld16(q + 16ull * (k + 64));
            v4u v2 = ld16(q + 16ull * (k + 128));
            v4u v3 = ld16(q + 16ull * (k + 192));
            acc += sum4(v0) + sum4(v1) + sum4(v2) + sum4(v3);
        }
        if (k + 64 < nint) {
            v4u v0 = ld16(q + 16ull * k);
            v4u v1 = ld16(q + 16ull * (k + 64));
            acc += sum4(v0) + sum4(v1);
            k += 128;
        }
        if (k < nint)
            acc += sum4(ld16(q + 16ull * k));
    }

    // One byte per lane: lanes 0-31 pseudo-header addresses (true pairing
    // relative to the address start, which is even in the packet), lanes
    // 32-47 the unaligned head [r0, min(c0, r1)), lanes 48-63 the tail
    // [max(c1, c0), r1) (absolute-address pairing, like the interior).
    uintptr_t bp = 0;
    bool true_pair = false;
    if (lane < 32) {
        if (kL4) {
            const uint32_t ao = v6 ? 8u : 12u, al = v6 ? 32u : 8u;
            if (lane < al && ao + lane < len) {
                bp = a + ao + lane;
                true_pair = true;
            }
        }
    } else if (lane < 48) {
        const uintptr_t he = c0 < r1 ? c0 : r1;
        const uintptr_t x = r0 + (lane - 32);
        if (x < he)
            bp = x;
    } else {
        const uintptr_t ts = c1 > c0 ? c1 : c0;
        const uintptr_t x = ts + (lane - 48);
        if (x < r1)
            bp = x;
    }
    uint32_t bv = 0;
    if (bp) {
        const uint32_t par = true_pair ? (lane & 1u) : (uint32_t)(bp & 1u);
        bv = ld8(bp) << (8u * par);
    }
    if (!true_pair)
        acc += bv;

    uint32_t f = fold16(acc);
    if (r0 & 1u)  // region pairs from an odd address: swap its folded sum
        f = bswap16(f);
    return f + (true_pair ? bv : 0u);
}

struct L4Params {
    const uint8_t *base;
    const wg_pkt_desc *desc;
    uint16_t *out;
    uint64_t n;
    uint64_t total_len;
    uint32_t seg;
    uint32_t cs;
    uint32_t flags;
};

enum Kind : int { kUniformL4 = 0, kDescL4 = 1, kDescPlain = 2 };

template <int kKind>
__global__ __launch_bounds__(256) void l4csum_wave_kernel(L4Params p) {
    const uint32_t lane = lane_id();
    const uint64_t wave0 = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t nw = (uint64_t)gridDim.x * 4u;
    for (uint64_t i = wave0; i < p.n; i += nw) {
        const uint8_t *pkt;
        uint32_t len, cs, fl;
        if (kKind == kUniformL4) {
            const uint64_t off = i * (uint64_t)p.seg;
            const uint64_t rem = p.total_len - off;
            len = rem < p.seg ? (uint32_t)rem : p.seg;
            pkt = p.base + off;
            cs = p.cs;
            fl = p.flags;
        } else {
            const wg_pkt_desc d = p.desc[i];
            pkt = p.base + d.offset;
            len = d.len;
            cs = kKind == kDescPlain ? 0u : d.csum_start;
            fl = d.flags;
        }
        const uint32_t part = packet_partial<kKind != kDescPlain>(pkt, len, cs, fl & WG_PKT_V6, lane);
        uint32_t s = wave_sum_u32(part);
        if (lane == 0) {
            if (kKind != kDescPlain) {
                // {0x00, proto, l4len>>8, l4len&0xff} as LE words
                // (include/netio/checksum.hpp:111-114, checksum.cpp:23,33).
                const uint32_t proto = (fl & WG_PKT_TCP) ? 6u : 17u;
                s += (proto << 8) + bswap16((len - cs) & 0xffffu);
            }
            p.out[i] = (uint16_t)(~fold16_32(s) & 0xffffu);
        }
    }
}

static int launch_l4(int kind, const L4Params &p, hipStream_t st) {
    if (p.n == 0)
        return WG_OK;
    const uint64_t want = (p.n + 3) / 4;
    uint64_t cap = tune().l4_blocks;
    uint64_t blocks = want < cap ? want : cap;
    if (blocks >= 8)
        blocks &= ~7ull;  // keep the XCD swizzle bijective
    dim3 grid((unsigned)blocks), block(256);
    switch (kind) {
    case kUniformL4:
        hipLaunchKernelGGL(l4csum_wave_kernel<kUniformL4>, grid, block, 0, st, p);
        break;
    case kDescL4:
        hipLaunchKernelGGL(l4csum_wave_kernel<kDescL4>, grid, block, 0, st, p);
        break;
    default:
        hipLaunchKernelGGL(l4csum_wave_kernel<kDescPlain>, grid, block, 0, st, p);
        break;
    }
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

}  // namespace wg

using namespace wg;

extern "C" int wg_l4csum_uniform(const uint8_t *dev_base, uint64_t total_len, uint32_t segment_size,
                                 uint16_t csum_start, uint32_t flags, uint16_t *dev_out,
                                 void *stream) {
    if (!segment_size || (total_len && (!dev_base || !dev_out)))
        return WG_ERR_INVALID;
    L4Params p{};
    p.base = dev_base;
    p.out = dev_out;
    p.n = (total_len + segment_size - 1) / segment_size;  // nr_segments(), offload.hpp:26-28
    p.total_len = total_len;
    p.seg = segment_size;
    p.cs = csum_start;
    p.flags = flags;
    return launch_l4(kUniformL4, p, static_cast<hipStream_t>(stream));
}

extern "C" int wg_l4csum_desc(const uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n,
                              uint16_t *dev_out, void *stream) {
    if (n && (!dev_base || !dev_desc || !dev_out || (reinterpret_cast<uintptr_t>(dev_desc) & 15)))
        return WG_ERR_INVALID;
    L4Params p{};
    p.base = dev_base;
    p.desc = dev_desc;
    p.out = dev_out;
    p.n = n;
    return launch_l4(kDescL4, p, static_cast<hipStream_t>(stream));
}

extern "C" int wg_checksum_desc(const uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n,
                                uint16_t *dev_out, void *stream) {
    if (n && (!dev_base || !dev_desc || !dev_out || (reinterpret_cast<uintptr_t>(dev_desc) & 15)))
        return WG_ERR_INVALID;
    L4Params p{};
    p.base = dev_base;
    p.desc = dev_desc;
    p.out = dev_out;
    p.n = n;
    return launch_l4(kDescPlain, p, static_cast<hipStream_t>(stream));
}
