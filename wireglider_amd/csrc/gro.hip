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
// Header-only work (tens of bytes per flow): one thread per flow, header
// chunks staged cooperatively through LDS.
#include <hip/hip_runtime.h>

#include "wg_device.hpp"
#include "wg_internal.hpp"
#include "wireglider_amd.h"

namespace wg {

__device__ __forceinline__ void stb(uint8_t *p, uint32_t v) { *p = (uint8_t)v; }
__device__ __forceinline__ void st_be16(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

// Fast path: the bytes finalize reads (v4: [0, csum_start); v6: [0, 40)) lie
// within 64 bytes of the header start.  They are fetched as (at most) five
// aligned 16-byte chunks — an aligned chunk holding a valid byte never
// crosses a page, and chunks past the last needed byte are clamped onto it —
// then funnel-shifted (v_alignbyte) into 16 header-relative dwords R[0..15],
// so every field sits at a static byte position.  The IPv4 length and
// checksum bytes are excluded from the header sum and the new length added,
// so nothing is read after it is written.
constexpr uint32_t kFastNeed = 64;

__device__ __forceinline__ uint32_t keep_below(uint32_t w, int m, uint32_t lim) {
    // bytes of header-relative dword m at positions < lim
    const int k = (int)lim - 4 * m;
    return k >= 4 ? w : (k <= 0 ? 0u : (w & ((1u << (8 * k)) - 1u)));
}

__device__ __forceinline__ uint32_t sum16x2(uint32_t w) { return (w & 0xffffu) + (w >> 16); }

__device__ __forceinline__ void st16_ne(uint8_t *p, uint32_t v) {  // native-order 16-bit store
    if (!((uintptr_t)p & 1u)) {
        *reinterpret_cast<uint16_t *>(p) = (uint16_t)v;
    } else {
        p[0] = (uint8_t)v;
        p[1] = (uint8_t)(v >> 8);
    }
}

// The finalize arithmetic on the header's aligned 16-B chunks W[0..19]
// (chunk c = the aligned chunk at (h & ~15) + 16c, clamped onto the last one
// holding a needed byte).
// Stores by aligned-type pointers: the compiler emits one dword / dwordx4
// store, and gfx950 global memory accepts the unaligned address.
__device__ __forceinline__ void st32_u(uint8_t *p, uint32_t v) {
    *reinterpret_cast<__attribute__((address_space(1))) uint32_t *>(reinterpret_cast<uintptr_t>(p)) = v;
}
__device__ __forceinline__ void st128_u(uint8_t *p, v4u v) {
    *reinterpret_cast<__attribute__((address_space(1))) v4u *>(reinterpret_cast<uintptr_t>(p)) = v;
}

// The fields go out in two wide stores instead of four or five narrow ones
// (stores at a 64-B lane stride are address-processing bound, so
// instructions, not bytes, are the cost; narrow stores of the changed 2-B
// fields only measured the same, profiles/r02_store_granularity.json): IPv4
// header bytes [0, 16) (ip_len and ip_sum with the 12 unchanged bytes around
// them) or the IPv6 payload length as one dword, and for UDP the length and
// the seed as one dword (csum_offset 6, adjacent fields).  Every byte written
// lies in the flow's own header and the unchanged ones get their own values
// back.
__device__ __forceinline__ void gro_fields(uint8_t *h, const wg_gro_desc &d, bool v6, bool tcp, uint64_t l4len,
                                           v4u k0, v4u k1, v4u k2, v4u k3, v4u k4) {
    const uint32_t W[20] = {k0[0], k0[1], k0[2], k0[3], k1[0], k1[1], k1[2], k1[3], k2[0], k2[1],
                            k2[2], k2[3], k3[0], k3[1], k3[2], k3[3], k4[0], k4[1], k4[2], k4[3]};
    const uint32_t s = (uint32_t)((uintptr_t)h & 15u);
    const uint32_t q = s >> 2, sh = s & 3u;
    uint32_t R[16];
#pragma unroll
    for (int m = 0; m < 16; m++) {
        const uint32_t lo = q == 0 ? W[m] : q == 1 ? W[m + 1] : q == 2 ? W[m + 2] : W[m + 3];
        const uint32_t hi = q == 0 ? W[m + 1] : q == 1 ? W[m + 2] : q == 2 ? W[m + 3] : W[m + 4];
        R[m] = __builtin_amdgcn_alignbyte(hi, lo, sh);
    }
    const uint32_t cs = d.csum_start;
    const uint32_t l16 = (uint32_t)l4len & 0xffffu;
    uint32_t sad, proto;
    if (!v6) {
        const uint32_t T = (uint32_t)((uint64_t)d.hdr_len + d.payload_bytes) & 0xffffu;
        uint32_t sip = (R[0] & 0xffffu) + sum16x2(R[1]) + (R[2] & 0xffffu);  // skip ip_len (2-3), ip_sum (10-11)
#pragma unroll
        for (int m = 3; m < 16; m++)
            sip += sum16x2(keep_below(R[m], m, cs));
        const uint32_t c = ~fold16_32(sip + bswap16(T)) & 0xffffu;  // :103-106
        st128_u(h, v4u{(R[0] & 0xffffu) | (bswap16(T) << 16), R[1], (R[2] & 0xffffu) | (c << 16), R[3]});
        sad = sum16x2(R[3]) + sum16x2(R[4]);
        proto = (R[2] >> 8) & 0xffu;
    } else {
        st32_u(h + 4, (R[1] & 0xffff0000u) | bswap16(l16));  // :95
        sad = 0;
#pragma unroll
        for (int m = 2; m < 10; m++)
            sad += sum16x2(R[m]);
        proto = (R[1] >> 16) & 0xffu;
    }
    const uint32_t seed = ~fold16_32(sad + (proto << 8) + bswap16(l16)) & 0xffffu;  // :108-112
    if (!tcp && d.csum_offset == 6) {
        st32_u(h + cs + 4, bswap16(l16) | (seed << 16));  // udp->len (:85-86) + seed (:114)
        return;
    }
    if (!tcp)
        st_be16(h + cs + 4, l16);           // udp->len, :85-86
    st16_ne(h + cs + d.csum_offset, seed);  // native order, :114
}

// General path (header fields beyond 64 bytes): byte loop in reference order.
__device__ __noinline__ void gro_slow(uint8_t *h, uint32_t H, uint32_t cs, uint32_t l4off, uint64_t payload_bytes,
                                     bool v6, uint64_t l4len) {
    uint32_t proto, ao, al;
    if (v6) {
        proto = h[6];
        ao = 8;
        al = 32;
        st_be16(h + 4, (uint32_t)l4len);
    } else {
        proto = h[9];
        ao = 12;
        al = 8;
        st_be16(h + 2, (uint32_t)((uint64_t)H + payload_bytes));
        uint32_t s = 0;
        for (uint32_t j = 0; j < cs; j++)
            s += (j == 10 || j == 11) ? 0u : (uint32_t)h[j] << (8u * (j & 1));
        const uint32_t c = ~fold16_32(s) & 0xffffu;
        stb(h + 10, c & 0xffu);
        stb(h + 11, c >> 8);
    }
    uint32_t ps = 0;
    for (uint32_t j = 0; j < al; j++)
        ps += (uint32_t)h[ao + j] << (8u * (j & 1u));
    ps += (proto << 8) + bswap16((uint32_t)l4len & 0xffffu);
    const uint32_t seed = ~fold16_32(ps) & 0xffffu;
    stb(h + l4off, seed & 0xffu);
    stb(h + l4off + 1, seed >> 8);
}

// The kernel: a thread per flow for the arithmetic, but the header chunks
// are fetched cooperatively: the block's 256 flows need up to 5 aligned 16-B
// chunks each; lane L loads chunk slots L, L+256, ... (slot k = chunk k % 5 of
// flow k / 5), so consecutive lanes read consecutive chunks of one flow and a
// wave-instruction touches a few contiguous lines instead of 64 scattered
// ones (thread-per-flow loads at a 64-B lane stride are address-processing
// bound: about one cache line per cycle per CU).  The chunks go through LDS
// to their flow's thread, which then runs gro_fields.  Five chunks cover
// every header of <= 64 bytes at any alignment; longer ones take the byte
// path.  (Measured and dropped: thread-per-flow loads, 4 chunks per flow,
// wave-owned staging without the block barrier, narrow field stores.)
constexpr uint32_t kGroBlock = 256;
constexpr uint32_t kGroChunks = 5;
static __device__ v4u g_gro_zero;  // load target of slots with nothing to stage

__device__ __forceinline__ uint32_t flow_of_slot(uint32_t slot) {  // slot / 5 for slot < 256 * 5
    return (slot * 52429u) >> 18;
}

__global__ __launch_bounds__(kGroBlock) void gro_finalize_lds_kernel(uint8_t *hdrs, wg_gro_desc *desc, uint64_t n) {
    constexpr uint32_t kNeedMax = kFastNeed;
    __shared__ v4u s_chunk[kGroBlock * kGroChunks];
    __shared__ uint64_t s_a0[kGroBlock];
    __shared__ uint32_t s_last[kGroBlock];  // last chunk index to load, or 0xff: nothing to stage
    const uint32_t t = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * kGroBlock + t;
    wg_gro_desc d{};
    bool live = i < n, fast = false, v6 = false, tcp = false;
    int8_t st = 0;
    uint32_t need = 0, cs = 0, l4off = 0;
    uint8_t *h = hdrs;
    if (live) {
        d = desc[i];
        h = hdrs + d.hdr_offset;
        const uint32_t H = d.hdr_len;
        cs = d.csum_start;
        l4off = cs + d.csum_offset;
        v6 = d.flags & WG_PKT_V6;
        tcp = d.flags & WG_PKT_TCP;
        const uint32_t iph = v6 ? 40u : 20u;
        if (cs < iph || cs > H || l4off < cs || l4off + 2 > H || (!tcp && cs + 8 > H))
            st = -3;
        else {
            need = v6 ? 40u : cs;
            fast = need <= kNeedMax;
        }
    }
    const uintptr_t hp = reinterpret_cast<uintptr_t>(h);
    s_a0[t] = hp & ~(uintptr_t)15;
    s_last[t] = fast ? (uint32_t)(((hp & 15u) + need - 1) >> 4) : 0xffu;
    __syncthreads();
    // All five loads issued before any is used, branch-free (slots of flows
    // with nothing to stage read the zero chunk): a load inside `if` made the
    // compiler wait for each before the next, five serial round trips.
    uint32_t lst[kGroChunks];
    uint64_t a0[kGroChunks];
#pragma unroll
    for (uint32_t k = 0; k < kGroChunks; k++) {  // every LDS read first (unconditional), then the loads
        const uint32_t f = flow_of_slot(t + kGroBlock * k);
        lst[k] = s_last[f];
        a0[k] = s_a0[f];
    }
    v4u v[kGroChunks];
#pragma unroll
    for (uint32_t k = 0; k < kGroChunks; k++) {
        const uint32_t slot = t + kGroBlock * k;
        const uint32_t c = slot - kGroChunks * flow_of_slot(slot);
        const uint32_t last = lst[k];
        const uintptr_t a = last != 0xffu ? a0[k] + 16u * (c < last ? c : last)
                                          : reinterpret_cast<uintptr_t>(&g_gro_zero);
        v[k] = ld16(a);
    }
#pragma unroll
    for (uint32_t k = 0; k < kGroChunks; k++)
        s_chunk[t + kGroBlock * k] = v[k];
    __syncthreads();
    if (!live)
        return;
    if (st == 0) {
        const uint64_t l4len = (uint64_t)(d.hdr_len - cs) + d.payload_bytes;  // :84
        if (fast) {
            const v4u *k = &s_chunk[t * kGroChunks];
            gro_fields(h, d, v6, tcp, l4len, k[0], k[1], k[2], k[3], k[4]);
        } else {
            if (!tcp)
                st_be16(h + cs + 4, (uint32_t)l4len);  // udp->len (uint16), :85-86
            gro_slow(h, d.hdr_len, cs, l4off, d.payload_bytes, v6, l4len);
        }
    }
    if (d.status != st)  // leave descriptor lines clean when the caller pre-zeroed status
        reinterpret_cast<int8_t *>(desc)[i * sizeof(wg_gro_desc) + offsetof(wg_gro_desc, status)] = st;
}

}  // namespace wg

using namespace wg;

extern "C" int wg_gro_finalize(uint8_t *dev_hdrs, wg_gro_desc *dev_desc, uint64_t n, void *stream) {
    if (!n)
        return WG_OK;
    if (!dev_hdrs || !dev_desc || (reinterpret_cast<uintptr_t>(dev_desc) & 7))
        return WG_ERR_INVALID;
    const uint64_t blocks = (n + 255) / 256;
    if (blocks > 0x7fffffffull)
        return WG_ERR_INVALID;
    hipLaunchKernelGGL(gro_finalize_lds_kernel, dim3((unsigned)blocks), dim3(kGroBlock), 0,
                       static_cast<hipStream_t>(stream), dev_hdrs, dev_desc, n);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}
