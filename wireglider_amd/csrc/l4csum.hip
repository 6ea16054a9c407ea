// l4csum.hip — batched L4 / plain Internet checksum on MI355X (gfx950).
//
// Replaces, at batch granularity, wireglider::calc_l4_checksum
// (reference checksum.cpp:8-36) and wireglider::checksum
// (include/netio/checksum.hpp:146-149).
//
// Structure: one wavefront per packet, P packets per wave iteration.  For
// each of its P packets a lane first ISSUES its loads — the 16-byte-aligned
// interior of the summed region through global_load_dwordx4 (64 lanes x 16 B
// = 1 KiB per instruction, coalesced; the first 2 KiB of every packet in this
// phase) and one global_load_ubyte that gathers the <=15-byte unaligned head
// and tail plus the pseudo-header address bytes (one lane per byte) — and
// only then FINISHES the packets one by one (rest of a long packet, fold,
// DPP butterfly, pseudo-header constants).  So P x ~1.5 KiB per wave are in
// flight before the first wait, which is what an HBM-bound stream needs.
// No LDS: every byte is used exactly once; staging it would only add LDS
// traffic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <mutex>

#include "wg_device.hpp"
#include "wg_internal.hpp"
#include "wg_l4wave.hpp"
#include "wireglider_amd.h"

namespace wg {

struct L4Params {
    const uint8_t *base;
    const wg_pkt_desc *desc;
    uint16_t *out;
    uint64_t n;
    uint64_t total_len;
    uint32_t seg;
    uint32_t cs;
    uint32_t flags;
    uint64_t quarter;  // l4csum_split_kernel: descriptors per quarter of the batch (a multiple of 4)
};

enum Kind : int { kUniformL4 = 0, kDescL4 = 1, kDescPlain = 2 };

template <int kKind>
__device__ __forceinline__ Geom load_geom(const L4Params &p, uint64_t i) {
    Geom g;
    if (i >= p.n) {  // padding slot of the last iteration: empty packet
        g.a = reinterpret_cast<uintptr_t>(p.base);
        g.len = 0;
        g.cs = 0;
        g.fl = 0;
        return g;
    }
    if constexpr (kKind == kUniformL4) {
        // PacketBatch segment i (include/util/packets.hpp:23-36)
        const uint64_t off = i * (uint64_t)p.seg;
        const uint64_t rem = p.total_len - off;
        g.a = reinterpret_cast<uintptr_t>(p.base) + off;
        g.len = rem < p.seg ? (uint32_t)rem : p.seg;
        g.cs = p.cs;
        g.fl = p.flags;
    } else {
        const wg_pkt_desc d = p.desc[i];
        g.a = reinterpret_cast<uintptr_t>(p.base) + d.offset;
        g.len = d.len;
        g.cs = kKind == kDescPlain ? 0u : d.csum_start;
        g.fl = d.flags;
    }
    return g;
}

// Descriptors of packets i0 .. i0+P-1 by ONE coalesced vector load (lane j
// holds descriptor j), made wave-uniform with v_readlane.
template <int P>
__device__ __forceinline__ v4u load_desc_vec(const L4Params &p, uint64_t i0, uint32_t lane) {
    const uint64_t di = i0 + (lane & (uint32_t)(P - 1));
    const uint64_t dc = di < p.n ? di : p.n - 1;
    return ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * dc);
}

template <int kKind, int P>
__device__ __forceinline__ void geoms_from_vec(const L4Params &p, uint64_t i0, const v4u &dv, Geom *g) {
#pragma unroll
    for (int j = 0; j < P; j++) {
        const bool live = i0 + j < p.n;  // else a padding slot: empty packet
        const uint64_t off = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dv.x, j) |
                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dv.y, j) << 32);
        const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)dv.w, j);
        g[j].a = reinterpret_cast<uintptr_t>(p.base) + (live ? off : 0u);
        g[j].len = live ? (uint32_t)__builtin_amdgcn_readlane((int)dv.z, j) : 0u;
        g[j].cs = kKind == kDescPlain || !live ? 0u : (w & 0xffffu);
        g[j].fl = live ? (w >> 16) & 0xffu : 0u;
    }
}

// Descriptor modes (kDM): 0 = scalar loads per iteration; 1 = one vector load
// per iteration (measured slower: the readlanes wait on it); 2 = scalar loads
// for a wave's first iteration, and each iteration's vector load of the NEXT
// iteration's descriptors issued right after its own packet loads, so from
// the second iteration on a wave starts its packet loads with no descriptor
// round trip in front of them (the launcher gives each wave l4_iters
// iterations).
template <int kKind, int P, bool kNT, int kDM, int O = 0>  // O: waves/SIMD target (0 = compiler's choice)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(O ? O : 1, O ? O : 8))) void l4csum_kernel(
    L4Params p) {
    constexpr bool kL4 = kKind != kDescPlain;
    constexpr int DM = kKind == kUniformL4 ? 0 : kDM;
    const uint32_t lane = lane_id();
    const uint64_t wave0 = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t step = (uint64_t)gridDim.x * 4u * P;
    v4u nextd = v4u{0, 0, 0, 0};
    bool have_next = false;
    for (uint64_t i0 = wave0 * P; i0 < p.n; i0 += step) {
        Geom g[P];
        Front f[P];
        if constexpr (DM == 1) {
            geoms_from_vec<kKind, P>(p, i0, load_desc_vec<P>(p, i0, lane), g);
        } else if constexpr (DM == 2) {
            if (have_next) {
                geoms_from_vec<kKind, P>(p, i0, nextd, g);
            } else {
#pragma unroll
                for (int j = 0; j < P; j++)
                    g[j] = load_geom<kKind>(p, i0 + j);
            }
        }
#pragma unroll
        for (int j = 0; j < P; j++) {
            if constexpr (DM == 0)
                g[j] = load_geom<kKind>(p, i0 + j);
            issue<kL4, kNT>(g[j], lane, f[j]);
        }
        if constexpr (DM == 2) {  // next iteration's descriptors, in flight during the finish
            have_next = i0 + step < p.n;
            nextd = load_desc_vec<P>(p, have_next ? i0 + step : i0, lane);
        }
        uint32_t res = 0;
#pragma unroll
        for (int j = 0; j < P; j++) {
            uint32_t s = wave_sum_u32(finish<kNT>(lane, f[j]));
            if (kL4) {
                // {0x00, proto, l4len>>8, l4len&0xff} as LE words
                // (include/netio/checksum.hpp:111-114); l4len is uint16_t
                // (checksum.cpp:23,33).
                const uint32_t proto = (g[j].fl & WG_PKT_TCP) ? 6u : 17u;
                s += (proto << 8) + bswap16((g[j].len - g[j].cs) & 0xffffu);
            }
            const uint32_t r = ~fold16_32(s) & 0xffffu;
            if (lane == (uint32_t)j)
                res = r;
        }
        if (lane < (uint32_t)P && i0 + lane < p.n)
            p.out[i0 + lane] = (uint16_t)res;
    }
}

template <int kKind, int P, bool kNT, int DM>
static void launch_occ(const L4Params &p, uint64_t blocks, hipStream_t st) {
    const uint32_t occ = tune().l4_occ;
    if constexpr (P == 4 && kNT) {
        if (occ == 7) {
            hipLaunchKernelGGL((l4csum_kernel<kKind, P, kNT, DM, 7>), dim3((unsigned)blocks), dim3(256), 0, st, p);
            return;
        }
        if (occ == 8) {
            hipLaunchKernelGGL((l4csum_kernel<kKind, P, kNT, DM, 8>), dim3((unsigned)blocks), dim3(256), 0, st, p);
            return;
        }
    }
    hipLaunchKernelGGL((l4csum_kernel<kKind, P, kNT, DM>), dim3((unsigned)blocks), dim3(256), 0, st, p);
}

template <int kKind, int P, bool kNT>
static void launch_variant(const L4Params &p, uint64_t blocks, hipStream_t st) {
    const uint32_t dm = kKind == kUniformL4 ? 0u : tune().l4_descv;
    if (dm == 1)
        launch_occ<kKind, P, kNT, 1>(p, blocks, st);
    else if (dm == 2)
        launch_occ<kKind, P, kNT, 2>(p, blocks, st);
    else
        launch_occ<kKind, P, kNT, 0>(p, blocks, st);
}

template <int kKind>
static void launch_kind(const L4Params &p, uint64_t blocks, uint32_t P, bool nt, hipStream_t st) {
    switch (P) {
    case 1: nt ? launch_variant<kKind, 1, true>(p, blocks, st) : launch_variant<kKind, 1, false>(p, blocks, st); break;
    case 2: nt ? launch_variant<kKind, 2, true>(p, blocks, st) : launch_variant<kKind, 2, false>(p, blocks, st); break;
    case 8: nt ? launch_variant<kKind, 8, true>(p, blocks, st) : launch_variant<kKind, 8, false>(p, blocks, st); break;
    default: nt ? launch_variant<kKind, 4, true>(p, blocks, st) : launch_variant<kKind, 4, false>(p, blocks, st); break;
    }
}

// ---------------------------------------------------------------------------
// Small-packet descriptor kernel (knob l4_small; SURVEY §8(d) config 4's
// small-packet stress).  A wave per packet spends ~150 wave-instructions
// (half of them on the CU's one scalar unit) on a 64-B packet, so 64-B
// batches are issue-bound at ~6 % of the HBM roofline.  Here a lane (or a
// lane quad, G below) takes one descriptor: a packet of <= kSmallMax bytes is
// summed from (at most) five aligned 16-B chunks — by a lane as 16
// packet-relative dwords funnel-shifted out of them, by a quad as masked
// absolute dwords — over the summed region and the pseudo-header address
// bytes; the lanes whose packet is longer are then taken by the whole wave,
// Q at a time, through the same issue / finish machinery as l4csum_kernel.
// Uniform PacketBatches with segment_size <= kSmallMax use it too (every
// segment is small).  Same arithmetic model (wg_device.hpp): one byte swap of
// a folded sum whose pairing starts at an odd position.
// ---------------------------------------------------------------------------
constexpr uint32_t kSmallMax = 64;  // bytes: five aligned 16-B chunks at any alignment

// Bytes of the dword at relative position p (a multiple of 4) that lie in [lo, hi).
__device__ __forceinline__ uint32_t dword_mask(uint32_t p, uint32_t lo, uint32_t hi) {
    const int a = (int)lo - (int)p, b = (int)hi - (int)p;
    const uint32_t mh = b >= 4 ? ~0u : (b <= 0 ? 0u : (1u << (8 * b)) - 1u);
    const uint32_t ml = a >= 4 ? ~0u : (a <= 0 ? 0u : (1u << (8 * a)) - 1u);
    return mh & ~ml;
}

__device__ __forceinline__ uint32_t half_sum(uint32_t w) { return (w & 0xffffu) + (w >> 16); }

// Packet-relative dword m (bytes 4m .. 4m+3 of the packet): keep the bytes
// at positions < lim / >= lo.
__device__ __forceinline__ uint32_t bytes_below(uint32_t w, uint32_t m, uint32_t lim) {
    const int k = (int)lim - 4 * (int)m;  // bytes of dword m at packet positions < lim
    return k >= 4 ? w : (k <= 0 ? 0u : (w & ((1u << (8 * k)) - 1u)));
}
__device__ __forceinline__ uint32_t bytes_from(uint32_t w, uint32_t m, uint32_t lo) {
    const int k = (int)lo - 4 * (int)m;
    return k <= 0 ? w : (k >= 4 ? 0u : (w & ~((1u << (8 * k)) - 1u)));
}

__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t j) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j);
}

// The lane path for one packet of <= kSmallMax bytes at a (length len):
// its five aligned 16-B chunks (default cache policy: a small packet's 128-B
// lines are shared with its neighbours' lanes, and non-temporal loads fetched
// them again — 64-B PacketBatch 42.9 -> 24.3 us), clamped onto the last
// chunk the packet touches; `use` false -> the zero chunk.
__device__ __forceinline__ void lane_chunks(uintptr_t a, uint32_t len, bool use, v4u W[5]) {
    const uintptr_t zero = reinterpret_cast<uintptr_t>(&g_zero16);
    const uintptr_t a0 = a & ~(uintptr_t)15;
    const uintptr_t alast = (a + len - 1) & ~(uintptr_t)15;
#pragma unroll
    for (uint32_t k = 0; k < 5; k++) {
        const uintptr_t ca = a0 + 16u * k;
        W[k] = ld16(use ? (ca > alast ? alast : ca) : zero);  // clamped chunks are masked below
    }
}

// ... summed: the chunks funnel-shifted into 16 packet-relative dwords
// (bytes past the packet zeroed), so the region and address masks are
// per-dword constants of len / csum_start and the addresses static dwords.
// Returns the pre-complement folded sum t (region, byte-swapped when it pairs
// from an odd packet offset, + pseudo-header when kL4); the caller's result
// is ~fold16_32(t).
template <bool kL4>
__device__ __forceinline__ uint32_t lane_sum(const v4u W[5], uintptr_t a, uint32_t len, uint32_t cs, uint32_t fl) {
    const uint32_t o0 = cs < len ? cs : len;
    const bool v6 = fl & WG_PKT_V6;
    const uint32_t Wd[20] = {W[0][0], W[0][1], W[0][2], W[0][3], W[1][0], W[1][1], W[1][2],
                             W[1][3], W[2][0], W[2][1], W[2][2], W[2][3], W[3][0], W[3][1],
                             W[3][2], W[3][3], W[4][0], W[4][1], W[4][2], W[4][3]};
    const uint32_t s = (uint32_t)(a & 15u), q4 = s >> 2, sh = s & 3u;
    uint32_t sr = 0, sq = 0;
#pragma unroll
    for (uint32_t m = 0; m < 16; m++) {
        const uint32_t lo = q4 == 0 ? Wd[m] : q4 == 1 ? Wd[m + 1] : q4 == 2 ? Wd[m + 2] : Wd[m + 3];
        const uint32_t hi = q4 == 0 ? Wd[m + 1] : q4 == 1 ? Wd[m + 2] : q4 == 2 ? Wd[m + 3] : Wd[m + 4];
        const uint32_t r = bytes_below(__builtin_amdgcn_alignbyte(hi, lo, sh), m, len);
        sr += half_sum(bytes_from(r, m, o0));
        if (kL4) {
            const bool in_addr = v6 ? (m >= 2u && m < 10u) : (m == 3u || m == 4u);  // v6 8-39, v4 12-19
            sq += in_addr ? half_sum(r) : 0u;
        }
    }
    sr = fold16_32(sr);
    if (o0 & 1u)  // packet pairing; the region pairs from an odd offset
        sr = bswap16(sr);
    uint32_t t = sr;
    if (kL4) {
        const uint32_t proto = (fl & WG_PKT_TCP) ? 6u : 17u;
        t += fold16_32(sq) + (proto << 8) + bswap16((len - cs) & 0xffffu);  // checksum.hpp:111-114, checksum.cpp:23,33
    }
    return t;
}

// The wave path: the packets of the lanes in mask m (lane j's packet at a,
// length len, csum_start cs, flags fl), Q at a time through the issue /
// finish machinery of l4csum_kernel (all Q packets' loads in flight before
// the first wait); packet j's result lands in lane j's res.
template <bool kL4, bool kNT, int Q, int U = 4>
__device__ __forceinline__ void wave_long(uint64_t m, uintptr_t a, uint32_t len, uint32_t cs, uint32_t fl,
                                          const uint8_t *base, uint32_t lane, uint32_t &res) {
    const uint32_t alo = (uint32_t)a, ahi = (uint32_t)((uint64_t)a >> 32);
    while (m) {
        Geom g[Q];
        uint32_t jj[Q];
#pragma unroll
        for (int k = 0; k < Q; k++) {
            const bool have = m != 0;
            const uint32_t j = have ? (uint32_t)__builtin_ctzll(m) : 0u;
            m = have ? m & (m - 1) : m;
            jj[k] = have ? j : 64u;
            g[k].a = have ? (uintptr_t)(((uint64_t)rdl(ahi, j) << 32) | rdl(alo, j)) : reinterpret_cast<uintptr_t>(base);
            g[k].len = have ? rdl(len, j) : 0u;
            g[k].cs = have ? rdl(cs, j) : 0u;
            g[k].fl = have ? rdl(fl, j) : 0u;
        }
        Front f[Q];
#pragma unroll
        for (int k = 0; k < Q; k++)
            issue<kL4, kNT>(g[k], lane, f[k]);
#pragma unroll
        for (int k = 0; k < Q; k++) {
            uint32_t t = wave_sum_u32(finish<kNT, U>(lane, f[k]));
            if (kL4) {
                const uint32_t proto = (g[k].fl & WG_PKT_TCP) ? 6u : 17u;
                t += (proto << 8) + bswap16((g[k].len - g[k].cs) & 0xffffu);
            }
            if (lane == jj[k])
                res = ~fold16_32(t) & 0xffffu;
        }
    }
}

// G: lanes per descriptor.  G = 1: a lane loads all five chunks; G = 4: a
// quad shares one descriptor, lane q of the quad loads chunks q and (q = 0)
// chunk 4, and the quad's partial sums meet by DPP — a wave then carries 16
// descriptors instead of 64, so its serial walk over the long packets is as
// short as the wave-per-packet kernel's four iterations.
template <int kKind, bool kNT, int Q, int G, bool kLate = false>  // Q: long packets the wave takes at a time (2, 4)
__global__ __launch_bounds__(256) void l4csum_small_kernel(L4Params p) {
    static_assert(G == 1 || G == 4, "lanes per descriptor");
    constexpr bool kL4 = kKind != kDescPlain;
    const uint32_t lane = lane_id();
    const uint32_t q = lane & (uint32_t)(G - 1);
    const uint64_t i = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * (256u / G) + threadIdx.x / G;
    const bool live = i < p.n;
    uintptr_t a;
    uint32_t len, cs, fl;
    if constexpr (kKind == kUniformL4) {  // PacketBatch segment i (include/util/packets.hpp:23-36)
        const uint64_t off = live ? i * (uint64_t)p.seg : 0u;
        const uint64_t rem = p.total_len - off;
        a = reinterpret_cast<uintptr_t>(p.base) + off;
        len = live ? (rem < p.seg ? (uint32_t)rem : p.seg) : 0u;
        cs = live ? p.cs : 0u;
        fl = live ? p.flags : 0u;
    } else {
        const v4u dv = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0));
        const uint64_t off = (uint64_t)dv.x | ((uint64_t)dv.y << 32);
        a = reinterpret_cast<uintptr_t>(p.base) + (live ? off : 0u);
        len = live ? dv.z : 0u;
        cs = kL4 && live ? (dv.w & 0xffffu) : 0u;
        fl = live ? (dv.w >> 16) & 0xffu : 0u;
    }
    const bool small = len <= kSmallMax;

    // ---- lane path: the packet's aligned chunks, all issued at once.
    // kLate: the loads go out before the wave path and are summed after it,
    // so they fly under the long packets' loads; otherwise loaded and summed
    // here, skipped by waves whose packets are all long (uniform branch).
    uint32_t res = 0;
    const bool any_small = __ballot(live && small) != 0;
    constexpr uint32_t kC = G == 1 ? 5u : 2u;  // chunks per lane
    v4u W[kC];
    uint32_t cidx[kC];
    const uint32_t s = (uint32_t)(a & 15u);
    auto load_chunks = [&]() {
        if constexpr (G == 1) {
            lane_chunks(a, len, small && len, W);
            return;
        }
        const uintptr_t zero = reinterpret_cast<uintptr_t>(&g_zero16);
        const uintptr_t a0 = a & ~(uintptr_t)15;
        const uintptr_t alast = (a + len - 1) & ~(uintptr_t)15;
        const bool any = small && len;
#pragma unroll
        for (uint32_t k = 0; k < kC; k++) {
            cidx[k] = G == 1 ? k : q + 4u * k;  // G = 4: chunks q and q + 4 (< 5 only for q = 0)
            const uintptr_t ca = a0 + 16u * cidx[k];
            const bool use = any && cidx[k] < 5u;
            // default-policy loads, not kNT: a small packet's 128-B lines are
            // shared with its neighbours' lanes (and the clamped duplicates),
            // so non-temporal loads fetched them again (64-B PacketBatch
            // 42.9 -> 24.3 us with cached loads)
            W[k] = ld16(use ? (ca > alast ? alast : ca) : zero);  // clamped chunks are masked below
        }
    };
    auto sum_chunks = [&]() {
        if constexpr (G == 1) {
            const uint32_t t = lane_sum<kL4>(W, a, len, cs, fl);
            if (small)
                res = ~fold16_32(t) & 0xffffu;
            return;
        }
        const uint32_t o0 = cs < len ? cs : len;
        const bool v6 = fl & WG_PKT_V6;
        const uint32_t ao = v6 ? 8u : 12u, al = v6 ? 32u : 8u;
        const uint32_t aend = ao + al < len ? ao + al : len;  // address bytes past the packet end are absent
        uint32_t sr = 0, sq = 0;
        uint32_t rodd;  // the region's pairing is odd relative to the summed dwords
        {
#pragma unroll
            for (uint32_t k = 0; k < kC; k++) {
#pragma unroll
                for (uint32_t d = 0; d < 4; d++) {
                    const uint32_t pos = 16u * cidx[k] + 4u * d, w = W[k][d];
                    sr += half_sum(w & dword_mask(pos, s + o0, s + len));
                    if (kL4)
                        sq += half_sum(w & dword_mask(pos, s + ao, s + (aend > ao ? aend : ao)));
                }
            }
            sr = group_sum_u32<4>(sr);  // the quad's partial sums (each < 2^20: no overflow)
            sq = group_sum_u32<4>(sq);
            rodd = (s + o0) & 1u;  // absolute-address pairing
        }
        sr = fold16_32(sr);
        if (rodd)  // the region pairs from an odd position
            sr = bswap16(sr);
        uint32_t t = sr;
        if (kL4) {
            sq = fold16_32(sq);
            if (G > 1 && (s & 1u))  // absolute pairing: the addresses pair from the packet start
                sq = bswap16(sq);
            const uint32_t proto = (fl & WG_PKT_TCP) ? 6u : 17u;
            t += sq + (proto << 8) + bswap16((len - cs) & 0xffffu);  // checksum.hpp:111-114, checksum.cpp:23,33
        }
        if (small)
            res = ~fold16_32(t) & 0xffffu;
    };
    if (kLate) {
        load_chunks();
    } else if (any_small) {
        load_chunks();
        sum_chunks();
    }

    // ---- wave path: the longer packets of this wave, Q at a time
    wave_long<kL4, kNT, Q>(__ballot(live && !small && q == 0), a, len, cs, fl, p.base, lane, res);
    if (kLate && any_small)
        sum_chunks();
    if (live && q == 0)
        p.out[i] = (uint16_t)res;
}

// Split-role descriptor kernel (knob l4_small = 5).  Descriptors come in
// groups of 4 consecutive ones; the batch is cut into 4 quarters of Q
// descriptors, and block b owns the 16 at [q*Q + 16b, q*Q + 16b + 16) of each
// quarter q (64 in all).  Its wave k owns one group per quarter,
// [q*Q + 16b + 4k, +4): 16 descriptors a quarter batch apart, like the
// wave-per-packet kernel's grid-stride iterations (consecutive packets per
// wave measured 3-4 % slower).
//  * WAVE role (every wave): every packet of its groups that hold a packet
//    longer than kSmallMax, 4 at a time through the wave-per-packet
//    machinery; small packets among long ones ride along in their issue
//    phase at next to no cost (config 4's mixed batch measured +2.5 % when
//    they went to the lane role instead).
//  * LANE role (wave 0): the block's all-small groups, a lane per packet,
//    summed from its 5 aligned chunks (4 KiB of loads in flight per wave).
// Wave 0 loads the block's 64 descriptors (lane l = descriptor
// (l >> 4) * Q + 16b + (l & 15); its own groups are lanes with (l & 15) < 4),
// waves 1-3 their 16: every descriptor read once from HBM.  An all-small
// batch keeps a lane per packet (waves 1-3 leave after one descriptor load),
// an all-long one keeps the short 16-packet waves with every descriptor in
// one vector load.  One launch, no host knowledge of the mix.
// kW = 8: 512-thread blocks, wave k owning group (k mod 4) of quarters
// 2 (k / 4) and 2 (k / 4) + 1 — 8 descriptors per wave, shorter-lived waves.
template <int kKind, bool kNT, int U = 4, int kW = 4>  // U: loads in flight per lane on a long packet's rest
__global__ __launch_bounds__(64 * kW) void l4csum_split_kernel(L4Params p) {
    constexpr bool kL4 = kKind != kDescPlain;
    constexpr uint32_t kQpw = 16u / kW;  // quarters per wave in the wave role (4 or 2)
    const uint32_t lane = lane_id();
    const uint32_t wib = wave_in_block();
    const uint64_t blk = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint64_t Q = p.quarter;
    // lane -> (quarter, offset in the block's 16 of that quarter)
    const uint32_t qq = wib == 0 ? lane >> 4 : kQpw * (wib >> 2) + ((lane >> 2) & (kQpw - 1u));
    const uint32_t oo = wib == 0 ? lane & 15u : 4u * (wib & 3u) + (lane & 3u);
    const uint64_t i = (uint64_t)qq * Q + 16u * blk + oo;
    const bool live = (wib == 0 || lane < 4u * kQpw) && 16u * blk < Q && i < p.n;
    const v4u d = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : p.n - 1));
    const uint64_t off = (uint64_t)d.x | ((uint64_t)d.y << 32);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p.base) + (live ? off : 0u);
    const uint32_t len = live ? d.z : 0u;
    const uint32_t cs = kL4 && live ? (d.w & 0xffffu) : 0u;
    const uint32_t fl = live ? (d.w >> 16) & 0xffu : 0u;
    // groups are 4 consecutive lanes in both layouts
    const uint64_t gl = __ballot(live && len > kSmallMax);
    const bool grp_long = ((gl >> (lane & ~3u)) & 0xfu) != 0;
    // ---- wave role: this wave's groups that hold a long packet
    const bool own = wib == 0 ? (lane & 15u) < 4u && (lane >> 4) < kQpw : true;
    const bool mine = live && own && grp_long;
    uint32_t res = 0;
    wave_long<kL4, kNT, 4, U>(__ballot(mine), a, len, cs, fl, p.base, lane, res);
    if (mine)
        p.out[i] = (uint16_t)res;
    // ---- lane role (wave 0): the block's all-small groups
    const bool small = wib == 0 && live && !grp_long;
    if (__ballot(small)) {  // wave-uniform; never true on waves 1-3
        v4u W[5];
        lane_chunks(a, len, small && len, W);
        const uint32_t t = lane_sum<kL4>(W, a, small ? len : 0u, cs, fl);
        if (small)
            p.out[i] = (uint16_t)(~fold16_32(t) & 0xffffu);
    }
}

// Walking descriptor kernel (knob l4_small = 6).  A wave per 64 descriptors
// whatever their sizes, laid out so that the waves resident at any moment
// touch one narrow window of the batch: lane l of wave w (of G) owns
// descriptor ((l >> 2) * G + w) * 4 + (l & 3) — sixteen 4-descriptor groups a
// sixteenth of the batch apart.  Small packets (<= kSmallMax) are summed in
// their lane (lane_chunks / lane_sum); the wave then walks its long packets in
// group order, 4 at a time, through the wave-per-packet issue / finish
// machinery.  An all-small batch costs n / 64 waves (the split kernel's n / 16
// waves spend three of every four on one descriptor load), an all-long batch
// 16 groups per wave.
template <int kKind, bool kNT, int U = 4>
__global__ __launch_bounds__(256) void l4csum_walk_kernel(L4Params p) {
    constexpr bool kL4 = kKind != kDescPlain;
    const uint32_t lane = lane_id();
    const uint64_t G = (uint64_t)gridDim.x * 4u;
    const uint64_t w = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t i = ((uint64_t)(lane >> 2) * G + w) * 4u + (lane & 3u);
    const bool live = i < p.n;
    const v4u d = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0u));
    const uint64_t off = (uint64_t)d.x | ((uint64_t)d.y << 32);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p.base) + (live ? off : 0u);
    const uint32_t len = live ? d.z : 0u;
    const uint32_t cs = kL4 && live ? (d.w & 0xffffu) : 0u;
    const uint32_t fl = live ? (d.w >> 16) & 0xffu : 0u;
    const bool small = live && len <= kSmallMax;
    uint32_t res = 0;
    if (__ballot(small)) {  // wave-uniform
        v4u W[5];
        lane_chunks(a, len, small && len, W);
        const uint32_t t = lane_sum<kL4>(W, a, small ? len : 0u, cs, fl);
        res = ~fold16_32(t) & 0xffffu;
    }
    wave_long<kL4, kNT, 4, U>(__ballot(live && !small), a, len, cs, fl, p.base, lane, res);
    if (live)
        p.out[i] = (uint16_t)res;
}

// Persistent walking kernel (knob l4_small = 7): the walking kernel's lane /
// wave split, but the grid is the device's resident wave capacity (or n / 64
// waves if fewer) and each wave takes ROUNDS of 16 groups — in round r lane l
// owns descriptor ((16 r + (l >> 2)) * G + w) * 4 + (l & 3) — so every wave
// gets the same number of groups to within one, whatever n (a grid of n / 64
// waves is 2.3 generations of resident waves for 1 M descriptors: its last
// partial generation ran at a third of the chip), and the waves resident at
// any moment still work on one narrow window of the batch.
template <int kKind, bool kNT, int U = 4>
__global__ __launch_bounds__(256) void l4csum_persist_kernel(L4Params p) {
    constexpr bool kL4 = kKind != kDescPlain;
    const uint64_t G = (uint64_t)gridDim.x * 4u;
    const uint64_t w = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    for (uint64_t r0 = 0; r0 * G * 4u < p.n; r0 += 16) {
        uint32_t lane = lane_id();
        asm volatile("" : "+v"(lane));  // lane-derived values recomputed per round, not held across it
        const uint64_t i = ((r0 + (lane >> 2)) * G + w) * 4u + (lane & 3u);
        const bool live = i < p.n;
        const v4u d = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0u));
        const uint64_t off = (uint64_t)d.x | ((uint64_t)d.y << 32);
        const uintptr_t a = reinterpret_cast<uintptr_t>(p.base) + (live ? off : 0u);
        const uint32_t len = live ? d.z : 0u;
        const uint32_t cs = kL4 && live ? (d.w & 0xffffu) : 0u;
        const uint32_t fl = live ? (d.w >> 16) & 0xffu : 0u;
        const bool small = live && len <= kSmallMax;
        uint32_t res = 0;
        if (__ballot(small)) {  // wave-uniform
            v4u W[5];
            lane_chunks(a, len, small && len, W);
            const uint32_t t = lane_sum<kL4>(W, a, small ? len : 0u, cs, fl);
            res = ~fold16_32(t) & 0xffffu;
        }
        wave_long<kL4, kNT, 4, U>(__ballot(live && !small), a, len, cs, fl, p.base, lane, res);
        if (live)
            p.out[i] = (uint16_t)res;
    }
}

// Resident 256-thread blocks of `kernel` on the current device (occupancy
// query x CUs), cached per device; 0 when the runtime cannot say.
template <typename K>
static uint64_t resident_blocks(K kernel) {
    static std::atomic<int64_t> cache[16];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0)
        return 0;
    if (dev < 16) {
        const int64_t c = cache[dev].load(std::memory_order_relaxed);
        if (c > 0)
            return (uint64_t)c;
    }
    int cus = 0, nb = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, 256, 0) != hipSuccess || cus <= 0 || nb <= 0)
        return 0;
    const int64_t v = (int64_t)cus * nb;
    if (dev < 16)
        cache[dev].store(v, std::memory_order_relaxed);
    return (uint64_t)v;
}

// Grid of a persistent walking kernel: n / 256 blocks, capped at the resident
// capacity, a multiple of 8 (XCD swizzle) when >= 8.
static uint64_t persist_grid(uint64_t n, uint64_t cap) {
    uint64_t b = (n + 255) / 256;
    if (cap >= 8 && b > (cap & ~7ull))
        b = cap & ~7ull;
    if (b >= 8)
        b = (b + 7) & ~7ull;  // <= the capped value: that is a multiple of 8
    return b;
}

// Block-per-descriptor kernel for batches of FEW, LONG packets (knob l4_coop:
// descriptor batches of n <= l4_coop; BASELINE config 1: 16,384 x 64 KiB).
// The split kernel sizes its grid by descriptor count — 1,024 waves for
// config 1, one per SIMD, each streaming 1 MiB with 8 KiB in flight, so the
// HBM pipe is never full (77 %).  Here W waves share one packet: wave 0 runs
// the issue phase (first 2 KiB, unaligned head / tail, pseudo-header bytes);
// the interior past that is dealt in rounds of W x 64 x U chunks, wave w
// taking the w-th 64 x U of each round, all U loads in flight.  Partial sums
// are of 16-B-aligned chunks, so they add directly; each wave folds its own
// (and byte-swaps it when the region pairs from an odd address — swapping
// distributes over one's-complement addition), and the W wave sums meet in
// LDS.  A short packet leaves waves 1..W-1 idle, which is why the host
// chooses this only for small n.
template <int kKind, bool kNT, int W, int U>
__global__ __launch_bounds__(64 * W) void l4csum_coop_kernel(L4Params p) {
    constexpr bool kL4 = kKind != kDescPlain;
    __shared__ uint32_t part[W];
    const uint32_t lane = lane_id();
    const uint32_t w = wave_in_block();
    const uint64_t i = xcd_swizzle(blockIdx.x, gridDim.x);
    if (i >= p.n)  // block-uniform: surplus blocks of the rounded grid
        return;
    const Geom g = load_geom<kKind>(p, i);
    Front f;
    if (w == 0) {
        issue<kL4, kNT>(g, lane, f);
    } else {
        // geometry of the interior only (as in issue)
        const uint32_t alo = (uint32_t)g.a;
        const uint32_t o0 = g.cs < g.len ? g.cs : g.len;
        const uint32_t oc0 = ((alo + o0 + 15u) & ~15u) - alo;
        const uint32_t b1 = ((alo + g.len) & ~15u) - alo + 16u;
        const uint32_t b0 = oc0 + 16u;
        f.nint = b1 > b0 ? (b1 - b0) >> 4 : 0u;
        f.c0 = g.a + oc0;
        f.r0odd = (alo + o0) & 1u;
        f.v0 = f.v1 = v4u{0, 0, 0, 0};
        f.bv = 0;
        f.bt = false;
    }
    Acc acc;
    if (f.nint > 128) {
        const uintptr_t q = f.c0;
        const uint32_t last = f.nint - 1;
        for (uint32_t k0 = 128 + 64u * U * w; k0 < f.nint; k0 += 64u * U * W) {
            v4u a[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t k = k0 + 64 * u + lane;
                a[u] = ld16x<kNT>(q + 16ull * (k < last ? k : last));
            }
#pragma unroll
            for (int u = 0; u < U; u++)
                if (k0 + 64 * u + lane < f.nint)
                    acc.add4(a[u]);
        }
    }
    acc.add4(f.v0);
    acc.add4(f.v1);
    if (!f.bt)
        acc.add(f.bv);
    uint32_t s = fold16(acc.value());
    if (f.r0odd)
        s = bswap16(s);
    s = wave_sum_u32(s + (f.bt ? f.bv : 0u));
    if (lane == 0)
        part[w] = s;
    __syncthreads();
    if (w == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int k = 0; k < W; k++)
            t += part[k];
        if (kL4) {
            const uint32_t proto = (g.fl & WG_PKT_TCP) ? 6u : 17u;
            t += (proto << 8) + bswap16((g.len - g.cs) & 0xffffu);
        }
        if (lane == 0)
            p.out[i] = (uint16_t)(~fold16_32(t) & 0xffffu);
    }
}

template <int kKind, bool kNT, int U>
static int launch_coop_u(const L4Params &p, uint32_t waves, hipStream_t st) {
    uint64_t blocks = p.n;
    if (blocks >= 8)
        blocks = (blocks + 7) & ~7ull;  // XCD swizzle bijective; surplus blocks exit
    if (blocks > 0x7fffffffull)
        return WG_ERR_INVALID;
    const dim3 grid((unsigned)blocks);
    switch (waves) {
    case 2: hipLaunchKernelGGL((l4csum_coop_kernel<kKind, kNT, 2, U>), grid, dim3(128), 0, st, p); break;
    case 8: hipLaunchKernelGGL((l4csum_coop_kernel<kKind, kNT, 8, U>), grid, dim3(512), 0, st, p); break;
    case 16: hipLaunchKernelGGL((l4csum_coop_kernel<kKind, kNT, 16, U>), grid, dim3(1024), 0, st, p); break;
    default: hipLaunchKernelGGL((l4csum_coop_kernel<kKind, kNT, 4, U>), grid, dim3(256), 0, st, p); break;
    }
    return WG_OK;
}

// 4 loads in flight per lane: with the work spread over a block's waves the
// rounds are short (16 waves: one round per 64 KiB packet), and U = 4 measured
// 2.7 % faster than 8 on config 1 (profiles/r02_coop_ab.json)
template <int kKind, bool kNT>
static int launch_coop(const L4Params &p, const Tune &t, hipStream_t st) {
    return launch_coop_u<kKind, kNT, 4>(p, t.l4_coop_waves, st);
}

template <int kKind, bool kNT>
static int launch_small(const L4Params &p, uint32_t mode, hipStream_t st) {
    const uint32_t per_block = mode >= 3 ? 64u : 256u;  // descriptors per 256-thread block
    uint64_t blocks = (p.n + per_block - 1) / per_block;
    L4Params q = p;
    if (mode == 5) {
        // quarters of Q descriptors (a multiple of 16: block b owns
        // [q*Q + 16b, +16) of each quarter, whole 4-descriptor groups); 4 Q >= n
        q.quarter = ((p.n + 3) / 4 + 15) & ~15ull;
        blocks = q.quarter / 16;
        if (blocks >= 8)
            blocks = (blocks + 7) & ~7ull;  // XCD swizzle bijective; surplus blocks have no live lane
    }
    if (mode == 6) {  // walking kernel: a wave per 64 descriptors
        blocks = (p.n + 255) / 256;
        if (blocks >= 8)
            blocks = (blocks + 7) & ~7ull;
    }
    if (blocks > 0x7fffffffull)
        return WG_ERR_INVALID;
    const dim3 grid((unsigned)blocks), blk(256);
    const Tune t = tune();
    if (mode == 7) {
        if (t.l4_unroll == 8) {
            auto k = l4csum_persist_kernel<kKind, kNT, 8>;
            hipLaunchKernelGGL(k, dim3((unsigned)persist_grid(p.n, resident_blocks(k))), blk, 0, st, p);
        } else {
            auto k = l4csum_persist_kernel<kKind, kNT, 4>;
            hipLaunchKernelGGL(k, dim3((unsigned)persist_grid(p.n, resident_blocks(k))), blk, 0, st, p);
        }
    } else if (mode == 6) {
        if (t.l4_unroll == 8)
            hipLaunchKernelGGL((l4csum_walk_kernel<kKind, kNT, 8>), grid, blk, 0, st, p);
        else
            hipLaunchKernelGGL((l4csum_walk_kernel<kKind, kNT, 4>), grid, blk, 0, st, p);
    } else if (mode == 5 && t.l4_split_waves == 8) {
        if (t.l4_unroll == 8)
            hipLaunchKernelGGL((l4csum_split_kernel<kKind, kNT, 8, 8>), grid, dim3(512), 0, st, q);
        else
            hipLaunchKernelGGL((l4csum_split_kernel<kKind, kNT, 4, 8>), grid, dim3(512), 0, st, q);
    } else if (mode == 5 && t.l4_unroll == 8)
        hipLaunchKernelGGL((l4csum_split_kernel<kKind, kNT, 8>), grid, blk, 0, st, q);
    else if (mode == 5)
        hipLaunchKernelGGL((l4csum_split_kernel<kKind, kNT>), grid, blk, 0, st, q);
    else if (mode == 4)
        hipLaunchKernelGGL((l4csum_small_kernel<kKind, kNT, 4, 4, true>), grid, blk, 0, st, p);
    else if (mode == 3)
        hipLaunchKernelGGL((l4csum_small_kernel<kKind, kNT, 4, 4>), grid, blk, 0, st, p);
    else if (mode == 2)
        hipLaunchKernelGGL((l4csum_small_kernel<kKind, kNT, 4, 1>), grid, blk, 0, st, p);
    else
        hipLaunchKernelGGL((l4csum_small_kernel<kKind, kNT, 2, 1>), grid, blk, 0, st, p);
    return WG_OK;
}

static int launch_l4(int kind, const L4Params &p, hipStream_t st) {
    if (p.n == 0)
        return WG_OK;
    const Tune t = tune();
    if (kind == kUniformL4 && p.seg <= kSmallMax && t.l4_small_uniform) {
        // every segment is small: the small-packet kernel, no trade-off
        const uint32_t mode = t.l4_small_uniform == 2 ? 2u : 3u;  // 1: lane quad per segment, 2: lane per segment
        const int rc = t.l4_nt ? launch_small<kUniformL4, true>(p, mode, st) : launch_small<kUniformL4, false>(p, mode, st);
        if (rc != WG_OK)
            return rc;
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    if (kind != kUniformL4 && p.n <= t.l4_coop) {
        // few descriptors: a block per packet (config 1's 64 KiB buffers)
        const int rc = kind == kDescL4 ? (t.l4_nt ? launch_coop<kDescL4, true>(p, t, st) : launch_coop<kDescL4, false>(p, t, st))
                                       : (t.l4_nt ? launch_coop<kDescPlain, true>(p, t, st)
                                                  : launch_coop<kDescPlain, false>(p, t, st));
        if (rc != WG_OK)
            return rc;
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    if (kind != kUniformL4 && t.l4_small) {
        int rc;
        if (kind == kDescL4)
            rc = t.l4_nt ? launch_small<kDescL4, true>(p, t.l4_small, st) : launch_small<kDescL4, false>(p, t.l4_small, st);
        else
            rc = t.l4_nt ? launch_small<kDescPlain, true>(p, t.l4_small, st)
                         : launch_small<kDescPlain, false>(p, t.l4_small, st);
        if (rc != WG_OK)
            return rc;
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    const uint32_t P = t.l4_ppw;
    uint64_t want = (p.n + 4ull * P - 1) / (4ull * P);
    if (kind != kUniformL4 && t.l4_descv == 2)  // l4_iters iterations per wave (descriptor prefetch)
        want = (want + t.l4_iters - 1) / t.l4_iters;
    uint64_t blocks = want < t.l4_blocks ? want : t.l4_blocks;
    if (blocks >= 8)
        blocks &= ~7ull;  // keep the XCD swizzle bijective
    const bool nt = t.l4_nt != 0;
    switch (kind) {
    case kUniformL4: launch_kind<kUniformL4>(p, blocks, P, nt, st); break;
    case kDescL4: launch_kind<kDescL4>(p, blocks, P, nt, st); break;
    default: launch_kind<kDescPlain>(p, blocks, P, nt, st); break;
    }
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

// ---------------------------------------------------------------------------
// Decap verify gates: the checksum decisions of
// evaluate_packet (include/worker/evaluator.hpp:112-149): size bounds,
// fill_fk_ip4 (worker/evaluator.cpp:14-40: ihl == 5, len == ip_len, no
// fragmentation, header checksum == 0) or fill_fk_ip6 (:42-58: plen), then
// the TCP / UDP length floors and calc_l4_checksum == 0
// (include/worker/evaluator.hpp:59-65, 89-94).  Per wave P packets, all loads
// issued straight after the descriptors: one byte load per packet brings
// header bytes 0-39 (decoded with v_readlane), the L4 issue machinery streams
// bytes [40, len), which belong to the L4 region whatever the family; the
// header bytes [ihs, 40) and the pseudo-header addresses are added from the
// byte load once the header is decoded.
// ---------------------------------------------------------------------------
typedef unsigned int v16u __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(4))) const v16u c_v16u;  // constant address space: scalar loads
typedef __attribute__((address_space(4))) const uint32_t c_u32;

struct VerifyParams {
    const uint8_t *base;
    const wg_pkt_desc *desc;  // null: a uniform PacketBatch (seg, total_len)
    uint8_t *verdict;
    uint16_t *l4;
    uint64_t n;
    uint64_t total_len = 0;
    uint32_t seg = 0;
    uint32_t last_len = 0;  // uniform: length of segment n - 1 (the only one that may be short)
    uint32_t *sample = nullptr;  // host-mapped word: small packets among 64 spread descriptors (verify_sample)
};

// The size mix of a descriptor batch, for the NEXT call's kernel choice
// (wg_verify_desc, verify_small = 7): lane k reads descriptor k*n/64 and the
// wave stores into two host-mapped words how many of those 64 packets are
// <= kSmallMax bytes and the summed length of the others (two dword stores;
// the host reads them without waiting).
__device__ __forceinline__ void verify_sample(const VerifyParams &p, uint32_t lane) {
    constexpr uint32_t kSmallLen = 64;  // = kSmallMax (declared with the small-packet kernels)
    const uint64_t i = ((uint64_t)lane * p.n) >> 6;
    const uint32_t len = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * i).z;
    const bool small = len <= kSmallLen;
    const uint32_t s = (uint32_t)__builtin_popcountll(__ballot(small));
    const uint32_t lb = wave_sum_u32(small ? 0u : (len < 65535u ? len : 65535u));
    if (lane < 2)
        __hip_atomic_store(p.sample + lane, lane ? lb : s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t j) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j);
}

// One group of P packets by the whole wave: ISSUE (header bytes and the
// packet bytes from 32 / 40 on), then `mid` (the caller's descriptor
// prefetch), then decode + finish; packet j's verdict and L4 result land in
// lane tgt[j]'s rv / rc.  Shared by verify_kernel and the long packets of
// verify_small_kernel.
template <int P, bool H, typename Mid>
__device__ __forceinline__ void verify_group(const uint8_t *base, const uint64_t *doff, const uint32_t *len,
                                             const uint32_t *tgt, uint32_t lane, uint32_t &rv, uint32_t &rc,
                                             Mid mid) {
    const uintptr_t zero = reinterpret_cast<uintptr_t>(&g_zero16);
    Geom g[P];
    Front f[P];
    uint32_t hv[P];
    // ISSUE, before any header is decoded: header bytes 0-39 one per lane,
    // and bytes [40, len) — inside the L4 region for IPv4 (ihs 20) and IPv6
    // (ihs 40) alike — through the L4 wave's issue phase.  Decoding first
    // would put a second memory round trip in front of the payload loads.
    // (Bytes of packets that then fail a gate are read but not used; every
    // read lies inside the descriptor's packet.)
#pragma unroll
    for (int j = 0; j < P; j++) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(base) + doff[j];
        g[j].a = a;
        g[j].fl = 0;
        if constexpr (H) {
            // longer packets fail the size gate (evaluator.hpp:118-121): only
            // their header bytes are read (region [32, 32) is empty)
            g[j].len = len[j] <= 65535u ? len[j] : 32u;
            g[j].cs = 32;
            issue<false, true, true>(g[j], lane, f[j]);
            hv[j] = f[j].hb;
        } else {
            const uint32_t hl = len[j] < 40u ? len[j] : 40u;
            hv[j] = ld8(hl ? a + (lane < hl ? lane : 0u) : zero);
            g[j].len = len[j] <= 65535u ? len[j] : 0u;
            g[j].cs = 40;
            issue<false, true>(g[j], lane, f[j]);
        }
    }
    mid();
    // decode (wave-uniform) and finish every packet
#pragma unroll
    for (int j = 0; j < P; j++) {
        const uint32_t L = len[j];
        uint32_t v = 0;
        bool ip_ok = false, tcp = false, l4 = false, v6 = false;
        uint32_t ihs = 20, proto = 0;
        // header byte `lane` in packet pairing (from byte 0); zero from lane
        // 32 (H) / 40 on and past the packet
        constexpr uint32_t kHdrEnd = H ? 32u : 40u;
        const uint32_t hb = lane < L && lane < kHdrEnd ? hv[j] << (8u * (lane & 1u)) : 0u;
        // IPv4 header sum over bytes 0-19
        const uint32_t hs = wave_sum_u32(lane < 20u ? hb : 0u);
        if (L >= 1) {
            const uint32_t b0 = rl(hv[j], 0);
            v6 = (b0 >> 4) == 6;
            if (v6)
                v |= WG_VERDICT_V6;
            ihs = v6 ? 40u : 20u;
            if (L >= ihs && L <= 65535u) {  // evaluator.hpp:118-121
                if (!v6) {
                    ip_ok = (b0 & 0xfu) == 5u &&                                   // ip_hl, evaluator.cpp:19
                            L == ((rl(hv[j], 2) << 8) | rl(hv[j], 3)) &&            // ip_len, :21
                            (((rl(hv[j], 6) << 8) | rl(hv[j], 7)) & ~0x4000u) == 0 &&  // ip_off & ~IP_DF, :24
                            fold16_32(hs) == 0xffffu;                             // checksum == 0, :27
                    proto = rl(hv[j], 9);
                } else {
                    ip_ok = L - 40u == ((rl(hv[j], 4) << 8) | rl(hv[j], 5));  // ip6_plen, :47
                    proto = rl(hv[j], 6);
                }
                if (ip_ok) {
                    v |= WG_VERDICT_IP_OK;
                    if (proto == 6u) {
                        v |= WG_VERDICT_TCP;
                        tcp = true;
                        l4 = L - ihs > 20u;  // evaluator.hpp:61
                    } else if (proto == 17u) {
                        v |= WG_VERDICT_UDP;
                        l4 = L - ihs > 8u;  // evaluator.hpp:91
                    }
                }
            }
        }
        // calc_l4_checksum(pkt, isv6, istcp, ihs) (checksum.cpp:8-36): bytes
        // [E, L) (issued above; E = 32 or 40) + header bytes [ihs, E) + the
        // pseudo-header addresses (v4 12-19, v6 8-39) below E, all in packet
        // pairing — ihs, E and the address offsets are even, so that is the
        // reference's pairing.  (v6 with E = 32: address bytes 32-39 are in
        // the issued region, and its L4 region starts at 40: each counted once.)
        const bool inl4 = lane >= ihs;  // hb is zero from lane E on
        const bool inps = v6 ? lane >= 8u : (lane >= 12u && lane < 20u);
        uint32_t s = wave_sum_u32(finish<true>(lane, f[j]) + (inl4 ? hb : 0u) + (inps ? hb : 0u));
        uint32_t c = 0;
        if (l4) {
            s += ((tcp ? 6u : 17u) << 8) + bswap16((L - ihs) & 0xffffu);
            c = ~fold16_32(s) & 0xffffu;
            if (c == 0)
                v |= WG_VERDICT_L4_OK;
        }
        if (lane == tgt[j]) {
            rv = v;
            rc = c;
        }
    }
}

// H: header bytes 0-31 ride in the L4 byte gather's idle lanes (issue<.., kHdr>)
// and the summed region starts at byte 32 — no separate header load; else a
// byte load of header bytes 0-39 per packet and the region from byte 40.
// kUni: a uniform PacketBatch instead of descriptors (wg_verify_uniform).
// kD64: a whole group's 4 descriptors (64 B) by one scalar load instead of a
// load per descriptor (which the compiler issues one after another, each
// waited for).
template <int P, int O = 0, int DM = 0, bool H = false, bool kUni = false, bool kD64 = false>  // O: waves/SIMD target (0 = compiler's choice); DM: descriptor mode 0 / 2
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(O ? O : 1, O ? O : 8))) void verify_kernel(
    VerifyParams p) {
    const uint32_t lane = lane_id();
    const uint64_t wave0 = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t step = (uint64_t)gridDim.x * 4u * P;
    const uintptr_t zero = reinterpret_cast<uintptr_t>(&g_zero16);
    // DM 2 (as the descriptor-batch L4 kernel): the next iteration's
    // descriptors by one vector load, in flight during this one's finish.
    // DM 0: one iteration per wave (the launcher covers the batch).
    v4u nextd = v4u{0, 0, 0, 0};
    bool have_next = false;
    for (uint64_t i0 = wave0 * P; i0 < p.n; i0 += step) {
    uint32_t len[P];
    uint64_t doff[P];
    if (DM == 2 && have_next) {
#pragma unroll
        for (int j = 0; j < P; j++) {
            doff[j] = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)nextd.x, j) |
                      ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)nextd.y, j) << 32);
            len[j] = i0 + j < p.n ? (uint32_t)__builtin_amdgcn_readlane((int)nextd.z, j) : 0u;
        }
    } else if (kUni) {
        // PacketBatch segment i0 + j (include/util/packets.hpp:23-36): one
        // 64-bit multiply and compare per wave (a 64-bit scalar compare has
        // no SALU form on gfx9, and this kernel's scalar unit is busy)
        const uint64_t o0 = i0 * (uint64_t)p.seg;
        const bool full = i0 + P < p.n;  // every segment of the group whole
#pragma unroll
        for (int j = 0; j < P; j++) {
            doff[j] = o0 + (uint32_t)j * p.seg;
            len[j] = full ? p.seg : (i0 + j + 1 < p.n ? p.seg : (i0 + j + 1 == p.n ? p.last_len : 0u));
        }
    } else if (kD64 && P == 4 && i0 + P <= p.n) {
        const v16u dd = *reinterpret_cast<const c_v16u *>(reinterpret_cast<uintptr_t>(p.desc + i0));
#pragma unroll
        for (int j = 0; j < P; j++) {
            doff[j] = ((uint64_t)dd[4 * j + 1] << 32) | dd[4 * j];
            len[j] = dd[4 * j + 2];
        }
    } else {
#pragma unroll
        for (int j = 0; j < P; j++) {
            const wg_pkt_desc d = p.desc[i0 + j < p.n ? i0 + j : p.n - 1];
            doff[j] = d.offset;
            len[j] = i0 + j < p.n ? d.len : 0u;
        }
    }
    uint32_t rv = 0, rc = 0;
    uint32_t tgt[P];
#pragma unroll
    for (int j = 0; j < P; j++)
        tgt[j] = (uint32_t)j;
    verify_group<P, H>(p.base, doff, len, tgt, lane, rv, rc, [&]() {
        if constexpr (DM == 2) {
            have_next = i0 + step < p.n;
            const uint64_t di = (have_next ? i0 + step : i0) + (lane & (uint32_t)(P - 1));
            nextd = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (di < p.n ? di : p.n - 1));
        }
    });
    if (lane < (uint32_t)P && i0 + lane < p.n) {
        p.verdict[i0 + lane] = (uint8_t)rv;
        if (p.l4)
            p.l4[i0 + lane] = (uint16_t)rc;
    }
    if constexpr (DM == 0)
        break;
    }
    if constexpr (!kUni) {
        if (p.sample && blockIdx.x == 0 && wave_in_block() == 0)
            verify_sample(p, lane);
    }
}

}  // namespace wg

using namespace wg;

namespace wg {

// Small-packet verify (knob verify_small; the same split as
// l4csum_small_kernel): a lane per descriptor.  A packet of <= kSmallMax
// bytes is decoded and summed in its lane from its five aligned 16-B chunks,
// funnel-shifted (v_alignbyte) into 16 packet-relative dwords R[0..15] with
// the bytes past the packet zeroed, so every gate field sits at a static
// byte position and every summed range (header [0, 20), L4 [ihs, len), the
// addresses) starts at an even packet offset: packet pairing throughout, as
// the reference pairs them.  The wave then takes the lanes with longer
// packets Q at a time through verify_group.

// G = 4: a lane quad per descriptor, every lane of it decoding the same
// packet (its loads hit the same addresses): a wave owns 16 descriptors, so
// its serial walk over the long packets is 4 groups instead of 16.
// The packets of the lanes in mask m (lane j: offset ohi:olo, length len),
// Q at a time through verify_group; packet j's verdict / L4 result land in
// lane j's rv / rc.
template <int Q>
__device__ __forceinline__ void verify_mask(uint64_t m, uint32_t olo, uint32_t ohi, uint32_t len, const uint8_t *base,
                                            uint32_t lane, uint32_t &rv, uint32_t &rc) {
    while (m) {
        uint64_t doff[Q];
        uint32_t ln[Q], tgt[Q];
#pragma unroll
        for (int k = 0; k < Q; k++) {
            const bool have = m != 0;
            const uint32_t j = have ? (uint32_t)__builtin_ctzll(m) : 0u;
            m = have ? m & (m - 1) : m;
            tgt[k] = have ? j : 64u;
            doff[k] = have ? (((uint64_t)rdl(ohi, j) << 32) | rdl(olo, j)) : 0u;
            ln[k] = have ? rdl(len, j) : 0u;
        }
        verify_group<Q, true>(base, doff, ln, tgt, lane, rv, rc, [] {});
    }
}

// The lane path of the small-packet verify kernels: packet (a, len), len <=
// kSmallMax, decoded and checked in one lane; verdict bits into rv, the L4
// result into rc.
// Its loads: the packet's five aligned 16-B chunks (clamped chunks lie past
// the packet and are zeroed by the decode).
__device__ __forceinline__ void verify_lane_load(uintptr_t a, uint32_t len, bool use, v4u W[5]) {
    const uintptr_t zero = reinterpret_cast<uintptr_t>(&g_zero16);
    const uintptr_t a0 = a & ~(uintptr_t)15;
    const uintptr_t alast = (a + len - 1) & ~(uintptr_t)15;
    const bool any = use && len;
#pragma unroll
    for (uint32_t c = 0; c < 5; c++) {
        const uintptr_t ca = a0 + 16u * c;
        W[c] = ld16(any ? (ca > alast ? alast : ca) : zero);
    }
}

__device__ __forceinline__ void verify_lane_decode(const v4u W[5], uintptr_t a, uint32_t len, uint32_t &rv,
                                                   uint32_t &rc);

__device__ __forceinline__ void verify_lane(uintptr_t a, uint32_t len, bool use, uint32_t &rv, uint32_t &rc) {
    v4u W[5];
    verify_lane_load(a, len, use, W);
    verify_lane_decode(W, a, len, rv, rc);
}

__device__ __forceinline__ void verify_lane_decode(const v4u W[5], uintptr_t a, uint32_t len, uint32_t &rv,
                                                   uint32_t &rc) {
    const uint32_t Wd[20] = {W[0][0], W[0][1], W[0][2], W[0][3], W[1][0], W[1][1], W[1][2], W[1][3],
                             W[2][0], W[2][1], W[2][2], W[2][3], W[3][0], W[3][1], W[3][2], W[3][3],
                             W[4][0], W[4][1], W[4][2], W[4][3]};
    const uint32_t s = (uint32_t)(a & 15u), q4 = s >> 2, sh = s & 3u;
    uint32_t R[16];
#pragma unroll
    for (uint32_t m = 0; m < 16; m++) {
        const uint32_t lo = q4 == 0 ? Wd[m] : q4 == 1 ? Wd[m + 1] : q4 == 2 ? Wd[m + 2] : Wd[m + 3];
        const uint32_t hi = q4 == 0 ? Wd[m + 1] : q4 == 1 ? Wd[m + 2] : q4 == 2 ? Wd[m + 3] : Wd[m + 4];
        R[m] = bytes_below(__builtin_amdgcn_alignbyte(hi, lo, sh), m, len);
    }
    uint32_t v = 0, c = 0;
    if (len >= 1) {
        const uint32_t b0 = R[0] & 0xffu;
        const bool v6 = (b0 >> 4) == 6;
        if (v6)
            v |= WG_VERDICT_V6;
        const uint32_t ihs = v6 ? 40u : 20u;
        bool ip_ok = false;
        uint32_t proto = 0;
        if (len >= ihs) {  // evaluator.hpp:118-121 (len <= 64 here)
            if (!v6) {
                const uint32_t hs = half_sum(R[0]) + half_sum(R[1]) + half_sum(R[2]) + half_sum(R[3]) +
                                    half_sum(R[4]);
                ip_ok = (b0 & 0xfu) == 5u &&                                  // ip_hl, evaluator.cpp:19
                        len == bswap16(R[0] >> 16) &&                          // ip_len, :21
                        (bswap16(R[1] >> 16) & ~0x4000u) == 0 &&              // ip_off & ~IP_DF, :24
                        fold16_32(hs) == 0xffffu;                             // checksum == 0, :27
                proto = (R[2] >> 8) & 0xffu;
            } else {
                ip_ok = len - 40u == bswap16(R[1] & 0xffffu);  // ip6_plen, :47
                proto = (R[1] >> 16) & 0xffu;
            }
        }
        bool l4 = false;
        if (ip_ok) {
            v |= WG_VERDICT_IP_OK;
            if (proto == 6u) {
                v |= WG_VERDICT_TCP;
                l4 = len - ihs > 20u;  // evaluator.hpp:61
            } else if (proto == 17u) {
                v |= WG_VERDICT_UDP;
                l4 = len - ihs > 8u;  // evaluator.hpp:91
            }
        }
        if (l4) {  // calc_l4_checksum(pkt, isv6, istcp, ihs), checksum.cpp:8-36
            uint32_t sum = (proto << 8) + bswap16((len - ihs) & 0xffffu);
#pragma unroll
            for (uint32_t m = 2; m < 16; m++) {
                const bool in_l4 = 4u * m >= ihs;
                const bool in_addr = v6 ? m < 10u : (m == 3u || m == 4u);  // v6 bytes 8-39, v4 12-19
                sum += (in_l4 ? half_sum(R[m]) : 0u) + (in_addr ? half_sum(R[m]) : 0u);
            }
            c = ~fold16_32(sum) & 0xffffu;
            if (c == 0)
                v |= WG_VERDICT_L4_OK;
        }
    }
    rv = v;
    rc = c;
}

template <int Q, int G = 1>
__global__ __launch_bounds__(256) void verify_small_kernel(VerifyParams p) {
    static_assert(G == 1 || G == 4, "lanes per descriptor");
    const uint32_t lane = lane_id();
    const uint32_t q = lane & (uint32_t)(G - 1);
    const uint64_t i = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * (256u / G) + threadIdx.x / G;
    const bool live = i < p.n;
    const v4u dv = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0));
    const uint32_t len = live ? dv.z : 0u;
    const uint32_t olo = live ? dv.x : 0u, ohi = live ? dv.y : 0u;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p.base) + (((uint64_t)ohi << 32) | olo);
    const bool small = len <= kSmallMax;
    uint32_t rv = 0, rc = 0;
    if (__ballot(live && small))
        verify_lane(a, len, small, rv, rc);
    // the longer packets of this wave, Q at a time
    verify_mask<Q>(__ballot(live && !small && q == 0), olo, ohi, len, p.base, lane, rv, rc);
    if (live && q == 0) {
        p.verdict[i] = (uint8_t)rv;
        if (p.l4)
            p.l4[i] = (uint16_t)rc;
    }
}

// Split-role verify kernel (knob verify_small = 3; the layout and the role
// split of l4csum_split_kernel): block b owns the 16 descriptors at
// [q*Q + 16b, +16) of each quarter q; groups of 4 consecutive descriptors
// whose packets are all <= kSmallMax bytes are decoded a lane per packet by
// wave 0, every other group by its wave through verify_group, 4 at a time.
template <int O = 0>  // O: waves/SIMD target (0 = compiler's choice)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(O ? O : 1, O ? O : 8))) void verify_split_kernel(VerifyParams p, uint64_t Q) {
    const uint32_t lane = lane_id();
    const uint32_t wib = wave_in_block();
    const uint64_t blk = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint32_t qq = wib == 0 ? lane >> 4 : (lane >> 2) & 3u;
    const uint32_t oo = wib == 0 ? lane & 15u : 4u * wib + (lane & 3u);
    const uint64_t i = (uint64_t)qq * Q + 16u * blk + oo;
    const bool live = (wib == 0 || lane < 16u) && 16u * blk < Q && i < p.n;
    const v4u d = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : p.n - 1));
    const uint32_t len = live ? d.z : 0u;
    const uint32_t olo = live ? d.x : 0u, ohi = live ? d.y : 0u;
    const uint64_t gl = __ballot(live && len > kSmallMax);
    const bool grp_long = ((gl >> (lane & ~3u)) & 0xfu) != 0;
    const bool own = wib == 0 ? (lane & 15u) < 4u : true;
    const bool mine = live && own && grp_long;
    uint32_t rv = 0, rc = 0;
    verify_mask<4>(__ballot(mine), olo, ohi, len, p.base, lane, rv, rc);
    const bool small = wib == 0 && live && !grp_long;
    if (__ballot(small)) {  // wave-uniform; never true on waves 1-3
        uint32_t sv = 0, sc = 0;
        verify_lane(reinterpret_cast<uintptr_t>(p.base) + (((uint64_t)ohi << 32) | olo), small ? len : 0u, small, sv,
                    sc);
        rv = small ? sv : rv;
        rc = small ? sc : rc;
    }
    if (mine || small) {
        p.verdict[i] = (uint8_t)rv;
        if (p.l4)
            p.l4[i] = (uint16_t)rc;
    }
}

// ---------------------------------------------------------------------------
// Two-role verify (knob verify_small 4 and 5).  The wave-per-packet kernel is
// fastest on long packets as one-shot 4-packet waves at 8 waves/SIMD, and the
// lane decode is fastest on small ones at 64 descriptors per wave; any layout
// that puts both roles in one wave costs the long packets occupancy or
// one-shot waves (verify_small 1-3).  Here the roles get separate waves:
//  - LANE role: a lane per descriptor; packets of <= kSmallMax bytes are
//    decoded in their lane (verify_lane), longer ones left alone;
//  - WAVE role: one-shot waves of 4 consecutive descriptors through
//    verify_group (the default kernel's body), taking only the packets longer
//    than kSmallMax; a wave whose 4 packets are all small exits after its
//    descriptor load.
// Every descriptor's result is stored by exactly one role.  verify_small = 4
// runs the roles as two launches, 5 as the two block ranges of one launch.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void verify_lane_role(const VerifyParams &p, uint64_t i) {
    const bool live = i < p.n;
    const v4u dv = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0));
    const uint32_t len = live ? dv.z : 0u;
    const bool small = live && len <= kSmallMax;
    if (!__ballot(small))  // wave-uniform: nothing small here
        return;
    uint32_t rv = 0, rc = 0;
    verify_lane(reinterpret_cast<uintptr_t>(p.base) + (((uint64_t)dv.y << 32) | dv.x), small ? len : 0u, small, rv,
                rc);
    if (small) {
        p.verdict[i] = (uint8_t)rv;
        if (p.l4)
            p.l4[i] = (uint16_t)rc;
    }
}

__device__ __forceinline__ void verify_wave_role(const VerifyParams &p, uint64_t i0, uint32_t lane) {
    constexpr int P = 4;
    uint64_t doff[P];
    uint32_t len[P], tgt[P];
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < P; j++) {
        const wg_pkt_desc d = p.desc[i0 + j < p.n ? i0 + j : p.n - 1];
        const uint32_t L = i0 + j < p.n ? d.len : 0u;
        const bool lg = L > kSmallMax;
        keep |= (uint32_t)lg << j;
        doff[j] = d.offset;
        len[j] = lg ? L : 0u;  // the lane role's packets: nothing issued
        tgt[j] = (uint32_t)j;
    }
    if (!keep)
        return;
    uint32_t rv = 0, rc = 0;
    verify_group<P, true>(p.base, doff, len, tgt, lane, rv, rc, [] {});
    if (lane < (uint32_t)P && ((keep >> lane) & 1u)) {
        p.verdict[i0 + lane] = (uint8_t)rv;
        if (p.l4)
            p.l4[i0 + lane] = (uint16_t)rc;
    }
}

__global__ __launch_bounds__(256) void verify_lane_kernel(VerifyParams p) {
    verify_lane_role(p, (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 256u + threadIdx.x);
}

// wg_verify_uniform with segment_size <= kSmallMax: every segment is small,
// so a lane per segment decodes it (no descriptors, no wave role).
__global__ __launch_bounds__(256) void verify_uniform_lane_kernel(VerifyParams p) {
    const uint64_t i = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 256u + threadIdx.x;
    const bool live = i < p.n;
    const uint64_t o = live ? i * (uint64_t)p.seg : 0u;
    const uint32_t len = live ? (p.total_len - o < p.seg ? (uint32_t)(p.total_len - o) : p.seg) : 0u;
    uint32_t rv = 0, rc = 0;
    verify_lane(reinterpret_cast<uintptr_t>(p.base) + o, len, live, rv, rc);
    if (live) {
        p.verdict[i] = (uint8_t)rv;
        if (p.l4)
            p.l4[i] = (uint16_t)rc;
    }
}

template <int O = 0, int BW = 4>  // BW: waves per block (4, or 16: fewer workgroups to dispatch)
__global__ __launch_bounds__(64 * BW) __attribute__((amdgpu_waves_per_eu(O ? O : 1, O ? O : 8))) void verify_long_kernel(
    VerifyParams p) {
    const uint64_t wave = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * (uint32_t)BW + wave_in_block();
    if (wave * 4u < p.n)
        verify_wave_role(p, wave * 4u, lane_id());
}

// One launch: blocks [0, nl) lane role (256 descriptors each), the rest wave
// role (16 descriptors each); both ranges multiples of 8 blocks (XCD swizzle).
template <int O = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(O ? O : 1, O ? O : 8))) void verify_roles_kernel(
    VerifyParams p, uint32_t nl) {
    if (blockIdx.x < nl) {
        verify_lane_role(p, (uint64_t)xcd_swizzle(blockIdx.x, nl) * 256u + threadIdx.x);
        return;
    }
    const uint64_t wave = (uint64_t)xcd_swizzle(blockIdx.x - nl, gridDim.x - nl) * 4u + wave_in_block();
    if (wave * 4u < p.n)
        verify_wave_role(p, wave * 4u, lane_id());
}

// ---------------------------------------------------------------------------
// Compacting verify (verify_small 6; 7 chooses per call between it and the
// wave kernel).  Two launches whose wave counts follow the batch's size mix
// instead of its descriptor count:
//  - verify_compact_lane_kernel, a lane per descriptor (n / 64 waves):
//    packets of <= kSmallMax bytes are decoded in their lane (verify_lane);
//    the longer ones are appended as 16-B entries {offset, len, index} to the
//    list of shard (blockIdx & 31) — one returning atomic per block, after the
//    block's four waves have counted their long lanes in LDS;
//  - verify_compact_long_kernel: waves take 4 consecutive entries of their
//    block's shard through verify_group (the wave kernel's body, 8
//    waves/SIMD) and store by index, grid-stride over the shard, so any grid
//    is correct and the host sizes it from the expected long count.
// A batch of ACK-sized packets thus costs n / 64 lane waves and an almost
// empty second launch, where n / 4 one-shot waves (the wave kernel, or any
// role split sized by descriptor count) cost ~30 us of wave launches alone
// (profiles/r03_verify_ab.json, verify_small 4 / 5 at 64 B).
// The counters come in two sets; a call uses set `parity` and its lane
// kernel zeroes the other, which the previous call's long kernel has finished
// reading (stream order), so no memset is launched per call.
// ---------------------------------------------------------------------------
constexpr uint32_t kVShards = 32;  // 4 per XCD: one returning atomic per word saturates at ~88/us
constexpr uint32_t kVCtrStride = 32;  // words between counters: a 128-B line each

struct VerifyCompact {
    v4u *ent;            // shard s's list at ent + s * cap
    uint64_t cap;        // entries per shard (>= 256 * ceil(lane-kernel blocks / 8))
    uint32_t *ctr;       // this call's counters (kVShards, stride kVCtrStride)
    uint32_t *ctr_next;  // the next call's, zeroed here
};

__global__ __launch_bounds__(256) void verify_compact_lane_kernel(VerifyParams p, VerifyCompact c) {
    __shared__ uint32_t s_cnt[4];
    __shared__ uint32_t s_base;
    const uint32_t lane = lane_id();
    const uint32_t wib = wave_in_block();
    const uint64_t i = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 256u + threadIdx.x;
    const bool live = i < p.n;
    const v4u dv = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0));
    const uint32_t len = live ? dv.z : 0u;
    const bool small = live && len <= kSmallMax;
    const bool lng = live && !small;
    if (blockIdx.x == 0 && threadIdx.x < kVShards)
        c.ctr_next[threadIdx.x * kVCtrStride] = 0;
    // the small packets: loads issued before the block synchronises
    uint32_t rv = 0, rc = 0;
    if (__ballot(small))  // wave-uniform
        verify_lane(reinterpret_cast<uintptr_t>(p.base) + (((uint64_t)dv.y << 32) | dv.x), small ? len : 0u, small,
                    rv, rc);
    // the long packets: block-aggregated append to this block's shard
    const uint64_t ml = __ballot(lng);
    if (lane == 0)
        s_cnt[wib] = (uint32_t)__builtin_popcountll(ml);
    __syncthreads();
    const uint32_t tot = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    if (tot) {  // block-uniform
        const uint32_t sh = blockIdx.x & (kVShards - 1);
        if (threadIdx.x == 0)
            s_base = atomicAdd(&c.ctr[sh * kVCtrStride], tot);
        __syncthreads();
        if (lng) {
            const uint32_t pre = (wib > 0 ? s_cnt[0] : 0u) + (wib > 1 ? s_cnt[1] : 0u) + (wib > 2 ? s_cnt[2] : 0u);
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(ml >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ml, 0u));
            c.ent[sh * c.cap + s_base + pre + r] = v4u{dv.x, dv.y, len, (uint32_t)i};
        }
    }
    if (small) {
        p.verdict[i] = (uint8_t)rv;
        if (p.l4)
            p.l4[i] = (uint16_t)rc;
    }
    if (p.sample && blockIdx.x == 0 && wib == 0)
        verify_sample(p, lane);
}

template <int O = 8, bool kLoop = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(O ? O : 1, O ? O : 8))) void verify_compact_long_kernel(
    VerifyParams p, VerifyCompact c) {
    constexpr int P = 4;
    __shared__ uint32_t s_idx[4][P];
    const uint32_t lane0 = lane_id();
    const uint32_t sh = blockIdx.x & (kVShards - 1);
    const uint32_t step = (gridDim.x / kVShards) * 4u * P;  // grid: a multiple of kVShards (32-bit: a shard's entries < 2^32)
    // The list and its count were written by the lane kernel (an earlier
    // launch) and are only read here: constant-address-space loads, so the
    // 4 entries (64 B) and the count are two scalar loads issued together.
    const c_v16u *e = reinterpret_cast<const c_v16u *>(reinterpret_cast<uintptr_t>(c.ent + sh * c.cap));
    uint32_t k0 = ((blockIdx.x / kVShards) * 4u + wave_in_block()) * P;
    v16u d = e[(k0 < c.cap ? k0 : c.cap - P) / P];  // past the count: read, not used
    const uint32_t cnt = *reinterpret_cast<const c_u32 *>(reinterpret_cast<uintptr_t>(c.ctr + sh * kVCtrStride));
    asm volatile("" ::"s"(d[0]), "s"(cnt));  // both in flight before the first wait
    while (k0 < cnt) {
        // the lane id laundered per iteration: the lane-derived constants of
        // verify_group are then recomputed in the body instead of hoisted and
        // held across the loop (which spilled at 64 VGPRs)
        uint32_t lane = lane0;
        asm volatile("" : "+v"(lane));
        uint64_t doff[P];
        uint32_t len[P], tgt[P];
#pragma unroll
        for (int j = 0; j < P; j++) {
            doff[j] = ((uint64_t)d[4 * j + 1] << 32) | d[4 * j];
            len[j] = k0 + j < cnt ? d[4 * j + 2] : 0u;
            tgt[j] = (uint32_t)j;
        }
        // the packets' indices parked in this wave's LDS words across the
        // group (held in registers they spill)
        if (lane < (uint32_t)P)
            s_idx[wave_in_block()][lane] = lane == 0 ? d[3] : lane == 1 ? d[7] : lane == 2 ? d[11] : d[15];
        uint32_t rv = 0, rc = 0;
        verify_group<P, true>(p.base, doff, len, tgt, lane, rv, rc, [] {});
        if (lane < (uint32_t)P && k0 + lane < cnt) {
            const uint32_t at = s_idx[wave_in_block()][lane];
            p.verdict[at] = (uint8_t)rv;
            if (p.l4)
                p.l4[at] = (uint16_t)rc;
        }
        if constexpr (!kLoop)
            break;
        k0 += step;
        if (k0 < cnt)
            d = e[k0 / P];
    }
}

// Walking verify (verify_small = 8): one launch of n / 64 waves whatever the
// size mix, the layout of l4csum_walk_kernel (lane l of wave w of G owns
// descriptor ((l >> 2) * G + w) * 4 + (l & 3): the resident waves work on one
// narrow window of the batch).  Packets of <= kSmallMax bytes are decoded in
// their lane (verify_lane); the wave then walks its longer packets in group
// order, 4 at a time, through verify_group.  Stateless: no host sample, no
// lists, nothing carried between calls.
// One round of the walking verify: lane l holds descriptor i (of group
// g = i / 4); small packets in their lane, long ones 4 at a time through
// verify_group with their offsets / lengths parked in LDS (s_geo: this wave's
// 3 x 64 words), results stored by index.
__device__ __forceinline__ void verify_walk_round(const VerifyParams &p, uint64_t i, uint32_t *s_geo) {
    const uint32_t lane = lane_id();
    const bool live = i < p.n;
    const v4u dv = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0u));
    const uint32_t len = live ? dv.z : 0u;
    const uint32_t olo = live ? dv.x : 0u, ohi = live ? dv.y : 0u;
    const bool small = live && len <= kSmallMax;
    uint32_t rv = 0, rc = 0;
    if (__ballot(small))  // wave-uniform
        verify_lane(reinterpret_cast<uintptr_t>(p.base) + (((uint64_t)ohi << 32) | olo), small ? len : 0u, small, rv,
                    rc);
    uint32_t r = rv | (rc << 8);  // one register across the walk
    uint64_t m = __ballot(live && !small);
    if (m) {
        s_geo[lane] = olo;
        s_geo[64 + lane] = ohi;
        s_geo[128 + lane] = len;
    }
    while (m) {
        uint32_t ln = lane_id();
        asm volatile("" : "+v"(ln));
        uint64_t doff[4];
        uint32_t lg[4], tgt[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool have = m != 0;
            const uint32_t j = have ? (uint32_t)__builtin_ctzll(m) : 0u;
            m = have ? m & (m - 1) : m;
            tgt[k] = have ? j : 64u;
            const uint32_t x = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_geo[j]);
            const uint32_t y = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_geo[64 + j]);
            const uint32_t z = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_geo[128 + j]);
            doff[k] = have ? (((uint64_t)y << 32) | x) : 0u;
            lg[k] = have ? z : 0u;
        }
        uint32_t v2 = 0, c2 = 0;
        verify_group<4, true>(p.base, doff, lg, tgt, ln, v2, c2, [] {});
        r = (ln == tgt[0] || ln == tgt[1] || ln == tgt[2] || ln == tgt[3]) ? (v2 | (c2 << 8)) : r;
    }
    if (live) {
        p.verdict[i] = (uint8_t)r;
        if (p.l4)
            p.l4[i] = (uint16_t)(r >> 8);
    }
}

// Persistent walking verify (verify_small = 9): the grid is the resident
// capacity (or n / 64 waves if fewer); wave w takes rounds of 16 groups,
// lane l of round r holding descriptor ((16 r + (l >> 2)) * G + w) * 4 + (l & 3):
// every wave gets the same number of groups to within one (l4csum_persist_kernel).
template <int O = 8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(O ? O : 1, O ? O : 8))) void verify_persist_kernel(
    VerifyParams p) {
    __shared__ uint32_t s_geo[4][3 * 64];
    const uint64_t G = (uint64_t)gridDim.x * 4u;
    const uint32_t wib = wave_in_block();
    const uint64_t w = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wib;
    for (uint64_t r0 = 0; r0 * G * 4u < p.n; r0 += 16) {
        uint32_t lane = lane_id();
        asm volatile("" : "+v"(lane));
        verify_walk_round(p, ((r0 + (lane >> 2)) * G + w) * 4u + (lane & 3u), s_geo[wib]);
    }
}

// Walk the long packets of mask m 4 at a time through verify_group, their
// geometry (olo / ohi / len of lane j) read from this wave's LDS words; each
// packet's verdict | L4 result << 8 lands in its lane's r.
__device__ __forceinline__ void verify_walk_lds(const VerifyParams &p, uint64_t m, const uint32_t *s_geo,
                                                uint32_t &r) {
    while (m) {
        // the lane id laundered per iteration: verify_group's lane-derived
        // constants are recomputed in the body, not held across the loop
        uint32_t ln = lane_id();
        asm volatile("" : "+v"(ln));
        uint64_t doff[4];
        uint32_t lg[4], tgt[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool have = m != 0;
            const uint32_t j = have ? (uint32_t)__builtin_ctzll(m) : 0u;
            m = have ? m & (m - 1) : m;
            tgt[k] = have ? j : 64u;
            const uint32_t x = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_geo[j]);
            const uint32_t y = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_geo[64 + j]);
            const uint32_t z = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_geo[128 + j]);
            doff[k] = have ? (((uint64_t)y << 32) | x) : 0u;
            lg[k] = have ? z : 0u;
        }
        uint32_t v2 = 0, c2 = 0;
        verify_group<4, true>(p.base, doff, lg, tgt, ln, v2, c2, [] {});
        r = (ln == tgt[0] || ln == tgt[1] || ln == tgt[2] || ln == tgt[3]) ? (v2 | (c2 << 8)) : r;
    }
}

// Split-role verify at 8 waves/SIMD (verify_small = 10): the layout of
// l4csum_split_kernel — block b owns the 16 descriptors [q*Q + 16b, +16) of
// each quarter q; wave k walks its own group of each quarter that holds a
// packet longer than kSmallMax (4 groups a quarter batch apart, as the
// wave-per-packet kernel's waves would take them); wave 0 then decodes the
// block's all-small groups a lane per packet.  The descriptors' geometry is
// parked in LDS across both roles (held in registers, verify_split_kernel
// spilled 60 B at 8 waves/SIMD).  An all-small batch costs n / 64 lane-waves
// (and three one-load waves per block), an all-long one the wave kernel's
// groups, 4 per wave.
template <int O = 8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(O ? O : 1, O ? O : 8))) void verify_split2_kernel(
    VerifyParams p, uint64_t Q) {
    __shared__ uint32_t s_geo[4][3 * 64];
    const uint32_t wib = wave_in_block();
    const uint64_t blk = xcd_swizzle(blockIdx.x, gridDim.x);
    uint64_t m_mine, m_small;
    {
        const uint32_t lane = lane_id();
        const uint32_t qq = wib == 0 ? lane >> 4 : (lane >> 2) & 3u;
        const uint32_t oo = wib == 0 ? lane & 15u : 4u * wib + (lane & 3u);
        const uint64_t i = (uint64_t)qq * Q + 16u * blk + oo;
        const bool live = (wib == 0 || lane < 16u) && 16u * blk < Q && i < p.n;
        const v4u d = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0u));
        const uint32_t len = live ? d.z : 0u;
        const uint64_t gl = __ballot(live && len > kSmallMax);
        const bool grp_long = ((gl >> (lane & ~3u)) & 0xfu) != 0;
        const bool own = wib == 0 ? (lane & 15u) < 4u : true;
        m_mine = __ballot(live && own && grp_long);
        m_small = __ballot(wib == 0 && live && !grp_long);
        s_geo[wib][lane] = live ? d.x : 0u;
        s_geo[wib][64 + lane] = live ? d.y : 0u;
        s_geo[wib][128 + lane] = len;
    }
    uint32_t r = 0;
    verify_walk_lds(p, m_mine, s_geo[wib], r);
    if (m_small) {  // wave-uniform; never true on waves 1-3
        uint32_t lane = lane_id();
        asm volatile("" : "+v"(lane));
        const bool small = (m_small >> lane) & 1u;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p.base) +
                            (((uint64_t)s_geo[wib][64 + lane] << 32) | s_geo[wib][lane]);
        uint32_t sv = 0, sc = 0;
        verify_lane(a, small ? s_geo[wib][128 + lane] : 0u, small, sv, sc);
        r = small ? (sv | (sc << 8)) : r;
    }
    uint32_t lane = lane_id();
    asm volatile("" : "+v"(lane));
    if (((m_mine | m_small) >> lane) & 1u) {
        const uint32_t qq = wib == 0 ? lane >> 4 : (lane >> 2) & 3u;
        const uint32_t oo = wib == 0 ? lane & 15u : 4u * wib + (lane & 3u);
        const uint64_t i = (uint64_t)qq * Q + 16u * blk + oo;
        p.verdict[i] = (uint8_t)r;
        if (p.l4)
            p.l4[i] = (uint16_t)(r >> 8);
    }
}

template <int O = 0, bool kLds = false>  // kLds: the long lanes' offsets / lengths parked in LDS across the walk
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(O ? O : 1, O ? O : 8))) void verify_walk_kernel(
    VerifyParams p) {
    __shared__ uint32_t s_geo[kLds ? 4 : 1][kLds ? 3 * 64 : 1];
    const uint32_t lane = lane_id();
    const uint64_t G = (uint64_t)gridDim.x * 4u;
    const uint64_t w = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t i = ((uint64_t)(lane >> 2) * G + w) * 4u + (lane & 3u);
    const bool live = i < p.n;
    const v4u dv = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0u));
    const uint32_t len = live ? dv.z : 0u;
    const uint32_t olo = live ? dv.x : 0u, ohi = live ? dv.y : 0u;
    const bool small = live && len <= kSmallMax;
    uint32_t rv = 0, rc = 0;
    if (__ballot(small))  // wave-uniform
        verify_lane(reinterpret_cast<uintptr_t>(p.base) + (((uint64_t)ohi << 32) | olo), small ? len : 0u, small, rv,
                    rc);
    // one register across the walk: verdict | L4 result << 8
    uint32_t r = rv | (rc << 8);
    uint64_t m = __ballot(live && !small);
    if constexpr (kLds) {
        const uint32_t wib = wave_in_block();
        if (m) {
            s_geo[wib][lane] = olo;
            s_geo[wib][64 + lane] = ohi;
            s_geo[wib][128 + lane] = len;
        }
    }
    while (m) {  // the long packets, 4 at a time in group order (verify_mask)
        // the lane id laundered per iteration: verify_group's lane-derived
        // constants are recomputed in the body, not held across the loop
        uint32_t ln = lane_id();
        asm volatile("" : "+v"(ln));
        uint64_t doff[4];
        uint32_t lg[4], tgt[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const bool have = m != 0;
            const uint32_t j = have ? (uint32_t)__builtin_ctzll(m) : 0u;
            m = have ? m & (m - 1) : m;
            tgt[k] = have ? j : 64u;
            if constexpr (kLds) {
                // same-address LDS reads (broadcast), made wave-uniform
                const uint32_t wib = wave_in_block();
                const uint32_t x = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_geo[wib][j]);
                const uint32_t y = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_geo[wib][64 + j]);
                const uint32_t z = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_geo[wib][128 + j]);
                doff[k] = have ? (((uint64_t)y << 32) | x) : 0u;
                lg[k] = have ? z : 0u;
            } else {
                doff[k] = have ? (((uint64_t)rdl(ohi, j) << 32) | rdl(olo, j)) : 0u;
                lg[k] = have ? rdl(len, j) : 0u;
            }
        }
        uint32_t v2 = 0, c2 = 0;
        verify_group<4, true>(p.base, doff, lg, tgt, ln, v2, c2, [] {});
        r = (ln == tgt[0] || ln == tgt[1] || ln == tgt[2] || ln == tgt[3]) ? (v2 | (c2 << 8)) : r;
    }
    // the index recomputed from a laundered lane id (held across the walk it spilled)
    uint32_t l2 = lane_id();
    asm volatile("" : "+v"(l2));
    const uint64_t i2 = ((uint64_t)(l2 >> 2) * G + w) * 4u + (l2 & 3u);
    if (i2 < p.n) {
        p.verdict[i2] = (uint8_t)r;
        if (p.l4)
            p.l4[i2] = (uint16_t)(r >> 8);
    }
}

}  // namespace wg

namespace {

// Per (device, stream) scratch of the compacting verify path: the entry
// lists, two counter sets, and the host-mapped sample word read by the next
// call.  Created on first use, grown (after draining the stream) when a
// batch needs more entries, never freed (a handful per process).  A stream
// whose state cannot be made (table full, allocation failure) runs the wave
// kernel: the same results by another kernel, never a host fallback.
struct VerifyState {
    int dev = -1;
    void *stream = nullptr;
    std::mutex mu;
    uint32_t *host_sample = nullptr;  // hipHostMalloc'd, mapped
    uint32_t *dev_sample = nullptr;
    uint32_t *ctr = nullptr;          // 2 sets x kVShards x kVCtrStride words
    wg::v4u *ent = nullptr;
    uint64_t cap = 0;                 // entries per shard
    uint32_t parity = 0;
};
constexpr uint32_t kSampleUnknown = 0xffffffffu;
constexpr size_t kMaxVerifyStates = 64;
std::mutex g_vstate_mu;
VerifyState *g_vstate[kMaxVerifyStates];
size_t g_nvstate = 0;

VerifyState *verify_state(void *stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return nullptr;
    std::lock_guard<std::mutex> g(g_vstate_mu);
    for (size_t k = 0; k < g_nvstate; k++)
        if (g_vstate[k]->dev == dev && g_vstate[k]->stream == stream)
            return g_vstate[k];
    if (g_nvstate == kMaxVerifyStates)
        return nullptr;
    VerifyState *s = new VerifyState;
    s->dev = dev;
    s->stream = stream;
    void *h = nullptr, *d = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        delete s;
        return nullptr;
    }
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&s->ctr), 2u * wg::kVShards * wg::kVCtrStride * 4u) != hipSuccess ||
        hipMemset(s->ctr, 0, 2u * wg::kVShards * wg::kVCtrStride * 4u) != hipSuccess) {
        (void)hipHostFree(h);
        if (s->ctr)
            (void)hipFree(s->ctr);
        delete s;
        return nullptr;
    }
    s->host_sample = static_cast<uint32_t *>(h);
    s->dev_sample = static_cast<uint32_t *>(d);
    __atomic_store_n(s->host_sample, kSampleUnknown, __ATOMIC_RELAXED);
    __atomic_store_n(s->host_sample + 1, 0u, __ATOMIC_RELAXED);
    g_vstate[g_nvstate++] = s;
    return s;
}

// Entry capacity for n descriptors (caller holds s->mu).
bool verify_reserve(VerifyState *s, uint64_t cap, hipStream_t st) {
    if (s->cap >= cap)
        return true;
    if (s->ent) {
        if (hipStreamSynchronize(st) != hipSuccess)
            return false;
        (void)hipFree(s->ent);
        s->ent = nullptr;
        s->cap = 0;
    }
    if (hipMalloc(reinterpret_cast<void **>(&s->ent), cap * wg::kVShards * 16u) != hipSuccess) {
        s->ent = nullptr;
        return false;
    }
    s->cap = cap;
    return true;
}

}  // namespace

namespace wg {

// The compacting path (caller holds s->mu).  Grid of the long kernel: est_long
// expected long packets (grid-stride, so a low estimate is only slower).
static int verify_compact_launch(VerifyParams p, VerifyState *s, uint64_t est_long, uint64_t kmin,
                                 hipStream_t st) {
    const uint64_t per_block = 256u;  // descriptors per lane-kernel block
    uint64_t nl = (p.n + per_block - 1) / per_block;
    if (nl >= 8)
        nl = (nl + 7) & ~7ull;
    const uint64_t cap = per_block * ((nl + kVShards - 1) / kVShards);
    if (nl > 0x7fffffffull || p.n >= (1ull << 32) || !verify_reserve(s, cap, st))
        return WG_ERR_RUNTIME;  // the caller runs the wave kernel instead
    VerifyCompact c{s->ent, s->cap, s->ctr + s->parity * kVShards * kVCtrStride,
                    s->ctr + (s->parity ^ 1u) * kVShards * kVCtrStride};
    s->parity ^= 1u;
    p.sample = s->dev_sample;
    hipLaunchKernelGGL(verify_compact_lane_kernel, dim3((unsigned)nl), dim3(256), 0, st, p, c);
    // long kernel: one 4-entry group per wave for the expected count (+1/8
    // and 32 waves of slack), at least one block per shard, at most n / 16
    uint64_t waves = (est_long + 3) / 4;
    waves += waves / 8 + 32;
    uint64_t nb = (waves + 3) / 4;
    nb = nb < kmin ? kmin : nb;  // a stale estimate: still every SIMD busy
    const uint64_t nbmax = (p.n + 15) / 16;
    nb = nb > nbmax ? nbmax : nb;
    nb = (nb + kVShards - 1) & ~(uint64_t)(kVShards - 1);
    hipLaunchKernelGGL((verify_compact_long_kernel<0, true>), dim3((unsigned)nb), dim3(256), 0, st, p, c);
    if (hipGetLastError() != hipSuccess) {
        // a launch that did not happen may have left a counter set dirty
        (void)hipMemsetAsync(s->ctr, 0, 2u * kVShards * kVCtrStride * 4u, st);
        return WG_ERR_LAUNCH;
    }
    return WG_OK;
}

}  // namespace wg

// verify_small = 7: the compacting path or the wave kernel, from the previous
// call's sample (smp of 64 spread packets <= 64 B, the others lb bytes in
// all).  Cost model, measured on MI355X (profiles/r03_verify_*):
// the wave kernel spends max(0.88 ns, group bytes / 6.5 TB/s) of chip time
// per 4-packet group whatever sizes the group mixes; the compacting path pays
// its lane kernel (~7 ps per descriptor + ~8 ps per small packet) and then
// the long packets' groups at 1.07x the wave kernel's per-group time.
static bool verify_pick_compact(uint64_t n, uint32_t smp, uint32_t lb, uint32_t min_small) {
    if (smp < min_small)
        return false;
    const double fs = smp / 64.0;
    const double l_all = (lb + 48.0 * smp) / 64.0;                   // mean length (small ones ~48 B)
    const double l_long = smp < 64 ? (double)lb / (64 - smp) : 0.0;  // mean length of the long ones
    auto group_s = [](double mean_len) { return std::max(0.88e-9, 4.0 * mean_len / 6.5e12); };
    const double t_wave = n / 4.0 * group_s(l_all);
    const double t_compact = n * (7e-12 + 8e-12 * fs) + 1.07 * (n * (1.0 - fs) / 4.0) * group_s(l_long);
    return t_compact < 0.97 * t_wave;
}

static uint64_t verify_wave_blocks(uint64_t n) {
    uint64_t blocks = (n + 15) / 16;  // one-shot 4-packet waves
    return blocks >= 8 ? (blocks + 7) & ~7ull : blocks;
}

extern "C" int wg_verify_desc(const uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n,
                              uint8_t *dev_verdict, uint16_t *dev_l4, void *stream) {
    if (!n)
        return WG_OK;
    if (!dev_base || !dev_desc || !dev_verdict || (reinterpret_cast<uintptr_t>(dev_desc) & 15))
        return WG_ERR_INVALID;
    VerifyParams p{dev_base, dev_desc, dev_verdict, dev_l4, n};
    const Tune t = tune();
    if (t.verify_small == 10) {  // split roles at 8 waves/SIMD: one stateless launch
        const uint64_t Q = ((n + 3) / 4 + 15) & ~15ull;  // as l4csum_split_kernel's quarters
        uint64_t sb = Q / 16;
        if (sb >= 8)
            sb = (sb + 7) & ~7ull;
        if (sb > 0x7fffffffull)
            return WG_ERR_INVALID;
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (t.verify_occ == 8)
            hipLaunchKernelGGL(verify_split2_kernel<8>, dim3((unsigned)sb), dim3(256), 0, st, p, Q);
        else
            hipLaunchKernelGGL(verify_split2_kernel<0>, dim3((unsigned)sb), dim3(256), 0, st, p, Q);
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    if (t.verify_small == 9) {  // persistent walking verify: one stateless launch at the resident capacity
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (t.verify_occ == 8) {
            auto k = verify_persist_kernel<8>;
            hipLaunchKernelGGL(k, dim3((unsigned)persist_grid(n, resident_blocks(k))), dim3(256), 0, st, p);
        } else {
            auto k = verify_persist_kernel<0>;
            hipLaunchKernelGGL(k, dim3((unsigned)persist_grid(n, resident_blocks(k))), dim3(256), 0, st, p);
        }
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    if (t.verify_small == 8) {  // walking verify: one stateless launch of n / 64 waves
        uint64_t blocks = (n + 255) / 256;
        if (blocks >= 8)
            blocks = (blocks + 7) & ~7ull;
        if (blocks > 0x7fffffffull)
            return WG_ERR_INVALID;
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (t.verify_occ == 8 && t.verify_dm == 2)  // (experiment) geometry parked in LDS
            hipLaunchKernelGGL((verify_walk_kernel<8, true>), dim3((unsigned)blocks), dim3(256), 0, st, p);
        else if (t.verify_occ == 8)
            hipLaunchKernelGGL(verify_walk_kernel<8>, dim3((unsigned)blocks), dim3(256), 0, st, p);
        else
            hipLaunchKernelGGL(verify_walk_kernel<0>, dim3((unsigned)blocks), dim3(256), 0, st, p);
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    if (t.verify_small >= 6) {
        // 6: the compacting path; 7 (default): the compacting path when the
        // previous call on this stream sampled >= verify_auto_t small packets
        // of 64, else the wave kernel (which samples this batch in turn).
        // Both give the same results; only the kernels differ.
        hipStream_t st = static_cast<hipStream_t>(stream);
        if (VerifyState *s = verify_state(stream)) {
            std::lock_guard<std::mutex> g(s->mu);
            const uint32_t smp = __atomic_load_n(s->host_sample, __ATOMIC_RELAXED);
            const uint32_t lb = __atomic_load_n(s->host_sample + 1, __ATOMIC_RELAXED);
            const bool known = smp <= 64u;
            if (t.verify_small == 6 || (known && verify_pick_compact(n, smp, lb, t.verify_auto_t))) {
                const uint64_t est = known ? (n * (64u - smp) + 63u) / 64u : n;
                const int rc = verify_compact_launch(p, s, est, t.verify_k2min, st);
                if (rc != WG_ERR_RUNTIME)
                    return rc;
            }
            p.sample = s->dev_sample;
            hipLaunchKernelGGL((verify_kernel<4, 8, 0, true, false, true>), dim3((unsigned)verify_wave_blocks(n)),
                               dim3(256), 0, st, p);
            return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
        }
    }
    if (t.verify_small == 4 || t.verify_small == 5) {
        hipStream_t st = static_cast<hipStream_t>(stream);
        uint64_t nl = (n + 255) / 256, nw = (n + 15) / 16;  // lane-role / wave-role blocks
        if (nl >= 8) nl = (nl + 7) & ~7ull;
        if (nw >= 8) nw = (nw + 7) & ~7ull;
        if (nl + nw > 0x7fffffffull)
            return WG_ERR_INVALID;
        if (t.verify_small == 4) {
            hipLaunchKernelGGL(verify_lane_kernel, dim3((unsigned)nl), dim3(256), 0, st, p);
            if (t.verify_wblk == 16) {
                uint64_t nw16 = (n + 63) / 64;
                if (nw16 >= 8) nw16 = (nw16 + 7) & ~7ull;
                hipLaunchKernelGGL((verify_long_kernel<8, 16>), dim3((unsigned)nw16), dim3(1024), 0, st, p);
            } else if (t.verify_occ == 8) {
                hipLaunchKernelGGL(verify_long_kernel<8>, dim3((unsigned)nw), dim3(256), 0, st, p);
            } else {
                hipLaunchKernelGGL(verify_long_kernel<0>, dim3((unsigned)nw), dim3(256), 0, st, p);
            }
        } else if (t.verify_occ == 8) {
            hipLaunchKernelGGL(verify_roles_kernel<8>, dim3((unsigned)(nl + nw)), dim3(256), 0, st, p, (uint32_t)nl);
        } else {
            hipLaunchKernelGGL(verify_roles_kernel<0>, dim3((unsigned)(nl + nw)), dim3(256), 0, st, p, (uint32_t)nl);
        }
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    if (t.verify_small == 3) {
        const uint64_t Q = ((n + 3) / 4 + 15) & ~15ull;  // as l4csum_split_kernel's quarters
        uint64_t sb = Q / 16;
        if (sb >= 8)
            sb = (sb + 7) & ~7ull;
        if (sb > 0x7fffffffull)
            return WG_ERR_INVALID;
        if (t.verify_occ == 8)
            hipLaunchKernelGGL(verify_split_kernel<8>, dim3((unsigned)sb), dim3(256), 0,
                               static_cast<hipStream_t>(stream), p, Q);
        else
            hipLaunchKernelGGL(verify_split_kernel<0>, dim3((unsigned)sb), dim3(256), 0,
                               static_cast<hipStream_t>(stream), p, Q);
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    if (t.verify_small) {
        const uint64_t per_block = t.verify_small == 2 ? 64u : 256u;  // descriptors per 256-thread block
        const uint64_t sb = (n + per_block - 1) / per_block;
        if (sb > 0x7fffffffull)
            return WG_ERR_INVALID;
        if (t.verify_small == 2)
            hipLaunchKernelGGL((verify_small_kernel<4, 4>), dim3((unsigned)sb), dim3(256), 0,
                               static_cast<hipStream_t>(stream), p);
        else
            hipLaunchKernelGGL((verify_small_kernel<4>), dim3((unsigned)sb), dim3(256), 0,
                               static_cast<hipStream_t>(stream), p);
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    const bool pf = t.verify_dm == 2;
    uint64_t blocks = (n + 15) / 16;
    if (pf) {
        blocks = (blocks + t.l4_iters - 1) / t.l4_iters;
        if (blocks >= 8)
            blocks &= ~7ull;  // XCD swizzle bijective; the grid-stride loop covers the rest
    } else if (blocks >= 8) {
        blocks = (blocks + 7) & ~7ull;  // one iteration per wave: round up
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)blocks);
    if (!pf && t.verify_hdr && t.verify_occ == 8)
        hipLaunchKernelGGL((verify_kernel<4, 8, 0, true>), grid, dim3(256), 0, st, p);
    else if (!pf && t.verify_hdr)
        hipLaunchKernelGGL((verify_kernel<4, 0, 0, true>), grid, dim3(256), 0, st, p);
    else if (pf && t.verify_occ == 6)
        hipLaunchKernelGGL((verify_kernel<4, 6, 2>), grid, dim3(256), 0, st, p);
    else if (pf)
        hipLaunchKernelGGL((verify_kernel<4, 0, 2>), grid, dim3(256), 0, st, p);
    else if (t.verify_occ == 8)
        hipLaunchKernelGGL((verify_kernel<4, 8, 0>), grid, dim3(256), 0, st, p);
    else
        hipLaunchKernelGGL((verify_kernel<4, 0, 0>), grid, dim3(256), 0, st, p);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_verify_uniform(const uint8_t *dev_base, uint64_t total_len, uint32_t segment_size,
                                 uint8_t *dev_verdict, uint16_t *dev_l4, void *stream) {
    if (!segment_size || (total_len && (!dev_base || !dev_verdict)))
        return WG_ERR_INVALID;
    if (!total_len)
        return WG_OK;
    const uint64_t nseg = (total_len + segment_size - 1) / segment_size;
    VerifyParams p{dev_base, nullptr, dev_verdict, dev_l4, nseg, total_len, segment_size,
                   (uint32_t)(total_len - (nseg - 1) * segment_size)};
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (segment_size <= kSmallMax) {  // every segment small: a lane each (no long packets to serve)
        uint64_t b = (p.n + 255) / 256;
        if (b >= 8) b = (b + 7) & ~7ull;
        if (b > 0x7fffffffull)
            return WG_ERR_INVALID;
        hipLaunchKernelGGL(verify_uniform_lane_kernel, dim3((unsigned)b), dim3(256), 0, st, p);
    } else {
        uint64_t blocks = (p.n + 15) / 16;  // one-shot 4-packet waves, as wg_verify_desc's default
        if (blocks >= 8) blocks = (blocks + 7) & ~7ull;
        if (blocks > 0x7fffffffull)
            return WG_ERR_INVALID;
        hipLaunchKernelGGL((verify_kernel<4, 8, 0, true, true>), dim3((unsigned)blocks), dim3(256), 0, st, p);
    }
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_l4csum_uniform(const uint8_t *dev_base, uint64_t total_len, uint32_t segment_size,
                                 uint16_t csum_start, uint32_t flags, uint16_t *dev_out, void *stream) {
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
