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
#include <cstdio>
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

// Descriptor modes (kDM): 0 = scalar descriptor loads per iteration (uniform
// batches need none); 2 = scalar loads for a wave's first iteration, and each
// iteration's vector load of the NEXT iteration's descriptors issued right
// after its own packet loads, so from the second iteration on a wave starts
// its packet loads with no descriptor round trip in front of them (the
// launcher gives each wave 4 iterations; one vector load per iteration
// without the prefetch measured slower: the readlanes wait on it).
template <int kKind, int P, bool kNT, int kDM>
__global__ __launch_bounds__(256) void l4csum_kernel(L4Params p) {
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
        if constexpr (DM == 2) {
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

// ---------------------------------------------------------------------------
// Small packets (SURVEY §8(d) config 4's small-packet stress).  A wave per
// packet spends ~150 wave-instructions (half of them on the CU's one scalar
// unit) on a 64-B packet, so 64-B batches are issue-bound at ~6 % of the HBM
// roofline by l4csum_kernel.  A lane takes a packet of <= kSmallMax bytes
// instead: summed from (at most) five aligned 16-B chunks funnel-shifted into
// 16 packet-relative dwords, over the summed region and the pseudo-header
// address bytes.  Same arithmetic model (wg_device.hpp): one byte swap of a
// folded sum whose pairing starts at an odd position.
// ---------------------------------------------------------------------------
constexpr uint32_t kSmallMax = 64;  // bytes: five aligned 16-B chunks at any alignment

// acc + both 16-bit halves of w in one instruction (v_sad_u16 against zero)
__device__ __forceinline__ uint32_t hacc(uint32_t acc, uint32_t w) { return __builtin_amdgcn_sad_u16(w, 0u, acc); }

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

// The same five chunks per lane, loaded by the whole wave together (the
// split kernel's lane role, knob lane_coop = 1): the wave's 320 chunk slots
// (lane j's chunk c = slot 5j + c) are dealt in order, instruction k giving
// lane l slot 64k + l, so one load instruction covers ~13 packets' windows
// (each lane learns packet j's window from lane j by two ds_bpermute)
// instead of one 16-B piece of each of 64 packets; the chunks go through the
// wave's 5 KiB of LDS rows (slot s at 16 s: each instruction's stores are
// 1 KiB in a row; lane l's reads at 80 l are conflict-free) back to their
// packet's lane.  Config 4's 64-B sub-batch 46.0 -> 45.3 us back to back,
// config 4 / 5 unchanged; the verify kernels' lane paths measured no gain
// or a loss (profiles/r06_coop_ab.txt).  Every lane of the wave
// must be active; the rows are used once per wave.
__device__ __forceinline__ void coop_chunks(uintptr_t a, uint32_t len, bool use, v4u W[5], v4u *rows) {
    uint64_t mine = (uint64_t)reinterpret_cast<uintptr_t>(&g_zero16);
    if (use && len) {  // the window lane_chunks loads: first chunk | index of the last (0-4) in its free low bits
        const uintptr_t a0 = a & ~(uintptr_t)15;
        mine = (uint64_t)a0 | (uint64_t)((((a + len - 1) & ~(uintptr_t)15) - a0) >> 4);
    }
    const uint32_t lo = (uint32_t)mine, hi = (uint32_t)(mine >> 32);
    const uint32_t lane = lane_id();
    v4u V[5];
#pragma unroll
    for (uint32_t k = 0; k < 5; k++) {
        const uint32_t sl = 64u * k + lane, j = sl / 5u, c = sl - 5u * j;
        const uint32_t jl = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(j << 2), (int)lo);
        const uint32_t jh = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(j << 2), (int)hi);
        const uint32_t n = jl & 15u;
        V[k] = ld16((uintptr_t)((((uint64_t)jh << 32) | (jl & ~15u)) + 16u * (c < n ? c : n)));
    }
#pragma unroll
    for (uint32_t k = 0; k < 5; k++)
        rows[64u * k + lane] = V[k];
    wave_lds_handoff();
#pragma unroll
    for (uint32_t c = 0; c < 5; c++)
        W[c] = rows[5u * lane + c];
}
constexpr uint32_t kCoopRows = 320;  // v4u per wave

// The lane paths' realignment: the packet's 16 dwords R[m] (bytes 4m..4m+3
// of the packet at a, bytes at positions >= len zeroed) from the 20 dwords of
// its five aligned chunks.  The dword offset q4 = (a & 15) >> 2 picks
// Wd[m + q4]:
//  * q4 the same in every lane of the wave (aligned batches): one scalar
//    branch to a straight-line copy for that q4 — no per-lane selects;
//  * q4 different across the wave (config 4's 64-B packets lie 8-B aligned
//    between 9000-B ones): two bit-mask select stages (by 2 dwords, then by
//    1) for every lane.  A 4-way ?: per word compiled to a branch ladder
//    that ran every case the wave held; plain ?: selects were turned into a
//    dynamically indexed copy of Wd in scratch.
// Measured (profiles/r06_barrel_ab.txt): the mask stages alone took config
// 4's 64-B sub-batch 50.9 -> 47.0 us but a uniform 64-B verify batch 12.3 ->
// 16.5 us (VALU it did not need); the scalar branch keeps the latter.
template <uint32_t Q>
__device__ __forceinline__ void realign_q(const uint32_t Wd[20], uint32_t sh, uint32_t len, uint32_t R[16]) {
#pragma unroll
    for (uint32_t m = 0; m < 16; m++)
        R[m] = bytes_below(__builtin_amdgcn_alignbyte(Wd[m + Q + 1], Wd[m + Q], sh), m, len);
}

__device__ __forceinline__ void lane_realign(const uint32_t Wd[20], uintptr_t a, uint32_t len, uint32_t R[16]) {
    const uint32_t s = (uint32_t)(a & 15u), q4 = s >> 2, sh = s & 3u;
    const uint32_t qf = (uint32_t)__builtin_amdgcn_readfirstlane((int)q4);
    if (__ballot(q4 != qf) == 0) {  // wave-uniform
        switch (qf) {
        case 0: realign_q<0>(Wd, sh, len, R); break;
        case 1: realign_q<1>(Wd, sh, len, R); break;
        case 2: realign_q<2>(Wd, sh, len, R); break;
        default: realign_q<3>(Wd, sh, len, R); break;
        }
        return;
    }
    const uint32_t m2 = 0u - ((q4 >> 1) & 1u), m1 = 0u - (q4 & 1u);
    const auto xw = [&](uint32_t i) { return Wd[i] ^ ((Wd[i] ^ Wd[i + 2]) & m2); };  // Wd[i + 2 * (q4 >> 1)]
    const auto pick = [&](uint32_t x0, uint32_t x1) { return x0 ^ ((x0 ^ x1) & m1); };
#pragma unroll
    for (uint32_t m = 0; m < 16; m++)
        R[m] = bytes_below(__builtin_amdgcn_alignbyte(pick(xw(m + 1), xw(m + 2)), pick(xw(m), xw(m + 1)), sh), m, len);
}

// ... summed: the chunks funnel-shifted into 16 packet-relative dwords
// (bytes past the packet zeroed), so the region and address masks are
// per-dword constants of len / csum_start and the addresses static dwords.
// Returns the pre-complement folded sum t (region, byte-swapped when it pairs
// from an odd packet offset, + pseudo-header when kL4); the caller's result
// is ~fold16_32(t).
template <bool kL4, bool kUni = false>
__device__ __forceinline__ uint32_t lane_sum(const v4u W[5], uintptr_t a, uint32_t len, uint32_t cs, uint32_t fl) {
    const uint32_t o0 = cs < len ? cs : len;
    const bool v6 = fl & WG_PKT_V6;
    const uint32_t Wd[20] = {W[0][0], W[0][1], W[0][2], W[0][3], W[1][0], W[1][1], W[1][2],
                             W[1][3], W[2][0], W[2][1], W[2][2], W[2][3], W[3][0], W[3][1],
                             W[3][2], W[3][3], W[4][0], W[4][1], W[4][2], W[4][3]};
    // kUni: a uniform PacketBatch's lane kernel (segments of one size: the
    // dword offset is the same across a wave when the size is a multiple of
    // 16) keeps the per-word 4-way select, whose branches then run one case
    // (the wave-uniform test of lane_realign in front cost a 64-B uniform
    // verify batch +3.4 %, profiles/r06_hybrid_ab.txt)
    uint32_t R[16];
    if constexpr (!kUni)
        lane_realign(Wd, a, len, R);
    const uint32_t s = (uint32_t)(a & 15u), q4 = s >> 2, sh = s & 3u;
    uint32_t sr = 0, sq = 0;
#pragma unroll
    for (uint32_t m = 0; m < 16; m++) {
        uint32_t r;
        if constexpr (kUni) {
            const uint32_t lo = q4 == 0 ? Wd[m] : q4 == 1 ? Wd[m + 1] : q4 == 2 ? Wd[m + 2] : Wd[m + 3];
            const uint32_t hi = q4 == 0 ? Wd[m + 1] : q4 == 1 ? Wd[m + 2] : q4 == 2 ? Wd[m + 3] : Wd[m + 4];
            r = bytes_below(__builtin_amdgcn_alignbyte(hi, lo, sh), m, len);
        } else {
            r = R[m];
        }
        sr = hacc(sr, bytes_from(r, m, o0));
        if (kL4) {
            if (m == 3u || m == 4u)  // v6 8-39, v4 12-19
                sq = hacc(sq, r);
            else if (m >= 2u && m < 10u)
                sq = v6 ? hacc(sq, r) : sq;
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

// Uniform PacketBatches of small segments (segment_size <= kSmallMax; knob
// l4_small_uniform = 2): every segment is small, so a lane per segment, summed
// by lane_chunks / lane_sum — no descriptors, no wave role.
__global__ __launch_bounds__(256) void l4csum_uniform_small_kernel(L4Params p) {
    const uint64_t i = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 256u + threadIdx.x;
    const bool live = i < p.n;
    // PacketBatch segment i (include/util/packets.hpp:23-36)
    const uint64_t off = live ? i * (uint64_t)p.seg : 0u;
    const uint64_t rem = p.total_len - off;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p.base) + off;
    const uint32_t len = live ? (rem < p.seg ? (uint32_t)rem : p.seg) : 0u;
    v4u W[5];
    lane_chunks(a, len, live && len, W);
    const uint32_t t = lane_sum<true, true>(W, a, len, live ? p.cs : 0u, live ? p.flags : 0u);
    if (live)
        p.out[i] = (uint16_t)(~fold16_32(t) & 0xffffu);
}

// Split-role descriptor kernel (knob l4_small = 5).  Descriptors come in
// groups of 4 consecutive ones; the batch is cut into 4 quarters of Q
// descriptors, and block b owns the 16 at [q*Q + 16b, q*Q + 16b + 16) of each
// quarter q (64 in all).  Its wave k owns one group per quarter,
// [q*Q + 16b + 4k, +4): 16 descriptors a quarter batch apart, like the
// wave-per-packet kernel's grid-stride iterations (consecutive packets per
// wave measured 3-4 % slower).
//  * WAVE role (every wave): every packet of its groups that hold a packet
//    longer than kSmallMax, one at a time through the wave-per-packet
//    machinery.  The long-packet path sets the kernel's register budget and
//    so the lane role's occupancy: 4 at a time held 94 VGPRs (5 waves per
//    SIMD), 2 held 74 (6), 1 holds 64 (8) — config 4's 64-B sub-batch 64 ->
//    56 -> 51 us, config 4 +0.7 % and +0.9 %, config 5 -0.3 % and 0 %
//    (profiles/r04_q2_ab.txt, r04_q1_ab.txt).  Small packets among long ones
//    ride along in their issue phase at next to no cost (config 4's mixed
//    batch measured +2.5 % when they went to the lane role instead).
//  * LANE role (wave 0): the block's all-small groups, a lane per packet,
//    summed from its 5 aligned chunks (4 KiB of loads in flight per wave).
// Wave 0 loads the block's 64 descriptors (lane l = descriptor
// (l >> 4) * Q + 16b + (l & 15); its own groups are lanes with (l & 15) < 4),
// waves 1-3 their 16: every descriptor read once from HBM.  An all-small
// batch keeps a lane per packet (waves 1-3 leave after one descriptor load),
// an all-long one keeps the short 16-packet waves with every descriptor in
// one vector load.  One launch, no host knowledge of the mix.
template <int kKind, bool kNT, int U = 4, bool kCoop = true>  // U: loads in flight per lane on a long packet's rest
__global__ __launch_bounds__(256) void l4csum_split_kernel(L4Params p) {
    constexpr bool kL4 = kKind != kDescPlain;
    __shared__ v4u s_rows[kCoop ? kCoopRows : 1];  // the lane role's (wave 0)
    const uint32_t lane = lane_id();
    const uint32_t wib = wave_in_block();
    const uint64_t blk = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint64_t Q = p.quarter;
    // lane -> (quarter, offset in the block's 16 of that quarter)
    const uint32_t qq = wib == 0 ? lane >> 4 : (lane >> 2) & 3u;
    const uint32_t oo = wib == 0 ? lane & 15u : 4u * wib + (lane & 3u);
    const uint64_t i = (uint64_t)qq * Q + 16u * blk + oo;
    const bool live = (wib == 0 || lane < 16u) && 16u * blk < Q && i < p.n;
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
    const bool own = wib == 0 ? (lane & 15u) < 4u : true;
    const bool mine = live && own && grp_long;
    uint32_t res = 0;
    wave_long<kL4, kNT, 1, U>(__ballot(mine), a, len, cs, fl, p.base, lane, res);
    if (mine)
        p.out[i] = (uint16_t)res;
    // ---- lane role (wave 0): the block's all-small groups
    const bool small = wib == 0 && live && !grp_long;
    if (__ballot(small)) {  // wave-uniform; never true on waves 1-3
        v4u W[5];
        if constexpr (kCoop)
            coop_chunks(a, len, small && len, W, s_rows);
        else
            lane_chunks(a, len, small && len, W);
        const uint32_t t = lane_sum<kL4>(W, a, small ? len : 0u, cs, fl);
        if (small)
            p.out[i] = (uint16_t)(~fold16_32(t) & 0xffffu);
    }
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
static int launch_split(const L4Params &p, hipStream_t st) {
    // quarters of Q descriptors (a multiple of 16: block b owns
    // [q*Q + 16b, +16) of each quarter, whole 4-descriptor groups); 4 Q >= n
    L4Params q = p;
    q.quarter = ((p.n + 3) / 4 + 15) & ~15ull;
    uint64_t blocks = q.quarter / 16;
    if (blocks >= 8)
        blocks = (blocks + 7) & ~7ull;  // XCD swizzle bijective; surplus blocks have no live lane
    if (blocks > 0x7fffffffull)
        return WG_ERR_INVALID;
    const Tune t = tune();
    const dim3 g((unsigned)blocks), b(256);
    if (t.l4_unroll == 8 && t.lane_coop)
        hipLaunchKernelGGL((l4csum_split_kernel<kKind, kNT, 8, true>), g, b, 0, st, q);
    else if (t.l4_unroll == 8)
        hipLaunchKernelGGL((l4csum_split_kernel<kKind, kNT, 8, false>), g, b, 0, st, q);
    else if (t.lane_coop)
        hipLaunchKernelGGL((l4csum_split_kernel<kKind, kNT, 4, true>), g, b, 0, st, q);
    else
        hipLaunchKernelGGL((l4csum_split_kernel<kKind, kNT, 4, false>), g, b, 0, st, q);
    return WG_OK;
}

static int launch_l4(int kind, const L4Params &p, hipStream_t st) {
    if (p.n == 0)
        return WG_OK;
    const Tune t = tune();
    int rc = WG_OK;
    if (kind == kUniformL4 && p.seg <= kSmallMax && t.l4_small_uniform) {
        // every segment is small: a lane per segment, no trade-off
        uint64_t b = (p.n + 255) / 256;
        if (b >= 8)
            b = (b + 7) & ~7ull;
        if (b > 0x7fffffffull)
            return WG_ERR_INVALID;
        hipLaunchKernelGGL(l4csum_uniform_small_kernel, dim3((unsigned)b), dim3(256), 0, st, p);
    } else if (kind != kUniformL4 && p.n <= t.l4_coop) {
        // few descriptors: a block per packet (config 1's 64 KiB buffers)
        rc = kind == kDescL4 ? (t.l4_nt ? launch_coop<kDescL4, true>(p, t, st) : launch_coop<kDescL4, false>(p, t, st))
                             : (t.l4_nt ? launch_coop<kDescPlain, true>(p, t, st)
                                        : launch_coop<kDescPlain, false>(p, t, st));
    } else if (kind != kUniformL4 && t.l4_small) {
        // descriptor batches: the split-role kernel (l4_small = 5, default)
        rc = kind == kDescL4 ? (t.l4_nt ? launch_split<kDescL4, true>(p, st) : launch_split<kDescL4, false>(p, st))
                             : (t.l4_nt ? launch_split<kDescPlain, true>(p, st)
                                        : launch_split<kDescPlain, false>(p, st));
    } else {
        // one wave per packet, 4 packets per wave (uniform batches, and
        // descriptor batches under l4_small = 0: 4 iterations per wave with
        // the next iteration's descriptors prefetched)
        uint64_t want = (p.n + 15) / 16;
        if (kind != kUniformL4)
            want = (want + 3) / 4;
        uint64_t blocks = want < t.l4_blocks ? want : t.l4_blocks;
        if (blocks >= 8)
            blocks &= ~7ull;  // keep the XCD swizzle bijective
        const dim3 g((unsigned)blocks), b(256);
        const bool nt = t.l4_nt != 0;
        if (kind == kUniformL4 && nt)
            hipLaunchKernelGGL((l4csum_kernel<kUniformL4, 4, true, 0>), g, b, 0, st, p);
        else if (kind == kUniformL4)
            hipLaunchKernelGGL((l4csum_kernel<kUniformL4, 4, false, 0>), g, b, 0, st, p);
        else if (kind == kDescL4 && nt)
            hipLaunchKernelGGL((l4csum_kernel<kDescL4, 4, true, 2>), g, b, 0, st, p);
        else if (kind == kDescL4)
            hipLaunchKernelGGL((l4csum_kernel<kDescL4, 4, false, 2>), g, b, 0, st, p);
        else if (nt)
            hipLaunchKernelGGL((l4csum_kernel<kDescPlain, 4, true, 2>), g, b, 0, st, p);
        else
            hipLaunchKernelGGL((l4csum_kernel<kDescPlain, 4, false, 2>), g, b, 0, st, p);
    }
    if (rc != WG_OK)
        return rc;
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
template <int P, typename Mid>
__device__ __forceinline__ void verify_group(const uint8_t *base, const uint64_t *doff, const uint32_t *len,
                                             const uint32_t *tgt, uint32_t lane, uint32_t &rv, uint32_t &rc,
                                             Mid mid) {
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
        // header bytes 0-31 ride in the byte gather's idle lanes; longer
        // packets fail the size gate (evaluator.hpp:118-121): only their
        // header bytes are read (region [32, 32) is empty)
        g[j].len = len[j] <= 65535u ? len[j] : 32u;
        g[j].cs = 32;
        issue<false, true, true>(g[j], lane, f[j]);
        hv[j] = f[j].hb;
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
        constexpr uint32_t kHdrEnd = 32u;
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

// The wave kernel: one-shot waves of 4 packets (one group) at 8 waves per
// SIMD.  Header bytes 0-31 ride in the L4 byte gather's idle lanes
// (verify_group) — no separate header load.  A group's 4 descriptors come by
// one 64-B scalar load (a load per descriptor, the compiler issues one after
// another, each waited for).  kUni: a uniform PacketBatch instead of
// descriptors (wg_verify_uniform).
template <bool kUni>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void verify_kernel(VerifyParams p) {
    constexpr int P = 4;
    const uint32_t lane = lane_id();
    const uint64_t i0 = ((uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block()) * P;
    if (i0 < p.n) {
        uint32_t len[P];
        uint64_t doff[P];
        if constexpr (kUni) {
            // PacketBatch segment i0 + j (include/util/packets.hpp:23-36): one
            // 64-bit multiply and compare per wave (a 64-bit scalar compare
            // has no SALU form on gfx9, and this kernel's scalar unit is busy)
            const uint64_t o0 = i0 * (uint64_t)p.seg;
            const bool full = i0 + P < p.n;  // every segment of the group whole
#pragma unroll
            for (int j = 0; j < P; j++) {
                doff[j] = o0 + (uint32_t)j * p.seg;
                len[j] = full ? p.seg : (i0 + j + 1 < p.n ? p.seg : (i0 + j + 1 == p.n ? p.last_len : 0u));
            }
        } else if (i0 + P <= p.n) {
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
        verify_group<P>(p.base, doff, len, tgt, lane, rv, rc, [] {});
        if (lane < (uint32_t)P && i0 + lane < p.n) {
            p.verdict[i0 + lane] = (uint8_t)rv;
            if (p.l4)
                p.l4[i0 + lane] = (uint16_t)rc;
        }
    }
    if constexpr (!kUni) {
        if (p.sample && blockIdx.x == 0 && wave_in_block() == 0)
            verify_sample(p, lane);
    }
}

}  // namespace wg

using namespace wg;

namespace wg {

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

template <bool kUni>
__device__ __forceinline__ void verify_lane_decode(const v4u W[5], uintptr_t a, uint32_t len, uint32_t &rv,
                                                   uint32_t &rc);

template <bool kUni = false>
__device__ __forceinline__ void verify_lane(uintptr_t a, uint32_t len, bool use, uint32_t &rv, uint32_t &rc) {
    v4u W[5];
    verify_lane_load(a, len, use, W);
    verify_lane_decode<kUni>(W, a, len, rv, rc);
}

template <bool kUni>
__device__ __forceinline__ void verify_lane_decode(const v4u W[5], uintptr_t a, uint32_t len, uint32_t &rv,
                                                   uint32_t &rc) {
    const uint32_t Wd[20] = {W[0][0], W[0][1], W[0][2], W[0][3], W[1][0], W[1][1], W[1][2], W[1][3],
                             W[2][0], W[2][1], W[2][2], W[2][3], W[3][0], W[3][1], W[3][2], W[3][3],
                             W[4][0], W[4][1], W[4][2], W[4][3]};
    uint32_t R[16];
    if constexpr (kUni) {  // as lane_sum's kUni: the per-word 4-way select
        const uint32_t s = (uint32_t)(a & 15u), q4 = s >> 2, sh = s & 3u;
#pragma unroll
        for (uint32_t m = 0; m < 16; m++) {
            const uint32_t lo = q4 == 0 ? Wd[m] : q4 == 1 ? Wd[m + 1] : q4 == 2 ? Wd[m + 2] : Wd[m + 3];
            const uint32_t hi = q4 == 0 ? Wd[m + 1] : q4 == 1 ? Wd[m + 2] : q4 == 2 ? Wd[m + 3] : Wd[m + 4];
            R[m] = bytes_below(__builtin_amdgcn_alignbyte(hi, lo, sh), m, len);
        }
    } else {
        lane_realign(Wd, a, len, R);
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
                const uint32_t hs = hacc(hacc(hacc(hacc(hacc(0u, R[0]), R[1]), R[2]), R[3]), R[4]);
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
            // the addresses (v6 bytes 8-39, v4 12-19) and the L4 bytes from
            // ihs (40 / 20) are each dword from 2 (v6) / 3 (v4) on, once
            uint32_t sum = (proto << 8) + bswap16((len - ihs) & 0xffffu);
            sum = v6 ? hacc(sum, R[2]) : sum;
#pragma unroll
            for (uint32_t m = 3; m < 16; m++) sum = hacc(sum, R[m]);
            c = ~fold16_32(sum) & 0xffffu;
            if (c == 0)
                v |= WG_VERDICT_L4_OK;
        }
    }
    rv = v;
    rc = c;
}

// wg_verify_uniform with segment_size <= kSmallMax: every segment is small,
// so a lane per segment decodes it (no descriptors, no wave role).
__global__ __launch_bounds__(256) void verify_uniform_lane_kernel(VerifyParams p) {
    const uint64_t i = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 256u + threadIdx.x;
    const bool live = i < p.n;
    const uint64_t o = live ? i * (uint64_t)p.seg : 0u;
    const uint32_t len = live ? (p.total_len - o < p.seg ? (uint32_t)(p.total_len - o) : p.seg) : 0u;
    uint32_t rv = 0, rc = 0;
    verify_lane<true>(reinterpret_cast<uintptr_t>(p.base) + o, len, live, rv, rc);
    if (live) {
        p.verdict[i] = (uint8_t)rv;
        if (p.l4)
            p.l4[i] = (uint16_t)rc;
    }
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
            // A shard receives at most cap entries per call (the host sizes
            // cap from the blocks per shard) when its counter started at 0,
            // which stream order guarantees (captured calls never come here);
            // the bound keeps a broken protocol from writing past the list.
            if (s_base + pre + r < c.cap) {
                c.ent[sh * c.cap + s_base + pre + r] = v4u{dv.x, dv.y, len, (uint32_t)i};
            } else {
                // never under the protocol; if it ever happens the packet
                // gets a defined verdict (0: not verified -> dropped, as a
                // failed gate), never a stale one, and the host is told
                // through the mapped sample area (word 2) on its next call
                p.verdict[i] = 0;
                if (p.l4)
                    p.l4[i] = 0xffffu;
                if (p.sample)
                    __hip_atomic_store(p.sample + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
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
    const uint32_t cnt0 = *reinterpret_cast<const c_u32 *>(reinterpret_cast<uintptr_t>(c.ctr + sh * kVCtrStride));
    asm volatile("" ::"s"(d[0]), "s"(cnt0));  // both in flight before the first wait
    const uint32_t cnt = cnt0 < c.cap ? cnt0 : (uint32_t)c.cap;  // never past the list (see the lane kernel)
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
        verify_group<P>(p.base, doff, len, tgt, lane, rv, rc, [] {});
        // (at < n: never otherwise under the protocol — the lane kernel wrote
        // i < n — but a broken one must not write outside the batch)
        const uint32_t at = lane < (uint32_t)P ? s_idx[wave_in_block()][lane] : 0u;
        if (lane < (uint32_t)P && k0 + lane < cnt && at < p.n) {
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

// Walking verify (verify_small = 8; the default's choice for all-small
// batches and for the first call on a stream): one stateless launch of n / 64
// waves whatever the size mix.  Lane l of wave w (of G) owns descriptor
// ((l >> 2) * G + w) * 4 + (l & 3) — sixteen 4-descriptor groups a sixteenth
// of the batch apart, so the waves resident at any moment work on one narrow
// window of the batch.  Packets of <= kSmallMax bytes are decoded in their
// lane (verify_lane); the wave then walks its longer packets in group order,
// 4 at a time, through verify_group.  Measured (profiles/r04_walk_verify_ab.json):
// 1 M x 64 B 0.0157 ms against the compacting path's 0.0174; long packets
// cost it 7-9 % against the one-shot wave kernel (a wave then lives for 16
// groups), so the cost model sends long-dominated batches there.
template <bool kConsec>
__global__ __launch_bounds__(256) void verify_walk_kernel(VerifyParams p) {
    const uint32_t lane = lane_id();
    const uint64_t G = (uint64_t)gridDim.x * 4u;
    const uint64_t w = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t i = kConsec ? w * 64u + lane : ((uint64_t)(lane >> 2) * G + w) * 4u + (lane & 3u);
    const bool live = i < p.n;
    const v4u dv = ld16(reinterpret_cast<uintptr_t>(p.desc) + 16ull * (live ? i : 0u));
    const uint32_t len = live ? dv.z : 0u;
    const uint32_t olo = live ? dv.x : 0u, ohi = live ? dv.y : 0u;
    const bool small = live && len <= kSmallMax;
    uint32_t rv = 0, rc = 0;
    if (__ballot(small))  // wave-uniform
        verify_lane(reinterpret_cast<uintptr_t>(p.base) + (((uint64_t)ohi << 32) | olo), small ? len : 0u, small, rv,
                    rc);
    uint32_t r = rv | (rc << 8);  // one register across the walk: verdict | L4 result << 8
    uint64_t m = __ballot(live && !small);
    while (m) {  // the long packets, 4 at a time in group order
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
            doff[k] = have ? (((uint64_t)rdl(ohi, j) << 32) | rdl(olo, j)) : 0u;
            lg[k] = have ? rdl(len, j) : 0u;
        }
        uint32_t v2 = 0, c2 = 0;
        verify_group<4>(p.base, doff, lg, tgt, ln, v2, c2, [] {});
        r = (ln == tgt[0] || ln == tgt[1] || ln == tgt[2] || ln == tgt[3]) ? (v2 | (c2 << 8)) : r;
    }
    // the index recomputed from a laundered lane id (held across the walk it spilled)
    uint32_t l2 = lane_id();
    asm volatile("" : "+v"(l2));
    const uint64_t i2 = kConsec ? w * 64u + l2 : ((uint64_t)(l2 >> 2) * G + w) * 4u + (l2 & 3u);
    if (i2 < p.n) {
        p.verdict[i2] = (uint8_t)r;
        if (p.l4)
            p.l4[i2] = (uint16_t)(r >> 8);
    }
    if (p.sample && blockIdx.x == 0 && wave_in_block() == 0)
        verify_sample(p, l2);
}

}  // namespace wg

namespace {

// Per-stream scratch of the compacting verify path: the entry lists, two
// counter sets, and the host-mapped sample words read by the next call.
//
// Protocol (per state): the counter set `parity` is this call's and its lane
// kernel zeroes the other, which the previous call's long kernel has finished
// reading — stream order.  So a state must only ever be used by ONE stream
// (or by streams whose earlier work on it has completed).
//
// Key.  A state belongs to the stream object the handle
// names, on the current device:
//  * an ordinary handle: the handle value.  The value can come back for a
//    new stream only after the old stream object is released, and the
//    runtime releases it only after the stream's work has completed:
//    hipStreamDestroy blocks until then on both HIP runtimes of this image
//    (ROCm 7.2 and PyTorch's 7.0: 21 ms for a pending 20 ms kernel), and even
//    under the documented return-immediately semantics the resources go only
//    once the device is done (tools/exp/stream_identity.hip,
//    profiles/r06_stream_identity.txt).  So a state inherited through a
//    reused value finds its counter set `parity` zero and its lists free;
//  * hipStreamPerThread: one handle value that is a different stream in every
//    host thread — keyed by a per-thread serial that is never reused, so no
//    two threads' streams share a state (round 5 keyed it by the value: four
//    threads on it ran their compacting kernels over one entry list, and the
//    stale entries read another batch's offsets — a GPU memory fault,
//    profiles/r06_mt_before_fix_perthread_vs6.err.txt);
//  * NULL / hipStreamLegacy: the legacy stream, one per device: threads
//    calling on it share its state, serialised by the state's mutex on the
//    host and by stream order on the device.
//
// Storage.  Sample words and counter sets of every state on a device come
// from one pool allocated once per device, right AFTER the device's first
// verify call has launched its (stateless) kernel; a stream's state is a
// table entry and a later stream's first call allocates nothing.  Entry
// lists are per state, allocated when the compacting path first runs there
// and grown (after draining the stream) when a batch needs more; never freed
// (a handful per process).  A stream whose state cannot be made (table full:
// 64 keys, allocation failure, or a call under stream capture) runs the
// stateless walking kernel: the same results by another kernel, never a host
// fallback.  Lookups go through a small per-thread cache, so a call takes no
// process-wide lock once its stream has a state.
struct VerifyState {
    int dev = -1;
    uint64_t key = 0;
    std::mutex mu;
    uint32_t *host_sample = nullptr;  // host-mapped (pool): [0] small count, [1] long bytes, [2] overflow flag
    uint32_t *dev_sample = nullptr;
    uint32_t *ctr = nullptr;          // 2 sets x kVShards x kVCtrStride words (pool)
    bool ctr_zeroed = false;          // zeroed on the stream by the first compacting call
    wg::v4u *ent = nullptr;
    uint64_t cap = 0;                 // entries per shard
    uint32_t parity = 0;
    int last_pick = -1;               // the path the previous call's sample priced (VerifyPath), -1 none
    bool overflow_reported = false;
};
constexpr uint32_t kSampleUnknown = 0xffffffffu;
constexpr size_t kMaxVerifyStates = 64;  // streams, over all devices
constexpr size_t kSampleWords = 16;      // 64 B per stream in the mapped pool
constexpr size_t kCtrWords = 2u * wg::kVShards * wg::kVCtrStride;
struct VerifyPool {
    int dev = -1;
    uint32_t *host = nullptr, *devp = nullptr;  // kMaxVerifyStates x kSampleWords, mapped
    uint32_t *ctr = nullptr;                    // kMaxVerifyStates x kCtrWords
    size_t used = 0;
};
constexpr size_t kMaxVerifyDevices = 64;
std::mutex g_vstate_mu;  // the table and the pools (state creation only)
VerifyState *g_vstate[kMaxVerifyStates];
size_t g_nvstate = 0;
VerifyPool g_vpool[kMaxVerifyDevices];
size_t g_nvpool = 0;
std::atomic<uint64_t> g_thread_serial{0};

// The device's pool (caller holds g_vstate_mu), made on first use; nullptr
// when an allocation fails (then the walking kernel serves that device).
VerifyPool *verify_pool(int dev) {
    for (size_t k = 0; k < g_nvpool; k++)
        if (g_vpool[k].dev == dev)
            return g_vpool[k].host ? &g_vpool[k] : nullptr;
    if (g_nvpool == kMaxVerifyDevices)
        return nullptr;
    VerifyPool &p = g_vpool[g_nvpool++];
    p.dev = dev;  // a failed allocation is remembered: never retried per call
    void *h = nullptr, *d = nullptr, *c = nullptr;
    if (hipHostMalloc(&h, kMaxVerifyStates * kSampleWords * 4u, hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess)
        return nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || hipMalloc(&c, kMaxVerifyStates * kCtrWords * 4u) != hipSuccess) {
        (void)hipHostFree(h);
        return nullptr;
    }
    p.host = static_cast<uint32_t *>(h);
    p.devp = static_cast<uint32_t *>(d);
    p.ctr = static_cast<uint32_t *>(c);
    return &p;
}

// The stream object's key on the current device (see above): the handle, or
// for hipStreamPerThread the calling thread's serial (top bit set: never a
// handle value).
struct VerifyKey {
    int dev;
    uint64_t key;
};

bool verify_key(void *stream, VerifyKey &k) {
    if (hipGetDevice(&k.dev) != hipSuccess)
        return false;
    if (stream == static_cast<void *>(hipStreamPerThread)) {
        static thread_local const uint64_t t_serial = g_thread_serial.fetch_add(1, std::memory_order_relaxed);
        k.key = t_serial | (1ull << 63);
    } else {
        k.key = (uint64_t)reinterpret_cast<uintptr_t>(stream);
    }
    return true;
}

// Per-thread lookup cache: (key -> state); a state never changes key.
struct VCacheEnt {
    int dev = -1;
    uint64_t key = 0;
    VerifyState *s = nullptr;
};
constexpr int kVCache = 4;
thread_local VCacheEnt t_vcache[kVCache];
thread_local int t_vcache_next = 0;

// The stream's state, or nullptr; with create, made when absent (nullptr when
// the table is full or an allocation fails).  No device work is queued or
// waited for here.
VerifyState *verify_state(const VerifyKey &k, bool create) {
    for (const VCacheEnt &c : t_vcache)
        if (c.s && c.dev == k.dev && c.key == k.key)
            return c.s;
    VerifyState *s = nullptr;
    {
        std::lock_guard<std::mutex> g(g_vstate_mu);
        for (size_t i = 0; i < g_nvstate && !s; i++)
            if (g_vstate[i]->dev == k.dev && g_vstate[i]->key == k.key)
                s = g_vstate[i];
        if (!s && create && g_nvstate < kMaxVerifyStates) {
            VerifyPool *pool = verify_pool(k.dev);
            if (pool && pool->used < kMaxVerifyStates) {
                const size_t slot = pool->used++;
                s = new VerifyState;
                s->dev = k.dev;
                s->key = k.key;
                s->host_sample = pool->host + slot * kSampleWords;
                s->dev_sample = pool->devp + slot * kSampleWords;
                s->ctr = pool->ctr + slot * kCtrWords;
                __atomic_store_n(s->host_sample, kSampleUnknown, __ATOMIC_RELAXED);
                __atomic_store_n(s->host_sample + 1, 0u, __ATOMIC_RELAXED);
                __atomic_store_n(s->host_sample + 2, 0u, __ATOMIC_RELAXED);
                g_vstate[g_nvstate++] = s;
            }
        }
    }
    if (s) {
        VCacheEnt &c = t_vcache[t_vcache_next];
        t_vcache_next = (t_vcache_next + 1) % kVCache;
        c = VCacheEnt{k.dev, k.key, s};
    }
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
        return WG_ERR_RUNTIME;  // the caller runs a stateless kernel instead
    if (!s->ctr_zeroed) {  // the stream's first compacting call: both counter sets, in stream order
        if (hipMemsetAsync(s->ctr, 0, 2u * kVShards * kVCtrStride * 4u, st) != hipSuccess)
            return WG_ERR_RUNTIME;
        s->ctr_zeroed = true;
    }
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

// verify_small = 7 (default): per call, one of three kernels from the size
// mixes the previous calls on this stream sampled (smp of 64 spread packets
// <= 64 B, the others lb bytes in all):
//  * the stream's first call: the walking kernel, launched before the
//    stream's state exists (the state is made after the launch, so the first
//    call waits on no allocation and writes no sample);
//  * each later sample prices a kernel: the walking kernel when the sample
//    is unknown or all small (one stateless launch within 7-9 % of the best
//    kernel on any mix, and the fastest on all-small batches), otherwise the
//    cheaper of the wave kernel and the compacting path by a cost model
//    measured on MI355X (profiles/r03_verify_*): the wave kernel
//    spends max(0.88 ns, group bytes / 6.5 TB/s) of chip time per 4-packet
//    group whatever sizes the group mixes; the compacting path pays its lane
//    kernel (~7 ps per descriptor + ~8 ps per small packet) and then the long
//    packets' groups at 1.07x the wave kernel's per-group time;
//  * a kernel other than the walking one runs only when the last TWO
//    samples priced it: a worker that alternates ACK-sized and MTU-sized
//    batches gets the walking kernel (at most 7-9 % over the best on its long
//    batches) instead of a kernel priced for the other shape (the wave kernel
//    on a 64-B batch is ~14x the walking kernel).
// Every kernel gives the same results; the choice only moves time.
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

enum VerifyPath { kPathWave, kPathCompact, kPathWalk };

// consec: each wave's 64 descriptors consecutive — for batches sampled all
// small (1 M x 64 B 0.0145 vs 0.0153 ms: each lane-load instruction of a
// wave covers one 4-KiB run of packets); otherwise sixteen 4-descriptor
// groups a sixteenth of the batch apart (long packets walked: 0.2707 vs
// 0.2772 ms on 1 M x 1500 B), profiles/r05_walk_layout_ab.txt
static int verify_launch_walk(const VerifyParams &p, hipStream_t st, bool consec = false) {
    uint64_t blocks = (p.n + 255) / 256;  // a wave per 64 descriptors
    if (blocks >= 8)
        blocks = (blocks + 7) & ~7ull;
    if (blocks > 0x7fffffffull)
        return WG_ERR_INVALID;
    if (consec)
        hipLaunchKernelGGL(verify_walk_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, p);
    else
        hipLaunchKernelGGL(verify_walk_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, p);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

// The wave kernel at its default geometry (one-shot 4-packet waves, 8 waves
// per SIMD, header bytes in the L4 gather, one 64-B descriptor load per group).
static int verify_launch_wave(const VerifyParams &p, hipStream_t st) {
    uint64_t blocks = (p.n + 15) / 16;
    if (blocks >= 8)
        blocks = (blocks + 7) & ~7ull;
    if (blocks > 0x7fffffffull)
        return WG_ERR_INVALID;
    hipLaunchKernelGGL(verify_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, p);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_verify_desc(const uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n,
                              uint8_t *dev_verdict, uint16_t *dev_l4, void *stream) {
    if (!n)
        return WG_OK;
    if (!dev_base || !dev_desc || !dev_verdict || (reinterpret_cast<uintptr_t>(dev_desc) & 15))
        return WG_ERR_INVALID;
    VerifyParams p{dev_base, dev_desc, dev_verdict, dev_l4, n};
    const Tune t = tune();
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (t.verify_small == 8)  // the walking kernel always
        return verify_launch_walk(p, st);
    if (t.verify_small == 6 || t.verify_small == 7) {
        // Stream capture: the host's choice and the compacting path's
        // alternating counter sets would be frozen into the graph (a replay
        // reuses one set without zeroing it), and the per-stream state cannot
        // be allocated while capturing — so captured calls take a stateless
        // kernel and leave the sample alone.
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        const bool capturing = hipStreamIsCapturing(st, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
        VerifyKey key;
        if (!verify_key(stream, key))
            return verify_launch_walk(p, st, true);
        VerifyState *s = verify_state(key, false);
        if (!s) {
            // the stream's first call (or capturing before it had state, or
            // no state free): the stateless kernel goes out first — in the
            // consecutive layout, the fastest on all-small batches and within
            // 2.4 % of the spread one on long ones — and the state
            // is made behind it for the next call
            const int rc = verify_launch_walk(p, st, true);
            if (!capturing)
                (void)verify_state(key, true);
            return rc;
        }
        std::lock_guard<std::mutex> g(s->mu);
        const uint32_t smp = __atomic_load_n(s->host_sample, __ATOMIC_RELAXED);
        const uint32_t lb = __atomic_load_n(s->host_sample + 1, __ATOMIC_RELAXED);
        if (__atomic_load_n(s->host_sample + 2, __ATOMIC_RELAXED) && !s->overflow_reported) {
            s->overflow_reported = true;
            std::fprintf(stderr, "wireglider_amd: wg_verify_desc entry list overflow on a stream "
                                 "(stream-order protocol broken?); affected packets got verdict 0\n");
        }
        const bool known = smp <= 64u;
        VerifyPath path = kPathCompact;
        if (t.verify_small == 7) {
            const VerifyPath priced = !known || smp == 64u ? kPathWalk
                                      : verify_pick_compact(n, smp, lb, t.verify_auto_t) ? kPathCompact
                                                                                          : kPathWave;
            path = (int)priced == s->last_pick ? priced : kPathWalk;
            if (!capturing)
                s->last_pick = (int)priced;
        }
        if (capturing) {
            path = path == kPathCompact ? kPathWalk : path;
        } else {
            p.sample = s->dev_sample;  // this batch's size mix, for the next call's choice
        }
        if (path == kPathCompact) {
            const uint64_t est = known ? (n * (64u - smp) + 63u) / 64u : n;
            const int rc = verify_compact_launch(p, s, est, t.verify_k2min, st);
            if (rc != WG_ERR_RUNTIME)
                return rc;
            path = kPathWalk;  // no entry lists for this batch: a stateless kernel instead
        }
        // all small by the sample, or no sample yet (as on the first call):
        // the consecutive walking layout; a sample with long packets: spread
        return path == kPathWalk ? verify_launch_walk(p, st, !known || smp == 64u) : verify_launch_wave(p, st);
    }
    return verify_launch_wave(p, st);  // verify_small = 0: the wave kernel
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
        hipLaunchKernelGGL(verify_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, p);
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
