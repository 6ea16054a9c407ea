// gso.hip — batched TSO/USO segmentation with per-segment checksum fixup on
// MI355X (gfx950).  Per super-buffer this is worker_impl::do_tun_gso_split
// (reference worker/offload.cpp:46-216) bit for bit, quirks included.
//
// One 256-thread workgroup per super-buffer; its four waves take the
// segments round-robin.  Per segment a wave, in ONE pass over the payload:
//   - streams the payload's destination-aligned 16-B chunks: ONE 16-B load
//     per chunk from its (unaligned) source address, stored at the aligned
//     destination and summed from the same registers;
//   - moves the <= 15-byte unaligned head/tail of the payload one byte per lane;
//   - rebuilds the header prefix one byte per lane with the reference's
//     fix-ups applied in the reference's order (IPv4 id/len or IPv6 plen ->
//     IPv4 header checksum -> TCP seq/FIN/PSH or UDP len -> L4 checksum).
// The reference touches every payload byte twice (std::copy at :165-166, then
// the checksum at :202); this kernel reads it once and writes it once.
//
// Register economy is the design constraint: the kernel is HBM-bound and its
// bytes in flight scale with resident waves, so everything per lane is a
// 32-bit offset from a wave-uniform base, the per-segment header values are
// looked up (v_writelane table + ds_bpermute) instead of selected, and the
// classification (plan pass) and the GSO_NONE in-place checksum (finalize
// pass) are kernels of their own.
#include <hip/hip_runtime.h>

#include "wg_device.hpp"
#include "wg_internal.hpp"
#include "wg_gso.hpp"
#include "wg_l4wave.hpp"
#include "wireglider_amd.h"

// v_writelane_b32 (no clang builtin in this toolchain: bind the LLVM
// intrinsic by name).
extern "C" __device__ int wg_writelane_i32(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

namespace wg {

__device__ __forceinline__ void st16_nt(uintptr_t addr, v4u v) {
    __builtin_nontemporal_store(v, reinterpret_cast<__attribute__((address_space(1))) v4u *>(addr));
}

// Variant bits (wg_tune_set("gso_ablate")), both correct: 1 = non-temporal
// payload stores (default-policy stores measured faster because the
// segment-edge byte stores then merge with the chunk stores in L2); 32 =
// blocks -> super-buffers in launch order instead of XCD-swizzled (the
// swizzle keeps consecutive super-buffers on one XCD).  Timing-only
// ablations with wrong output live in tools/exp, never in this library.
// 64 is not an ablation but the headers-only mode of wg_encap_batch: every
// segment's header and the payload up to the header's 64-B block boundary
// are written (checksums over the whole loaded payload as always), the rest
// of the payload is not — the AEAD reads it from the input instead.
enum : int { kAblNtStore = 1, kAblNoSwizzle = 32, kHdrOnly = 64 };

template <int A>
__device__ __forceinline__ void st16x(uintptr_t addr, v4u v) {
    if constexpr (A & kAblNtStore)
        st16_nt(addr, v);
    else
        *reinterpret_cast<__attribute__((address_space(1))) v4u *>(addr) = v;
}

// Per-super-buffer plan, written by gso_plan_kernel into the caller's
// wg_gso_result slot (24 B; gso_finalize_kernel overwrites it with the
// result): the classification and the invariant header sums, so the split
// kernel's waves start their payload loads one (scalar) load after launch
// instead of after the descriptor -> prefix -> classification chain.
struct GsoPlan {
    uint16_t hdr_len, cs;
    uint16_t l4off;
    uint8_t kind;     // kPlan* bits
    uint8_t flags13;  // TCP flags byte of the prefix; -status when not split
    uint16_t gso, nseg;
    uint16_t id0, ip_base;  // sums folded to 16 bits (zero-preserving, congruent)
    uint16_t l4h_base, ps_sum;
    uint32_t seq0;
};
static_assert(sizeof(GsoPlan) == sizeof(wg_gso_result), "plan lives in the result slot");
// kind bits: the split-path family / protocol (v6, tcp: the unmasked :151
// test), the classification's isv6 (:48) and ecn (bits 2-3), GSO_NONE +
// NEEDS_CSUM in place, split.
enum : uint32_t { kPlanV6 = 1, kPlanTcp = 2, kPlanEcnShift = 2, kPlanIsV6 = 0x10, kPlanInplace = 0x40, kPlanSplit = 0x80 };
struct PlanRaw {  // GsoPlan as dwords (little-endian field order above)
    uint32_t w[6];
};
struct DescRaw {  // wg_gso_desc dwords 0-4: in_offset, out_offset, in_len
    uint32_t w[5];
};

// Wave-uniform record loads through the constant address space: s_load.
template <typename T>
__device__ __forceinline__ T sload(const T *p) {
#if __HIP_DEVICE_COMPILE__
    return *reinterpret_cast<__attribute__((address_space(4))) const T *>(reinterpret_cast<uintptr_t>(p));
#else
    return *p;
#endif
}

// One output segment of the full split by one wave, in two phases so a wave may have several
// segments' loads in flight: seg_issue() issues every load of the segment
// (branch-free: clamped offsets, masked use); seg_finish() stores, sums and
// writes the header.  Only the loaded data and the segment index cross the
// phase boundary; the (scalar) geometry is recomputed.
struct SegGeom {
    uintptr_t seg, oa, c0, sa;
    uintptr_t base;  // source of output chunk 0 (unaligned), or the zero chunk when there is none
    uint32_t datalen, pktlen, nint, he, ts;
    bool last;
};

__device__ __forceinline__ SegGeom seg_geom(const Ctx &c, uintptr_t out_base, uint32_t i) {
    SegGeom g;
    g.seg = out_base + (uintptr_t)i * (c.hdr_len + c.gso);
    const uint32_t off = i * c.gso;
    g.datalen = c.rest - off < c.gso ? c.rest - off : c.gso;
    g.pktlen = c.hdr_len + g.datalen;
    g.last = i + 1 == c.nseg;
    g.oa = g.seg + c.hdr_len;       // payload, destination
    g.sa = c.in + c.hdr_len + off;  // payload, source
    const uintptr_t ob = g.oa + g.datalen;
    g.c0 = (g.oa + 15) & ~(uintptr_t)15;  // destination-aligned interior chunks [c0, c1)
    const uintptr_t c1 = ob & ~(uintptr_t)15;
    g.nint = c1 > g.c0 ? (uint32_t)((c1 - g.c0) >> 4) : 0u;
    // head [oa, he) and tail [ts, datalen) as offsets from oa, <= 15 bytes each
    g.he = (uint32_t)((g.c0 < ob ? g.c0 : ob) - g.oa);
    g.ts = (uint32_t)((c1 > g.c0 ? c1 : g.c0) - g.oa);
    // Interior chunk k = ONE 16-B load at its unaligned source address
    // c0 + 16k + (sa - oa): inside the payload, so always in bounds; an empty
    // interior points every lane at the static zero chunk.
    g.base = g.nint ? g.c0 + (g.sa - g.oa) : reinterpret_cast<uintptr_t>(&g_zero16);
    return g;
}

// Payload head on lanes 0-15, tail on lanes 16-31: this lane's byte offset
// from oa (the source byte is at the same offset from sa), or kNoEdge.
constexpr uint32_t kNoEdge = 0xffffffffu;
__device__ __forceinline__ uint32_t edge_off(const SegGeom &g, uint32_t lane) {
    const uint32_t xt = g.ts + lane - 16u;
    if (lane < 16 && lane < g.he)
        return lane;
    if (lane >= 16 && lane < 32 && xt < g.datalen)
        return xt;
    return kNoEdge;
}

struct SegFront {
    uint32_t i, pb;
    v4u lo0, lo1;  // interior chunks lane, lane + 64
};

template <int Abl>
__device__ __forceinline__ void seg_issue(const Ctx &c, uintptr_t out_base, uint32_t i, uint32_t lane, SegFront &f) {
    const SegGeom g = seg_geom(c, out_base, i);
    f.i = i;
    const uint32_t last = g.nint ? g.nint - 1 : 0u;
    f.lo0 = ld16(g.base + 16u * (lane < last ? lane : last));
    f.lo1 = ld16(g.base + 16u * (lane + 64 < last ? lane + 64 : last));
    const uint32_t eo = edge_off(g, lane);
    f.pb = ld8(g.sa + (eo != kNoEdge ? eo : 0u));
}

template <int Abl>
__device__ __forceinline__ void seg_finish(const Ctx &c, uintptr_t out_base, const SegFront &f, uint32_t lane) {
    const SegGeom g = seg_geom(c, out_base, f.i);
    const uint32_t i = f.i, pktlen = g.pktlen;
    Acc acc;
    // payload: store and sum (destination-aligned chunks: absolute pairing)
    if (lane < g.nint) {
        st16x<Abl>(g.c0 + 16u * lane, f.lo0);
        acc.add4(f.lo0);
    }
    if (lane + 64 < g.nint) {
        st16x<Abl>(g.c0 + 16u * (lane + 64), f.lo1);
        acc.add4(f.lo1);
    }
    if (g.nint > 128) {  // long segments (gso > ~2 KiB)
        for (uint32_t k = lane + 128; k < g.nint; k += 64) {
            const v4u v = ld16(g.base + 16u * k);
            st16x<Abl>(g.c0 + 16u * k, v);
            acc.add4(v);
        }
    }
    const uint32_t eo = edge_off(g, lane);
    if (eo != kNoEdge) {
        st8(g.oa + eo, f.pb);
        acc.add(f.pb << (8u * (((uint32_t)g.oa + eo) & 1u)));
    }

    // checksums: the invariant header sums plus this segment's fields
    // (exact integer sums, so the 0x0000 / 0xFFFF split stays exact)
    uint32_t ipcs = 0;
    if (!c.v6)
        ipcs = ~fold16_32(c.ip_base + bswap16(pktlen & 0xffffu) + bswap16((c.id0 + i) & 0xffffu)) & 0xffffu;
    const uint32_t seq = c.seq0 + c.gso * i;
    const uint32_t flags = g.last ? c.flags13 : (c.flags13 & ~0x09u);  // FIN/PSH only on the last segment
    uint32_t l4h = c.l4h_base;
    if (c.tcp)
        l4h += bswap16(seq >> 16) + bswap16(seq & 0xffffu) + (flags << 8);
    else
        l4h += bswap16((pktlen - c.cs) & 0xffffu);
    uint32_t lp = fold16(acc.value());
    if ((g.seg + c.cs) & 1u)  // payload summed in absolute pairing; the L4 region pairs from seg + cs
        lp = bswap16(lp);
    uint32_t T = wave_sum_u32(lp) + l4h + c.ps_sum;
    T += ((c.tcp ? 6u : 17u) << 8) + bswap16((pktlen - c.cs) & 0xffffu);
    const uint32_t l4cs = ~fold16_32(T) & 0xffffu;
    // write the header prefix: each byte is the prefix byte or one byte of a
    // per-segment value, by its field code (checksums in native order,
    // :185-186, :203-204).  The values go into lanes 1-7 of one VGPR and
    // every lane fetches its field with ONE ds_bpermute (full EXEC).
    uint32_t tbl = 0;
    tbl = (uint32_t)wg_writelane_i32((int)pktlen, kFldPkt, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)(c.id0 + i), kFldId, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)ipcs, kFldIpcs, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)l4cs, kFldL4cs, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)seq, kFldSeq, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)(pktlen - c.cs), kFldUlen, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)flags, kFldFlags, (int)tbl);
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((c.hc0 & 7u) << 2), (int)tbl);
    const uint32_t b0 = (c.hc0 & 7u) ? (r0 >> (c.hc0 >> 8)) & 0xffu : c.hb0;
    if (lane < c.hdr_len)
        st8(g.seg + lane, b0);
    if (c.hdr_len > 64) {
        const uint32_t r1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((c.hc1 & 7u) << 2), (int)tbl);
        const uint32_t b1 = (c.hc1 & 7u) ? (r1 >> (c.hc1 >> 8)) & 0xffu : c.hb1;
        if (lane + 64 < c.hdr_len)
            st8(g.seg + lane + 64, b1);
        if (c.hdr_len > 128) {
            HdrVals hv;
            hv.v[0] = 0;
            hv.v[kFldPkt] = pktlen;
            hv.v[kFldId] = c.id0 + i;
            hv.v[kFldIpcs] = ipcs;
            hv.v[kFldL4cs] = l4cs;
            hv.v[kFldSeq] = seq;
            hv.v[kFldUlen] = pktlen - c.cs;
            hv.v[kFldFlags] = flags;
            for (uint32_t j = lane + 128; j < c.hdr_len; j += 64)
                st8(g.seg + j, hdr_byte_slow(hv, hdr_code(c, j), ld8(c.in + j)));
        }
    }
}

// The headers-only split (wg_encap_batch) on raw buffer ops.  Most of its
// lanes have nothing to store (only the header's 64-B block of payload is
// written), so every access is a buffer op at a 32-bit offset from the
// super-buffer's input / output base and an idle lane gets the offset kOob:
// the range check drops its store and returns 0 for its load (adding
// nothing to the sum) — no EXEC save / restore per conditional access and no
// 64-bit address arithmetic per lane.  3-4 % faster than seg_issue /
// seg_finish on the encap step; 1 % slower than them on the full split
// (config 3), which therefore stays on global_* ops.
struct HSegGeom {
    uint32_t seg, oa, sa;  // segment start, payload destination (from c.out), payload source (from c.in)
    uint32_t c0, src0;     // first destination-aligned interior chunk, and its (unaligned) source
    uint32_t datalen, pktlen, nint, he, ts;
    bool last;
};

__device__ __forceinline__ HSegGeom hseg_geom(const Ctx &c, uint32_t i) {
    HSegGeom g;
    g.seg = i * (c.hdr_len + c.gso);
    const uint32_t off = i * c.gso;
    g.datalen = c.rest - off < c.gso ? c.rest - off : c.gso;
    g.pktlen = c.hdr_len + g.datalen;
    g.last = i + 1 == c.nseg;
    g.oa = g.seg + c.hdr_len;
    g.sa = c.hdr_len + off;
    // destination-aligned interior chunks [A0, A1) in "absolute low bits"
    // terms (offset + omis), head [oa, A0) and tail [A1, ob) <= 15 bytes each
    const uint32_t x0 = g.oa + c.omis, xb = x0 + g.datalen;
    const uint32_t A0 = (x0 + 15u) & ~15u, A1 = xb & ~15u;
    g.nint = A1 > A0 ? (A1 - A0) >> 4 : 0u;
    g.c0 = A0 - c.omis;
    g.he = (A0 < xb ? A0 : xb) - x0;
    g.ts = (A1 > A0 ? A1 : A0) - x0;
    g.src0 = g.c0 + (g.sa - g.oa);  // mod 2^32: src0 + 16k is the true, small offset
    return g;
}

__device__ __forceinline__ uint32_t hedge_off(const HSegGeom &g, uint32_t lane) {
    const uint32_t xt = g.ts + lane - 16u;
    const bool h = lane < 16 && lane < g.he;
    const bool t = lane >= 16 && lane < 32 && xt < g.datalen;
    return h ? lane : (t ? xt : kNoEdge);
}

__device__ __forceinline__ void hseg_issue(const Ctx &c, uint32_t i, uint32_t lane, SegFront &f) {
    const HSegGeom g = hseg_geom(c, i);
    f.i = i;
    f.lo0 = bld16(c.rin, lane < g.nint ? g.src0 + 16u * lane : kOob);
    f.lo1 = bld16(c.rin, lane + 64 < g.nint ? g.src0 + 16u * lane + 1024u : kOob);
    const uint32_t eo = hedge_off(g, lane);
    f.pb = bld8(c.rin, eo != kNoEdge ? g.sa + eo : kOob);
}

__device__ __forceinline__ void hseg_finish(const Ctx &c, const SegFront &f, uint32_t lane) {
    const HSegGeom g = hseg_geom(c, f.i);
    const uint32_t i = f.i, pktlen = g.pktlen;
    Acc acc;
    // every payload byte is summed; only those in the header's last 64-B
    // block are stored (every such chunk is among the first 64)
    const uint32_t hlim = g.seg + ((c.hdr_len + 63u) & ~63u);
    const uint32_t d0 = g.c0 + 16u * lane;
    bst16(c.rout, (lane < g.nint && d0 < hlim) ? d0 : kOob, f.lo0);
    acc.add4(f.lo0);
    acc.add4(f.lo1);
    for (uint32_t k0 = 128; k0 < g.nint; k0 += 64) {  // long segments (gso > ~2 KiB)
        const uint32_t k = k0 + lane;
        acc.add4(bld16(c.rin, k < g.nint ? g.src0 + 16u * k : kOob));
    }
    const uint32_t eo = hedge_off(g, lane);
    const uint32_t eoff = g.oa + eo;
    bst8(c.rout, (eo != kNoEdge && eoff < hlim) ? eoff : kOob, f.pb);
    acc.add(f.pb << (8u * ((eoff + c.omis) & 1u)));  // pb = 0 on lanes without an edge byte

    uint32_t ipcs = 0;
    if (!c.v6)
        ipcs = ~fold16_32(c.ip_base + bswap16(pktlen & 0xffffu) + bswap16((c.id0 + i) & 0xffffu)) & 0xffffu;
    const uint32_t seq = c.seq0 + c.gso * i;
    const uint32_t flags = g.last ? c.flags13 : (c.flags13 & ~0x09u);
    uint32_t l4h = c.l4h_base;
    if (c.tcp)
        l4h += bswap16(seq >> 16) + bswap16(seq & 0xffffu) + (flags << 8);
    else
        l4h += bswap16((pktlen - c.cs) & 0xffffu);
    uint32_t lp = fold16(acc.value());
    if ((g.seg + c.cs + c.omis) & 1u)
        lp = bswap16(lp);
    uint32_t T = wave_sum_u32(lp) + l4h + c.ps_sum;
    T += ((c.tcp ? 6u : 17u) << 8) + bswap16((pktlen - c.cs) & 0xffffu);
    const uint32_t l4cs = ~fold16_32(T) & 0xffffu;
    // the header prefix, as in seg_finish
    uint32_t tbl = 0;
    tbl = (uint32_t)wg_writelane_i32((int)pktlen, kFldPkt, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)(c.id0 + i), kFldId, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)ipcs, kFldIpcs, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)l4cs, kFldL4cs, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)seq, kFldSeq, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)(pktlen - c.cs), kFldUlen, (int)tbl);
    tbl = (uint32_t)wg_writelane_i32((int)flags, kFldFlags, (int)tbl);
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((c.hc0 & 7u) << 2), (int)tbl);
    const uint32_t b0 = (c.hc0 & 7u) ? (r0 >> (c.hc0 >> 8)) & 0xffu : c.hb0;
    bst8(c.rout, lane < c.hdr_len ? g.seg + lane : kOob, b0);
    if (c.hdr_len > 64) {
        const uint32_t r1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((c.hc1 & 7u) << 2), (int)tbl);
        const uint32_t b1 = (c.hc1 & 7u) ? (r1 >> (c.hc1 >> 8)) & 0xffu : c.hb1;
        bst8(c.rout, lane + 64 < c.hdr_len ? g.seg + lane + 64u : kOob, b1);
        if (c.hdr_len > 128) {
            HdrVals hv;
            hv.v[0] = 0;
            hv.v[kFldPkt] = pktlen;
            hv.v[kFldId] = c.id0 + i;
            hv.v[kFldIpcs] = ipcs;
            hv.v[kFldL4cs] = l4cs;
            hv.v[kFldSeq] = seq;
            hv.v[kFldUlen] = pktlen - c.cs;
            hv.v[kFldFlags] = flags;
            for (uint32_t j = lane + 128; j < c.hdr_len; j += 64)
                st8(c.out + g.seg + j, hdr_byte_slow(hv, hdr_code(c, j), ld8(c.in + j)));
        }
    }
}

// One segment's loads / completion: the headers-only split on buffer ops,
// everything else on global_* ops.
template <int Abl>
__device__ __forceinline__ void seg_go(const Ctx &c, uintptr_t out_base, uint32_t i, uint32_t lane, SegFront &f) {
    if constexpr (Abl & kHdrOnly)
        hseg_issue(c, i, lane, f);
    else
        seg_issue<Abl>(c, out_base, i, lane, f);
}
template <int Abl>
__device__ __forceinline__ void seg_done(const Ctx &c, uintptr_t out_base, const SegFront &f, uint32_t lane) {
    if constexpr (Abl & kHdrOnly)
        hseg_finish(c, f, lane);
    else
        seg_finish<Abl>(c, out_base, f, lane);
}

// Main kernel.  The flat grid walks (super-buffer, group) units: unit u is
// group u % G of super-buffer u / G, so the G blocks of one super-buffer are
// consecutive in dispatch order (and, after the XCD swizzle, on one XCD).
// Group g's waves take segment slots g*W .. g*W+W-1 of the super-buffer
// (stride G*W); blockIdx.y (grid y) further splits the slots.  More groups
// mean shorter waves, each paying the per-wave setup (plan + descriptor,
// template bytes, field codes) again: G = 3 x W = 4 measured best.
// S = segments per wave step: 0 one at a time (occupancy hides latency),
// 1 ping-pong pipeline (the next segment's loads in flight while this one
// finishes), 2-4 that many, a slot stride apart, issued then all finished (4,
// the default: with 3 groups of 4 waves a 45-segment super-buffer's wave
// sends all its ~4 segments' loads out at once).
template <int W, int S, int Abl>
__global__ __launch_bounds__(64 * W) void gso_split_kernel(GsoParams p) {
    constexpr uint32_t kStep = S ? S : 1;
    const uint32_t lane = lane_id();
    const uint32_t G = p.groups;
    const uint32_t gstride = gridDim.y * G * W * kStep;
    const uint64_t units = (p.list ? sload(p.list) : p.n) * G;
    const uint64_t u0 = (Abl & kAblNoSwizzle) ? blockIdx.x : xcd_swizzle(blockIdx.x, gridDim.x);
    for (uint64_t u = u0; u < units; u += gridDim.x) {
        const uint64_t ub = G == 1 ? u : u / G;
        const uint64_t b = p.list ? sload(p.list + 1 + ub) : ub;
        const uint32_t gw = (blockIdx.y * G + (uint32_t)(u - ub * G)) * W + wave_in_block();  // segment slot
        // plan and descriptor as raw dwords: one s_load each (16-bit struct
        // fields would become dependent vector loads), unpacked by shifts
        const DescRaw dr = sload(reinterpret_cast<const DescRaw *>(p.desc + b));  // first 20 B of the 40-B descriptor
        const PlanRaw pr = sload(reinterpret_cast<const PlanRaw *>(p.res) + b);
        // all eleven dwords in one scalar round trip: without this the
        // compiler sinks each load below the first branch that needs it
        // and chains three waits before the first payload load
        asm volatile("" ::"s"(pr.w[0]), "s"(pr.w[1]), "s"(pr.w[2]), "s"(pr.w[3]), "s"(pr.w[4]), "s"(pr.w[5]),
                     "s"(dr.w[0]), "s"(dr.w[1]), "s"(dr.w[2]), "s"(dr.w[3]), "s"(dr.w[4]));
        const uint32_t kind = (pr.w[1] >> 16) & 0xffu, nseg = pr.w[2] >> 16;
        if (!(kind & kPlanSplit) || gw >= nseg)
            continue;  // passthrough / error (in-place work: gso_finalize_kernel) or no segment for this slot
        if constexpr (Abl & kHdrOnly) {
            if (p.synth && syn_eligible(pr.w[0] & 0xffffu, pr.w[0] >> 16, pr.w[1] & 0xffffu)) {
                const uint32_t H = pr.w[0] & 0xffffu, gso = pr.w[2] & 0xffffu;
                uint32_t bytes;
                if (encap_fit((uint64_t)(dr.w[4] - H) + (uint64_t)nseg * H, H + gso, p.fit_segs, p.fit_size,
                              p.fit_cap, bytes))
                    continue;  // wg_encap_batch's AEAD writes these headers itself
            }
        }
        const uint64_t in_off = (uint64_t)dr.w[0] | ((uint64_t)dr.w[1] << 32);
        const uint64_t out_off = (uint64_t)dr.w[2] | ((uint64_t)dr.w[3] << 32);
        const uint32_t in_len = dr.w[4];
        Ctx c;
        c.in = reinterpret_cast<uintptr_t>(p.in) + in_off;
        c.in_len = in_len;
        c.hdr_len = pr.w[0] & 0xffffu;
        c.cs = pr.w[0] >> 16;
        c.l4off = pr.w[1] & 0xffffu;
        c.gso = pr.w[2] & 0xffffu;
        c.nseg = nseg;
        c.rest = in_len - c.hdr_len;
        c.v6 = kind & kPlanV6;
        c.tcp = kind & kPlanTcp;
        c.id0 = pr.w[3] & 0xffffu;
        c.seq0 = pr.w[5];
        c.ip_base = pr.w[3] >> 16;
        c.l4h_base = pr.w[4] & 0xffffu;
        c.ps_sum = pr.w[4] >> 16;
        c.flags13 = pr.w[1] >> 24;
        // this lane's template bytes (used when the first header is written)
        // and field codes
        c.hb0 = ld8(c.in + (lane < c.hdr_len ? lane : 0u));
        c.hb1 = ld8(c.in + (lane + 64 < c.hdr_len ? lane + 64 : 0u));
        const uintptr_t out_base = reinterpret_cast<uintptr_t>(p.out) + out_off;
        if constexpr (Abl & kHdrOnly) {
            c.out = out_base;
            c.omis = (uint32_t)out_base & 15u;
            c.rin = make_rsrc(c.in);
            c.rout = make_rsrc(out_base);
        }
        if constexpr (S == 0) {
            c.hc0 = hdr_code(c, lane);
            c.hc1 = hdr_code(c, lane + 64);
            for (uint32_t i = gw; i < c.nseg; i += gstride) {
                SegFront A;
                seg_go<Abl>(c, out_base, i, lane, A);
                seg_done<Abl>(c, out_base, A, lane);
            }
        } else if constexpr (S == 1) {
            const uint32_t last = c.nseg - 1;
            uint32_t i = gw;
            SegFront A, B;
            seg_go<Abl>(c, out_base, i, lane, A);
            // the header field codes are needed only when the first header is
            // written: computed while the first segment's loads are in flight
            c.hc0 = hdr_code(c, lane);
            c.hc1 = hdr_code(c, lane + 64);
            if (i + gstride > last) {  // the slot's only segment: no second slot to fill
                seg_done<Abl>(c, out_base, A, lane);
                continue;
            }
            for (;;) {
                const uint32_t i1 = i + gstride;
                seg_go<Abl>(c, out_base, i1 < last ? i1 : last, lane, B);
                seg_done<Abl>(c, out_base, A, lane);
                if (i1 > last)
                    break;
                const uint32_t i2 = i1 + gstride;
                seg_go<Abl>(c, out_base, i2 < last ? i2 : last, lane, A);
                seg_done<Abl>(c, out_base, B, lane);
                if (i2 > last)
                    break;
                i = i2;
            }
        } else {
            c.hc0 = hdr_code(c, lane);
            c.hc1 = hdr_code(c, lane + 64);
            // the wave's S segments a slot stride apart (gw, gw + G W, ...):
            // config 3 -0.85 %, UDP_L4 -0.73 % against S consecutive ones
            // (profiles/r05_gso/ab_spread_segments.txt)
            const uint32_t sstr = gstride / S;
            for (uint32_t i0 = gw; i0 < c.nseg; i0 += gstride) {
                SegFront f[S];
#pragma unroll
                for (int k = 0; k < S; k++)
                    seg_go<Abl>(c, out_base, i0 + k * sstr < c.nseg ? i0 + k * sstr : c.nseg - 1, lane, f[k]);
#pragma unroll
                for (int k = 0; k < S; k++)
                    if (i0 + k * sstr < c.nseg)
                        seg_done<Abl>(c, out_base, f[k], lane);
            }
        }
    }
}

// Plan pass, ONE THREAD per super-buffer: classification (:48-134), the
// per-super-buffer fields (IPv4 id, TCP seq read after the :145-149 zeroing)
// and the invariant header sums into the GsoPlan.  This is scalar,
// branchy work on a few dozen bytes; a thread does it for 64 super-buffers
// per wave where a wave per super-buffer spent ~400 instructions of one
// wave each (130 us for config 3, instruction-issue bound).  Each thread
// stages its prefix (bytes [0, min(in_len, 128)), nine aligned 16-B chunks)
// in its own LDS area, then reads bytes from there; bytes >= 128 (headers
// past 128 bytes: rare) are loaded directly.  No barrier: a thread only
// touches its own area.  GSO_NONE + NEEDS_CSUM super-buffers are marked
// kPlanInplace; gso_finalize_kernel does their checksums (:56-78).
constexpr uint32_t kPlanBlock = 256, kPreChunks = 9;
constexpr uint32_t kPreStride = 4 * kPreChunks + 1;  // dwords per thread: odd, so threads' bytes spread over the banks

__global__ __launch_bounds__(kPlanBlock) void gso_plan_kernel(GsoParams p) {
    __shared__ uint32_t s_pre[kPlanBlock * kPreStride];
    const uint32_t t = threadIdx.x;
    const uint64_t b = (uint64_t)blockIdx.x * kPlanBlock + t;
    if (b >= p.n)
        return;
    const wg_gso_desc dsc = p.desc[b];
    const uintptr_t in = reinterpret_cast<uintptr_t>(p.in) + dsc.in_offset;
    const uint32_t win = dsc.in_len < 128u ? dsc.in_len : 128u;  // staged bytes
    const uint32_t o = (uint32_t)(in & 15u);
    // branch-free: chunks past the window re-read its last chunk (an aligned
    // 16-B chunk holding a byte of the buffer lies inside its page)
    const uintptr_t base = win ? (in & ~(uintptr_t)15) : reinterpret_cast<uintptr_t>(&g_zero16);
    const uint32_t last = win ? (o + win - 1u) >> 4 : 0u;
    v4u ch[kPreChunks];
#pragma unroll
    for (uint32_t k = 0; k < kPreChunks; k++)
        ch[k] = ld16(base + 16u * (k < last ? k : last));
    uint32_t *my = &s_pre[t * kPreStride];
#pragma unroll
    for (uint32_t k = 0; k < kPreChunks; k++) {
        my[4 * k] = ch[k].x;
        my[4 * k + 1] = ch[k].y;
        my[4 * k + 2] = ch[k].z;
        my[4 * k + 3] = ch[k].w;
    }
    const uint8_t *mb = reinterpret_cast<const uint8_t *>(my) + o;
    auto byte = [&](uint32_t j) -> uint32_t { return j < win ? (uint32_t)mb[j] : ld8(in + j); };

    Ctx c;
    Cls cl = classify_by(dsc, reinterpret_cast<uintptr_t>(p.in), c, byte);
    // Super-buffers longer than 65,535 bytes (tun never delivers one: the IP
    // length fields are 16-bit) are out of contract for splitting and in-place
    // checksumming: status -3 rather than 16-bit plan fields that wrap.
    if (dsc.in_len > 65535u && (!cl.pass || cl.inplace)) {
        cl.status = -3;
        cl.pass = true;
        cl.inplace = false;
    }
    GsoPlan pl{};
    pl.hdr_len = (uint16_t)c.hdr_len;
    const uint32_t cls_bits = (cl.isv6 ? kPlanIsV6 : 0u) | (cl.ecn << kPlanEcnShift);
    if (!cl.pass) {
        c.id0 = (byte(4) << 8) | byte(5);
        // seq0 is read after the prefix's L4 checksum field was zeroed
        // (:149 before :152-154), which matters when the two overlap.
        c.seq0 = 0;
        if (c.tcp) {
            for (uint32_t q = 0; q < 4; q++) {
                const uint32_t j = c.cs + 4 + q;
                const uint32_t bb = (j == c.l4off || j == c.l4off + 1) ? 0u : byte(j);
                c.seq0 |= bb << (8u * (3u - q));
            }
        }
        hdr_bases_thread(c, byte);
        pl.cs = (uint16_t)c.cs;
        pl.l4off = (uint16_t)c.l4off;
        pl.kind = (uint8_t)(kPlanSplit | cls_bits | (c.v6 ? kPlanV6 : 0u) | (c.tcp ? kPlanTcp : 0u));
        pl.flags13 = (uint8_t)c.flags13;
        pl.gso = (uint16_t)c.gso;
        pl.nseg = (uint16_t)c.nseg;
        pl.id0 = (uint16_t)c.id0;
        pl.ip_base = (uint16_t)fold16_32(c.ip_base);
        pl.l4h_base = (uint16_t)fold16_32(c.l4h_base);
        pl.ps_sum = (uint16_t)fold16_32(c.ps_sum);
        pl.seq0 = c.seq0;
    } else {
        // passthrough / error: the status rides in flags13 (as -status)
        const bool tcp = cl.inplace && (cl.isv6 ? byte(6) : byte(9)) == 6;  // :67-70
        pl.cs = (uint16_t)c.cs;
        pl.l4off = (uint16_t)c.l4off;
        pl.kind = (uint8_t)(cls_bits | (cl.inplace ? kPlanInplace : 0u) | (c.v6 ? kPlanV6 : 0u) |
                            (tcp ? kPlanTcp : 0u));
        pl.flags13 = (uint8_t)(-cl.status);
    }
    reinterpret_cast<GsoPlan *>(p.res)[b] = pl;
    if (p.list) {
        // still split here unless wg_encap_batch's AEAD synthesizes it
        uint32_t bytes;
        const bool split =
            !cl.pass && !(p.synth && syn_eligible(c.hdr_len, c.cs, c.l4off) &&
                          encap_fit((uint64_t)(dsc.in_len - c.hdr_len) + (uint64_t)c.nseg * c.hdr_len,
                                    c.hdr_len + c.gso, p.fit_segs, p.fit_size, p.fit_cap, bytes));
        const uint64_t m = __ballot(split);  // the wave's active threads
        if (split) {
            const uint32_t lane = lane_id(), lead = (uint32_t)__builtin_ctzll(m);
            uint32_t base = 0;
            if (lane == lead)
                base = atomicAdd(p.list, (uint32_t)__builtin_popcountll(m));
            base = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lead << 2), (int)base);
            p.list[1u + base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull))] = (uint32_t)b;
        }
    }
}

// Finalize (same stream, after the split kernel), thread per super-buffer
// from its plan: the PacketBatch record, and the reference's in-place zeroing
// of the input prefix's ip_sum / L4 checksum field (:145-149) — only once
// every block of the split kernel has read that prefix, hence a separate
// launch.  Then each wave checksums its GSO_NONE + NEEDS_CSUM super-buffers
// in place (:56-78), one at a time, the whole wave per super-buffer.
__global__ __launch_bounds__(256) void gso_finalize_kernel(GsoParams p) {
    const uint32_t lane = lane_id();
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = b < p.n;
    GsoPlan pl{};
    uint64_t in_off = 0;
    uint32_t in_len = 0;
    if (live) {
        pl = reinterpret_cast<const GsoPlan *>(p.res)[b];
        in_off = p.desc[b].in_offset;
        in_len = p.desc[b].in_len;
    }
    const uint32_t kind = pl.kind;
    const uintptr_t in = reinterpret_cast<uintptr_t>(p.in) + in_off;
    if (live) {
        const bool split = kind & kPlanSplit;
        wg_gso_result r;
        const int status = split ? 0 : -(int)pl.flags13;
        r.hdr_len = pl.hdr_len;
        r.isv6 = (kind & kPlanIsV6) ? 1 : 0;
        r.ecn = (uint8_t)((kind >> kPlanEcnShift) & 3u);
        r.status = (int8_t)status;
        r.passthrough = split ? 0 : 1;
        r.out_len = split ? (uint64_t)(in_len - pl.hdr_len) + (uint64_t)pl.nseg * pl.hdr_len : (status ? 0 : in_len);
        r.segment_size = split ? (uint32_t)pl.hdr_len + pl.gso : (status ? 0u : in_len);
        for (int k = 0; k < 6; k++) r.pad[k] = 0;
        p.res[b] = r;
        if (split) {
            if (!(kind & kPlanV6)) {
                st8(in + 10, 0);
                st8(in + 11, 0);
            }
            st8(in + pl.l4off, 0);
            st8(in + pl.l4off + 1, 0);
        }
    }
    uint64_t todo = __ballot(live && (kind & kPlanInplace));
    while (todo) {
        const uint32_t j = (uint32_t)__builtin_ctzll(todo);
        todo &= todo - 1;
        Ctx c;
        // through uint32_t: readlane returns int, and int -> uintptr_t would
        // sign-extend an address whose bit 31 is set
        c.in = (uintptr_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)in, (int)j) |
               ((uintptr_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(in >> 32), (int)j) << 32);
        c.in_len = (uint32_t)__builtin_amdgcn_readlane((int)in_len, (int)j);
        c.cs = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pl.cs, (int)j);
        c.l4off = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pl.l4off, (int)j);
        const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)kind, (int)j);
        c.v6 = kj & kPlanV6;
        c.tcp = kj & kPlanTcp;
        do_inplace(c, lane);
    }
}

}  // namespace wg

using namespace wg;

template <int S, int Abl>
static void launch_split(const GsoParams &p, dim3 g, uint32_t waves, hipStream_t st) {
    switch (waves) {
    case 1: hipLaunchKernelGGL((gso_split_kernel<1, S, Abl>), g, dim3(64), 0, st, p); break;
    case 2: hipLaunchKernelGGL((gso_split_kernel<2, S, Abl>), g, dim3(128), 0, st, p); break;
    case 8: hipLaunchKernelGGL((gso_split_kernel<8, S, Abl>), g, dim3(512), 0, st, p); break;
    default: hipLaunchKernelGGL((gso_split_kernel<4, S, Abl>), g, dim3(256), 0, st, p); break;
    }
}

namespace wg {
// plan -> split -> finalize for n super-buffers (wg_gso_split; hdr_only:
// wg_encap_batch's headers-only split, synth: without the super-buffers
// whose headers its AEAD synthesizes)
int gso_split_launch(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                     wg_gso_result *dev_res, bool hdr_only, hipStream_t st, const EncapFit *synth, uint32_t *list) {
    const Tune t = tune();
    const bool syn = hdr_only && synth;
    GsoParams p{dev_in,
                dev_desc,
                n,
                dev_out,
                dev_res,
                t.gso_groups,
                syn ? 1u : 0u,
                syn ? synth->msg_cap : 0u,
                syn ? synth->max_segments : 0u,
                syn ? synth->max_segment_size : 0u,
                syn ? list : nullptr};
    if (p.list && hipMemsetAsync(p.list, 0, sizeof(uint32_t), st) != hipSuccess)
        return WG_ERR_RUNTIME;
    // 1. plans (into dev_res), thread per super-buffer
    const uint64_t pb = (n + kPlanBlock - 1) / kPlanBlock;
    if (pb > 0x7fffffffull)
        return WG_ERR_INVALID;
    hipLaunchKernelGGL(gso_plan_kernel, dim3((unsigned)pb), dim3(kPlanBlock), 0, st, p);
    if (!debug_sync(st, "gso_plan_kernel"))
        return WG_ERR_LAUNCH;
    // 2. the split
    const uint64_t units = n * t.gso_groups;
    // list mode: a fixed grid walks the listed super-buffers (usually few)
    const uint64_t cap = p.list ? 4096u : t.gso_blocks;
    uint64_t blocks = units < cap ? units : cap;
    if (blocks >= 8)
        blocks &= ~7ull;  // the XCD swizzle wants a multiple of 8 (the grid-stride loop covers the rest)
    const dim3 g((unsigned)blocks, t.gso_split);
    if (hdr_only) {
        switch (t.encap_spw) {  // the encap step's own value: it stores headers only (3 there, 4 for the full split)
        case 1: launch_split<1, kHdrOnly>(p, g, t.gso_waves, st); break;
        case 2: launch_split<2, kHdrOnly>(p, g, t.gso_waves, st); break;
        case 3: launch_split<3, kHdrOnly>(p, g, t.gso_waves, st); break;
        case 4: launch_split<4, kHdrOnly>(p, g, t.gso_waves, st); break;
        default: launch_split<0, kHdrOnly>(p, g, t.gso_waves, st); break;
        }
    } else {
        switch (t.gso_ablate) {  // correct A/B variants
        case 1: launch_split<0, 1>(p, g, 4, st); break;
        case 32: launch_split<0, 32>(p, g, 4, st); break;
        default:
            switch (t.gso_spw) {
            case 1: launch_split<1, 0>(p, g, t.gso_waves, st); break;
            case 2: launch_split<2, 0>(p, g, t.gso_waves, st); break;
            case 3: launch_split<3, 0>(p, g, t.gso_waves, st); break;
            case 4: launch_split<4, 0>(p, g, t.gso_waves, st); break;
            default: launch_split<0, 0>(p, g, t.gso_waves, st); break;
            }
        }
    }
    if (hipGetLastError() != hipSuccess || !debug_sync(st, "gso_split_kernel"))
        return WG_ERR_LAUNCH;
    // 3. PacketBatch records + the input prefix zeroing + in-place checksums
    hipLaunchKernelGGL(gso_finalize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p);
    if (!debug_sync(st, "gso_finalize_kernel"))
        return WG_ERR_LAUNCH;
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}
}  // namespace wg

extern "C" int wg_gso_split(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                            wg_gso_result *dev_res, void *stream) {
    if (!n)
        return WG_OK;
    if (!dev_in || !dev_desc || !dev_out || !dev_res || (reinterpret_cast<uintptr_t>(dev_desc) & 7) ||
        (reinterpret_cast<uintptr_t>(dev_res) & 7))
        return WG_ERR_INVALID;
    return gso_split_launch(dev_in, dev_desc, n, dev_out, dev_res, false, static_cast<hipStream_t>(stream));
}
