// gso.hip — batched TSO/USO segmentation with per-segment checksum fixup on
// MI355X (gfx950).  Per super-buffer this is worker_impl::do_tun_gso_split
// (reference worker/offload.cpp:46-216) bit for bit, quirks included.
//
// One 256-thread workgroup per super-buffer; its four waves take the
// segments round-robin.  Per segment a wave, in ONE pass over the payload:
//   - streams the payload's output-aligned 16-B chunks: two aligned source
//     loads per chunk, re-aligned in registers with v_alignbyte (the shift
//     source - destination is uniform per segment), stored non-temporally,
//     and summed from the same registers;
//   - moves the <= 15-byte unaligned head/tail of the payload one byte per lane;
//   - rebuilds the header prefix one byte per lane with the reference's
//     fix-ups applied in the reference's order (IPv4 id/len or IPv6 plen ->
//     IPv4 header checksum -> TCP seq/FIN/PSH or UDP len -> L4 checksum).
// The reference touches every payload byte twice (std::copy at :165-166, then
// the checksum at :202); this kernel reads it once and writes it once.
#include <hip/hip_runtime.h>

#include "wg_device.hpp"
#include "wg_internal.hpp"
#include "wg_l4wave.hpp"
#include "wireglider_amd.h"

namespace wg {

enum : uint32_t {
    kNeedsCsum = 1,
    kGsoNone = 0,
    kGsoTcp4 = 1,
    kGsoTcp6 = 4,
    kGsoUdpL4 = 5,  // include/worker/offload.hpp:11-15
    kGsoEcn = 0x80,
};

struct GsoParams {
    uint8_t *in;
    const wg_gso_desc *desc;
    uint64_t n;
    uint8_t *out;
    wg_gso_result *res;
};

// Wave-uniform byte load (every lane reads the same address).
__device__ __forceinline__ uint32_t ubyte_u(uintptr_t a) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)ld8(a));
}

struct Ctx {
    uintptr_t in;
    uint32_t in_len, cs, l4off, hdr_len, gso, nseg;
    uint32_t rest;  // payload bytes after the prefix
    uint32_t id0, seq0;
    bool v6, tcp;
    // Per-super-buffer header sums over the bytes that do NOT change from
    // segment to segment (computed once by each wave, hdr_bases()):
    uint32_t ip_base;   // IPv4 header [0, cs) minus len/id, ip_sum = 0 (pairing from byte 0)
    uint32_t l4h_base;  // L4 header [cs, hdr_len) minus seq/flags (TCP) or len (UDP) (pairing from cs)
    uint32_t ps_sum;    // pseudo-header addresses
    uint32_t flags13;   // TCP flags byte of the prefix
    uint32_t hb0, hb1;  // this lane's prefix bytes lane, lane + 64 (one load for the whole wave)
};

// Prefix byte j, wave-uniform: from the registers of the one prefix load
// when j < 128, else a direct load.
__device__ __forceinline__ uint32_t pbyte(const Ctx &c, uint32_t j) {
    if (j < 64)
        return (uint32_t)__builtin_amdgcn_readlane((int)c.hb0, (int)j);
    if (j < 128)
        return (uint32_t)__builtin_amdgcn_readlane((int)c.hb1, (int)(j - 64));
    return ubyte_u(c.in + j);
}

// Is prefix byte j one of the per-segment L4 header fields?
__device__ __forceinline__ bool l4_varying(const Ctx &c, uint32_t j) {
    return c.tcp ? ((j >= c.cs + 4 && j < c.cs + 8) || j == c.cs + 13) : (j == c.cs + 4 || j == c.cs + 5);
}

// One pass over the prefix per wave: exact integer sums of the invariant
// header bytes (the reference's values after the :145-149 zeroing).
__device__ void hdr_bases(Ctx &c, uint32_t lane) {
    const uint32_t ao = c.v6 ? 8u : 12u, al = c.v6 ? 32u : 8u;
    uint32_t ip = 0, l4 = 0, ps = 0;
    for (uint32_t j = lane; j < c.hdr_len; j += 64) {
        uint32_t b = j < 64 ? c.hb0 : (j < 128 ? c.hb1 : ld8(c.in + j));
        if ((!c.v6 && (j == 10 || j == 11)) || j == c.l4off || j == c.l4off + 1)
            b = 0;
        if (j < c.cs) {
            if (!(!c.v6 && j >= 2 && j <= 5))
                ip += b << (8u * (j & 1u));
        } else if (!l4_varying(c, j)) {
            l4 += b << (8u * ((j - c.cs) & 1u));
        }
        if (j >= ao && j < ao + al)
            ps += b << (8u * ((j - ao) & 1u));
    }
    c.ip_base = wave_sum_u32(ip);
    c.l4h_base = wave_sum_u32(l4);
    c.ps_sum = wave_sum_u32(ps);
    const uint32_t j13 = c.cs + 13;
    c.flags13 = (c.tcp && j13 < c.hdr_len && j13 != c.l4off && j13 != c.l4off + 1) ? pbyte(c, j13) : 0u;
}

// Prefix byte j of segment i after the IP fix-ups (offload.cpp:145-149
// zeroing of ip_sum / L4 field, then :168-183).
__device__ __forceinline__ uint32_t stage_ip(const Ctx &c, uint32_t j, uint32_t b, uint32_t i, uint32_t pktlen) {
    if (!c.v6 && (j == 10 || j == 11))
        b = 0;
    if (j == c.l4off || j == c.l4off + 1)
        b = 0;
    if (c.v6) {
        const uint32_t plen = pktlen - c.cs;  // ip6_plen (uint16 on store)
        if (j == 4) b = (plen >> 8) & 0xffu;
        if (j == 5) b = plen & 0xffu;
    } else {
        if (j == 2) b = (pktlen >> 8) & 0xffu;  // ip_len
        if (j == 3) b = pktlen & 0xffu;
        if (i) {
            const uint32_t id = c.id0 + i;  // ip_id += i (uint16)
            if (j == 4) b = (id >> 8) & 0xffu;
            if (j == 5) b = id & 0xffu;
        }
    }
    return b;
}

// ... then the L4 header fix-ups (:189-200).  `istcp` is the UNMASKED
// gso_type test of :151, so TCP|ECN super-buffers get the UDP fix-up.
__device__ __forceinline__ uint32_t stage_l4(const Ctx &c, uint32_t j, uint32_t b, uint32_t i, uint32_t pktlen,
                                             bool last) {
    if (j < c.cs)
        return b;
    if (c.tcp) {
        if (j >= c.cs + 4 && j < c.cs + 8) {
            const uint32_t seq = c.seq0 + c.gso * i;
            b = (seq >> (8u * (c.cs + 7u - j))) & 0xffu;
        } else if (j == c.cs + 13 && !last) {
            b &= ~0x09u;  // FIN, PSH only on the last segment
        }
    } else {
        const uint32_t ulen = pktlen - c.cs;
        if (j == c.cs + 4) b = (ulen >> 8) & 0xffu;
        if (j == c.cs + 5) b = ulen & 0xffu;
    }
    return b;
}

// Bytes delta..delta+15 of the 32-byte window lo|hi; q = delta >> 2 is
// wave-uniform (scalar branch), r = delta & 3 goes to v_alignbyte.
__device__ __forceinline__ v4u funnel(v4u lo, v4u hi, uint32_t q, uint32_t r) {
    uint32_t w0, w1, w2, w3, w4;
    switch (q) {
    case 0: w0 = lo.x; w1 = lo.y; w2 = lo.z; w3 = lo.w; w4 = hi.x; break;
    case 1: w0 = lo.y; w1 = lo.z; w2 = lo.w; w3 = hi.x; w4 = hi.y; break;
    case 2: w0 = lo.z; w1 = lo.w; w2 = hi.x; w3 = hi.y; w4 = hi.z; break;
    default: w0 = lo.w; w1 = hi.x; w2 = hi.y; w3 = hi.z; w4 = hi.w; break;
    }
    v4u v;
    v.x = __builtin_amdgcn_alignbyte(w1, w0, r);
    v.y = __builtin_amdgcn_alignbyte(w2, w1, r);
    v.z = __builtin_amdgcn_alignbyte(w3, w2, r);
    v.w = __builtin_amdgcn_alignbyte(w4, w3, r);
    return v;
}

__device__ __forceinline__ void st16_nt(uintptr_t addr, v4u v) {
    __builtin_nontemporal_store(v, reinterpret_cast<__attribute__((address_space(1))) v4u *>(addr));
}

// Variant bits (wg_tune_set("gso_ablate")): 1 = non-temporal payload
// stores (a correct variant; default-policy stores measured faster because
// the segment-edge byte stores then merge with the chunk stores in L2).
// Timing-only (WRONG output, to price one part of the kernel, guide §5.4
// rule 17): 2 = no byte stores (header / payload head & tail), 4 = no
// re-alignment window (one source chunk per output chunk).
enum : int { kAblNtStore = 1, kAblNoByteStores = 2, kAblOneLoad = 4 };

template <int A>
__device__ __forceinline__ void st16x(uintptr_t addr, v4u v) {
    if constexpr (A & kAblNtStore)
        st16_nt(addr, v);
    else
        *reinterpret_cast<__attribute__((address_space(1))) v4u *>(addr) = v;
}

__device__ __forceinline__ void st8(uintptr_t addr, uint32_t b) {
    *reinterpret_cast<__attribute__((address_space(1))) uint8_t *>(addr) = (uint8_t)b;
}

// One output segment by one wave, in two phases so a wave can have several
// segments' loads in flight: seg_issue() issues every load of the segment
// (branch-free: clamped addresses, masked use); seg_finish() re-aligns,
// stores, sums and writes the header.  Only the loaded data and the segment
// index cross the phase boundary; the (scalar) geometry is recomputed, which
// keeps the scalar register file from spilling.
struct SegGeom {
    uintptr_t seg, oa, ob, d, c0, c1, sa, smin, smax, a0;
    uint32_t datalen, pktlen, nint, q, r;
    bool last;
};

__device__ __forceinline__ SegGeom seg_geom(const Ctx &c, uintptr_t out_base, uint32_t i) {
    SegGeom g;
    g.seg = out_base + (uintptr_t)i * (c.hdr_len + c.gso);
    const uint32_t off = i * c.gso;
    g.datalen = c.rest - off < c.gso ? c.rest - off : c.gso;
    g.pktlen = c.hdr_len + g.datalen;
    g.last = i + 1 == c.nseg;
    g.oa = g.seg + c.hdr_len;  // payload, destination
    g.ob = g.seg + g.pktlen;
    g.sa = c.in + c.hdr_len + off;  // payload, source
    g.d = g.sa - g.oa;              // source = destination + d (mod 2^64)
    const uint32_t delta = (uint32_t)(g.d & 15u);
    g.q = delta >> 2;
    g.r = delta & 3u;
    g.c0 = (g.oa + 15) & ~(uintptr_t)15;  // destination-aligned interior chunks
    g.c1 = g.ob & ~(uintptr_t)15;
    g.nint = g.c1 > g.c0 ? (uint32_t)((g.c1 - g.c0) >> 4) : 0u;
    g.smin = g.sa & ~(uintptr_t)15;
    g.smax = (g.sa + g.datalen - 1) & ~(uintptr_t)15;
    g.a0 = (g.c0 + g.d) & ~(uintptr_t)15;
    return g;
}

struct SegFront {
    uint32_t i, pb;
    v4u lo0, lo1;  // source chunks a0 + 16 * lane and a0 + 16 * (lane + 64)
};

// Source chunk m of the segment, clamped into the chunks that hold payload
// bytes: the clamp never changes a byte an in-range output chunk needs, and
// keeps every load in bounds.
__device__ __forceinline__ v4u src_chunk(const SegGeom &g, uint64_t m) {
    uintptr_t A = g.a0 + 16ull * m;
    A = A < g.smin ? g.smin : (A > g.smax ? g.smax : A);
    return ld16(A);
}

// Output chunk k needs source chunks k and k + 1 (re-alignment window):
// chunk k + 1 of lane l is chunk k of lane l + 1, fetched by a lane shuffle;
// lane 63 takes it from `next` (lane 0's chunk of the following row).
__device__ __forceinline__ v4u next_chunk(v4u lo, v4u next, uint32_t lane) {
    v4u h;
    h.x = (uint32_t)__shfl_down((int)lo.x, 1);
    h.y = (uint32_t)__shfl_down((int)lo.y, 1);
    h.z = (uint32_t)__shfl_down((int)lo.z, 1);
    h.w = (uint32_t)__shfl_down((int)lo.w, 1);
    if (lane == 63)
        h = next;
    return h;
}

__device__ __forceinline__ v4u lane0(v4u v) {
    v4u r;
    r.x = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.x);
    r.y = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.y);
    r.z = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.z);
    r.w = (uint32_t)__builtin_amdgcn_readfirstlane((int)v.w);
    return r;
}

// Payload head [oa, min(c0, ob)) on lanes 0-15, tail [max(c1, c0), ob) on
// lanes 16-31: this lane's byte address, or 0.
__device__ __forceinline__ uintptr_t edge_byte(const SegGeom &g, uint32_t lane) {
    const uintptr_t he = g.c0 < g.ob ? g.c0 : g.ob;
    const uintptr_t ts = g.c1 > g.c0 ? g.c1 : g.c0;
    const uintptr_t xh = g.oa + lane, xt = ts + (lane - 16);
    if (lane < 16 && xh < he)
        return xh;
    if (lane >= 16 && lane < 32 && xt < g.ob)
        return xt;
    return 0;
}

template <int Abl>
__device__ __forceinline__ void seg_issue(const Ctx &c, uintptr_t out_base, uint32_t i, uint32_t lane, SegFront &f) {
    const SegGeom g = seg_geom(c, out_base, i);
    f.i = i;
    f.lo0 = src_chunk(g, lane);
    f.lo1 = src_chunk(g, lane + 64);
    const uintptr_t xb = edge_byte(g, lane);
    f.pb = ld8(xb ? xb + g.d : g.sa);
}

template <int Abl>
__device__ __forceinline__ void seg_finish(const Ctx &c, uintptr_t out_base, const SegFront &f, uint32_t lane) {
    const SegGeom g = seg_geom(c, out_base, f.i);
    const uint32_t i = f.i, pktlen = g.pktlen;
    Acc acc;
    // payload: re-align, store, sum
    if (g.nint) {
        const v4u nx1 = g.nint > 127 ? lane0(src_chunk(g, 128)) : f.lo1;
        const v4u hi0 = next_chunk(f.lo0, lane0(f.lo1), lane);
        const v4u hi1 = next_chunk(f.lo1, nx1, lane);
        if (lane < g.nint) {
            const v4u v = funnel(f.lo0, (Abl & kAblOneLoad) ? f.lo0 : hi0, g.q, g.r);
            st16x<Abl>(g.c0 + 16ull * lane, v);
            acc.add4(v);
        }
        if (lane + 64 < g.nint) {
            const v4u v = funnel(f.lo1, (Abl & kAblOneLoad) ? f.lo1 : hi1, g.q, g.r);
            st16x<Abl>(g.c0 + 16ull * (lane + 64), v);
            acc.add4(v);
        }
        for (uint32_t k = lane + 128; k < g.nint; k += 64) {  // long segments (gso > ~2 KiB)
            const v4u lo = src_chunk(g, k);
            const v4u v = funnel(lo, src_chunk(g, k + 1), g.q, g.r);
            st16x<Abl>(g.c0 + 16ull * k, v);
            acc.add4(v);
        }
    }
    const uintptr_t xb = edge_byte(g, lane);
    if (xb) {
        if (!(Abl & kAblNoByteStores))
            st8(xb, f.pb);
        acc.add(f.pb << (8u * (uint32_t)(xb & 1u)));
    }

    // checksums: the invariant header sums plus this segment's fields
    // (exact integer sums, so the 0x0000 / 0xFFFF split stays exact)
    uint32_t ipcs = 0;
    if (!c.v6)
        ipcs = ~fold16_32(c.ip_base + bswap16(pktlen & 0xffffu) + bswap16((c.id0 + i) & 0xffffu)) & 0xffffu;
    uint32_t l4h = c.l4h_base;
    if (c.tcp) {
        const uint32_t seq = c.seq0 + c.gso * i;
        l4h += bswap16(seq >> 16) + bswap16(seq & 0xffffu) + ((g.last ? c.flags13 : (c.flags13 & ~0x09u)) << 8);
    } else {
        l4h += bswap16((pktlen - c.cs) & 0xffffu);
    }
    uint32_t lp = fold16(acc.value());
    if ((g.seg + c.cs) & 1u)  // payload summed in absolute pairing; the L4 region pairs from seg + cs
        lp = bswap16(lp);
    uint32_t T = wave_sum_u32(lp) + l4h + c.ps_sum;
    T += ((c.tcp ? 6u : 17u) << 8) + bswap16((pktlen - c.cs) & 0xffffu);
    const uint32_t l4cs = ~fold16_32(T) & 0xffffu;
    const uint32_t j0 = lane, j1 = lane + 64;

    // write the header prefix (checksums in native order, :185-186, :203-204)
    auto final_byte = [&](uint32_t j, uint32_t s4) {
        if (!c.v6 && j == 10) return ipcs & 0xffu;
        if (!c.v6 && j == 11) return ipcs >> 8;
        if (j == c.l4off) return l4cs & 0xffu;
        if (j == c.l4off + 1) return l4cs >> 8;
        return s4;
    };
    auto s4 = [&](uint32_t j, uint32_t b) { return stage_l4(c, j, stage_ip(c, j, b, i, pktlen), i, pktlen, g.last); };
    if (Abl & kAblNoByteStores) {
        if (lane == 0 && l4cs == 0x12345u) st8(g.seg, 0);  // keep the sums live
        return;
    }
    if (j0 < c.hdr_len) st8(g.seg + j0, final_byte(j0, s4(j0, c.hb0)));
    if (j1 < c.hdr_len) st8(g.seg + j1, final_byte(j1, s4(j1, c.hb1)));
    for (uint32_t j = lane + 128; j < c.hdr_len; j += 64) {
        const uint32_t b2 = stage_ip(c, j, ld8(c.in + j), i, pktlen);
        st8(g.seg + j, final_byte(j, stage_l4(c, j, b2, i, pktlen, g.last)));
    }
}

// GSO_NONE + NEEDS_CSUM (offload.cpp:56-78): both checksums in place, one wave.
__device__ void do_inplace(const Ctx &c, uint32_t lane) {
    // IPv4 header checksum over [0, cs) with ip_sum zeroed.
    uint32_t ipcs = 0;
    if (!c.v6) {
        uint32_t part = 0;
        for (uint32_t j = lane; j < c.cs; j += 64) {
            uint32_t b = ld8(c.in + j);
            if (j == 10 || j == 11) b = 0;
            part += b << (8u * (j & 1u));
        }
        ipcs = ~fold16_32(wave_sum_u32(part)) & 0xffffu;
    }
    // L4 over the bytes as they are, then replace the checksum field's
    // contribution by zero: adding 0xFFFF - x is subtracting x mod 0xFFFF,
    // and the total is never zero (the pseudo-header carries the protocol),
    // so the fold only depends on the sum mod 0xFFFF.
    Geom g;
    g.a = c.in;
    g.len = c.in_len;
    g.cs = c.cs;
    g.fl = (c.v6 ? WG_PKT_V6 : 0u) | (c.tcp ? WG_PKT_TCP : 0u);
    Front f;
    issue<true, false>(g, lane, f);
    const uint32_t f0 = ld8(c.in + c.l4off), f1 = ld8(c.in + c.l4off + 1);
    uint32_t T = wave_sum_u32(finish<false>(lane, f));
    const uint32_t fw = ((c.l4off - c.cs) & 1u) ? ((f0 << 8) | f1) : (f0 | (f1 << 8));
    T += 0xffffu - fw;
    T += ((c.tcp ? 6u : 17u) << 8) + bswap16((c.in_len - c.cs) & 0xffffu);
    const uint32_t l4cs = ~fold16_32(T) & 0xffffu;
    if (lane == 0) {
        if (!c.v6) {
            st8(c.in + 10, ipcs & 0xffu);
            st8(c.in + 11, ipcs >> 8);
        }
        st8(c.in + c.l4off, l4cs & 0xffu);
        st8(c.in + c.l4off + 1, l4cs >> 8);
    }
}

// Classification of one super-buffer (mirrors :48-134 and the oracle).
// kUniform: called by a whole wave (wave-uniform byte loads).
struct Cls {
    int status;
    bool pass, inplace;
    uint32_t isv6, ecn;
};

template <bool kUniform>
__device__ __forceinline__ uint32_t ldb(const Ctx &c, uint32_t j) {
    if constexpr (kUniform)
        return pbyte(c, j);
    else
        return ld8(c.in + j);
}

template <bool kUniform>
__device__ __forceinline__ Cls classify(const wg_gso_desc &dsc, uintptr_t in_base, Ctx &c) {
    c.in = in_base + dsc.in_offset;
    c.in_len = dsc.in_len;
    c.cs = dsc.vnet.csum_start;
    c.l4off = (uint32_t)dsc.vnet.csum_start + dsc.vnet.csum_offset;  // :47
    c.hdr_len = dsc.vnet.hdr_len;
    c.gso = dsc.vnet.gso_size;
    c.rest = 0;
    c.nseg = 0;
    c.v6 = false;
    const uint32_t gtype = dsc.vnet.gso_type;
    Cls r{0, true, false, 0u, 0u};
    if (c.in_len < 1) {
        r.status = -3;
        return r;
    }
    if constexpr (kUniform) {
        // the whole wave loads prefix bytes 0-127 at once; every byte the
        // classification and the header work need is then a readlane
        const uint32_t lane = lane_id();
        c.hb0 = ld8(c.in + (lane < c.in_len ? lane : 0u));
        c.hb1 = ld8(c.in + (lane + 64 < c.in_len ? lane + 64 : 0u));
    }
    r.isv6 = (ldb<kUniform>(c, 0) >> 4) == 6;  // :48
    const uint32_t iph_min = r.isv6 ? 40u : 20u;
    if (c.in_len < iph_min) {
        r.status = -3;
        return r;
    }
    r.ecn = r.isv6 ? ((ldb<kUniform>(c, 1) >> 4) & 3u) : (ldb<kUniform>(c, 1) & 3u);  // :49-53
    c.v6 = r.isv6;
    const uint32_t g = gtype & ~kGsoEcn;  // :55
    bool seg = false;
    if (g == kGsoNone) {
        if (dsc.vnet.flags & kNeedsCsum) {
            if (c.cs < iph_min || c.cs > c.in_len || c.l4off + 2 > c.in_len)
                r.status = -3;
            else
                r.inplace = true;
        }
    } else if (g == kGsoTcp4 || g == kGsoTcp6) {
        if (c.cs > c.in_len) {
            r.status = -3;
        } else if (c.in_len - c.cs >= 20) {                                        // :91
            const uint32_t thlen = 4u * (ldb<kUniform>(c, c.cs + 12) >> 4);  // doff, :100
            if (thlen >= 20) {                                                    // :101
                c.hdr_len = c.cs + thlen;                                         // :110
                seg = true;
            }
        }
    } else if (g == kGsoUdpL4) {
        c.hdr_len = c.cs + 8;  // :114
        seg = true;
    }
    if (seg && c.in_len >= c.hdr_len) {  // :126-134
        if (c.cs < iph_min || c.l4off < c.cs || c.l4off + 2 > c.hdr_len) {
            r.status = -3;
        } else {
            c.rest = c.in_len - c.hdr_len;
            if (c.rest && !c.gso) {
                r.status = -1;  // the reference loops forever
            } else {
                c.nseg = c.gso ? (c.rest + c.gso - 1) / c.gso : 0;
                if ((uint64_t)dsc.out_cap < (uint64_t)c.in_len + (uint64_t)c.nseg * c.hdr_len)
                    r.status = -2;  // reserve_size assert, :139-143
                else
                    r.pass = false;
            }
        }
    }
    c.tcp = gtype == kGsoTcp4 || gtype == kGsoTcp6;  // :151, unmasked
    return r;
}

// Main kernel: blockIdx.x walks super-buffers, blockIdx.y splits a
// super-buffer's segments over gridDim.y blocks of W waves (so waves are
// short-lived; the copy roofline on MI355X wants many small one-shot waves).
template <int W, int S, int Abl>  // W waves per block, S segments in flight per wave
__global__ __launch_bounds__(64 * W) void gso_split_kernel(GsoParams p) {
    const uint32_t lane = lane_id();
    const uint32_t gw = blockIdx.y * W + wave_in_block();  // wave index within the super-buffer
    const uint32_t gstride = gridDim.y * W * S;
    for (uint64_t b = blockIdx.x; b < p.n; b += gridDim.x) {
        const wg_gso_desc dsc = p.desc[b];
        Ctx c;
        const Cls cl = classify<true>(dsc, reinterpret_cast<uintptr_t>(p.in), c);
        if (!cl.pass) {
            if (gw * S >= c.nseg)
                continue;
            c.id0 = (pbyte(c, 4) << 8) | pbyte(c, 5);
            // seq0 is read after the prefix's L4 checksum field was zeroed
            // (:149 before :152-154), which matters when the two overlap.
            c.seq0 = 0;
            if (c.tcp) {
                for (uint32_t k = 0; k < 4; k++) {
                    const uint32_t j = c.cs + 4 + k;
                    const uint32_t bb = (j == c.l4off || j == c.l4off + 1) ? 0u : pbyte(c, j);
                    c.seq0 |= bb << (8u * (3u - k));
                }
            }
            hdr_bases(c, lane);
            const uintptr_t out_base = reinterpret_cast<uintptr_t>(p.out) + dsc.out_offset;
            if constexpr (S == 1) {
                // ping-pong software pipeline: the next segment's loads are in
                // flight while this one is re-aligned, stored and summed
                const uint32_t last = c.nseg - 1;
                uint32_t i = gw;
                SegFront A, B;
                seg_issue<Abl>(c, out_base, i, lane, A);
                for (;;) {
                    const uint32_t i1 = i + gstride;
                    seg_issue<Abl>(c, out_base, i1 < last ? i1 : last, lane, B);
                    seg_finish<Abl>(c, out_base, A, lane);
                    if (i1 > last)
                        break;
                    const uint32_t i2 = i1 + gstride;
                    seg_issue<Abl>(c, out_base, i2 < last ? i2 : last, lane, A);
                    seg_finish<Abl>(c, out_base, B, lane);
                    if (i2 > last)
                        break;
                    i = i2;
                }
            } else {
                for (uint32_t i0 = gw * S; i0 < c.nseg; i0 += gstride) {
                    SegFront f[S];
#pragma unroll
                    for (int k = 0; k < S; k++)
                        seg_issue<Abl>(c, out_base, i0 + k < c.nseg ? i0 + k : c.nseg - 1, lane, f[k]);
#pragma unroll
                    for (int k = 0; k < S; k++)
                        if (i0 + k < c.nseg)
                            seg_finish<Abl>(c, out_base, f[k], lane);
                }
            }
        } else if (cl.inplace && gw == 0) {
            c.tcp = (cl.isv6 ? pbyte(c, 6) : pbyte(c, 9)) == 6;  // :67-70
            do_inplace(c, lane);
        }
    }
}

// Finalize (same stream, after the main kernel): the PacketBatch record per
// super-buffer, and the reference's in-place zeroing of the input prefix's
// ip_sum / L4 checksum field (:145-149) — only once every block of the main
// kernel has read that prefix, hence a separate launch.
__global__ __launch_bounds__(256) void gso_finalize_kernel(GsoParams p) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < p.n; b += stride) {
        const wg_gso_desc dsc = p.desc[b];
        Ctx c;
        const Cls cl = classify<false>(dsc, reinterpret_cast<uintptr_t>(p.in), c);
        wg_gso_result r;
        r.out_len = cl.pass ? c.in_len : (uint64_t)c.rest + (uint64_t)c.nseg * c.hdr_len;
        r.segment_size = cl.pass ? c.in_len : c.hdr_len + c.gso;
        r.hdr_len = (uint16_t)c.hdr_len;
        r.isv6 = (uint8_t)cl.isv6;
        r.ecn = (uint8_t)cl.ecn;
        r.status = (int8_t)cl.status;
        r.passthrough = cl.pass ? 1 : 0;
        for (int k = 0; k < 6; k++) r.pad[k] = 0;
        if (cl.status != 0) {
            r.out_len = 0;
            r.segment_size = 0;
        }
        p.res[b] = r;
        if (!cl.pass) {
            if (!c.v6) {
                st8(c.in + 10, 0);
                st8(c.in + 11, 0);
            }
            st8(c.in + c.l4off, 0);
            st8(c.in + c.l4off + 1, 0);
        }
    }
}

}  // namespace wg

using namespace wg;

extern "C" int wg_gso_split(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                            wg_gso_result *dev_res, void *stream) {
    if (!n)
        return WG_OK;
    if (!dev_in || !dev_desc || !dev_out || !dev_res || (reinterpret_cast<uintptr_t>(dev_desc) & 7) ||
        (reinterpret_cast<uintptr_t>(dev_res) & 7))
        return WG_ERR_INVALID;
    GsoParams p{dev_in, dev_desc, n, dev_out, dev_res};
    const Tune &t = tune();
    const uint64_t blocks = n < t.gso_blocks ? n : t.gso_blocks;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 g((unsigned)blocks, t.gso_split);
    if (t.gso_ablate) {  // timing-only variants (wrong output), 4 waves x 1 segment
        switch (t.gso_ablate) {
        case 1: hipLaunchKernelGGL((gso_split_kernel<4, 1, 1>), g, dim3(256), 0, st, p); break;
        case 2: hipLaunchKernelGGL((gso_split_kernel<4, 1, 2>), g, dim3(256), 0, st, p); break;
        case 3: hipLaunchKernelGGL((gso_split_kernel<4, 1, 3>), g, dim3(256), 0, st, p); break;
        case 4: hipLaunchKernelGGL((gso_split_kernel<4, 1, 4>), g, dim3(256), 0, st, p); break;
        case 6: hipLaunchKernelGGL((gso_split_kernel<4, 1, 6>), g, dim3(256), 0, st, p); break;
        default: hipLaunchKernelGGL((gso_split_kernel<4, 1, 7>), g, dim3(256), 0, st, p); break;
        }
        uint64_t fb = (n + 255) / 256;
        hipLaunchKernelGGL(gso_finalize_kernel, dim3((unsigned)(fb < 65536 ? fb : 65536)), dim3(256), 0, st, p);
        return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
    }
    const uint32_t key = t.gso_waves * 10 + t.gso_spw;
    switch (key) {
    case 41: hipLaunchKernelGGL((gso_split_kernel<4, 1, 0>), g, dim3(256), 0, st, p); break;
    case 42: hipLaunchKernelGGL((gso_split_kernel<4, 2, 0>), g, dim3(256), 0, st, p); break;
    case 81: hipLaunchKernelGGL((gso_split_kernel<8, 1, 0>), g, dim3(512), 0, st, p); break;
    case 82: hipLaunchKernelGGL((gso_split_kernel<8, 2, 0>), g, dim3(512), 0, st, p); break;
    case 161: hipLaunchKernelGGL((gso_split_kernel<16, 1, 0>), g, dim3(1024), 0, st, p); break;
    default: hipLaunchKernelGGL((gso_split_kernel<16, 2, 0>), g, dim3(1024), 0, st, p); break;
    }
    if (hipGetLastError() != hipSuccess)
        return WG_ERR_LAUNCH;
    {
        uint64_t fb = (n + 255) / 256;
        hipLaunchKernelGGL(gso_finalize_kernel, dim3((unsigned)(fb < 65536 ? fb : 65536)), dim3(256), 0, st, p);
    }
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}
