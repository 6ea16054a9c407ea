// wg_gso.hpp — per-super-buffer state shared by the GSO split kernels
// (gso.hip):
// classification of do_tun_gso_split (reference worker/offload.cpp:46-134),
// the invariant header sums, the per-segment header field codes, and the
// GSO_NONE + NEEDS_CSUM in-place path.
#pragma once

#include <hip/hip_runtime.h>

#include "wg_device.hpp"
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
    uint32_t groups;  // blocks per super-buffer (flat grid: block u -> super-buffer u / groups)
    // headers-only split of wg_encap_batch with header synthesis: skip the
    // super-buffers whose segments the AEAD encrypts (encap_fit) and builds
    // (syn_eligible); every other one is split as usual
    uint32_t synth, fit_cap, fit_segs, fit_size;
    // nullable: the plan kernel lists the super-buffers still to split here
    // ([0] count, then indices) and the split kernel walks that list (synth
    // with nearly every super-buffer synthesized: no wave per skipped one)
    uint32_t *list;
};

struct Ctx {
    uintptr_t in;
    uint32_t in_len, cs, l4off, hdr_len, gso, nseg;
    uint32_t rest;  // payload bytes after the prefix
    uint32_t id0, seq0;
    bool v6, tcp;
    // Per-super-buffer header sums over the bytes that do NOT change from
    // segment to segment (hdr_bases_thread(), in the plan pass):
    uint32_t ip_base;   // IPv4 header [0, cs) minus len/id, ip_sum = 0 (pairing from byte 0)
    uint32_t l4h_base;  // L4 header [cs, hdr_len) minus seq/flags (TCP) or len (UDP) (pairing from cs)
    uint32_t ps_sum;    // pseudo-header addresses
    uint32_t flags13;   // TCP flags byte of the prefix
    uint32_t hb0, hb1;  // split kernel: this lane's prefix bytes lane, lane + 64
    uint32_t hc0, hc1;  // per-segment field code of prefix bytes lane, lane + 64 (hdr_code)
    // split kernel: the super-buffer's output base, its low 4 address bits
    // (destination chunks are 16-B aligned in absolute terms), and buffer
    // resources over the input super-buffer and its output area
    uintptr_t out;
    uint32_t omis;
    rsrc_t rin, rout;
};

// Is prefix byte j one of the per-segment L4 header fields?
__device__ __forceinline__ bool l4_varying(const Ctx &c, uint32_t j) {
    return c.tcp ? ((j >= c.cs + 4 && j < c.cs + 8) || j == c.cs + 13) : (j == c.cs + 4 || j == c.cs + 5);
}

// Field code of prefix byte j in every output segment: which per-segment
// value replaces it (bits 0-2, a field index; 0 = the prefix byte as is) and
// which byte of that value (shift, bits 8-12).  Priority as in the
// reference's write order: checksums (written last, :185-186, :203-204) over
// the length/id/seq fix-ups.  The per-segment values sit in lanes 1-7 of one
// VGPR (v_writelane) and each header lane fetches its field with one
// ds_bpermute (seg_finish, gso.hip).
enum : uint32_t { kFldTmpl = 0, kFldPkt = 1, kFldId = 2, kFldIpcs = 3, kFldL4cs = 4, kFldSeq = 5, kFldUlen = 6,
                  kFldFlags = 7 };

__device__ __forceinline__ uint32_t hdr_code(const Ctx &c, uint32_t j) {
    if (!c.v6 && (j == 10 || j == 11))
        return kFldIpcs | ((j == 11 ? 8u : 0u) << 8);  // native order
    if (j == c.l4off || j == c.l4off + 1)
        return kFldL4cs | ((j == c.l4off + 1 ? 8u : 0u) << 8);
    if (c.v6) {
        if (j == 4 || j == 5)  // ip6_plen = pktlen - cs (big endian)
            return kFldUlen | ((j == 4 ? 8u : 0u) << 8);
    } else {
        if (j == 2 || j == 3)  // ip_len
            return kFldPkt | ((j == 2 ? 8u : 0u) << 8);
        if (j == 4 || j == 5)  // ip_id
            return kFldId | ((j == 4 ? 8u : 0u) << 8);
    }
    if (j >= c.cs) {
        if (c.tcp) {
            if (j >= c.cs + 4 && j < c.cs + 8)
                return kFldSeq | ((8u * (c.cs + 7u - j)) << 8);
            if (j == c.cs + 13)  // TCP flags: the prefix's, FIN/PSH cleared except on the last segment
                return kFldFlags;
        } else if (j == c.cs + 4 || j == c.cs + 5) {
            return kFldUlen | ((j == c.cs + 4 ? 8u : 0u) << 8);
        }
    }
    return kFldTmpl;
}

// Exact integer sums of the invariant header bytes (the reference's values
// after the :145-149 zeroing), by ONE thread over its super-buffer's prefix
// bytes (`byte(j)`, j < hdr_len): IPv4 header [0, cs) without len / id /
// ip_sum, L4 header [cs, hdr_len) without its checksum and per-segment
// fields, and the pseudo-header addresses.  Every total stays below 2^32
// (at most 32,768 16-bit words), so the later 16-bit folds are exact.
template <class ByteFn>
__device__ __forceinline__ void hdr_bases_thread(Ctx &c, ByteFn byte) {
    const uint32_t ao = c.v6 ? 8u : 12u, al = c.v6 ? 32u : 8u;
    uint32_t ip = 0, l4 = 0, ps = 0;
    for (uint32_t j = 0; j < c.hdr_len; j++) {
        uint32_t b = byte(j);
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
    c.ip_base = ip;
    c.l4h_base = l4;
    c.ps_sum = ps;
    const uint32_t j13 = c.cs + 13;
    c.flags13 = (c.tcp && j13 < c.hdr_len && j13 != c.l4off && j13 != c.l4off + 1) ? byte(j13) : 0u;
}

__device__ __forceinline__ void st8(uintptr_t addr, uint32_t b) {
    *reinterpret_cast<__attribute__((address_space(1))) uint8_t *>(addr) = (uint8_t)b;
}

// The per-segment field values, indexed by kFld* (entry 0 unused).
struct HdrVals {
    uint32_t v[8];
};

// Header byte by field code, for header bytes past the first 128 (rare: the
// general path; the first 128 use the ds_bpermute lookup).
__device__ __forceinline__ uint32_t hdr_byte_slow(const HdrVals &h, uint32_t code, uint32_t tb) {
    const uint32_t f = code & 7u;
    uint32_t v = tb;
#pragma unroll
    for (uint32_t k = 1; k < 8; k++)
        v = f == k ? (h.v[k] >> (code >> 8)) & 0xffu : v;
    return v;
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

// Classification of one super-buffer (mirrors :48-134 and the oracle), by
// one thread (gso_plan_kernel).
struct Cls {
    int status;
    bool pass, inplace;
    uint32_t isv6, ecn;
};

// byte(j): prefix byte j of the super-buffer (only called for j < in_len).
template <class ByteFn>
__device__ __forceinline__ Cls classify_by(const wg_gso_desc &dsc, uintptr_t in_base, Ctx &c, ByteFn byte) {
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
    r.isv6 = (byte(0) >> 4) == 6;  // :48
    const uint32_t iph_min = r.isv6 ? 40u : 20u;
    if (c.in_len < iph_min) {
        r.status = -3;
        return r;
    }
    r.ecn = r.isv6 ? ((byte(1) >> 4) & 3u) : (byte(1) & 3u);  // :49-53
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
            const uint32_t thlen = 4u * (byte(c.cs + 12) >> 4);  // doff, :100
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

}  // namespace wg
