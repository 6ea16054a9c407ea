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
#include "wg_gso.hpp"
#include "wg_l4wave.hpp"
#include "wireglider_amd.h"

namespace wg {

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
// 32 = blocks -> super-buffers in launch order instead of XCD-swizzled (a
// correct variant; the swizzle keeps consecutive super-buffers on one XCD,
// +2.7 % on config 3).
enum : int { kAblNtStore = 1, kAblNoByteStores = 2, kAblOneLoad = 4, kAblNoSwizzle = 32 };

template <int A>
__device__ __forceinline__ void st16x(uintptr_t addr, v4u v) {
    if constexpr (A & kAblNtStore)
        st16_nt(addr, v);
    else
        *reinterpret_cast<__attribute__((address_space(1))) v4u *>(addr) = v;
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
__device__ __forceinline__ v4u next_chunk(v4u lo, v4u next) {
    // DPP wave_shl:1 — lane l reads lane l + 1; lane 63 has no source and
    // keeps `old` = next (bound_ctrl off).  (A ds_bpermute shuffle measured
    // the same, tools/ab_gso.py.)
    v4u h;
    h.x = (uint32_t)__builtin_amdgcn_update_dpp((int)next.x, (int)lo.x, 0x130, 0xf, 0xf, false);
    h.y = (uint32_t)__builtin_amdgcn_update_dpp((int)next.y, (int)lo.y, 0x130, 0xf, 0xf, false);
    h.z = (uint32_t)__builtin_amdgcn_update_dpp((int)next.z, (int)lo.z, 0x130, 0xf, 0xf, false);
    h.w = (uint32_t)__builtin_amdgcn_update_dpp((int)next.w, (int)lo.w, 0x130, 0xf, 0xf, false);
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
        const v4u hi0 = next_chunk(f.lo0, lane0(f.lo1));
        const v4u hi1 = next_chunk(f.lo1, nx1);
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
    // write the header prefix: each byte is the prefix byte or one byte of a
    // per-segment value, by its precomputed field code (checksums in native
    // order, :185-186, :203-204)
    if (Abl & kAblNoByteStores) {
        if (lane == 0 && l4cs == 0x12345u) st8(g.seg, 0);  // keep the sums live
        return;
    }
    const HdrVals hv{pktlen, c.id0 + i, ipcs, l4cs, c.seq0 + c.gso * i, pktlen - c.cs, g.last ? 0xffu : 0xf6u};
    if (lane < c.hdr_len) st8(g.seg + lane, hdr_byte(hv, c.hc0, c.hb0));
    if (lane + 64 < c.hdr_len) st8(g.seg + lane + 64, hdr_byte(hv, c.hc1, c.hb1));
    for (uint32_t j = lane + 128; j < c.hdr_len; j += 64)
        st8(g.seg + j, hdr_byte(hv, hdr_code(c, j), ld8(c.in + j)));
}

// Main kernel: blockIdx.x walks super-buffers, blockIdx.y splits a
// super-buffer's segments over gridDim.y blocks of W waves (so waves are
// short-lived; the copy roofline on MI355X wants many small one-shot waves).
template <int W, int S, int Abl>  // W waves per block, S segments in flight per wave
__global__ __launch_bounds__(64 * W) void gso_split_kernel(GsoParams p) {
    const uint32_t lane = lane_id();
    const uint32_t gw = blockIdx.y * W + wave_in_block();  // wave index within the super-buffer
    const uint32_t gstride = gridDim.y * W * S;
    const uint64_t b0 = (Abl & kAblNoSwizzle) ? blockIdx.x : xcd_swizzle(blockIdx.x, gridDim.x);
    for (uint64_t b = b0; b < p.n; b += gridDim.x) {
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

static void launch_gso_finalize(const GsoParams &p, hipStream_t st) {
    const uint64_t fb = (p.n + 255) / 256;
    hipLaunchKernelGGL(gso_finalize_kernel, dim3((unsigned)(fb < 65536 ? fb : 65536)), dim3(256), 0, st, p);
}

extern "C" int wg_gso_split(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                            wg_gso_result *dev_res, void *stream) {
    if (!n)
        return WG_OK;
    if (!dev_in || !dev_desc || !dev_out || !dev_res || (reinterpret_cast<uintptr_t>(dev_desc) & 7) ||
        (reinterpret_cast<uintptr_t>(dev_res) & 7))
        return WG_ERR_INVALID;
    GsoParams p{dev_in, dev_desc, n, dev_out, dev_res};
    const Tune &t = tune();
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint64_t blocks = n < t.gso_blocks ? n : t.gso_blocks;
    if (blocks >= 8)
        blocks &= ~7ull;  // the XCD swizzle wants a multiple of 8 (the grid-stride loop covers the rest)
    const dim3 g((unsigned)blocks, t.gso_split);
    if (t.gso_ablate) {  // A/B variants, 4 waves x 1 segment (1, 32 correct; 2, 4 timing-only)
        switch (t.gso_ablate) {
        case 1: hipLaunchKernelGGL((gso_split_kernel<4, 1, 1>), g, dim3(256), 0, st, p); break;
        case 2: hipLaunchKernelGGL((gso_split_kernel<4, 1, 2>), g, dim3(256), 0, st, p); break;
        case 3: hipLaunchKernelGGL((gso_split_kernel<4, 1, 3>), g, dim3(256), 0, st, p); break;
        case 4: hipLaunchKernelGGL((gso_split_kernel<4, 1, 4>), g, dim3(256), 0, st, p); break;
        case 6: hipLaunchKernelGGL((gso_split_kernel<4, 1, 6>), g, dim3(256), 0, st, p); break;
        case 32: hipLaunchKernelGGL((gso_split_kernel<4, 1, 32>), g, dim3(256), 0, st, p); break;
        default: hipLaunchKernelGGL((gso_split_kernel<4, 1, 7>), g, dim3(256), 0, st, p); break;
        }
        launch_gso_finalize(p, st);
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
    launch_gso_finalize(p, st);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}
