// NOT BUILT — kept as the record of a measured negative result (DESIGN.md
// §6.2).  A plan pre-pass + one-wave-per-output-segment "chunk stream" GSO
// engine (unaligned 16-B source loads, whole-chunk non-temporal stores,
// header chunks assembled from an LDS template).  Bit-exact against the
// oracle on tests/test_gpu_gso.py, but on config 3 it measured 26.8 ms
// (one-shot waves), 11.9 ms (persistent, residency-sized grid) and 13.9 ms
// (persistent + two-slot pipeline) against 6.4 ms for gso.hip: each wave's
// plan -> load dependency chain and ~500 VALU per segment (vs ~230) left it
// latency/issue bound.  It compiled against the tree at commit 4eca7b8
// (wireglider_amd/csrc/, with GsoPlan in this file).
// gso_rows.hip — the default GSO split engine: do_tun_gso_split (reference
// worker/offload.cpp:46-216) for a batch of super-buffers, laid out for the
// MI355X memory system rather than per segment.
//
//   1. gso_plan_kernel (one wave per super-buffer): classification
//      (:48-134), the invariant header sums and the per-super-buffer fields
//      (IPv4 id, TCP seq read after the :145-149 zeroing) into a 64-B plan;
//      GSO_NONE + NEEDS_CSUM super-buffers are checksummed in place here.
//   2. gso_seg_kernel: one-shot waves, one output segment each (4 waves of
//      one super-buffer per block, XCD-swizzled so a super-buffer's blocks
//      share one L2).  The segment's output is a run of destination-aligned
//      16-B chunks: a chunk inside the payload is ONE unaligned 16-B load from
//      its source (in + p - i * hdr_len) and ONE non-temporal 16-B store,
//      summed from the same registers; the few chunks that touch a header (or
//      the end of the output) are assembled byte by byte from a per-wave LDS
//      copy of the header template and the segment's fields once its L4
//      checksum is known.  A chunk straddling two segments belongs to the
//      segment its first byte is in, so every output byte is written by
//      exactly one full-chunk store (byte stores only at the two ends of the
//      output) and HBM sees whole lines.
//   3. gso_finalize_kernel (gso.hip): PacketBatch records and the in-place
//      zeroing of the input prefix (:145-149) after every block has read it.
//
// Measured on BASELINE config 3: the layout experiments in
// tools/exp/gso_shape.hip put this structure at the copy-probe ceiling,
// where one looping block per super-buffer tops out ~15 % lower.
#include <hip/hip_runtime.h>

#include "wg_device.hpp"
#include "wg_gso.hpp"
#include "wg_internal.hpp"
#include "wireglider_amd.h"

namespace wg {

struct GsoPlan {
    uint64_t in_off, out_off;  // the super-buffer's wg_gso_desc offsets
    uint32_t h_cs;             // hdr_len | csum_start << 16
    uint32_t l4_fl;            // l4off | fl << 16 | kind << 24 (fl: bit0 v6, bit1 tcp = unmasked :151 test)
    uint32_t G, nseg, rest, in_len;
    uint32_t id0, seq0, ip_base, l4h_base, ps_sum, flags13;
};
static_assert(sizeof(GsoPlan) == 64, "plan record is one 64-B line");

enum : uint32_t { kPlanRows = 0, kPlanNone = 1 };
constexpr uint32_t kTmplMax = 256;  // header bytes staged in LDS per wave
constexpr uint32_t kWinMax = 16;    // mixed-chunk source windows staged in LDS per wave

struct SegParams {
    const uint8_t *in;
    uint8_t *out;
    const GsoPlan *plan;
    uint64_t n;
    uint32_t Rw;  // waves (segment slots) per super-buffer, a multiple of 4
    uint32_t Q;   // stripes: super-buffers processed concurrently
};

// ---------------------------------------------------------------- plan ----

__global__ __launch_bounds__(256) void gso_plan_kernel(const uint8_t *in, const wg_gso_desc *desc, uint64_t n,
                                                       GsoPlan *plan) {
    const uint32_t lane = lane_id();
    const uint64_t w0 = (uint64_t)blockIdx.x * 4u + wave_in_block();
    const uint64_t ws = (uint64_t)gridDim.x * 4u;
    for (uint64_t b = w0; b < n; b += ws) {
        const wg_gso_desc dsc = desc[b];
        Ctx c;
        const Cls cl = classify<true>(dsc, reinterpret_cast<uintptr_t>(in), c);
        GsoPlan pl{};
        uint32_t kind = kPlanNone;
        if (!cl.pass) {
            c.id0 = (pbyte(c, 4) << 8) | pbyte(c, 5);
            c.seq0 = 0;
            if (c.tcp) {  // read after the checksum field was zeroed (:149 before :152-154)
                for (uint32_t k = 0; k < 4; k++) {
                    const uint32_t j = c.cs + 4 + k;
                    const uint32_t bb = (j == c.l4off || j == c.l4off + 1) ? 0u : pbyte(c, j);
                    c.seq0 |= bb << (8u * (3u - k));
                }
            }
            hdr_bases(c, lane);
            kind = c.nseg ? kPlanRows : kPlanNone;
            pl.in_off = dsc.in_offset;
            pl.out_off = dsc.out_offset;
            pl.h_cs = c.hdr_len | (c.cs << 16);
            pl.G = c.gso;
            pl.nseg = c.nseg;
            pl.rest = c.rest;
            pl.in_len = c.in_len;
            pl.id0 = c.id0;
            pl.seq0 = c.seq0;
            pl.ip_base = c.ip_base;
            pl.l4h_base = c.l4h_base;
            pl.ps_sum = c.ps_sum;
            pl.flags13 = c.flags13;
        } else if (cl.inplace) {
            c.tcp = (cl.isv6 ? pbyte(c, 6) : pbyte(c, 9)) == 6;  // :67-70
            do_inplace(c, lane);
        }
        pl.l4_fl = (c.l4off & 0xffffu) | ((c.v6 ? 1u : 0u) << 16) | ((c.tcp ? 2u : 0u) << 16) | (kind << 24);
        if (lane == 0)
            plan[b] = pl;
    }
}

// ---------------------------------------------------------------- rows ----

// Unaligned 16-byte load (gfx950 global loads take any byte address; the
// measured cost over an aligned load is ~1 %, tools/exp/unaligned.hip).
__device__ __forceinline__ v4u ldu16_nt(uintptr_t a) {
    return __builtin_nontemporal_load(reinterpret_cast<g_v4u *>(a));
}

__device__ __forceinline__ void stu16_nt(uintptr_t a, v4u v) {
    __builtin_nontemporal_store(v, reinterpret_cast<__attribute__((address_space(1))) v4u *>(a));
}

// Branch-free source window: 16 bytes at in[src], the load clamped to
// in[in_len - 16, in_len) (no lane ever reads outside its super-buffer; every
// load is issued unconditionally so a row's loads are all in flight at once)
// and shifted back in registers by win_shift (delta = 0 for all but the
// super-buffer's last chunks).
__device__ __forceinline__ v4u win_issue(uintptr_t in, uint32_t in_len, int64_t src, uint32_t &delta) {
    const int64_t sc = src < 0 ? 0 : src;
    const int64_t mx = (int64_t)in_len - 16;
    const int64_t base = sc > mx ? mx : sc;
    const int64_t d = sc - base;
    delta = (uint32_t)(d > 15 ? 15 : d);
    return ldu16_nt(in + (uintptr_t)base);
}

__device__ __forceinline__ v4u win_shift(v4u w, uint32_t delta) {
    const uint32_t q = delta >> 2, r = delta & 3u;
    const uint32_t W[8] = {w.x, w.y, w.z, w.w, 0u, 0u, 0u, 0u};
    v4u o;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t lo = q == 0 ? W[j] : q == 1 ? W[j + 1] : q == 2 ? W[j + 2] : W[j + 3];
        const uint32_t hi = q == 0 ? W[j + 1] : q == 1 ? W[j + 2] : q == 2 ? W[j + 3] : W[j + 4];
        o[j] = __builtin_amdgcn_alignbyte(hi, lo, r);
    }
    return o;
}

// Bytes [lo, hi) of a 4-byte word that holds bytes [4j, 4j + 4).
__device__ __forceinline__ uint32_t byte_mask(int j, int lo, int hi) {
    auto below = [](int k) -> uint32_t { return k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : ((1u << (8 * k)) - 1u)); };
    return below(hi - 4 * j) & ~below(lo - 4 * j);
}

__device__ __forceinline__ uint32_t halves(uint32_t w) { return (w & 0xffffu) + (w >> 16); }

// Unpacked plan (wave-uniform).
struct SegCtx {
    uintptr_t in, ob, oal;  // input, output start, output start rounded down to 16
    uint32_t a;             // ob & 15
    uint32_t H, cs, l4off, G, nseg, rest, in_len, out_len, S;
    bool v6, tcp;
};

__device__ __forceinline__ HdrVals seg_vals(const SegCtx &c, const GsoPlan &pl, uint32_t s, uint32_t l4cs) {
    const uint32_t dl = s + 1 < c.nseg ? c.G : c.rest - s * c.G;
    const uint32_t pkt = c.H + dl, id = pl.id0 + s;
    uint32_t ipcs = 0;
    if (!c.v6)
        ipcs = ~fold16_32(pl.ip_base + bswap16(pkt & 0xffffu) + bswap16(id & 0xffffu)) & 0xffffu;
    const uint32_t fm = s + 1 == c.nseg ? 0xffu : 0xf6u;
    return HdrVals{pkt, id, ipcs, l4cs, pl.seq0 + c.G * s, pkt - c.cs, fm};
}

__device__ __forceinline__ SegCtx make_ctx(const SegParams &p, const GsoPlan &pl) {
    SegCtx c;
    c.in = reinterpret_cast<uintptr_t>(p.in) + pl.in_off;
    c.ob = reinterpret_cast<uintptr_t>(p.out) + pl.out_off;
    c.a = (uint32_t)(c.ob & 15u);
    c.oal = c.ob - c.a;
    c.H = pl.h_cs & 0xffffu;
    c.cs = pl.h_cs >> 16;
    c.l4off = pl.l4_fl & 0xffffu;
    c.v6 = (pl.l4_fl >> 16) & 1u;
    c.tcp = (pl.l4_fl >> 17) & 1u;
    c.G = pl.G;
    c.nseg = pl.nseg;
    c.rest = pl.rest;
    c.in_len = pl.in_len;
    c.out_len = pl.rest + pl.nseg * c.H;
    c.S = c.H + c.G;
    return c;
}

// Plan record through the constant address space, so the (wave-uniform)
// load is an s_load into SGPRs.
__device__ __forceinline__ GsoPlan load_plan(const GsoPlan *plan, uint64_t i) {
#if __HIP_DEVICE_COMPILE__
    typedef __attribute__((address_space(4))) const GsoPlan c_plan;
    return ((c_plan *)(reinterpret_cast<uintptr_t>(plan)))[i];
#else
    return plan[i];
#endif
}

// Per-segment geometry (wave-uniform).  All per-lane offsets are 32-bit and
// relative to the segment's first owned chunk; only the bases are 64-bit.
struct SegGeo {
    uint64_t s0;           // segment start in the output
    uintptr_t src_b;       // in + i * G: source of segment-relative byte r is src_b + r
    uintptr_t dst_b;       // destination of the first owned chunk
    int64_t src_o;         // i * G
    int seglen, r_f, jh, jt;
    uint32_t i, nk, nhead, nm;
    bool last;
};

__device__ __forceinline__ SegGeo seg_geo(const SegCtx &c, uint32_t i) {
    SegGeo g;
    g.i = i;
    g.s0 = (uint64_t)i * c.S;
    const uint32_t dl = i + 1 < c.nseg ? c.G : c.rest - i * c.G;
    g.seglen = (int)(c.H + dl);
    g.last = i + 1 == c.nseg;
    const uint64_t sa = g.s0 + c.a;                    // segment start, aligned coordinates
    const uint64_t kf = i == 0 ? 0 : (sa + 15) >> 4;  // first chunk owned
    const uint64_t ke = (g.last ? (uint64_t)c.out_len + c.a + 15 : sa + c.S + 15) >> 4;
    g.nk = (uint32_t)(ke - kf);
    g.r_f = (int)((int64_t)(kf << 4) - (int64_t)sa);
    // chunks that are not pure payload: a head run over the header and a
    // tail run past the payload end (next header / output end)
    int jh = ((int)c.H - g.r_f + 15) >> 4;
    g.jh = jh < (int)g.nk ? jh : (int)g.nk;
    const int jt = (g.seglen - g.r_f) >> 4;
    g.jt = jt > g.jh ? jt : g.jh;
    g.nhead = (uint32_t)g.jh;
    g.nm = g.nhead + (g.nk - (uint32_t)g.jt);
    g.src_o = (int64_t)i * c.G;
    g.src_b = c.in + (uint64_t)g.src_o;
    g.dst_b = c.oal + (kf << 4);
    return g;
}

template <int U>
struct SegFront2 {
    v4u wv[U];
    int dlt[U];
    uint32_t tb;
};

// Issue every load of one row of chunks (branch-free; clamped into the
// super-buffer, shifted back later).
template <int U>
__device__ __forceinline__ void seg_issue2(const SegCtx &c, const SegGeo &g, uint32_t rb, uint32_t lane,
                                           SegFront2<U> &f) {
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int r = g.r_f + 16 * (int)(rb + lane + 64u * u);
        int64_t o = g.src_o + r;
        o = o < 0 ? 0 : o;
        const int64_t mx = (int64_t)c.in_len - 16;
        const int64_t ob = o > mx ? mx : o;
        f.dlt[u] = (int)(o - ob);
        f.wv[u] = ldu16_nt(c.in + (uintptr_t)ob);
    }
    f.tb = rb == 0 ? ld8(c.in + (lane < c.H ? lane : 0u)) : 0u;
}

// Store / sum one issued row; stage the mixed chunks' windows and (first
// row) the header template in LDS.  Returns this lane's folded payload sum.
template <int U>
__device__ __forceinline__ uint32_t seg_row(const SegCtx &c, const Ctx &cc, const SegGeo &g, uint32_t rb,
                                            uint32_t lane, SegFront2<U> &f, uint8_t *tmpl, uint16_t *code,
                                            uint8_t *win) {
    bool shift = false;
#pragma unroll
    for (int u = 0; u < U; u++)
        shift |= f.dlt[u] != 0;
    if (__ballot(shift)) {  // only the super-buffer's last chunks
#pragma unroll
        for (int u = 0; u < U; u++)
            f.wv[u] = win_shift(f.wv[u], (uint32_t)(f.dlt[u] > 15 ? 15 : f.dlt[u]));
    }
    uint32_t part = 0;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t j = rb + lane + 64u * u;
        const int r = g.r_f + 16 * (int)j;
        const v4u v = f.wv[u];
        if (j < g.nk && r >= (int)c.H && r + 16 <= g.seglen) {
            stu16_nt(g.dst_b + 16u * (uint64_t)j, v);
            part += halves(v.x) + halves(v.y) + halves(v.z) + halves(v.w);
        } else if (j < g.nk) {
            int t0 = (int)c.H - r, t1 = g.seglen - r;
            t0 = t0 < 0 ? 0 : (t0 > 16 ? 16 : t0);
            t1 = t1 < t0 ? t0 : (t1 > 16 ? 16 : t1);
#pragma unroll
            for (int q4 = 0; q4 < 4; q4++)
                part += halves(v[q4] & byte_mask(q4, t0, t1));
            const uint32_t m = (int)j < g.jh ? j : g.nhead + (j - (uint32_t)g.jt);
            if (m < kWinMax)
                *reinterpret_cast<v4u *>(win + 16 * m) = v;
        }
    }
    if (rb == 0) {
        if (lane < c.H) {  // kTmplMax >= 64
            tmpl[lane] = (uint8_t)f.tb;
            code[lane] = (uint16_t)hdr_code(cc, lane);
        }
        for (uint32_t x = lane + 64; x < (c.H < kTmplMax ? c.H : kTmplMax); x += 64) {  // hdr_len > 64
            tmpl[x] = (uint8_t)ld8(c.in + x);
            code[x] = (uint16_t)hdr_code(cc, x);
        }
    }
    return fold16_32(part);
}

// Everything after the first row's loads: the remaining rows, the L4
// checksum, and the mixed chunks one byte per lane.
template <int U>
__device__ __forceinline__ void seg_finish2(const SegCtx &c, const Ctx &cc, const GsoPlan &pl, const SegGeo &g,
                                            uint32_t lane, SegFront2<U> &f, uint8_t *tmpl, uint16_t *code,
                                            uint8_t *win) {
    uint32_t acc = seg_row<U>(c, cc, g, 0, lane, f, tmpl, code, win);
    for (uint32_t rb = 64u * U; rb < g.nk; rb += 64u * U) {  // segments longer than one row
        SegFront2<U> f2;
        seg_issue2<U>(c, g, rb, lane, f2);
        acc += seg_row<U>(c, cc, g, rb, lane, f2, tmpl, code, win);
    }
    // L4 checksum (:201-204): payload sum (absolute pairing; the L4 region
    // pairs from seg + cs) + invariant header sums + this segment's fields +
    // pseudo-header
    uint32_t lp = fold16_32(wave_sum_u32(fold16_32(acc)));
    if ((c.ob + g.s0 + c.cs) & 1u)
        lp = bswap16(lp);
    const uint32_t pkt = (uint32_t)g.seglen, seq = pl.seq0 + c.G * g.i;
    uint32_t l4h = pl.l4h_base;
    if (c.tcp)
        l4h += bswap16(seq >> 16) + bswap16(seq & 0xffffu) + ((g.last ? pl.flags13 : (pl.flags13 & ~0x09u)) << 8);
    else
        l4h += bswap16((pkt - c.cs) & 0xffffu);
    const uint32_t T = lp + l4h + pl.ps_sum + ((c.tcp ? 6u : 17u) << 8) + bswap16((pkt - c.cs) & 0xffffu);
    const uint32_t l4cs = ~fold16_32(T) & 0xffffu;
    const HdrVals hA = seg_vals(c, pl, g.i, l4cs);
    const HdrVals hB = seg_vals(c, pl, g.i + 1, 0u);  // only its first <= 15 (IP-level) bytes are used
    // LDS: a wave's ds ops execute in program order, so the staged windows /
    // template are visible to every lane; only the compiler must not move
    // them (wave_barrier is a code-motion barrier)
    __builtin_amdgcn_wave_barrier();
    // the mixed chunks' bytes, one byte per lane: a store instruction covers
    // whole chunks and completes the lines the payload stores left open
    for (uint32_t b = lane; b < 16u * g.nm; b += 64) {
        const uint32_t m = b >> 4, t = b & 15u;
        const uint32_t j = m < g.nhead ? m : (uint32_t)g.jt + (m - g.nhead);
        const int pr = g.r_f + 16 * (int)j + (int)t;  // byte rel. segment start
        if (pr < 0 || (g.last && pr >= g.seglen))
            continue;
        const bool second = pr >= (int)c.S;
        const uint32_t x = (uint32_t)(second ? pr - (int)c.S : pr);
        uint32_t byte;
        if (x < c.H) {
            const HdrVals &hv = second ? hB : hA;
            if (x < kTmplMax)
                byte = hdr_byte(hv, code[x], tmpl[x]);
            else
                byte = hdr_byte(hv, hdr_code(cc, x), ld8(c.in + x));
        } else if (m < kWinMax) {
            byte = win[b];
        } else {  // more than kWinMax mixed chunks (tiny segments)
            byte = ld8(g.src_b + (intptr_t)pr);
        }
        st8(g.dst_b + 16u * (uint64_t)j + t, byte);
    }
    __builtin_amdgcn_wave_barrier();  // the next segment rewrites the LDS staging
}

__device__ __forceinline__ Ctx hdr_ctx(const SegCtx &c) {
    Ctx cc;  // the fields hdr_code reads
    cc.v6 = c.v6;
    cc.tcp = c.tcp;
    cc.cs = c.cs;
    cc.l4off = c.l4off;
    return cc;
}

// Persistent grid sized to the resident waves: block (stripe q, slot group)
// -> wave slot r0; the wave takes segment r0 (+ Rw, ...) of super-buffers
// q, q + Q, q + 2Q, ...  All Q x Rw waves advance through the batch
// together, so the bytes in flight at any moment are one contiguous window
// of ~Q super-buffers (DRAM page locality), and a stripe's blocks are
// consecutive (one XCD's L2).  Each wave is a two-stage software pipeline:
// the next super-buffer's plan and first-row loads are issued before the
// current segment is stored, summed and headed.
template <int U>  // chunks per lane per row: one row covers segments up to 64 * U * 16 - 16 bytes
__global__ __launch_bounds__(256) void gso_seg_kernel(SegParams p) {
    __shared__ uint8_t s_tmpl[4][kTmplMax];
    __shared__ uint16_t s_code[4][kTmplMax];
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4][16 * kWinMax];

    const uint32_t lb = xcd_swizzle(blockIdx.x, gridDim.x);
    const uint32_t bps = p.Rw >> 2;
    const uint32_t q = lb / bps;
    const uint32_t w = wave_in_block(), lane = lane_id();
    const uint32_t r0 = (lb % bps) * 4u + w;
    if (q >= p.Q)
        return;
    uint8_t *tmpl = s_tmpl[w];
    uint16_t *code = s_code[w];
    uint8_t *win = s_win[w];

    // next super-buffer (from `sb`, step Q) that has a segment r0
    auto find = [&](uint64_t sb, GsoPlan &pl) -> uint64_t {
        for (; sb < p.n; sb += p.Q) {
            pl = load_plan(p.plan, sb);
            if ((pl.l4_fl >> 24) == kPlanRows && r0 < pl.nseg)
                return sb;
        }
        return p.n;
    };
    // two work slots, alternating roles (no copies of registers whose loads
    // are still in flight: that would force a wait)
    GsoPlan plA, plB;
    SegCtx cA, cB;
    SegGeo gA, gB;
    SegFront2<U> fA, fB;
    uint64_t sbA = find(q, plA);
    if (sbA >= p.n)
        return;
    cA = make_ctx(p, plA);
    gA = seg_geo(cA, r0);
    seg_issue2<U>(cA, gA, 0, lane, fA);
    auto rest_of = [&](const SegCtx &c, const Ctx &cc, const GsoPlan &pl) {
        for (uint32_t i = r0 + p.Rw; i < c.nseg; i += p.Rw) {  // more segments than slots
            const SegGeo g = seg_geo(c, i);
            SegFront2<U> f;
            seg_issue2<U>(c, g, 0, lane, f);
            seg_finish2<U>(c, cc, pl, g, lane, f, tmpl, code, win);
        }
    };
    for (;;) {
        const uint64_t sbB = find(sbA + p.Q, plB);
        if (sbB < p.n) {
            cB = make_ctx(p, plB);
            gB = seg_geo(cB, r0);
            seg_issue2<U>(cB, gB, 0, lane, fB);
        }
        {
            const Ctx cc = hdr_ctx(cA);
            seg_finish2<U>(cA, cc, plA, gA, lane, fA, tmpl, code, win);
            rest_of(cA, cc, plA);
        }
        if (sbB >= p.n)
            break;
        sbA = find(sbB + p.Q, plA);
        if (sbA < p.n) {
            cA = make_ctx(p, plA);
            gA = seg_geo(cA, r0);
            seg_issue2<U>(cA, gA, 0, lane, fA);
        }
        {
            const Ctx cc = hdr_ctx(cB);
            seg_finish2<U>(cB, cc, plB, gB, lane, fB, tmpl, code, win);
            rest_of(cB, cc, plB);
        }
        if (sbA >= p.n)
            break;
    }
}

}  // namespace wg

using namespace wg;

// Launch the plan and segment kernels (gso.hip launches the finalize kernel).
namespace wg {
int gso_rows_launch(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out, void *ws,
                    hipStream_t st) {
    GsoPlan *plan = static_cast<GsoPlan *>(ws);
    uint64_t pb = (n + 3) / 4;
    if (pb > 65536)
        pb = 65536;
    hipLaunchKernelGGL(gso_plan_kernel, dim3((unsigned)pb), dim3(256), 0, st, dev_in, dev_desc, n, plan);
    if (hipGetLastError() != hipSuccess)
        return WG_ERR_LAUNCH;
    const uint32_t Rw = (tune().gso_rows + 3u) & ~3u;
    uint32_t Q = tune().gso_stripes;
    if (!Q) {  // size the persistent grid to the resident blocks (one stripe = Rw / 4 blocks)
        static int resident = 0;  // blocks resident on the device (same for every MI355X)
        if (!resident) {
            int per_cu = 0, cus = 0, dev = 0;
            hipGetDevice(&dev);
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gso_seg_kernel<2>, 256, 0);
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            resident = per_cu > 0 && cus > 0 ? per_cu * cus : 1024;
        }
        Q = (uint32_t)resident / (Rw / 4);
        Q = Q ? Q : 1;
    }
    if (Q > n)
        Q = (uint32_t)n;
    uint64_t blocks = (uint64_t)Q * (Rw / 4);
    blocks = (blocks + 7) & ~7ull;  // XCD swizzle needs a multiple of 8
    SegParams p{dev_in, dev_out, plan, n, Rw, Q};
    hipLaunchKernelGGL((gso_seg_kernel<2>), dim3((unsigned)blocks), dim3(256), 0, st, p);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}
}  // namespace wg
