// wg_l4wave.hpp — one packet's L4 / plain checksum by one wavefront,
// split into an ISSUE phase (all loads, branch-free) and a FINISH phase
// (long-packet remainder, fold, pairing fix-up).  Shared by the batch
// checksum kernels (l4csum.hip) and the in-place path of the GSO kernel.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wg_device.hpp"
#include "wireglider_amd.h"

namespace wg {

struct Geom {
    uintptr_t a;  // packet start
    uint32_t len, cs, fl;
};

// Always-valid, always-zero 16 B: the load target of lanes (and packets)
// with nothing to read, so the issue phase needs no branches — a branch
// around a load makes the compiler wait for it inside the branch.
static __device__ v4u g_zero16;

// Per-packet state between the issue and finish phases.
struct Front {
    v4u v0, v1;      // interior chunks lane, lane + 64 (masked to zero)
    uint32_t bv;     // gathered byte, already shifted to its pairing
    bool bt;         // bv is in TRUE pairing (pseudo-header address byte)
    uint32_t hb;     // kHdr: packet byte `lane` (lanes 0-31), raw; else 0
    uint32_t r0odd;  // the summed region starts at an odd address
    uintptr_t c0;    // first aligned interior chunk
    uint32_t nint;   // interior chunk count
};

// Issue phase.  Summed region [r0, r1) = [a + cs, a + len) (empty when
// cs >= len).  Interior = whole aligned chunks [c0, c1); the unaligned head
// [r0, min(c0, r1)) and tail [max(c1, c0), r1) are <= 15 bytes each.
// Branch-free: out-of-range lanes re-read a valid chunk and are masked.
// The geometry is 32-bit offsets from the packet start (alignment depends
// only on the address's low bits): 64-bit scalar compares have no SALU form
// on gfx9 and cost a VALU compare plus exec bookkeeping each, and the scalar
// unit (one per CU) is what the per-packet work is bound by.  Requires
// len < 2^32 - 32.
// kHdr (plain sums only): the byte gather's otherwise idle lanes 0-31 bring
// packet bytes 0-31 into f.hb (raw, not summed by finish) — the verify
// kernel's header, with no extra load instruction.
template <bool kL4, bool kNT, bool kHdr = false>
__device__ __forceinline__ void issue(const Geom &g, uint32_t lane, Front &f) {
    static_assert(!(kL4 && kHdr), "kHdr uses the pseudo-header lanes");
    const uintptr_t zero = reinterpret_cast<uintptr_t>(&g_zero16);
    const uint32_t alo = (uint32_t)g.a;
    const uint32_t o0 = g.cs < g.len ? g.cs : g.len;                // r0 - a
    const uint32_t oc0 = ((alo + o0 + 15u) & ~15u) - alo;           // c0 - a, in [o0, o0 + 15]
    const uint32_t b1 = ((alo + g.len) & ~15u) - alo + 16u;         // c1 - a + 16 (c1 - a >= -15)
    const uint32_t b0 = oc0 + 16u;
    const uint32_t nint = b1 > b0 ? (b1 - b0) >> 4 : 0u;
    const uintptr_t c0 = g.a + oc0;
    f.r0odd = (alo + o0) & 1u;
    f.c0 = c0;
    f.nint = nint;
    // wave-uniform base and clamp, per-lane 32-bit offset
    const uintptr_t base = nint ? c0 : zero;
    const uint32_t last = nint ? nint - 1 : 0u;
    const uint32_t k0 = lane < last ? lane : last;
    const uint32_t k1 = lane + 64 < last ? lane + 64 : last;
    const v4u t0 = ld16x<kNT>(base + 16u * k0);
    const v4u t1 = ld16x<kNT>(base + 16u * k1);
    const v4u z = v4u{0, 0, 0, 0};
    f.v0 = lane < nint ? t0 : z;
    f.v1 = lane + 64 < nint ? t1 : z;

    // One byte per lane: lanes 0-31 pseudo-header addresses (pairing
    // relative to the address start, an even packet offset: 12 for v4, 8 for
    // v6 — checksum.cpp:14-28), lanes 32-47 the head, lanes 48-63 the tail
    // (absolute-address pairing, like the interior).
    const bool v6 = g.fl & WG_PKT_V6;
    const uint32_t ao = v6 ? 8u : 12u, al = v6 ? 32u : 8u;
    // Per-lane 32-bit offsets from a wave-uniform base (packet start, or the
    // zero chunk for an empty packet): no per-lane 64-bit addresses.
    const bool bt = kL4 && lane < al && ao + lane < g.len;
    const uint32_t heo = oc0 < g.len ? oc0 : g.len;   // head end
    const uint32_t tso = nint ? b1 - 16u : oc0;       // tail start
    const uint32_t xh = o0 + lane - 32u, xt = tso + lane - 48u;
    const bool bh = lane >= 32 && lane < 48 && xh < heo;
    const bool btl = lane >= 48 && xt < g.len;
    const bool bhd = kHdr && lane < 32u && lane < g.len;
    const uint32_t off = bt ? ao + lane : (bh ? xh : (btl ? xt : (bhd ? lane : 0u)));
    const uint32_t par = bt ? (lane & 1u) : ((alo + off) & 1u);
    const uint32_t byte = ld8((g.len ? g.a : zero) + off);
    f.bv = (bt || bh || btl) ? byte << (8u * par) : 0u;
    f.bt = bt;
    f.hb = bhd ? byte : 0u;
}

// Finish phase: this lane's share of the packet's sum in TRUE pairing.
// U: loads in flight per lane while streaming a long packet's rest (4 or 8).
template <bool kNT, int U = 4>
__device__ __forceinline__ uint32_t finish(uint32_t lane, const Front &f) {
    static_assert(U == 4 || U == 8, "loads in flight");
    Acc acc;
    if (f.nint > 128) {  // long packet (> ~2 KiB): stream the rest, U loads in flight
        const uintptr_t q = f.c0;
        const uint32_t last = f.nint - 1;
        // wave-uniform trip count: every round issues U loads (lanes past the
        // end re-read the last chunk and are masked), so the remainder is one
        // round trip too.  The first round goes out BEFORE the issue phase's
        // chunks are consumed (loads return in order: the adds of v0 / v1 wait
        // for those alone), so a packet of up to 128 + 64 U chunks costs one
        // memory round trip, not two.
        uint32_t k0 = 128;
        v4u a[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t k = k0 + 64 * u + lane;
            a[u] = ld16x<kNT>(q + 16ull * (k < last ? k : last));
        }
        acc.add4(f.v0);
        acc.add4(f.v1);
        for (;;) {
#pragma unroll
            for (int u = 0; u < U; u++)
                if (k0 + 64 * u + lane < f.nint)
                    acc.add4(a[u]);
            k0 += 64 * U;
            if (k0 >= f.nint)
                break;
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t k = k0 + 64 * u + lane;
                a[u] = ld16x<kNT>(q + 16ull * (k < last ? k : last));
            }
        }
    } else {
        acc.add4(f.v0);
        acc.add4(f.v1);
    }
    if (!f.bt)
        acc.add(f.bv);
    uint32_t s = fold16(acc.value());
    if (f.r0odd)  // region pairs from an odd address: swap its folded sum
        s = bswap16(s);
    return s + (f.bt ? f.bv : 0u);
}

}  // namespace wg
