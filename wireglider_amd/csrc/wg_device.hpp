// wg_device.hpp — gfx950 device primitives for the one's-complement engine.
//
// Arithmetic model: every byte b at absolute
// address x contributes b << (8 * (x & 1)) to a plain integer sum; that sum
// is congruent mod 0xFFFF to the RFC 1071 sum paired at even addresses, and
// is zero only if every byte is zero.  A region whose word pairing starts at
// an odd address (the reference pairs relative to the span start,
// include/netio/checksum.hpp:30-100) is corrected by one byte swap of its
// folded value (x * 256 mod 0xFFFF == bswap16(x)).  Folding is end-around and
// zero-preserving, so the reference's 0x0000-vs-0xFFFF split falls out
// exactly: the final result is 0xFFFF only when the whole sum is zero.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wg {

// 64 -> 16 bit end-around fold; result in [0, 0xFFFF], 0 iff x == 0.
__device__ __forceinline__ uint32_t fold16(uint64_t x) {
    uint64_t t = (x & 0xffffffffull) + (x >> 32);  // <= 2^33
    uint32_t u = (uint32_t)(t & 0xffffu) + (uint32_t)((t >> 16) & 0xffffu) + (uint32_t)(t >> 32);
    u = (u & 0xffffu) + (u >> 16);
    u = (u & 0xffffu) + (u >> 16);
    return u;
}

__device__ __forceinline__ uint32_t fold16_32(uint32_t u) {
    u = (u & 0xffffu) + (u >> 16);
    u = (u & 0xffffu) + (u >> 16);
    return u;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) {
    return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
}

// Native 4 x u32 vector (trivially copyable in every address space).
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t sum4(v4u v) {
    return (uint64_t)v.x + (uint64_t)v.y + (uint64_t)v.z + (uint64_t)v.w;
}

// 64-bit accumulator as two u32 with explicit carry: 2 VALU per dword
// (v_add_co_u32 + v_addc_co_u32), no zero-extension moves.
struct Acc {
    uint32_t lo = 0, hi = 0;
    __device__ __forceinline__ void add(uint32_t x) {
        uint32_t c;
        lo = __builtin_addc(lo, x, 0u, &c);
        hi += c;
    }
    __device__ __forceinline__ void add4(v4u v) {
        add(v.x);
        add(v.y);
        add(v.z);
        add(v.w);
    }
    __device__ __forceinline__ uint64_t value() const { return ((uint64_t)hi << 32) | lo; }
};

// DPP controls (GFX9 encoding).
enum : int {
    kDppQuadPerm1032 = 0xB1,  // quad_perm:[1,0,3,2]
    kDppQuadPerm2301 = 0x4E,  // quad_perm:[2,3,0,1]
    kDppRowHalfMirror = 0x141,
    kDppRowMirror = 0x140,
};

// Sum of v over all 64 lanes, returned wave-uniform.  EXEC must be full.
// In-row butterfly by DPP (4 VALU), then 4 readlanes across the rows.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppQuadPerm1032, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppQuadPerm2301, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppRowHalfMirror, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppRowMirror, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// Sum over aligned groups of G lanes (G = 4, 8 or 16); every lane of a group
// receives its group's total.  EXEC must be full.
template <int G>
__device__ __forceinline__ uint32_t group_sum_u32(uint32_t v) {
    static_assert(G == 4 || G == 8 || G == 16, "group size");
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppQuadPerm1032, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppQuadPerm2301, 0xF, 0xF, false);
    if (G >= 8)
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppRowHalfMirror, 0xF, 0xF, false);
    if (G >= 16)
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppRowMirror, 0xF, 0xF, false);
    return v;
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Cross-lane LDS handoff within one wave: every LDS write this wave issued
// before is visible to its reads after (release / acquire at wavefront scope
// around a scheduling barrier), instead of relying on LDS issue order.
__device__ __forceinline__ void wave_lds_handoff() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave index within the grid, provably uniform to the compiler.
__device__ __forceinline__ uint32_t wave_in_block() {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

// XCD-aware block remap (guide T1): blocks b and b+8 share an XCD under the
// observed round-robin dispatch, so give each XCD a contiguous run of virtual
// block ids.  Speed only; any placement is correct.  Needs nblocks % 8 == 0
// for the bijection, otherwise identity.
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t b, uint32_t nblocks) {
    if (nblocks & 7u)
        return b;
    return (b & 7u) * (nblocks >> 3) + (b >> 3);
}

// Loads through the GLOBAL address space (global_load_*, not flat_*: flat
// ops count against both vmcnt and lgkmcnt and return out of order).
typedef __attribute__((address_space(1))) const v4u g_v4u;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

// 16-byte load of an aligned chunk at absolute address `addr`.
__device__ __forceinline__ v4u ld16(uintptr_t addr) {
    return *reinterpret_cast<g_v4u *>(addr);
}

// Non-temporal variant (global_load_dwordx4 ... nt): for once-read streams.
__device__ __forceinline__ v4u ld16_nt(uintptr_t addr) {
    return __builtin_nontemporal_load(reinterpret_cast<g_v4u *>(addr));
}

template <bool kNT>
__device__ __forceinline__ v4u ld16x(uintptr_t addr) {
    if constexpr (kNT)
        return ld16_nt(addr);
    else
        return ld16(addr);
}

__device__ __forceinline__ uint32_t ld8(uintptr_t addr) {
    return *reinterpret_cast<g_u8 *>(addr);
}

// Raw buffer access (buffer_load / buffer_store through a 128-bit resource
// built from a wave-uniform base): a 32-bit per-lane byte offset instead of
// a 64-bit address, and the hardware range check as a free lane mask — a
// lane whose offset is kOob (past kRsrcRecords) loads 0 and stores nothing,
// with no EXEC manipulation.  Callers keep every real offset below
// kRsrcRecords (a super-buffer's input < 2^16 bytes; its split output at
// most ~2^30: 32,767 one-byte segments behind a 32,768-byte header).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOob = 0x80000000u;
constexpr int kRsrcRecords = 0x7fffffff;

__device__ __forceinline__ rsrc_t make_rsrc(uintptr_t base) {
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), (short)0, kRsrcRecords, 0x00020000);
}
__device__ __forceinline__ v4u bld16(rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t bld8(rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
}
__device__ __forceinline__ void bst16(rsrc_t r, uint32_t off, v4u v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}
__device__ __forceinline__ void bst8(rsrc_t r, uint32_t off, uint32_t b) {
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b, r, off, 0, 0);
}

// A PacketBatch of out_len bytes in segments of S: its encap messages and
// their bytes, or 0 / 0 when a bound is exceeded (more than max_segments
// segments, segments over max_segment_size, messages over msg_cap bytes).
// The encap counter scan (aead.hip encap_scan_local) and the headers-only
// split's synthesis skip (gso.hip) agree through this one function.
__device__ __forceinline__ uint32_t encap_fit(uint64_t out_len, uint32_t S, uint32_t max_segments,
                                             uint32_t max_segment_size, uint32_t msg_cap, uint32_t &bytes) {
    bytes = 0;
    if (!S || !out_len)
        return 0;
    const uint64_t ns = (out_len + S - 1) / S;
    const uint64_t last = out_len - (ns - 1) * S;
    const uint64_t b = (ns - 1) * (32ull + ((S + 15u) & ~15u)) + 32ull + ((last + 15u) & ~15ull);
    if (ns > max_segments || S > max_segment_size || b > msg_cap)
        return 0;
    bytes = (uint32_t)b;
    return (uint32_t)ns;
}

// wg_encap_batch header synthesis (knob encap_synth, aead.hip): a split
// super-buffer whose segments' headers the AEAD builds itself — the header in
// whole dwords of one 64-B block (every TCP / UDP header is), the L4 sum
// starting on a dword (the lanes' word sums then pair as the checksum does), the checksum field 2-B aligned, csum_start past
// the 20-B IPv4 header (the classification guarantees it for split plans; the
// MAC correction assumes the field lies past the block's first 16 bytes).
// The headers-only split skips exactly these (gso.hip), the AEAD builds
// exactly these.
__device__ __forceinline__ bool syn_eligible(uint32_t hdr_len, uint32_t cs, uint32_t l4off) {
    return hdr_len <= 64u && (hdr_len & 3u) == 0u && cs >= 20u && (cs & 3u) == 0u && (l4off & 1u) == 0u &&
           l4off + 2u <= hdr_len && cs + 8u <= hdr_len;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

}  // namespace wg
