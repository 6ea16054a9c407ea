// aead.hip — batched WireGuard data-message AEAD on MI355X (gfx950), SURVEY §8 f4.
//
// Per packet this is Peer::encrypt / Peer::decrypt (reference
// proto/proto.cpp:544-583, 496-523) over crypto_aead_chacha20poly1305_ietf
// (libsodium, i.e. RFC 8439), for the batches the workers build:
//   encap: every segment of a PacketBatch into consecutive data messages
//          (worker/encap.cpp:136-141; counter = encrypt_nonce++ per call);
//   decap: every message of a UDP GRO batch (worker/decap_ref.cpp:78-86).
//
// Layout: a group of lanes per packet (exactly the lanes its blocks need, up
// to 32; 64 lanes in passes for packets past 96 blocks), K consecutive
// ChaCha20 blocks per lane (knob aead_k; by default 2 or 3 per batch, see
// launch_aead): block counter c is lane c / K's.  Counter 0 (group lane 0's
// first block) is the Poly1305 key; the lane writing it also writes the
// DataHeader and handles the length block; counter c >= 1 is the keystream
// for the 64 bytes [64(c-1), 64c) of the padded payload, XORed and stored.
// Poly1305 runs in the lanes too: each lane Horner-evaluates its (up to) 4K
// 16-B ciphertext blocks with r, multiplies the result by r^(blocks after
// it) — a suffix product of r^(n_j) over the later lanes, log2(lanes)
// cross-lane steps — and the group sums the products (normalised 26-bit
// limbs, so 32 of them fit a dword) before one multiplication by r (the
// length block comes last), the reduction mod 2^130 - 5 and + s.  The
// per-lane fixed costs (powers of r, the scan, the term) are paid once per K
// blocks.  A lane's blocks are computed two at a time with their quarter
// rounds interleaved, and K = 3's third beside them: a 1,500-B packet takes
// K = 3 in 9 lanes, 7 packets per wave.
// ChaCha20 and Poly1305 are integer-VALU work (~1,000 and ~200
// instructions per 64-B block lane), so this kernel is bound by VALU issue,
// not HBM.
#include <hip/hip_runtime.h>

#include "wg_device.hpp"
#include "wg_internal.hpp"
#include "wireglider_amd.h"


namespace wg {

// ---------------------------------------------------------------------------
// ChaCha20 block function (RFC 8439 §2.3)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }

#define WG_QR(a, b, c, d)                                                                                            \
    a += b; d ^= a; d = rotl(d, 16);                                                                                 \
    c += d; b ^= c; b = rotl(b, 12);                                                                                 \
    a += b; d ^= a; d = rotl(d, 8);                                                                                  \
    c += d; b ^= c; b = rotl(b, 7);

struct AeadKey {
    uint32_t k[8];
};

__device__ __forceinline__ void chacha20_block(const AeadKey &key, uint32_t ctr, uint32_t n0, uint32_t n1, uint32_t n2,
                                               uint32_t out[16]) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = key.k[0], x5 = key.k[1], x6 = key.k[2], x7 = key.k[3];
    uint32_t x8 = key.k[4], x9 = key.k[5], x10 = key.k[6], x11 = key.k[7];
    uint32_t x12 = ctr, x13 = n0, x14 = n1, x15 = n2;
#pragma unroll 2
    for (int i = 0; i < 10; i++) {
        WG_QR(x0, x4, x8, x12);
        WG_QR(x1, x5, x9, x13);
        WG_QR(x2, x6, x10, x14);
        WG_QR(x3, x7, x11, x15);
        WG_QR(x0, x5, x10, x15);
        WG_QR(x1, x6, x11, x12);
        WG_QR(x2, x7, x8, x13);
        WG_QR(x3, x4, x9, x14);
    }
    out[0] = x0 + 0x61707865u;
    out[1] = x1 + 0x3320646eu;
    out[2] = x2 + 0x79622d32u;
    out[3] = x3 + 0x6b206574u;
    out[4] = x4 + key.k[0];
    out[5] = x5 + key.k[1];
    out[6] = x6 + key.k[2];
    out[7] = x7 + key.k[3];
    out[8] = x8 + key.k[4];
    out[9] = x9 + key.k[5];
    out[10] = x10 + key.k[6];
    out[11] = x11 + key.k[7];
    out[12] = x12 + ctr;
    out[13] = x13 + n0;
    out[14] = x14 + n1;
    out[15] = x15 + n2;
}
// Two consecutive blocks (counters ctr, ctr + 1) with their quarter rounds
// interleaved: 8 independent columns per step instead of 4, for a lane's
// first two blocks (aead_k = 2), so a wave has twice the independent VALU
// work between dependent instructions.
__device__ __forceinline__ void chacha20_block2(const AeadKey &key, uint32_t ctr, uint32_t n0, uint32_t n1,
                                                uint32_t n2, uint32_t o0[16], uint32_t o1[16]) {
    uint32_t x[16], y[16];
    const uint32_t init[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key.k[0], key.k[1], key.k[2],
                               key.k[3],    key.k[4],    key.k[5],    key.k[6],    key.k[7], ctr,      n0,
                               n1,          n2};
#pragma unroll
    for (int m = 0; m < 16; m++) x[m] = y[m] = init[m];
    y[12] = ctr + 1u;
#pragma unroll 2
    for (int i = 0; i < 10; i++) {
        WG_QR(x[0], x[4], x[8], x[12]);
        WG_QR(y[0], y[4], y[8], y[12]);
        WG_QR(x[1], x[5], x[9], x[13]);
        WG_QR(y[1], y[5], y[9], y[13]);
        WG_QR(x[2], x[6], x[10], x[14]);
        WG_QR(y[2], y[6], y[10], y[14]);
        WG_QR(x[3], x[7], x[11], x[15]);
        WG_QR(y[3], y[7], y[11], y[15]);
        WG_QR(x[0], x[5], x[10], x[15]);
        WG_QR(y[0], y[5], y[10], y[15]);
        WG_QR(x[1], x[6], x[11], x[12]);
        WG_QR(y[1], y[6], y[11], y[12]);
        WG_QR(x[2], x[7], x[8], x[13]);
        WG_QR(y[2], y[7], y[8], y[13]);
        WG_QR(x[3], x[4], x[9], x[14]);
        WG_QR(y[3], y[4], y[9], y[14]);
    }
#pragma unroll
    for (int m = 0; m < 16; m++) {
        o0[m] = x[m] + init[m];
        o1[m] = y[m] + (m == 12 ? ctr + 1u : init[m]);
    }
}
// Columns 1-3 of round 1 involve key, constants and nonce only, never the
// block counter (state word 12 is column 0's): one lane's blocks share them,
// so they are computed once per lane and every block starts from them
// (36 of ~960 quarter-round operations per block).
struct ChaPre {
    uint32_t v[12];  // x1 x5 x9 x13, x2 x6 x10 x14, x3 x7 x11 x15 after round 1's column quarter rounds
};

__device__ __forceinline__ ChaPre chacha_pre(const AeadKey &key, uint32_t n0, uint32_t n1, uint32_t n2) {
    uint32_t x1 = 0x3320646eu, x5 = key.k[1], x9 = key.k[5], x13 = n0;
    uint32_t x2 = 0x79622d32u, x6 = key.k[2], x10 = key.k[6], x14 = n1;
    uint32_t x3 = 0x6b206574u, x7 = key.k[3], x11 = key.k[7], x15 = n2;
    WG_QR(x1, x5, x9, x13);
    WG_QR(x2, x6, x10, x14);
    WG_QR(x3, x7, x11, x15);
    return ChaPre{{x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15}};
}

// Round 1 of a block from the shared columns: column 0 (the counter's), the
// precomputed columns 1-3, then the diagonals.
__device__ __forceinline__ void chacha_round1(const AeadKey &key, uint32_t ctr, const ChaPre &pc, uint32_t x[16]) {
    x[0] = 0x61707865u;
    x[4] = key.k[0];
    x[8] = key.k[4];
    x[12] = ctr;
    WG_QR(x[0], x[4], x[8], x[12]);
#pragma unroll
    for (int c = 0; c < 3; c++) {
        x[1 + c] = pc.v[4 * c];
        x[5 + c] = pc.v[4 * c + 1];
        x[9 + c] = pc.v[4 * c + 2];
        x[13 + c] = pc.v[4 * c + 3];
    }
    WG_QR(x[0], x[5], x[10], x[15]);
    WG_QR(x[1], x[6], x[11], x[12]);
    WG_QR(x[2], x[7], x[8], x[13]);
    WG_QR(x[3], x[4], x[9], x[14]);
}

// chacha20_block / chacha20_block2 from the shared round-1 columns.
__device__ __forceinline__ void chacha20_block_pre(const AeadKey &key, uint32_t ctr, uint32_t n0, uint32_t n1,
                                                   uint32_t n2, const ChaPre &pc, uint32_t out[16]) {
    uint32_t x[16];
    chacha_round1(key, ctr, pc, x);
#pragma unroll 3
    for (int i = 1; i < 10; i++) {
        WG_QR(x[0], x[4], x[8], x[12]);
        WG_QR(x[1], x[5], x[9], x[13]);
        WG_QR(x[2], x[6], x[10], x[14]);
        WG_QR(x[3], x[7], x[11], x[15]);
        WG_QR(x[0], x[5], x[10], x[15]);
        WG_QR(x[1], x[6], x[11], x[12]);
        WG_QR(x[2], x[7], x[8], x[13]);
        WG_QR(x[3], x[4], x[9], x[14]);
    }
    const uint32_t init[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key.k[0], key.k[1], key.k[2],
                               key.k[3],    key.k[4],    key.k[5],    key.k[6],    key.k[7], ctr,      n0,
                               n1,          n2};
#pragma unroll
    for (int m = 0; m < 16; m++)
        out[m] = x[m] + init[m];
}

__device__ __forceinline__ void chacha20_block2_pre(const AeadKey &key, uint32_t ctr, uint32_t n0, uint32_t n1,
                                                    uint32_t n2, const ChaPre &pc, uint32_t o0[16], uint32_t o1[16]) {
    uint32_t x[16], y[16];
    chacha_round1(key, ctr, pc, x);
    chacha_round1(key, ctr + 1u, pc, y);
#pragma unroll 3
    for (int i = 1; i < 10; i++) {
        WG_QR(x[0], x[4], x[8], x[12]);
        WG_QR(y[0], y[4], y[8], y[12]);
        WG_QR(x[1], x[5], x[9], x[13]);
        WG_QR(y[1], y[5], y[9], y[13]);
        WG_QR(x[2], x[6], x[10], x[14]);
        WG_QR(y[2], y[6], y[10], y[14]);
        WG_QR(x[3], x[7], x[11], x[15]);
        WG_QR(y[3], y[7], y[11], y[15]);
        WG_QR(x[0], x[5], x[10], x[15]);
        WG_QR(y[0], y[5], y[10], y[15]);
        WG_QR(x[1], x[6], x[11], x[12]);
        WG_QR(y[1], y[6], y[11], y[12]);
        WG_QR(x[2], x[7], x[8], x[13]);
        WG_QR(y[2], y[7], y[8], y[13]);
        WG_QR(x[3], x[4], x[9], x[14]);
        WG_QR(y[3], y[4], y[9], y[14]);
    }
    const uint32_t init[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key.k[0], key.k[1], key.k[2],
                               key.k[3],    key.k[4],    key.k[5],    key.k[6],    key.k[7], ctr,      n0,
                               n1,          n2};
#pragma unroll
    for (int m = 0; m < 16; m++) {
        o0[m] = x[m] + init[m];
        o1[m] = y[m] + (m == 12 ? ctr + 1u : init[m]);
    }
}
#undef WG_QR

// ---------------------------------------------------------------------------
// Poly1305 arithmetic mod 2^130 - 5 in five 26-bit limbs (RFC 8439 §2.5)
// ---------------------------------------------------------------------------
struct L5 {
    uint32_t v[5];
};

__device__ __forceinline__ L5 l5_one() { return L5{{1u, 0u, 0u, 0u, 0u}}; }
__device__ __forceinline__ L5 l5_zero() { return L5{{0u, 0u, 0u, 0u, 0u}}; }

// 16 little-endian bytes (four dwords) + 2^128 * hibit as limbs
__device__ __forceinline__ L5 l5_from_words(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t hibit) {
    L5 a;
    a.v[0] = w0 & 0x3ffffffu;
    a.v[1] = ((w0 >> 26) | (w1 << 6)) & 0x3ffffffu;
    a.v[2] = ((w1 >> 20) | (w2 << 12)) & 0x3ffffffu;
    a.v[3] = ((w2 >> 14) | (w3 << 18)) & 0x3ffffffu;
    a.v[4] = (w3 >> 8) | (hibit << 24);
    return a;
}

__device__ __forceinline__ L5 l5_sel(bool c, const L5 &a, const L5 &b) {
    L5 o;
#pragma unroll
    for (int i = 0; i < 5; i++) o.v[i] = c ? a.v[i] : b.v[i];
    return o;
}

__device__ __forceinline__ L5 l5_add(const L5 &a, const L5 &b) {
    L5 c;
#pragma unroll
    for (int i = 0; i < 5; i++) c.v[i] = a.v[i] + b.v[i];
    return c;
}

// a * b mod p, partially reduced (limbs < 2^26 + a little); inputs with
// limbs below ~2^27 (the products then stay below 2^58 after five terms).
__device__ __forceinline__ L5 l5_mul(const L5 &a, const L5 &b) {
    const uint32_t b0 = b.v[0], b1 = b.v[1], b2 = b.v[2], b3 = b.v[3], b4 = b.v[4];
    const uint32_t s1 = b1 * 5u, s2 = b2 * 5u, s3 = b3 * 5u, s4 = b4 * 5u;
    const uint32_t a0 = a.v[0], a1 = a.v[1], a2 = a.v[2], a3 = a.v[3], a4 = a.v[4];
    uint64_t d0 = (uint64_t)a0 * b0 + (uint64_t)a1 * s4 + (uint64_t)a2 * s3 + (uint64_t)a3 * s2 + (uint64_t)a4 * s1;
    uint64_t d1 = (uint64_t)a0 * b1 + (uint64_t)a1 * b0 + (uint64_t)a2 * s4 + (uint64_t)a3 * s3 + (uint64_t)a4 * s2;
    uint64_t d2 = (uint64_t)a0 * b2 + (uint64_t)a1 * b1 + (uint64_t)a2 * b0 + (uint64_t)a3 * s4 + (uint64_t)a4 * s3;
    uint64_t d3 = (uint64_t)a0 * b3 + (uint64_t)a1 * b2 + (uint64_t)a2 * b1 + (uint64_t)a3 * b0 + (uint64_t)a4 * s4;
    uint64_t d4 = (uint64_t)a0 * b4 + (uint64_t)a1 * b3 + (uint64_t)a2 * b2 + (uint64_t)a3 * b1 + (uint64_t)a4 * b0;
    L5 h;
    uint32_t c = (uint32_t)(d0 >> 26);
    h.v[0] = (uint32_t)d0 & 0x3ffffffu;
    d1 += c;
    c = (uint32_t)(d1 >> 26);
    h.v[1] = (uint32_t)d1 & 0x3ffffffu;
    d2 += c;
    c = (uint32_t)(d2 >> 26);
    h.v[2] = (uint32_t)d2 & 0x3ffffffu;
    d3 += c;
    c = (uint32_t)(d3 >> 26);
    h.v[3] = (uint32_t)d3 & 0x3ffffffu;
    d4 += c;
    c = (uint32_t)(d4 >> 26);
    h.v[4] = (uint32_t)d4 & 0x3ffffffu;
    h.v[0] += c * 5u;
    c = h.v[0] >> 26;
    h.v[0] &= 0x3ffffffu;
    h.v[1] += c;
    return h;
}

// The Horner step x = (x + m + 2^128) * r mod p for one 16-B block, in
// radix 2^32 (four 32-bit words + a small fifth): r is CLAMPED (RFC 8439
// §2.5: r_j < 2^28, r_1..r_3 divisible by 4), so 2^128 r_j = 2^130 (r_j / 4)
// == 5 r_j / 4 = s_j (mod p) folds the columns past 2^128 back exactly, each
// column is four or five products below 2^60.4 (no 64-bit overflow), and the
// product takes 16 + 3 multiplies instead of radix 2^26's 25 (the layout of
// OpenSSL's 32-bit Poly1305).  h[4] stays <= 4 between steps.
struct P32 {
    uint32_t h[5];
};

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// 32-bit carry chains (v_add_co / v_addc_co) and the column carries folded
// into the next column's multiply-add chain as its addend: no 64-bit adds of
// zero-extended words (each of those cost a register-pair move).
__device__ __forceinline__ P32 p32_step(const P32 &x, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
                                        const uint32_t r[4], const uint32_t sr[4]) {
    uint32_t c;
    const uint32_t t0 = __builtin_addc(x.h[0], m0, 0u, &c);
    const uint32_t t1 = __builtin_addc(x.h[1], m1, c, &c);
    const uint32_t t2 = __builtin_addc(x.h[2], m2, c, &c);
    const uint32_t t3 = __builtin_addc(x.h[3], m3, c, &c);
    const uint32_t t4 = x.h[4] + 1u + c;  // + 2^128: the block's pad bit
    const uint64_t d0 = mad64(t3, sr[1], mad64(t2, sr[2], mad64(t1, sr[3], (uint64_t)t0 * r[0])));
    const uint64_t d1 =
        mad64(t4, sr[1], mad64(t3, sr[2], mad64(t2, sr[3], mad64(t1, r[0], mad64(t0, r[1], d0 >> 32)))));
    const uint64_t d2 =
        mad64(t4, sr[2], mad64(t3, sr[3], mad64(t2, r[0], mad64(t1, r[1], mad64(t0, r[2], d1 >> 32)))));
    const uint64_t d3 =
        mad64(t4, sr[3], mad64(t3, r[0], mad64(t2, r[1], mad64(t1, r[2], mad64(t0, r[3], d2 >> 32)))));
    const uint32_t h4 = t4 * r[0] + (uint32_t)(d3 >> 32);
    const uint32_t cc = (h4 >> 2) + (h4 & ~3u);  // 5 * (h4 >> 2): 2^130 == 5
    P32 o;
    o.h[0] = __builtin_addc((uint32_t)d0, cc, 0u, &c);
    o.h[1] = __builtin_addc((uint32_t)d1, 0u, c, &c);
    o.h[2] = __builtin_addc((uint32_t)d2, 0u, c, &c);
    o.h[3] = __builtin_addc((uint32_t)d3, 0u, c, &c);
    o.h[4] = (h4 & 3u) + c;
    return o;
}

// radix 2^32 -> five 26-bit limbs (h[4] <= 4: limb 4 < 2^27)
__device__ __forceinline__ L5 p32_to_l5(const P32 &x) {
    return l5_from_words(x.h[0], x.h[1], x.h[2], x.h[3], x.h[4]);
}

// Shuffles within groups of G lanes (ds_bpermute).
template <int G>
__device__ __forceinline__ uint32_t grp_down(uint32_t v, uint32_t lane, uint32_t off) {
    const uint32_t g = lane & (G - 1u);
    const uint32_t src = g + off < (uint32_t)G ? lane + off : lane;
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
template <int G>
__device__ __forceinline__ L5 l5_down(const L5 &a, uint32_t lane, uint32_t off) {
    L5 b;
#pragma unroll
    for (int i = 0; i < 5; i++) b.v[i] = grp_down<G>(a.v[i], lane, off);
    return b;
}
template <int G>
__device__ __forceinline__ uint32_t grp_sum(uint32_t v, uint32_t lane) {
#pragma unroll
    for (uint32_t off = 1; off < (uint32_t)G; off <<= 1)
        v += (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane ^ off) << 2), (int)v);
    return v;
}

// The same for a group size known only at run time (gs lanes from base, any
// gs <= 32): `g` is the lane's index in its group.
__device__ __forceinline__ uint32_t grp_down_rt(uint32_t v, uint32_t lane, uint32_t g, uint32_t gs, uint32_t off) {
    const uint32_t src = g + off < gs ? lane + off : lane;
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((src & 63u) << 2), (int)v);
}
__device__ __forceinline__ L5 l5_down_rt(const L5 &a, uint32_t lane, uint32_t g, uint32_t gs, uint32_t off) {
    L5 b;
#pragma unroll
    for (int i = 0; i < 5; i++) b.v[i] = grp_down_rt(a.v[i], lane, g, gs, off);
    return b;
}

// Carry-normalise (value unchanged mod p): every limb < 2^26 but limb 1,
// which may exceed it by a few units.  Limbs in must be < 2^32 - 2^29.
__device__ __forceinline__ L5 l5_norm(L5 h) {
    uint32_t c;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        c = h.v[0] >> 26; h.v[0] &= 0x3ffffffu; h.v[1] += c;
        c = h.v[1] >> 26; h.v[1] &= 0x3ffffffu; h.v[2] += c;
        c = h.v[2] >> 26; h.v[2] &= 0x3ffffffu; h.v[3] += c;
        c = h.v[3] >> 26; h.v[3] &= 0x3ffffffu; h.v[4] += c;
        c = h.v[4] >> 26; h.v[4] &= 0x3ffffffu; h.v[0] += c * 5u;
    }
    c = h.v[0] >> 26; h.v[0] &= 0x3ffffffu; h.v[1] += c;
    return h;
}

// Group sum of normalised limbs: 32 lanes x (2^26 + small) fits 32 bits; 64
// lanes might not, so G = 64 sums two 32-lane halves, normalises, then adds.
template <int G>
__device__ __forceinline__ L5 l5_grp_sum(L5 a, uint32_t lane) {
    constexpr int H = G < 32 ? G : 32;
#pragma unroll
    for (int k = 0; k < 5; k++) a.v[k] = grp_sum<H>(a.v[k], lane);
    if constexpr (G == 64) {
        a = l5_norm(a);
#pragma unroll
        for (int k = 0; k < 5; k++)
            a.v[k] += (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane ^ 32u) << 2), (int)a.v[k]);
    }
    return a;
}

// Full reduction mod p of a limb sum (limbs < 2^32), + s mod 2^128 -> tag words.
__device__ __forceinline__ void poly_finish(L5 h, const uint32_t s[4], uint32_t tag[4]) {
    uint32_t h0 = h.v[0], h1 = h.v[1], h2 = h.v[2], h3 = h.v[3], h4 = h.v[4];
    uint32_t c;
    for (int k = 0; k < 2; k++) {  // two carry rounds: limbs < 2^32 -> < 2^26 (+ tiny)
        c = h0 >> 26; h0 &= 0x3ffffffu; h1 += c;
        c = h1 >> 26; h1 &= 0x3ffffffu; h2 += c;
        c = h2 >> 26; h2 &= 0x3ffffffu; h3 += c;
        c = h3 >> 26; h3 &= 0x3ffffffu; h4 += c;
        c = h4 >> 26; h4 &= 0x3ffffffu; h0 += c * 5u;
    }
    c = h0 >> 26; h0 &= 0x3ffffffu; h1 += c;
    uint32_t g0 = h0 + 5u;
    c = g0 >> 26; g0 &= 0x3ffffffu;
    uint32_t g1 = h1 + c;
    c = g1 >> 26; g1 &= 0x3ffffffu;
    uint32_t g2 = h2 + c;
    c = g2 >> 26; g2 &= 0x3ffffffu;
    uint32_t g3 = h3 + c;
    c = g3 >> 26; g3 &= 0x3ffffffu;
    const uint32_t g4 = h4 + c - (1u << 26);
    const uint32_t mask = (g4 >> 31) - 1u;  // all ones when h >= p
    h0 = (h0 & ~mask) | (g0 & mask);
    h1 = (h1 & ~mask) | (g1 & mask);
    h2 = (h2 & ~mask) | (g2 & mask);
    h3 = (h3 & ~mask) | (g3 & mask);
    h4 = (h4 & ~mask) | (g4 & mask);
    const uint64_t f0 = (uint64_t)(uint32_t)(h0 | (h1 << 26)) + s[0];
    const uint64_t f1 = (uint64_t)(uint32_t)((h1 >> 6) | (h2 << 20)) + s[1] + (f0 >> 32);
    const uint64_t f2 = (uint64_t)(uint32_t)((h2 >> 12) | (h3 << 14)) + s[2] + (f1 >> 32);
    const uint64_t f3 = (uint64_t)(uint32_t)((h3 >> 18) | (h4 << 8)) + s[3] + (f2 >> 32);
    tag[0] = (uint32_t)f0;
    tag[1] = (uint32_t)f1;
    tag[2] = (uint32_t)f2;
    tag[3] = (uint32_t)f3;
}

// ---------------------------------------------------------------------------
// Byte movement
// ---------------------------------------------------------------------------
static __device__ v4u g_aead_zero16;

__device__ __forceinline__ uint32_t keep_below(uint32_t w, uint32_t m, uint32_t lim) {
    // bytes of dword m below lim: all of them, none, or the low lim % 4 of
    // the one dword lim falls in (m is a compile-time index at every call:
    // two compares against constants and one mask shared by the dwords)
    const uint32_t part = (1u << (8u * (lim & 3u))) - 1u;
    return lim >= 4u * m + 4u ? w : (lim > 4u * m ? w & part : 0u);
}

// The 64 bytes at a (of which the first `n` belong to the packet, n may be
// 0..64; the rest read as zero) as 16 dwords.  The aligned 16-B chunks
// covering them are loaded; chunks past the packet's last byte read the
// zero chunk, and only the chunk holding that last byte has bytes to clear
// (those at or past a + n: another packet's), masked there BEFORE the
// funnel shift — one chunk's four masks instead of a byte mask on each of
// the sixteen shifted dwords.  No load leaves the packet's own aligned chunks.
__device__ __forceinline__ void load64(uintptr_t a, uint32_t n, uint32_t W[16]) {
    const uintptr_t a0 = a & ~(uintptr_t)15;
    const uintptr_t zero = reinterpret_cast<uintptr_t>(&g_aead_zero16);
    const uint32_t e = (uint32_t)a % 16u + n;          // end of the packet's bytes, relative to a0 (<= 79)
    const uint32_t cl = n ? (e - 1u) >> 4 : 5u;         // chunk holding the last byte (5: none)
    const uint32_t eb = e - 16u * cl;                   // its bytes to keep: [0, eb), 1..16
    uint32_t mk[4];
#pragma unroll
    for (uint32_t d = 0; d < 4; d++) {
        const uint32_t k = eb > 4u * d ? (eb - 4u * d < 4u ? eb - 4u * d : 4u) : 0u;
        mk[d] = k >= 4u ? ~0u : (1u << (8u * k)) - 1u;
    }
    v4u c[5];
#pragma unroll
    for (uint32_t k = 0; k < 5; k++) {
        c[k] = ld16(k <= cl && cl < 5u ? a0 + 16u * k : zero);
#pragma unroll
        for (uint32_t d = 0; d < 4; d++)
            c[k][d] = k == cl ? c[k][d] & mk[d] : c[k][d];
    }
    const v4u c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3], c4 = c[4];
    // dword m of the result funnels dwords m + q and m + q + 1 of the chunks,
    // q = (a / 4) mod 4 per lane: chosen by q's two bits over NAMED values
    // (selects between elements of an array became a scratch array indexed
    // at run time; a select chain on q became exec-mask branches per dword)
    const uint32_t sh = (uint32_t)a & 3u;
    const bool q1 = a & 4u, q2 = a & 8u;
    const uint32_t t0 = q1 ? c0[1] : c0[0];
    const uint32_t t1 = q1 ? c0[2] : c0[1];
    const uint32_t t2 = q1 ? c0[3] : c0[2];
    const uint32_t t3 = q1 ? c1[0] : c0[3];
    const uint32_t t4 = q1 ? c1[1] : c1[0];
    const uint32_t t5 = q1 ? c1[2] : c1[1];
    const uint32_t t6 = q1 ? c1[3] : c1[2];
    const uint32_t t7 = q1 ? c2[0] : c1[3];
    const uint32_t t8 = q1 ? c2[1] : c2[0];
    const uint32_t t9 = q1 ? c2[2] : c2[1];
    const uint32_t t10 = q1 ? c2[3] : c2[2];
    const uint32_t t11 = q1 ? c3[0] : c2[3];
    const uint32_t t12 = q1 ? c3[1] : c3[0];
    const uint32_t t13 = q1 ? c3[2] : c3[1];
    const uint32_t t14 = q1 ? c3[3] : c3[2];
    const uint32_t t15 = q1 ? c4[0] : c3[3];
    const uint32_t t16 = q1 ? c4[1] : c4[0];
    const uint32_t t17 = q1 ? c4[2] : c4[1];
    const uint32_t t18 = q1 ? c4[3] : c4[2];
    W[0] = __builtin_amdgcn_alignbyte(q2 ? t3 : t1, q2 ? t2 : t0, sh);
    W[1] = __builtin_amdgcn_alignbyte(q2 ? t4 : t2, q2 ? t3 : t1, sh);
    W[2] = __builtin_amdgcn_alignbyte(q2 ? t5 : t3, q2 ? t4 : t2, sh);
    W[3] = __builtin_amdgcn_alignbyte(q2 ? t6 : t4, q2 ? t5 : t3, sh);
    W[4] = __builtin_amdgcn_alignbyte(q2 ? t7 : t5, q2 ? t6 : t4, sh);
    W[5] = __builtin_amdgcn_alignbyte(q2 ? t8 : t6, q2 ? t7 : t5, sh);
    W[6] = __builtin_amdgcn_alignbyte(q2 ? t9 : t7, q2 ? t8 : t6, sh);
    W[7] = __builtin_amdgcn_alignbyte(q2 ? t10 : t8, q2 ? t9 : t7, sh);
    W[8] = __builtin_amdgcn_alignbyte(q2 ? t11 : t9, q2 ? t10 : t8, sh);
    W[9] = __builtin_amdgcn_alignbyte(q2 ? t12 : t10, q2 ? t11 : t9, sh);
    W[10] = __builtin_amdgcn_alignbyte(q2 ? t13 : t11, q2 ? t12 : t10, sh);
    W[11] = __builtin_amdgcn_alignbyte(q2 ? t14 : t12, q2 ? t13 : t11, sh);
    W[12] = __builtin_amdgcn_alignbyte(q2 ? t15 : t13, q2 ? t14 : t12, sh);
    W[13] = __builtin_amdgcn_alignbyte(q2 ? t16 : t14, q2 ? t15 : t13, sh);
    W[14] = __builtin_amdgcn_alignbyte(q2 ? t17 : t15, q2 ? t16 : t14, sh);
    W[15] = __builtin_amdgcn_alignbyte(q2 ? t18 : t16, q2 ? t17 : t15, sh);
}

__device__ __forceinline__ void st16(uintptr_t addr, v4u v) {
    *reinterpret_cast<__attribute__((address_space(1))) v4u *>(addr) = v;
}
__device__ __forceinline__ void st8b(uintptr_t addr, uint32_t v) {
    *reinterpret_cast<__attribute__((address_space(1))) uint8_t *>(addr) = (uint8_t)v;
}

// Store the first n (0..64) bytes of W at `a` (any alignment): whole 16-B
// stores for full chunks, bytes for the partial one.
__device__ __forceinline__ void store_n(uintptr_t a, const uint32_t W[16], uint32_t n) {
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
        const uint32_t b0 = 16u * q;
        if (b0 + 16u <= n) {
            st16(a + b0, v4u{W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3]});
        } else if (b0 < n) {
            // the partial chunk byte by byte, static register indices (a
            // run-time index would put W in scratch)
#pragma unroll
            for (uint32_t j = 0; j < 15; j++)
                if (b0 + j < n)
                    st8b(a + b0 + j, W[4 * q + (j >> 2)] >> (8u * (j & 3u)));
        }
    }
}

// ---------------------------------------------------------------------------
// The kernel
// ---------------------------------------------------------------------------
struct AeadParams {
    const uint8_t *in;
    uint8_t *out;
    int8_t *status;
    uint64_t total_len;
    uint64_t n;          // packets (encrypt) / messages (decrypt)
    uint32_t seg;        // segment_size of the input batch
    uint32_t receiver;   // encrypt: DataHeader.receiver_index
    uint64_t counter0;   // encrypt: counter of packet 0
    AeadKey key;
    uint32_t grp;        // aead_kernel<0, ...>: lanes per packet (1..32)
    uint8_t *verdict;    // decrypt + verify: WG_VERDICT_* per message (kVer)
    uint16_t *l4;        // decrypt + verify: the L4 checksum result per message (kVer)
    // encap (kGso): packet pi is segment pi % gm of super-buffer pi / gm
    const uint8_t *gin;          // wg_gso_split's input (passthrough batches)
    const wg_gso_desc *gdesc;
    const wg_gso_result *gres;
    const uint64_t *msg_off;     // where super-buffer i's messages go
    const uint32_t *work;        // [n] local exclusive prefixes of nmsg, [n + b] block prefixes
    wg_encap_result *eres;
    uint32_t gm;                 // max segments per super-buffer
    uint32_t gmode;              // kGso: 1 segments from `in` (wg_encap_encrypt), 2 headers from `in`,
                                 // payload from `gin` (wg_encap_batch)
    const uint64_t *ctr_base;    // kGso, nullable: messages of earlier chunks, added to counter0
                                 // (the host path's chained chunks)
    uint32_t lstride;            // kStage: bytes per message slot in LDS (32 + pad16(seg))
    uint32_t lds_wave;           // kStage: LDS bytes per wave (packets per wave x lstride)
    uint32_t synth;              // kGso == 2: eligible segments' headers built here (kSyn; encap_synth)
};

// The decap verify gates (wg_verify_desc, SURVEY §8 f1: evaluate_packet,
// include/worker/evaluator.hpp:112-149, worker/evaluator.cpp:14-58) decided
// from a packet's first 64 bytes R[16] (zero past len): the verdict bits,
// the protocol, the header length, whether the L4 checksum is computed, and
// the sums the L4 checksum needs besides the packet's own word sum: the
// header words [0, ihs) (subtracted) and the pseudo-header addresses.
struct HdrGate {
    uint32_t v, proto, ihs, hsum, asum;
    bool l4;
};

// acc + both 16-bit halves of w in one instruction (v_sad_u16 against zero)
__device__ __forceinline__ uint32_t hacc(uint32_t acc, uint32_t w) { return __builtin_amdgcn_sad_u16(w, 0u, acc); }

__device__ __forceinline__ HdrGate hdr_gate(const uint32_t R[16], uint32_t len) {
    HdrGate h{0u, 0u, 20u, 0u, 0u, false};
    if (len < 1u)
        return h;
    const uint32_t b0 = R[0] & 0xffu;
    const bool v6 = (b0 >> 4) == 6;
    h.v = v6 ? WG_VERDICT_V6 : 0u;
    h.ihs = v6 ? 40u : 20u;
    bool ip_ok = false;
    if (len >= h.ihs && len <= 65535u) {  // evaluator.hpp:118-121
        if (!v6) {
            const uint32_t hs = hacc(hacc(hacc(hacc(hacc(0u, R[0]), R[1]), R[2]), R[3]), R[4]);
            ip_ok = (b0 & 0xfu) == 5u &&                      // ip_hl, evaluator.cpp:19
                    len == bswap16(R[0] >> 16) &&              // ip_len, :21
                    (bswap16(R[1] >> 16) & ~0x4000u) == 0 &&  // ip_off & ~IP_DF, :24
                    fold16_32(hs) == 0xffffu;                 // header checksum == 0, :27
            h.proto = (R[2] >> 8) & 0xffu;
        } else {
            ip_ok = len - 40u == bswap16(R[1] & 0xffffu);  // ip6_plen, :47
            h.proto = (R[1] >> 16) & 0xffu;
        }
    }
    if (ip_ok) {
        h.v |= WG_VERDICT_IP_OK;
        if (h.proto == 6u) {
            h.v |= WG_VERDICT_TCP;
            h.l4 = len - h.ihs > 20u;  // evaluator.hpp:61
        } else if (h.proto == 17u) {
            h.v |= WG_VERDICT_UDP;
            h.l4 = len - h.ihs > 8u;  // evaluator.hpp:91
        }
    }
#pragma unroll
    for (uint32_t m = 0; m < 10; m++) {
        h.hsum = 4u * m < h.ihs ? hacc(h.hsum, R[m]) : h.hsum;
        h.asum = (v6 ? (m >= 2u && m < 10u) : (m == 3u || m == 4u)) ? hacc(h.asum, R[m]) : h.asum;  // v6 8-39, v4 12-19
    }
    return h;
}

constexpr uint64_t kRejectAfterMessages = ~0ull - (1ull << 13);  // include/proto/proto.hpp:36

// ---------------------------------------------------------------------------
// Encap header synthesis (wg_encap_batch, knob encap_synth).  A split
// segment's first 64 bytes are built by its group's lane 0 before the
// keystream, from the tun super-buffer itself: its prefix (ip_sum and the L4
// checksum field zeroed by the split's finalize pass,
// worker/offload.cpp:145-149) with the segment's fields (:168-199), then the
// payload, stored where the headers-only split would have written them.  The
// L4 checksum needs the whole segment's words, which the group's lanes sum
// as they encrypt their blocks (the totals ride along in the tag's group
// reduction); block 0 is encrypted with the field at zero, and at the end its
// two ciphertext bytes and the MAC are corrected (Poly1305 is linear in each
// 16-B block).  So the split pass only plans and finalizes these
// super-buffers: no per-segment wave, no payload read besides the
// encryption's own.  Eligible (syn_eligible, wg_device.hpp): the header in
// whole dwords of one 64-B block, csum_start a multiple of 4, the checksum
// field 2-B aligned — every plain IPv4 / IPv6 TCP or UDP header; other
// super-buffers keep the split's segments.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

struct SynSeg {
    uintptr_t tpl;  // the super-buffer (its prefix is every segment's header template)
    uint32_t tlen;  // its length
    uint32_t cs, l4off, hdr, gso, idx;
    bool tcp, v6, last;
};

// Segment q's plaintext [0, 64) — the template's header with the segment's
// fields, then the payload — stored at hdst (the segment slot, where the
// headers-only split would have written it; the encryption reads block 0
// back from there like any split header, so its lanes' word sums cover the
// header as stored).  The IP fields sit at fixed dwords and are set in
// registers; the L4 fields (TCP seq / flags, UDP length) sit at run-time
// offsets and are stored over the written block byte by byte (selecting
// dwords by a run-time index costs a select chain per dword).  rest: the L4
// sum's terms other than the segment's words from block 0 on — pseudo-header
// addresses, protocol, L4 length, and 32 * 0xFFFF minus block 0's words below
// csum_start (subtracting x mod 0xFFFF is adding 0xFFFF - x), plus pv, the
// two bytes at the checksum field once every field is set (the reference
// sums them, then overwrites them, :202-204): the field is stored as zero
// here (pv only differs from zero when the field overlaps the TCP seq or the
// UDP length), so the encryption needs no register for pv and the end just
// writes the checksum over a zero field.
__device__ __forceinline__ void syn_block0(const SynSeg &q, uintptr_t psrc, uintptr_t hdst, uint32_t pktlen,
                                           uint32_t &rest) {
    const uint32_t nin = pktlen < 64u ? pktlen : 64u;
    uint32_t T[16], M[16];
    if (nin == 64u && q.tlen >= 64u) {
        // both 64-B windows inside the super-buffer: four 16-B loads each at
        // the addresses as they are (the usual case)
#pragma unroll
        for (uint32_t c = 0; c < 4; c++) {
            const v4u t = ld16(q.tpl + 16u * c), v = ld16(psrc + 16u * c);
#pragma unroll
            for (uint32_t e = 0; e < 4; e++) {
                T[4 * c + e] = t[e];
                M[4 * c + e] = v[e];
            }
        }
    } else {
        // a real branch, taken only for short segments / super-buffers
        asm volatile("" ::: "memory");
        load64(q.tpl, q.hdr, T);  // the template (split super-buffers hold >= hdr bytes)
        load64(psrc, nin, M);     // payload byte j of the segment at psrc + j (j >= hdr), zero past nin
    }
    const uint32_t hw4 = q.hdr >> 2, cw = q.cs >> 2;  // both multiples of 4 (syn_eligible)
    const uint32_t l4len = bswap16((pktlen - q.cs) & 0xffffu);
    uint32_t ips = 0, ps = 0;
#pragma unroll
    for (uint32_t m = 0; m < 16; m++) {
        uint32_t w = m < hw4 ? T[m] : M[m];
        if (m == 0u && !q.v6)
            w = (w & 0xffffu) | (bswap16(pktlen & 0xffffu) << 16);  // ip_len (offload.cpp:183)
        if (m == 1u) {
            if (!q.v6)
                w = (w & 0xffff0000u) | bswap16((bswap16(w & 0xffffu) + q.idx) & 0xffffu);  // ip_id (:178-182)
            else
                w = (w & 0xffff0000u) | l4len;  // ip6_plen (:170-172)
        }
        M[m] = w;
        if (m < 15u)
            ips = m < cw ? hacc(ips, w) : ips;  // [0, cs), ip_sum zero (cw <= 14)
        if (m >= 2u && m < 10u)
            ps = (q.v6 || m == 3u || m == 4u) ? hacc(ps, w) : ps;  // addresses: v6 8-39, v4 12-19
    }
    const uint32_t ipcs = ~fold16_32(ips) & 0xffffu;
    if (!q.v6)
        M[2] = (M[2] & 0xffffu) | (ipcs << 16);  // ip_sum, native order (:184-186); the template's was zeroed (:147)
    if (nin == 64u) {
#pragma unroll
        for (uint32_t c = 0; c < 4; c++) st16(hdst + 16u * c, v4u{M[4 * c], M[4 * c + 1], M[4 * c + 2], M[4 * c + 3]});
    } else {
        store_n(hdst, M, nin);
    }
    const uintptr_t l4 = hdst + q.cs, t4 = q.tpl + q.cs;
    const uint32_t f0 = q.l4off - q.cs - 4u, f1 = f0 + 1u;  // the field's bytes from L4 byte 4 (wrap: none)
    uint32_t pv;
    if (q.tcp) {
        // seq (:192; seq0 read after the :149 zeroing) and FIN / PSH on the
        // last segment only (:193-195)
        const uint32_t s0 = (ld8(t4 + 4) << 24) | (ld8(t4 + 5) << 16) | (ld8(t4 + 6) << 8) | ld8(t4 + 7);
        const uint32_t sq = s0 + q.gso * q.idx;
        st8b(l4 + 4, sq >> 24);
        st8b(l4 + 5, sq >> 16);
        st8b(l4 + 6, sq >> 8);
        st8b(l4 + 7, sq);
        if (!q.last)
            st8b(l4 + 13, ld8(t4 + 13) & ~0x09u);  // (a flags byte inside the field is zero already)
        pv = (f0 < 4u ? (sq >> (24u - 8u * f0)) & 0xffu : 0u) | ((f1 < 4u ? (sq >> (24u - 8u * f1)) & 0xffu : 0u) << 8);
    } else {
        st8b(l4 + 4, l4len);  // udp len (:199)
        st8b(l4 + 5, l4len >> 8);
        pv = (f0 < 2u ? (l4len >> (8u * f0)) & 0xffu : 0u) | ((f1 < 2u ? (l4len >> (8u * f1)) & 0xffu : 0u) << 8);
    }
    st8b(hdst + q.l4off, 0u);  // the field zero until the checksum is written
    st8b(hdst + q.l4off + 1u, 0u);
    const uint32_t hw = ips + (q.v6 ? 0u : ipcs);  // block 0's words below csum_start, as stored
    rest = ps + ((q.tcp ? 6u : 17u) << 8) + l4len + pv + (32u * 0xffffu - hw);
}

// kDec = false: encrypt packet i (bytes [i*seg, +len) of `in`) into the data
// message at out + i*stride, stride = 16 + pad16(seg) + 16.
// kDec = true: decrypt message i (bytes [i*seg, +len) of `in`) into
// out + i*(seg - 32); status[i] = 0 / -1.
// G lanes per packet, K consecutive ChaCha20 blocks per lane: a pass covers
// counters [pass*G*K, +G*K), lane g the K from pass*G*K + g*K; counter 0 is
// the Poly1305 key block, counter c >= 1 the payload's 64-B block c - 1.
// G = 0: the group size is p.grp (any 1..32, set at launch as the lanes a
// packet needs: a 1,500-B packet's 25 blocks at K = 3 take 9 lanes, 7
// packets fill 63 of a wave's 64 lanes), one pass.
// kVer (decrypt only): the decap verify gates over each plaintext as it is
// produced (decrypt + evaluate_packet in one pass: no second read of the
// plaintext from HBM).  Every lane sums its plaintext's 16-bit words (blocks
// start at even offsets: packet-relative pairing); the lane holding payload
// block 0 decides the header gates from its 16 dwords (hdr_gate); the L4
// sum is the group's total minus the header words [0, ihs) plus the
// pseudo-header — exact, because subtracting x mod 0xFFFF is adding
// 0xFFFF - x and the total is never zero (the protocol word), so its fold
// only depends on the sum mod 0xFFFF.
// kGso (encrypt only): the packets are the segments of wg_gso_split's
// PacketBatches, super-buffer by super-buffer (worker/encap.cpp:136-141 for
// each tun read's batch), counters in order over all of them (the scan of
// encap_scan_*), messages at the caller's per-super-buffer offsets.
// kGso = 1: segment s of a split super-buffer is read whole from the split
// output; kGso = 2: only its first 64-B blocks up to the end of the header
// are (the headers-only split writes exactly those bytes), every later
// block from the input itself, where plaintext byte q >= hdr_len of segment
// s is input byte s * gso + q — one source per block, no merge.
// kStage (encrypt, groups of exactly the lanes needed): every message is
// assembled in the wave's LDS slot (header, ciphertext blocks, tag) and then
// written out slot by slot with consecutive lanes on consecutive 16-B chunks,
// so each store instruction covers whole lines: written straight from the
// lanes, a block's 64 B straddle two 64-B sectors (the ciphertext starts 16 B
// into the message) that are completed at different times, and the memory
// wrote ~1.48x the message bytes (profiles/pmc_aead.json).
template <int G, int K, bool kDec, bool kVer = false, int kGso = 0, bool kStage = false, bool kSyn = false>
__global__ __launch_bounds__(256) void aead_kernel(AeadParams p) {
    static_assert(!kStage || (!kDec && G == 0), "staged messages: encrypt, exact-size groups");
    static_assert(!kSyn || (kStage && kGso == 2 && K >= 2), "header synthesis: wg_encap_batch with staged messages, "
                                                             "block 0 in group lane 0");
    extern __shared__ v4u aead_lds[];
    constexpr bool kFlex = G == 0;
    const uint32_t GG = kFlex ? p.grp : (uint32_t)G;  // lanes per packet
    const uint32_t kPer = kFlex ? 64u / GG : 64u / (uint32_t)(G ? G : 1);  // packets per wave
    const uint32_t kPass = GG * (uint32_t)K;  // counters per pass
    const uint32_t lane = lane_id();
    const uint32_t slot = kFlex ? lane / GG : lane / (uint32_t)(G ? G : 1);  // packet of the wave
    const uint32_t g = kFlex ? lane - slot * GG : lane & (uint32_t)(G - 1);
    const uint64_t wave = (uint64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    const uint64_t i = wave * kPer + slot;
    bool live = slot < kPer && i < p.n;
    const uint64_t ii = live ? i : 0;
    uint64_t off = ii * p.seg;
    uint32_t len = live ? (uint32_t)(p.total_len - off < p.seg ? p.total_len - off : p.seg) : 0u;
    // kGso: segment s of super-buffer sb
    uint64_t sb = 0;
    uint32_t gs = 0, gstride = 0;
    uintptr_t gsrc = 0, gdst = 0;
    uintptr_t hsrc = 0;  // kGso == 2: the segment slot, holding plaintext [0, hl)
    uint32_t hl = 0;     // kGso == 2: hdr_len rounded up to whole 64-B blocks (0: passthrough)
    uint64_t gctr = 0;
    // encrypt: the end of the contiguous source region holding the packet's
    // plaintext (blocks at or past hl for kGso == 2): a partial last block
    // whose 64-B window ends inside it is loaded whole and masked
    uintptr_t send = 0;
    // kSyn: this segment's header is built here (syn_block0) when eligible
    bool syn = false;
    // the rest of the L4 sum folded to 16 bits | the checksum field's offset << 16
    uint32_t syn_rl = 0;
    if constexpr (kGso) {
        sb = ii / p.gm;
        gs = (uint32_t)(ii - sb * p.gm);
        const wg_encap_result er = p.eres[sb];  // nmsg from encap_scan_local
        const wg_gso_result gr = p.gres[sb];
        const wg_gso_desc gd = p.gdesc[sb];
        live = live && gs < er.nmsg;
        const uint32_t S = gr.segment_size;
        const uint64_t so = (uint64_t)gs * S;
        len = live ? (uint32_t)(gr.out_len - so < S ? gr.out_len - so : S) : 0u;
        if constexpr (kGso == 2) {
            hl = gr.passthrough ? 0u : ((uint32_t)gr.hdr_len + 63u) & ~63u;
            hsrc = reinterpret_cast<uintptr_t>(p.in) + gd.out_offset + so;
            gsrc = reinterpret_cast<uintptr_t>(p.gin) + gd.in_offset +
                   (gr.passthrough ? so : (uint64_t)gs * (S - gr.hdr_len));
            send = reinterpret_cast<uintptr_t>(p.gin) + gd.in_offset + gd.in_len;
            if constexpr (kSyn) {
                // in group lane 0, before the keystream (few registers live
                // here); the lane reads block 0 back from the slot later
                const uint32_t cs = gd.vnet.csum_start, l4 = cs + gd.vnet.csum_offset;
                syn = live && !gr.passthrough && syn_eligible(gr.hdr_len, cs, l4);
                syn_rl = l4 << 16;
                if (syn && g == 0u) {
                    SynSeg sq;
                    sq.tpl = reinterpret_cast<uintptr_t>(p.gin) + gd.in_offset;
                    sq.tlen = gd.in_len;
                    sq.cs = cs;
                    sq.l4off = l4;
                    sq.hdr = gr.hdr_len;
                    sq.gso = S - gr.hdr_len;
                    sq.idx = gs;
                    sq.tcp = gd.vnet.gso_type == 1u || gd.vnet.gso_type == 4u;  // unmasked (:151): TCP|ECN is fixed up as UDP
                    sq.v6 = gr.isv6;
                    sq.last = gs + 1u == er.nmsg;
                    uint32_t rest;
                    syn_block0(sq, gsrc, hsrc, len, rest);
                    syn_rl |= fold16_32(rest);
                }
            }
        } else {
            gsrc = (gr.passthrough ? reinterpret_cast<uintptr_t>(p.gin) + gd.in_offset
                                   : reinterpret_cast<uintptr_t>(p.in) + gd.out_offset) + so;
            send = gr.passthrough ? reinterpret_cast<uintptr_t>(p.gin) + gd.in_offset + gd.in_len
                                  : reinterpret_cast<uintptr_t>(p.in) + gd.out_offset + gr.out_len;
        }
        gstride = 32u + ((S + 15u) & ~15u);
        gdst = reinterpret_cast<uintptr_t>(p.out) + p.msg_off[sb] + (uint64_t)gs * gstride;
        gctr = p.counter0 + (p.ctr_base ? *p.ctr_base : 0ull) + p.work[p.n / p.gm + sb / 1024u] + p.work[sb] + gs;
    }
    // payload geometry
    uint64_t counter;
    uint32_t plen;  // encrypt: plaintext bytes; decrypt: ciphertext bytes
    uint32_t pad;   // bytes of the Poly1305 ciphertext region (pad16)
    uintptr_t src, dst;
    int8_t st = 0;
    if constexpr (!kDec) {
        counter = kGso ? gctr : p.counter0 + ii;
        plen = len;
        pad = (len + 15u) & ~15u;
        src = kGso ? gsrc : reinterpret_cast<uintptr_t>(p.in) + off;
        if constexpr (!kGso)
            send = reinterpret_cast<uintptr_t>(p.in) + p.total_len;
        dst = kGso ? gdst : reinterpret_cast<uintptr_t>(p.out) + ii * (32ull + ((p.seg + 15u) & ~15u));
        if (counter >= kRejectAfterMessages)  // proto.cpp:560-562: EncryptError::NoSession
            st = -1;
    } else {
        const uintptr_t msg = reinterpret_cast<uintptr_t>(p.in) + off;
        // DataHeader counter (bytes 8-15), only when the message holds a header
        const uint32_t hdr_ok = len >= 16u;
        uint32_t c0 = 0, c1 = 0;
        if (hdr_ok) {
            c0 = ld8(msg + 8) | (ld8(msg + 9) << 8) | (ld8(msg + 10) << 16) | (ld8(msg + 11) << 24);
            c1 = ld8(msg + 12) | (ld8(msg + 13) << 8) | (ld8(msg + 14) << 16) | (ld8(msg + 15) << 24);
        }
        counter = ((uint64_t)c1 << 32) | c0;
        if (len < 16u || counter > kRejectAfterMessages || len < 32u)  // proto.cpp:497-501; clen < ABYTES
            st = -1;
        plen = st ? 0u : len - 32u;
        pad = (plen + 15u) & ~15u;
        src = msg + 16;
        dst = reinterpret_cast<uintptr_t>(p.out) + ii * (uint64_t)(p.seg > 32u ? p.seg - 32u : 0u);
    }
    const uint32_t n0 = 0, n1 = (uint32_t)counter, n2 = (uint32_t)(counter >> 32);  // nonce: 0^4 || le64(counter)
    const bool act = live && st == 0;
    // kStage: this packet's message slot in LDS (16-B units)
    const uint32_t lslot = kStage ? (wave_in_block() * p.lds_wave + slot * p.lstride) / 16u : 0u;

    // Each lane's first block of pass 0 (counter g*K) up front: group lane
    // 0's is block 0, the Poly1305 key (r, s), which every lane needs first.
    // One pass (G < 64): the lane's blocks two at a time, each pair
    // interleaved (chacha20_block2), the first pair up front (8 independent
    // columns per step: -8 %, profiles/r02_aead_pair_ab.json)
    constexpr bool kPair = K >= 2 && G < 64;
    // K = 3, one pass: the lane's third block computed up front too, so its
    // quarter rounds sit in the same straight-line code as the first two
    // blocks' XOR / store / Poly1305 chains (dependent multiply-adds).
    // 3 waves/SIMD, and still faster: the waves wait on dependent VALU
    // issue, not on memory (forcing 4 waves/SIMD spills and loses half the
    // gain; encrypt -6.5 %, encap -4 %, profiles/r03_aead_tri_ab.json)
    constexpr bool kTri = K == 3 && G < 64;
    uint32_t ks[16], ks1[16], ks2[kTri ? 16 : 1];
    const ChaPre pc = chacha_pre(p.key, n0, n1, n2);
    if constexpr (kPair)
        chacha20_block2_pre(p.key, g * (uint32_t)K, n0, n1, n2, pc, ks, ks1);
    else
        chacha20_block_pre(p.key, g * (uint32_t)K, n0, n1, n2, pc, ks);
    if constexpr (kTri)
        chacha20_block_pre(p.key, g * (uint32_t)K + 2u, n0, n1, n2, pc, ks2);
    const uint32_t base_lane = kFlex ? slot * GG : lane & ~(uint32_t)(G - 1);
    uint32_t rw[4], sw[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        rw[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(base_lane << 2), (int)ks[k]);
        sw[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(base_lane << 2), (int)ks[4 + k]);
    }
    // r clamped (RFC 8439 §2.5)
    rw[0] &= 0x0fffffffu;
    rw[1] &= 0x0ffffffcu;
    rw[2] &= 0x0ffffffcu;
    rw[3] &= 0x0ffffffcu;
    const L5 r = l5_from_words(rw[0], rw[1], rw[2], rw[3], 0u);
    const uint32_t srw[4] = {0u, rw[1] + (rw[1] >> 2), rw[2] + (rw[2] >> 2), rw[3] + (rw[3] >> 2)};  // 5 r_j / 4

    const uint32_t nblk = (pad + 63u) / 64u;  // payload blocks: counters 1 .. nblk
    const uint32_t npass = G == 64 ? (nblk + kPass) / kPass : 1u;  // (nblk + 1) counters
    // wave-uniform pass count (G = 64: one packet per wave); passes run last
    // to first, F carrying r^(16-B blocks after the pass)
    const uint32_t passes = G == 64 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)npass) : 1u;
    L5 F = l5_one();
    L5 acc = l5_zero();
    uint32_t vsum = 0;                          // kVer: this lane's plaintext word sum
    uint32_t psum = 0;  // kSyn: the segment's words from block 0 on (this lane's blocks)
    HdrGate gate{0u, 0u, 20u, 0u, 0u, false};   // kVer: set in the lane holding payload block 0
    for (uint32_t pp = passes; pp-- > 0;) {
        const uint32_t cf = pp * kPass + g * (uint32_t)K;  // this lane's first counter
        // This lane's 16-B Poly1305 blocks in the pass follow from the
        // geometry alone: payload blocks [lo, hi) (counter c is block c - 1)
        // cut at pad.  So its weight r^nq and the suffix product over the
        // later lanes are computed here, before the block loop, and the
        // powers of r are dead by the time the keystream needs registers.
        uint32_t nq = 0;
        if (act) {
            const uint32_t lo = cf ? cf - 1u : 0u;
            const uint32_t hi = cf + K - 1u < nblk ? cf + K - 1u : nblk;
            nq = hi > lo ? ((64u * hi < pad ? 64u * hi : pad) - 64u * lo) / 16u : 0u;
        }
        L5 S;
        L5 synw;  // kSyn: r^(nq - k), the weight of chunk k = l4off / 16 (the checksum's) in group lane 0's sum
        {
            // r^nq = r^(4a) r^b from r, r^2 and r^4, r^8 (K >= 2), r^12, r^16
            // (K = 4); limb-wise selects (a select between whole L5 values
            // became a scratch array indexed at run time)
            const L5 r2 = l5_mul(r, r);
            const uint32_t a4 = nq >> 2, b = nq & 3u;
            const L5 r4 = l5_mul(r2, r2);
            L5 QA = l5_sel(a4 == 1u, r4, l5_one());
            if constexpr (K >= 2) {
                const L5 r8 = l5_mul(r4, r4);
                QA = l5_sel(a4 == 2u, r8, QA);
                if constexpr (K >= 3) {
                    const L5 r12 = l5_mul(r8, r4);
                    QA = l5_sel(a4 == 3u, r12, QA);
                    if constexpr (K == 4)
                        QA = l5_sel(a4 == 4u, l5_mul(r8, r8), QA);
                }
            }
            const L5 rb = l5_sel(b >= 2u, r2, l5_sel(b == 1u, r, l5_one()));
            const L5 r3 = l5_mul(r2, r);
            const L5 QB = l5_sel(b == 3u, r3, rb);
            S = l5_sel(b == 0u, QA, l5_sel(a4 == 0u, QB, l5_mul(QA, QB)));
            if constexpr (kSyn) {
                // chunk k opens group lane 0's Horner sum at block 0 (1 <= k
                // <= 3; lane 0's first counter is the key: nq <= 4(K - 1),
                // e <= 7)
                const uint32_t e = syn && g == 0u && nq > (syn_rl >> 20) ? nq - (syn_rl >> 20) : 0u;
                const uint32_t eb = e & 3u;
                const L5 WB = l5_sel(eb == 3u, r3, l5_sel(eb == 2u, r2, l5_sel(eb == 1u, r, l5_one())));
                synw = l5_mul(l5_sel(e >= 4u, r4, l5_one()), WB);
            }
        }
        L5 E;
        if constexpr (kFlex) {
            for (uint32_t o = 1; o < GG; o <<= 1) {  // wave-uniform trip count
                const L5 t = l5_down_rt(S, lane, g, GG, o);
                if (g + o < GG)
                    S = l5_mul(S, t);
            }
            E = l5_sel(g + 1u >= GG, l5_one(), l5_down_rt(S, lane, g, GG, 1u));
        } else {
#pragma unroll
            for (uint32_t o = 1; o < (uint32_t)G; o <<= 1) {
                const L5 t = l5_down<G ? G : 1>(S, lane, o);
                if (g + o < (uint32_t)G)
                    S = l5_mul(S, t);
            }
            // exclusive: product over lanes after this one
            E = l5_sel(g + 1u >= (uint32_t)G, l5_one(), l5_down<G ? G : 1>(S, lane, 1u));
        }
        // the later passes' blocks (F == 1 with one pass: wave-uniform test)
        const L5 EF = passes > 1 ? l5_mul(E, F) : E;
        if constexpr (kSyn) {
            // the L4 checksum field's weight, times EF, parked in the message
            // slot's header / tag positions (written only at the end) until
            // the checksum is known: no registers held across the blocks
            const L5 w = l5_mul(synw, EF);
            if (syn && g == 0u) {
                aead_lds[lslot] = v4u{w.v[0], w.v[1], w.v[2], w.v[3]};
                reinterpret_cast<uint32_t *>(aead_lds)[4u * (lslot + 1u + pad / 16u)] = w.v[4];
            }
        }
        if (passes > 1 && pp > 0) {
            // F *= product of the whole pass (group lane 0 holds S over lanes >= 0)
            L5 Sall;
#pragma unroll
            for (int k = 0; k < 5; k++)
                Sall.v[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(base_lane << 2), (int)S.v[k]);
            F = l5_mul(F, Sall);
        }

        // the lane's K blocks: keystream, XOR, store, Horner with r (radix 2^32)
        P32 x{{0u, 0u, 0u, 0u, 0u}};
        auto block = [&](uint32_t c, uint32_t kb[16]) {
            const uint32_t d = c - 1u;  // payload block
            const bool has = act && c >= 1u && d < nblk;
            const uint32_t boff = has ? 64u * d : 0u;
            const uint32_t nin = has ? (plen - boff < 64u ? plen - boff : 64u) : 0u;  // payload bytes in the block
            const uint32_t nct = has ? (pad - boff < 64u ? pad - boff : 64u) : 0u;    // Poly1305 bytes in the block
            // plaintext (encrypt) / ciphertext (decrypt); kGso == 2: blocks
            // below hl from the segment slot
            const uintptr_t bsrc = (kGso == 2 && boff < hl ? hsrc : src) + boff;
            const uintptr_t bdst = kDec ? dst + boff : dst + 16 + boff;
            // encrypt: a packet's last block whose 64-B window lies inside
            // the source region takes the whole-block path too, masked to its
            // payload bytes (ciphertext stores and Poly1305 steps only below
            // pad, both whole 16-B chunks): the general path then runs only
            // for windows at a region's end
            const bool tail = !kDec && has && nin < 64u && !(kGso == 2 && boff < hl) && bsrc + 64u <= send;
            uint32_t W[16];
            if (nin == 64u || tail) {
                // A whole block inside the payload (every block of a packet
                // but its last): four 16-B loads at the source address as it
                // is (gfx950 global loads take any alignment; all 64 bytes
                // are the packet's), no masks, four 16-B stores, four
                // unmasked Poly1305 steps.  Lanes whose block is the packet's
                // last, or none, take the general path below; per wave that
                // path runs only in the iterations where some lane needs it.
#pragma unroll
                for (uint32_t q = 0; q < 4; q++) {
                    const v4u v = ld16(bsrc + 16u * q);
#pragma unroll
                    for (uint32_t e = 0; e < 4; e++) W[4 * q + e] = v[e];
                }
                // wave-uniform: some lane holds a packet's last block here
                const bool anyt = !kDec && __ballot(tail) != 0;
                if (anyt) {
#pragma unroll
                    for (int m = 0; m < 16; m++)
                        W[m] = keep_below(W[m], (uint32_t)m, nin);  // padding plaintext is zero (proto.cpp:568-572)
                }
                if constexpr (kSyn) {
#pragma unroll
                    for (int m = 0; m < 16; m++) psum = hacc(psum, W[m]);  // the segment's L4 words
                }
#pragma unroll
                for (int m = 0; m < 16; m++) {
                    if constexpr (!kDec)
                        W[m] ^= kb[m];  // ciphertext
                    else
                        kb[m] ^= W[m];  // plaintext
                }
                const uint32_t *o = kDec ? kb : W;
                if (anyt) {
                    const uint32_t nqc = nct / 16u;  // ciphertext chunks below pad
#pragma unroll
                    for (uint32_t q = 0; q < 4; q++) {
                        if (q < nqc) {
                            const v4u v{o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
                            if constexpr (kStage)
                                aead_lds[lslot + (16u + boff) / 16u + q] = v;
                            else
                                st16(bdst + 16u * q, v);
                        }
                        const P32 t = p32_step(x, W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3], rw, srw);
#pragma unroll
                        for (int k = 0; k < 5; k++)
                            x.h[k] = q < nqc ? t.h[k] : x.h[k];
                    }
                } else {
#pragma unroll
                    for (uint32_t q = 0; q < 4; q++) {
                        const v4u v{o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
                        if constexpr (kStage)
                            aead_lds[lslot + (16u + boff) / 16u + q] = v;
                        else
                            st16(bdst + 16u * q, v);
                    }
#pragma unroll
                    for (uint32_t q = 0; q < 4; q++)
                        x = p32_step(x, W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3], rw, srw);
                }
            } else if (has) {
                // zero past the payload
                load64(bsrc, nin, W);
                if constexpr (kSyn) {
#pragma unroll
                    for (int m = 0; m < 16; m++) psum = hacc(psum, W[m]);  // the segment's L4 words
                }
                const uint32_t nqc = nct / 16u;  // whole 16-B Poly1305 chunks in the block (nct is a multiple of 16)
#pragma unroll
                for (int m = 0; m < 16; m++) {
                    if constexpr (!kDec) {
                        // padding plaintext bytes are zero (proto.cpp:568-572):
                        // their ciphertext is the keystream itself
                        W[m] = (uint32_t)m / 4u < nqc ? W[m] ^ kb[m] : 0u;  // ciphertext, what Poly1305 sees
                    } else if constexpr (kVer) {
                        kb[m] = keep_below(W[m] ^ kb[m], (uint32_t)m, nin);  // plaintext (the gates read it whole)
                    } else {
                        kb[m] = W[m] ^ kb[m];  // plaintext; store_n writes its first nin bytes only
                    }
                }
                // decrypt stores the plaintext now; a bad tag zeroes it below
                // (the final bytes are libsodium's either way)
                if constexpr (kStage) {
#pragma unroll
                    for (uint32_t q = 0; q < 4; q++)
                        if (q < nqc)
                            aead_lds[lslot + (16u + boff) / 16u + q] = v4u{W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3]};
                } else {
                    store_n(bdst, kDec ? kb : W, kDec ? nin : nct);
                }
#pragma unroll
                for (uint32_t q = 0; q < 4; q++) {
                    const P32 t = p32_step(x, W[4 * q], W[4 * q + 1], W[4 * q + 2], W[4 * q + 3], rw, srw);
#pragma unroll
                    for (int k = 0; k < 5; k++)
                        x.h[k] = q < nqc ? t.h[k] : x.h[k];
                }
            }
            if constexpr (kVer) {
                // the plaintext's words; the first 64 bytes decide the gates
                if (has) {
#pragma unroll
                    for (int m = 0; m < 16; m++) vsum = hacc(vsum, kb[m]);
                    if (d == 0u)
                        gate = hdr_gate(kb, plen);
                }
            }
        };
        uint32_t j0 = 0;
        if (pp == 0) {  // pass 0 starts with the block(s) computed up front
            block(cf, ks);
            j0 = 1;
            if constexpr (kPair) {
                block(cf + 1u, ks1);
                j0 = 2;
            }
            if constexpr (kTri) {
                block(cf + 2u, ks2);
                j0 = 3;
            }
        }
        if constexpr (kPair) {
            uint32_t j = j0;
#pragma unroll 1
            for (; j + 1u < (uint32_t)K; j += 2) {
                uint32_t kb[16], kb1[16];
                chacha20_block2(p.key, cf + j, n0, n1, n2, kb, kb1);
                block(cf + j, kb);
                block(cf + j + 1u, kb1);
            }
            if (j < (uint32_t)K) {  // K odd: the last block alone
                uint32_t kb[16];
                chacha20_block(p.key, cf + j, n0, n1, n2, kb);
                block(cf + j, kb);
            }
        } else {
#pragma unroll 1
            for (uint32_t j = j0; j < (uint32_t)K; j++) {
                uint32_t kb[16];
                chacha20_block(p.key, cf + j, n0, n1, n2, kb);
                block(cf + j, kb);
            }
        }
        // this lane's term: x * r^(blocks after it in this pass) * F; the
        // common factor r (the length block after everything) is applied
        // once to the group's sum
        if (nq)
            acc = l5_add(acc, l5_mul(p32_to_l5(x), EF));
        if constexpr (kSyn) {
            // a refused message (counter exhausted) encrypts nothing, but
            // its segment's header still needs the checksum: its lanes sum
            // their blocks' plaintext here (wave-uniform test, rare)
            if (__ballot(syn && !act) != 0ull && syn && !act) {
                for (uint32_t j = 0; j < (uint32_t)K; j++) {
                    const uint32_t c = g * (uint32_t)K + j, d = c - 1u;
                    if (c >= 1u && d < nblk) {
                        const uint32_t boff = 64u * d;
                        uint32_t W[16];
                        load64((boff < hl ? hsrc : src) + boff, plen - boff < 64u ? plen - boff : 64u, W);
#pragma unroll
                        for (int m = 0; m < 16; m++) psum = hacc(psum, W[m]);
                    }
                }
            }
        }
    }
    // the length block: le64(0) || le64(pad / payload length), times r
    const uint32_t mlen = kDec ? plen : pad;  // AEAD ct length (encrypt: the padded plaintext)
    const L5 lenblk = l5_from_words(0u, 0u, mlen, 0u, 1u);
    if (g == 0u && act)
        acc = l5_add(acc, lenblk);
    // group sum, times r (every term's last factor), every lane finishes
    L5 tot;
    if constexpr (kFlex) {
        // reduction tree by down-shifts (lane g sums [g, g + 2^k)), then the
        // group's first lane broadcasts: any group size
        L5 a = l5_norm(acc);
        uint32_t L = psum;  // kSyn: the segment's L4 words, summed along
        for (uint32_t o = 1; o < GG; o <<= 1) {
            const L5 t = l5_down_rt(a, lane, g, GG, o);
            uint32_t tl = 0;
            if constexpr (kSyn)
                tl = grp_down_rt(L, lane, g, GG, o);
            if (g + o < GG) {
                a = l5_add(a, t);
                L += tl;
            }
        }
        if constexpr (kSyn) {
            // group lane 0 now holds the segment's L4 word total: the
            // checksum, and the MAC's correction added to the group's sum
            if (syn && g == 0u) {
                const uint32_t l4cs = ~fold16_32(fold16_32(L) + (syn_rl & 0xffffu)) & 0xffffu;  // stored native (offload.cpp:202-204)
                // block 0 was encrypted with a zero field: its two
                // ciphertext bytes in the staged message, then the MAC
                uint16_t *lb = reinterpret_cast<uint16_t *>(aead_lds);
                const uint32_t syn_l4 = syn_rl >> 16;
                const uint32_t hw = (lslot * 16u + 16u + syn_l4) >> 1;
                const uint32_t oc = lb[hw];
                const uint32_t nc = (oc ^ l4cs) & 0xffffu;
                lb[hw] = (uint16_t)nc;
                st8b(hsrc + syn_l4, l4cs);  // and the segment's header in the slot
                st8b(hsrc + syn_l4 + 1u, l4cs >> 8);
                // its 16-B block (the lane's chunk l4off / 16) changes by
                // (nc - oc) * 256^(l4off % 16): add that times its weight mod p
                const uint32_t pb = syn_l4 & 15u;
                const bool up = nc >= oc;
                const uint32_t dv = (up ? nc - oc : oc - nc) << (8u * (pb & 3u));
                const uint32_t wq = pb >> 2;
                L5 dl = l5_from_words(wq == 0u ? dv : 0u, wq == 1u ? dv : 0u, wq == 2u ? dv : 0u, wq == 3u ? dv : 0u, 0u);
                if (!up) {  // -x == 2p - x (mod p); every limb of 2p exceeds x's
                    const uint32_t tp[5] = {0x7fffff6u, 0x7fffffeu, 0x7fffffeu, 0x7fffffeu, 0x7fffffeu};
#pragma unroll
                    for (int k = 0; k < 5; k++) dl.v[k] = tp[k] - dl.v[k];
                }
                // its weight r^(nq - k) * EF, parked in the slot by the S step
                // (and the slot's ciphertext written by the group's lanes):
                // an explicit wave-scope LDS handoff, not LDS issue order
                wave_lds_handoff();
                const uint32_t *lw = reinterpret_cast<const uint32_t *>(aead_lds);
                const v4u w4 = aead_lds[lslot];
                const L5 synw{{w4[0], w4[1], w4[2], w4[3], lw[4u * (lslot + 1u + pad / 16u)]}};
                a = l5_add(a, l5_mul(dl, synw));
            }
        }
#pragma unroll
        for (int k = 0; k < 5; k++)
            a.v[k] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(base_lane << 2), (int)a.v[k]);
        tot = l5_mul(l5_norm(a), r);
    } else {
        tot = l5_mul(l5_norm(l5_grp_sum<G ? G : 1>(l5_norm(acc), lane)), r);
    }
    uint32_t tagw[4];
    poly_finish(tot, sw, tagw);
    if constexpr (!kDec) {
        if (g == 0u && live) {
            if (act) {
                const v4u hdr{4u, p.receiver, n1, n2};  // DataHeader (proto.cpp:563-566)
                const v4u tag{tagw[0], tagw[1], tagw[2], tagw[3]};
                if constexpr (kStage) {
                    aead_lds[lslot] = hdr;
                    aead_lds[lslot + 1u + pad / 16u] = tag;
                } else {
                    st16(dst, hdr);
                    st16(dst + 16 + pad, tag);
                }
            }
            if constexpr (kGso) {
                if (gs == 0u)
                    p.eres[sb].counter0 = counter;
                // the first refused message ends the batch's output: the
                // reference advances its outbuf only over accepted messages
                // (worker/encap.cpp:138-140) while encrypt_nonce still counts
                // the refused ones (proto.cpp:556-562), and counters only
                // grow, so the accepted messages are a prefix of full-stride
                // ones
                if (st != 0 && (gs == 0u || counter - 1u < kRejectAfterMessages))
                    p.eres[sb].msg_bytes = gs * gstride;
            } else if (p.status) {
                p.status[ii] = st;
            }
        }
        if constexpr (kStage) {
            // every lane's blocks, headers and tags are in the slots: the
            // copy-out reads what other lanes of the wave wrote
            wave_lds_handoff();
            // the wave's messages, slot by slot: consecutive lanes on
            // consecutive 16-B chunks of one message (refused / empty slots
            // write nothing, as unstaged)
            const uint32_t mch = act ? (32u + pad) / 16u : 0u;  // the message's 16-B chunks
            const uint32_t dlo = (uint32_t)dst, dhi = (uint32_t)(dst >> 32);
            const uint32_t wl = wave_in_block() * p.lds_wave / 16u;
            const uint32_t l16 = p.lstride / 16u;
            // every slot a full-size message and the wave's messages back to
            // back in memory as they are in LDS (consecutive packets; a
            // super-buffer's segments): one flat copy of the whole run
            const uintptr_t base0 = (uintptr_t)(uint32_t)__builtin_amdgcn_readlane((int)dlo, 0) |
                                    ((uintptr_t)(uint32_t)__builtin_amdgcn_readlane((int)dhi, 0) << 32);
            const bool off = g == 0u && slot < kPer && (mch != l16 || dst != base0 + (uint64_t)slot * p.lstride);
            if (__ballot(off) == 0ull) {
                for (uint32_t t = lane; t < kPer * l16; t += 64u)
                    st16(base0 + 16u * t, aead_lds[wl + t]);
            } else {
                for (uint32_t s = 0; s < kPer; s++) {  // wave-uniform
                    const int src_lane = (int)(s * GG);
                    const uint32_t n16 = (uint32_t)__builtin_amdgcn_readlane((int)mch, src_lane);
                    if (n16 == 0u)
                        continue;
                    const uintptr_t base = (uintptr_t)(uint32_t)__builtin_amdgcn_readlane((int)dlo, src_lane) |
                                           ((uintptr_t)(uint32_t)__builtin_amdgcn_readlane((int)dhi, src_lane) << 32);
                    const uint32_t ls = wl + s * l16;
                    for (uint32_t t = lane; t < n16; t += 64u)
                        st16(base + 16u * t, aead_lds[ls + t]);
                }
            }
        }
    } else {
        // tag check (crypto_verify_16); on a mismatch libsodium zeroes the
        // message: overwrite this lane's plaintext blocks.  Messages rejected
        // before the MAC wrote nothing and stay untouched.
        const uintptr_t tsrc = src + plen;
        uint32_t got[4] = {0, 0, 0, 0};
        if (act) {
#pragma unroll
            for (int k = 0; k < 4; k++)
                got[k] = ld8(tsrc + 4 * k) | (ld8(tsrc + 4 * k + 1) << 8) | (ld8(tsrc + 4 * k + 2) << 16) |
                         (ld8(tsrc + 4 * k + 3) << 24);
        }
        const uint32_t diff = (got[0] ^ tagw[0]) | (got[1] ^ tagw[1]) | (got[2] ^ tagw[2]) | (got[3] ^ tagw[3]);
        const bool tag_ok = diff == 0;
        if (act && !tag_ok) {
            const uint32_t Z[16] = {};
            for (uint32_t pp = 0; pp < passes; pp++) {
                for (uint32_t j = 0; j < (uint32_t)K; j++) {
                    const uint32_t c = pp * kPass + g * (uint32_t)K + j;
                    const uint32_t d = c - 1u;
                    if (c >= 1u && d < nblk) {
                        const uint32_t boff = 64u * d;
                        store_n(dst + boff, Z, plen - boff < 64u ? plen - boff : 64u);
                    }
                }
            }
        }
        if (g == 0u && live)
            p.status[ii] = (int8_t)(st ? st : (tag_ok ? 0 : -1));
        if constexpr (kVer) {
            // the group's word sum (< 2^32: at most 32,768 words), to every lane
            uint32_t tsum = vsum;
            if constexpr (kFlex) {
                for (uint32_t o = 1; o < GG; o <<= 1) {
                    const uint32_t t = grp_down_rt(tsum, lane, g, GG, o);
                    if (g + o < GG)
                        tsum += t;
                }
                tsum = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(base_lane << 2), (int)tsum);
            } else {
                tsum = grp_sum<G ? G : 1>(tsum, lane);
            }
            // the lane holding payload block 0 (counter 1) writes the verdict
            const uint32_t h0 = 1u / (uint32_t)K < GG ? 1u / (uint32_t)K : 0u;  // (an empty plaintext: a 1-lane group)
            if (g == h0 && live) {
                const bool ok = act && tag_ok;  // rejected / failed messages: no packet
                uint32_t c = 0;
                if (ok && gate.l4) {
                    const uint32_t T = fold16_32(tsum) + (0xffffu - fold16_32(gate.hsum)) + fold16_32(gate.asum) +
                                       (gate.proto << 8) + bswap16((plen - gate.ihs) & 0xffffu);
                    c = ~fold16_32(T) & 0xffffu;
                }
                p.verdict[ii] = (uint8_t)(ok ? (gate.v | (gate.l4 && c == 0u ? WG_VERDICT_L4_OK : 0u)) : 0u);
                p.l4[ii] = (uint16_t)c;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Encap counter scan: each super-buffer's message count (its PacketBatch's
// segments, 0 on a GSO error or a bound exceeded), exclusive prefix over the
// batch — block-local (encap_scan_local) then over the block totals
// (encap_scan_blocks) — so the AEAD kernel gives segment s of super-buffer i
// the counter counter0 + prefix(i) + s, as the reference's serial
// encrypt_nonce++ would.
// ---------------------------------------------------------------------------
struct EncapScan {
    const wg_gso_result *gres;
    wg_encap_result *eres;
    uint32_t *work;
    uint64_t *total;
    uint64_t n;
    uint32_t msg_cap, max_segments, max_segment_size;
    const uint64_t *base;  // nullable: added to *total (chained chunks of the host path)
};

__device__ __forceinline__ uint32_t block_excl_scan_1024(uint32_t v, uint32_t *lds, uint32_t t, uint32_t &tot) {
    // Hillis-Steele inclusive scan over 1,024 threads in LDS
    lds[t] = v;
    __syncthreads();
    for (uint32_t o = 1; o < 1024u; o <<= 1) {
        const uint32_t a = t >= o ? lds[t - o] : 0u;
        __syncthreads();
        lds[t] += a;
        __syncthreads();
    }
    tot = lds[1023];
    return lds[t] - v;
}

__global__ __launch_bounds__(1024) void encap_scan_local(EncapScan q) {
    __shared__ uint32_t lds[1024];
    const uint32_t t = threadIdx.x;
    const uint64_t i = (uint64_t)blockIdx.x * 1024u + t;
    uint32_t nm = 0, bytes = 0;
    if (i < q.n) {
        const wg_gso_result r = q.gres[i];
        const uint32_t S = r.segment_size;
        if (r.status == 0)
            nm = encap_fit(r.out_len, S, q.max_segments, q.max_segment_size, q.msg_cap, bytes);
        q.eres[i].nmsg = nm;
        q.eres[i].msg_bytes = bytes;
        q.eres[i].counter0 = 0;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan_1024(nm, lds, t, tot);
    if (i < q.n)
        q.work[i] = ex;
    if (t == 0)
        q.work[q.n + blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void encap_scan_blocks(EncapScan q, uint32_t nb) {
    __shared__ uint32_t lds[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t v = t < nb ? q.work[q.n + t] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan_1024(v, lds, t, tot);
    if (t < nb)
        q.work[q.n + t] = ex;
    if (t == 0 && q.total)
        q.total[0] = (q.base ? q.base[0] : 0ull) + tot;
}

}  // namespace wg

using namespace wg;

static AeadKey key_words(const uint8_t key[32]) {
    AeadKey k;
    for (int i = 0; i < 8; i++)
        k.k[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
                 ((uint32_t)key[4 * i + 3] << 24);
    return k;
}

// LDS per block of the staged encrypt kernel: at most this, so three blocks
// (12 waves) still fit a CU's 160 KiB; larger messages per wave are stored
// straight from the lanes
constexpr uint32_t kStageMaxBlockLds = 53248;

template <int G, int K, bool kDec>
static void launch_gk(const AeadParams &p, uint64_t blocks, hipStream_t st) {
    if constexpr (!kDec) {
        if constexpr (G == 0) {
            const uint32_t shm = 4u * p.lds_wave;
            if (p.lds_wave && shm <= kStageMaxBlockLds) {
                if (!p.eres)
                    hipLaunchKernelGGL((aead_kernel<0, K, false, false, 0, true>), dim3((unsigned)blocks), dim3(256),
                                       shm, st, p);
                else if (p.gmode == 2 && p.synth)
                    hipLaunchKernelGGL((aead_kernel<0, K, false, false, 2, true, true>), dim3((unsigned)blocks),
                                       dim3(256), shm, st, p);
                else if (p.gmode == 2)
                    hipLaunchKernelGGL((aead_kernel<0, K, false, false, 2, true>), dim3((unsigned)blocks), dim3(256),
                                       shm, st, p);
                else
                    hipLaunchKernelGGL((aead_kernel<0, K, false, false, 1, true>), dim3((unsigned)blocks), dim3(256),
                                       shm, st, p);
                return;
            }
        }
        if (p.eres) {  // encap: GSO segments
            if (p.gmode == 2)
                hipLaunchKernelGGL((aead_kernel<G, K, false, false, 2>), dim3((unsigned)blocks), dim3(256), 0, st, p);
            else
                hipLaunchKernelGGL((aead_kernel<G, K, false, false, 1>), dim3((unsigned)blocks), dim3(256), 0, st, p);
            return;
        }
    } else {
        if (p.verdict) {  // decrypt + verify
            hipLaunchKernelGGL((aead_kernel<G, K, true, true>), dim3((unsigned)blocks), dim3(256), 0, st, p);
            return;
        }
    }
    hipLaunchKernelGGL((aead_kernel<G, K, kDec>), dim3((unsigned)blocks), dim3(256), 0, st, p);
}

template <int K, bool kDec>
static void launch_k(const AeadParams &p, uint32_t G, uint64_t blocks, hipStream_t st) {
    if (G == 0)
        launch_gk<0, K, kDec>(p, blocks, st);
    else if (G == 1)
        launch_gk<1, K, kDec>(p, blocks, st);
    else
        launch_gk<64, K, kDec>(p, blocks, st);
}

// Launch geometry for payloads up to maxpay bytes: counters per packet are
// the key block + the padded payload's 64-B blocks; K (knob aead_k)
// consecutive blocks per lane; a group of exactly the lanes needed (up to
// 32: 64 / lanes packets per wave), else 64 lanes in several passes
struct AeadGeom {
    uint32_t K, lanes, G, per_wave, lstride, lds_wave;
    bool staged;  // the kStage kernel runs (encrypt)
};
static AeadGeom aead_geom(uint32_t maxpay, uint32_t seg, bool dec, const Tune &t) {
    const uint32_t nblk = (((maxpay + 15u) & ~15u) + 63u) / 64u;
    uint32_t K = t.aead_k;
    if (K == 0) {
        // auto: K = 2 or 3, whichever moves more packets per unit of lane
        // work with exact-size groups (64 / lanes packets per wave, K blocks
        // each lane): 1,500 B (25 blocks) -> K = 3, 9 lanes, 7 packets per
        // wave (63 of 64 lanes); 64 B (2 blocks) -> K = 2, 64 per wave
        const uint32_t c = nblk + 1u;
        const uint32_t l2 = (c + 1u) / 2u, l3 = (c + 2u) / 3u;
        const uint32_t w2 = l2 <= 32u ? 64u / l2 : 0u, w3 = l3 <= 32u ? 64u / l3 : 0u;
        K = 2u * w3 > 3u * w2 ? 3u : 2u;  // w3 / 3 > w2 / 2
    }
    AeadGeom a;
    a.K = K;
    a.lanes = (nblk + 1u + K - 1u) / K;
    a.G = a.lanes <= 1u ? 1u : a.lanes <= 32u ? 0u : 64u;
    a.per_wave = a.G ? 64u / a.G : 64u / a.lanes;
    // staged messages (encrypt, exact-size groups): one LDS slot per packet
    a.lstride = 32u + ((seg + 15u) & ~15u);
    a.lds_wave = (!dec && a.G == 0 && t.aead_stage) ? a.per_wave * a.lstride : 0u;
    a.staged = a.lds_wave && 4u * a.lds_wave <= kStageMaxBlockLds;
    return a;
}

template <bool kDec>
static int launch_aead(AeadParams &p, uint32_t maxpay, hipStream_t st, const Tune &t) {
    const AeadGeom a = aead_geom(maxpay, p.seg, kDec, t);
    const uint32_t K = a.K, G = a.G, per_wave = a.per_wave;
    p.grp = a.lanes;
    p.lstride = a.lstride;
    p.lds_wave = a.lds_wave;
    if (p.synth && !a.staged)
        return WG_ERR_INVALID;  // internal: synthesis was decided from the same geometry
    const uint64_t per_block = 4u * per_wave;  // packets per 256-thread block
    uint64_t blocks = (p.n + per_block - 1) / per_block;
    if (blocks >= 8)
        blocks = (blocks + 7) & ~7ull;  // XCD swizzle bijective; surplus waves have no live packet
    if (blocks > 0x7fffffffull)
        return WG_ERR_INVALID;
    if (K == 2)
        launch_k<2, kDec>(p, G, blocks, st);
    else
        launch_k<3, kDec>(p, G, blocks, st);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_aead_encrypt_batch(const uint8_t *dev_in, uint64_t total_len, uint32_t segment_size,
                                     const uint8_t key[32], uint32_t receiver_index, uint64_t counter0,
                                     uint8_t *dev_out, int8_t *dev_status, void *stream) {
    if (!segment_size || segment_size > 65535u || !key)
        return WG_ERR_INVALID;
    if (!total_len)
        return WG_OK;
    if (!dev_in || !dev_out || (reinterpret_cast<uintptr_t>(dev_out) & 15))
        return WG_ERR_INVALID;
    AeadParams p{};
    p.in = dev_in;
    p.out = dev_out;
    p.status = dev_status;
    p.total_len = total_len;
    p.n = (total_len + segment_size - 1) / segment_size;
    p.seg = segment_size;
    p.receiver = receiver_index;
    p.counter0 = counter0;
    p.key = key_words(key);
    return launch_aead<false>(p, segment_size, static_cast<hipStream_t>(stream), tune());
}

extern "C" int wg_aead_decrypt_batch(const uint8_t *dev_in, uint64_t total_len, uint32_t segment_size,
                                     const uint8_t key[32], uint8_t *dev_out, int8_t *dev_status, void *stream) {
    if (!segment_size || segment_size > 65535u + 32u || !key)
        return WG_ERR_INVALID;
    if (!total_len)
        return WG_OK;
    if (!dev_in || !dev_out || !dev_status)
        return WG_ERR_INVALID;
    AeadParams p{};
    p.in = dev_in;
    p.out = dev_out;
    p.status = dev_status;
    p.total_len = total_len;
    p.n = (total_len + segment_size - 1) / segment_size;
    p.seg = segment_size;
    p.key = key_words(key);
    return launch_aead<true>(p, segment_size > 32u ? segment_size - 32u : 0u, static_cast<hipStream_t>(stream), tune());
}


extern "C" int wg_aead_decrypt_verify_batch(const uint8_t *dev_in, uint64_t total_len, uint32_t segment_size,
                                            const uint8_t key[32], uint8_t *dev_out, int8_t *dev_status,
                                            uint8_t *dev_verdict, uint16_t *dev_l4, void *stream) {
    if (!segment_size || segment_size > 65535u + 32u || !key)
        return WG_ERR_INVALID;
    if (!total_len)
        return WG_OK;
    if (!dev_in || !dev_out || !dev_status || !dev_verdict || !dev_l4)
        return WG_ERR_INVALID;
    AeadParams p{};
    p.in = dev_in;
    p.out = dev_out;
    p.status = dev_status;
    p.verdict = dev_verdict;
    p.l4 = dev_l4;
    p.total_len = total_len;
    p.n = (total_len + segment_size - 1) / segment_size;
    p.seg = segment_size;
    p.key = key_words(key);
    return launch_aead<true>(p, segment_size > 32u ? segment_size - 32u : 0u, static_cast<hipStream_t>(stream), tune());
}

// the encap scans + the AEAD over GSO output (gmode 1: whole segments in
// dev_seg; 2: headers in dev_seg, payload in dev_in)
static int encap_launch(const uint8_t *dev_in, const uint8_t *dev_seg, const wg_gso_desc *dev_desc,
                        const wg_gso_result *dev_gso_res, uint64_t n, const uint8_t key[32], uint32_t receiver_index,
                        uint64_t counter0, const uint64_t *dev_msg_offset, uint32_t msg_cap, uint32_t max_segments,
                        uint32_t max_segment_size, uint8_t *dev_msgs, wg_encap_result *dev_res, uint32_t *dev_work,
                        uint64_t *dev_total, uint32_t gmode, const uint64_t *dev_base, hipStream_t st,
                        const Tune &t, bool synth) {
    EncapScan q{dev_gso_res, dev_res, dev_work, dev_total, n, msg_cap, max_segments, max_segment_size, dev_base};
    const uint32_t nb = (uint32_t)((n + 1023) / 1024);
    hipLaunchKernelGGL(encap_scan_local, dim3(nb), dim3(1024), 0, st, q);
    hipLaunchKernelGGL(encap_scan_blocks, dim3(1), dim3(1024), 0, st, q, nb);
    if (hipGetLastError() != hipSuccess)
        return WG_ERR_LAUNCH;
    AeadParams p{};
    p.in = dev_seg;
    p.out = dev_msgs;
    p.status = nullptr;
    p.n = n * max_segments;  // packet pi = segment pi % max_segments of super-buffer pi / max_segments
    p.seg = max_segment_size;
    p.total_len = p.n * (uint64_t)max_segment_size;  // unused by the kGso geometry
    p.receiver = receiver_index;
    p.counter0 = counter0;
    p.key = key_words(key);
    p.gin = dev_in;
    p.gdesc = dev_desc;
    p.gres = dev_gso_res;
    p.msg_off = dev_msg_offset;
    p.work = dev_work;
    p.eres = dev_res;
    p.gm = max_segments;
    p.gmode = gmode;
    p.ctr_base = dev_base;
    p.synth = synth ? 1u : 0u;
    return launch_aead<false>(p, max_segment_size, st, t);
}

// An empty batch still reports its message count: *dev_total = 0 (or the
// chained base), so counter0 + *dev_total stays the peer's next nonce.
static int encap_empty_total(uint64_t *dev_total, const uint64_t *dev_base, hipStream_t st) {
    if (!dev_total)
        return WG_OK;
    const hipError_t e = dev_base ? hipMemcpyAsync(dev_total, dev_base, sizeof(uint64_t), hipMemcpyDeviceToDevice, st)
                                  : hipMemsetAsync(dev_total, 0, sizeof(uint64_t), st);
    return e == hipSuccess ? WG_OK : WG_ERR_RUNTIME;
}

// the arguments both encap entry points share
static bool encap_args_ok(const uint8_t *key, uint64_t n, const void *dev_in, const void *dev_seg,
                          const wg_gso_desc *dev_desc, const wg_gso_result *dev_gso_res,
                          const uint64_t *dev_msg_offset, uint32_t max_segments, uint32_t max_segment_size,
                          const uint8_t *dev_msgs, const wg_encap_result *dev_res, const uint32_t *dev_work) {
    if (!key || !max_segments || !max_segment_size || max_segment_size > 65535u || n > (1ull << 20))
        return false;
    if (!n)
        return true;
    if (!dev_in || !dev_seg || !dev_desc || !dev_gso_res || !dev_msg_offset || !dev_msgs || !dev_res || !dev_work ||
        (reinterpret_cast<uintptr_t>(dev_msgs) & 15) || (reinterpret_cast<uintptr_t>(dev_gso_res) & 7) ||
        (reinterpret_cast<uintptr_t>(dev_desc) & 7) || (reinterpret_cast<uintptr_t>(dev_res) & 7) ||
        (reinterpret_cast<uintptr_t>(dev_msg_offset) & 7) || (reinterpret_cast<uintptr_t>(dev_work) & 3))
        return false;
    // the counter scan keeps per-super-buffer prefixes and block totals in
    // 32 bits: every message of the call must have a distinct 32-bit index,
    // or two segments would share a nonce
    return (uint64_t)max_segments * n < (1ull << 32);
}

extern "C" int wg_encap_encrypt(const uint8_t *dev_in, const uint8_t *dev_seg, const wg_gso_desc *dev_desc,
                                const wg_gso_result *dev_gso_res, uint64_t n, const uint8_t key[32],
                                uint32_t receiver_index, uint64_t counter0, const uint64_t *dev_msg_offset,
                                uint32_t msg_cap, uint32_t max_segments, uint32_t max_segment_size, uint8_t *dev_msgs,
                                wg_encap_result *dev_res, uint32_t *dev_work, uint64_t *dev_total, void *stream) {
    if (!encap_args_ok(key, n, dev_in, dev_seg, dev_desc, dev_gso_res, dev_msg_offset, max_segments, max_segment_size,
                       dev_msgs, dev_res, dev_work))
        return WG_ERR_INVALID;
    if (!n)
        return encap_empty_total(dev_total, nullptr, static_cast<hipStream_t>(stream));
    return encap_launch(dev_in, dev_seg, dev_desc, dev_gso_res, n, key, receiver_index, counter0, dev_msg_offset,
                        msg_cap, max_segments, max_segment_size, dev_msgs, dev_res, dev_work, dev_total, 1u,
                        nullptr, static_cast<hipStream_t>(stream), tune(), false);
}

namespace wg {

// Side stream + events for the pipelined encap step (knob encap_parts): one
// set per host thread and device, created on first use and kept.
struct EncapSide {
    int device = -1;
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr;
    hipEvent_t split_done[8] = {};
};
static thread_local EncapSide g_side;

static int encap_side(EncapSide &e) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return WG_ERR_NODEV;
    if (e.device == dev)
        return WG_OK;
    e = EncapSide{};  // a new device: the old objects are left to the runtime (device switches are rare)
    if (hipStreamCreateWithFlags(&e.side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&e.fork, hipEventDisableTiming) != hipSuccess)
        return WG_ERR_RUNTIME;
    for (hipEvent_t &ev : e.split_done)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
            return WG_ERR_RUNTIME;
    e.device = dev;
    return WG_OK;
}

int encap_batch_launch(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                       wg_gso_result *dev_gso_res, const uint8_t key[32], uint32_t receiver_index, uint64_t counter0,
                       const uint64_t *dev_msg_offset, uint32_t msg_cap, uint32_t max_segments,
                       uint32_t max_segment_size, uint8_t *dev_msgs, wg_encap_result *dev_res, uint32_t *dev_work,
                       uint64_t *dev_total, const uint64_t *dev_base, hipStream_t st) {
    if (!encap_args_ok(key, n, dev_in, dev_out, dev_desc, dev_gso_res, dev_msg_offset, max_segments, max_segment_size,
                       dev_msgs, dev_res, dev_work))
        return WG_ERR_INVALID;
    if (!n)
        return encap_empty_total(dev_total, dev_base, st);
    // one knob snapshot for the split and the AEAD: header synthesis
    // (encap_synth) needs the staged kernel, and the split must skip exactly
    // the super-buffers the AEAD synthesizes
    const Tune t = tune();
    const bool synth = t.encap_synth && aead_geom(max_segment_size, max_segment_size, false, t).staged;
    const EncapFit fit{msg_cap, max_segments, max_segment_size};
    const uint32_t parts = t.encap_parts;
    if (parts <= 1 || n < 2ull * parts) {
        // the split's list of super-buffers left to it lives in dev_work,
        // which the scans only use after the split
        const int rc = gso_split_launch(dev_in, dev_desc, n, dev_out, dev_gso_res, true, st, synth ? &fit : nullptr,
                                        dev_work);
        if (rc != WG_OK)
            return rc;
        return encap_launch(dev_in, dev_out, dev_desc, dev_gso_res, n, key, receiver_index, counter0, dev_msg_offset,
                            msg_cap, max_segments, max_segment_size, dev_msgs, dev_res, dev_work, dev_total, 2u,
                            dev_base, st, t, synth);
    }
    // Pipelined: the batch in `parts` slices of super-buffers; slice k's
    // headers-only split runs on a side stream while slice k-1's scans and
    // AEAD run on the caller's stream (the split waits on memory, the AEAD on
    // VALU issue).  Counters chain on the device: slice k starts at
    // counter0 + *base + the messages of slices < k (ctr[k], kept at the end
    // of dev_work past every slice's scan area), the last slice writing
    // *dev_total.
    EncapSide &e = g_side;
    int rc = encap_side(e);
    if (rc != WG_OK)
        return rc;
    // dev_work is 4 * (n + 1024) bytes; a slice's scan uses [0, cnt + cnt / 1024 + 1) dwords
    // and cnt <= n / 2 here, so the last 2 * (parts + 2) dwords are free (8-B aligned below)
    const uintptr_t wend = reinterpret_cast<uintptr_t>(dev_work) + 4ull * (n + 1024);
    uint64_t *ctr = reinterpret_cast<uint64_t *>((wend - 8ull * (parts + 2)) & ~(uintptr_t)7);
    if (hipMemsetAsync(ctr, 0, sizeof(uint64_t), st) != hipSuccess)
        return WG_ERR_RUNTIME;
    if (dev_base && hipMemcpyAsync(ctr, dev_base, sizeof(uint64_t), hipMemcpyDeviceToDevice, st) != hipSuccess)
        return WG_ERR_RUNTIME;
    if (hipEventRecord(e.fork, st) != hipSuccess || hipStreamWaitEvent(e.side, e.fork, 0) != hipSuccess)
        return WG_ERR_RUNTIME;
    for (uint32_t k = 0; k < parts; k++) {
        const uint64_t i0 = n * k / parts, cnt = n * (k + 1) / parts - i0;
        rc = gso_split_launch(dev_in, dev_desc + i0, cnt, dev_out, dev_gso_res + i0, true, e.side,
                              synth ? &fit : nullptr);
        if (rc != WG_OK)
            return rc;
        if (hipEventRecord(e.split_done[k], e.side) != hipSuccess ||
            hipStreamWaitEvent(st, e.split_done[k], 0) != hipSuccess)
            return WG_ERR_RUNTIME;
        rc = encap_launch(dev_in, dev_out, dev_desc + i0, dev_gso_res + i0, cnt, key, receiver_index, counter0,
                          dev_msg_offset + i0, msg_cap, max_segments, max_segment_size, dev_msgs, dev_res + i0,
                          dev_work, k + 1 == parts ? dev_total : ctr + k + 1, 2u, ctr + k, st, t, synth);
        if (rc != WG_OK)
            return rc;
    }
    return WG_OK;
}

}  // namespace wg

extern "C" int wg_encap_batch(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                              wg_gso_result *dev_gso_res, const uint8_t key[32], uint32_t receiver_index,
                              uint64_t counter0, const uint64_t *dev_msg_offset, uint32_t msg_cap,
                              uint32_t max_segments, uint32_t max_segment_size, uint8_t *dev_msgs,
                              wg_encap_result *dev_res, uint32_t *dev_work, uint64_t *dev_total, void *stream) {
    return encap_batch_launch(dev_in, dev_desc, n, dev_out, dev_gso_res, key, receiver_index, counter0,
                              dev_msg_offset, msg_cap, max_segments, max_segment_size, dev_msgs, dev_res, dev_work,
                              dev_total, nullptr, static_cast<hipStream_t>(stream));
}
