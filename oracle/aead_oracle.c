/*
 * aead_oracle.c — CPU restatement of wireglider's data-message AEAD
 * (SURVEY §8 f4): Peer::encrypt / Peer::decrypt (reference proto/proto.cpp:
 * 496-523, 544-583) over libsodium's crypto_aead_chacha20poly1305_ietf
 * (libsodium is an un-vendored dependency, Makefile:107-109, no pinned
 * version; its published algorithm is RFC 8439: ChaCha20 §2.3-2.4,
 * Poly1305 §2.5, the AEAD construction §2.8).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the GPU kernels
 * (wireglider_amd/csrc/aead.hip) and bench.py's CPU baseline.  Pinned by the
 * RFC 8439 test vectors and by vectors generated with the system OpenSSL's
 * independent implementation (tests/golden/aead/).
 */
#include "orc_pin.h"
#include "csum_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static inline uint32_t ld_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline void st_le32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}
static inline void st_le64(uint8_t *p, uint64_t v) {
    st_le32(p, (uint32_t)v);
    st_le32(p + 4, (uint32_t)(v >> 32));
}

#define QR(a, b, c, d)                                                                                               \
    do {                                                                                                             \
        a += b; d ^= a; d = rotl32(d, 16);                                                                           \
        c += d; b ^= c; b = rotl32(b, 12);                                                                           \
        a += b; d ^= a; d = rotl32(d, 8);                                                                            \
        c += d; b ^= c; b = rotl32(b, 7);                                                                            \
    } while (0)

/* RFC 8439 §2.3: the ChaCha20 block function (key 32 B, 32-bit block
 * counter, nonce 12 B) -> 64 bytes of keystream. */
void orc_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865u;
    s[1] = 0x3320646eu;
    s[2] = 0x79622d32u;
    s[3] = 0x6b206574u;
    for (int i = 0; i < 8; i++) s[4 + i] = ld_le32(key + 4 * i);
    s[12] = counter;
    for (int i = 0; i < 3; i++) s[13 + i] = ld_le32(nonce + 4 * i);
    memcpy(x, s, sizeof x);
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]);
        QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]);
        QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]);
        QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);
        QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) st_le32(out + 4 * i, x[i] + s[i]);
}

/* RFC 8439 §2.4: out = in XOR keystream(counter, counter + 1, ...). */
void orc_chacha20_xor(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], const uint8_t *in,
                      uint8_t *out, size_t len) {
    uint8_t ks[64];
    for (size_t off = 0; off < len; off += 64, counter++) {
        orc_chacha20_block(key, counter, nonce, ks);
        const size_t n = len - off < 64 ? len - off : 64;
        for (size_t j = 0; j < n; j++) out[off + j] = in[off + j] ^ ks[j];
    }
}

/* RFC 8439 §2.5: Poly1305 over msg with the one-time key (r || s).  The
 * accumulator in five 26-bit limbs, products in 64 bits. */
void orc_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]) {
    /* r clamped (§2.5: r &= 0x0ffffffc0ffffffc0ffffffc0fffffff) */
    const uint32_t r0 = ld_le32(key) & 0x3ffffff;
    const uint32_t r1 = (ld_le32(key + 3) >> 2) & 0x3ffff03;
    const uint32_t r2 = (ld_le32(key + 6) >> 4) & 0x3ffc0ff;
    const uint32_t r3 = (ld_le32(key + 9) >> 6) & 0x3f03fff;
    const uint32_t r4 = (ld_le32(key + 12) >> 8) & 0x00fffff;
    const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0;
    for (size_t off = 0; off < len; off += 16) {
        uint8_t blk[17] = {0};
        const size_t n = len - off < 16 ? len - off : 16;
        memcpy(blk, msg + off, n);
        blk[n] = 1; /* §2.5: the 0x01 byte after the (possibly short) block */
        h0 += ld_le32(blk) & 0x3ffffff;
        h1 += (ld_le32(blk + 3) >> 2) & 0x3ffffff;
        h2 += (ld_le32(blk + 6) >> 4) & 0x3ffffff;
        h3 += (ld_le32(blk + 9) >> 6) & 0x3ffffff;
        h4 += (ld_le32(blk + 12) >> 8) | ((uint32_t)blk[16] << 24);
        const uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
        uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 + (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
        uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
        uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
        uint64_t d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 + (uint64_t)h3 * r1 + (uint64_t)h4 * r0;
        uint32_t c = (uint32_t)(d0 >> 26);
        h0 = (uint32_t)d0 & 0x3ffffff;
        d1 += c;
        c = (uint32_t)(d1 >> 26);
        h1 = (uint32_t)d1 & 0x3ffffff;
        d2 += c;
        c = (uint32_t)(d2 >> 26);
        h2 = (uint32_t)d2 & 0x3ffffff;
        d3 += c;
        c = (uint32_t)(d3 >> 26);
        h3 = (uint32_t)d3 & 0x3ffffff;
        d4 += c;
        c = (uint32_t)(d4 >> 26);
        h4 = (uint32_t)d4 & 0x3ffffff;
        h0 += c * 5;
        c = h0 >> 26;
        h0 &= 0x3ffffff;
        h1 += c;
    }
    /* full carry, then h mod 2^130 - 5 */
    uint32_t c = h1 >> 26;
    h1 &= 0x3ffffff;
    h2 += c;
    c = h2 >> 26;
    h2 &= 0x3ffffff;
    h3 += c;
    c = h3 >> 26;
    h3 &= 0x3ffffff;
    h4 += c;
    c = h4 >> 26;
    h4 &= 0x3ffffff;
    h0 += c * 5;
    c = h0 >> 26;
    h0 &= 0x3ffffff;
    h1 += c;
    uint32_t g0 = h0 + 5;
    c = g0 >> 26;
    g0 &= 0x3ffffff;
    uint32_t g1 = h1 + c;
    c = g1 >> 26;
    g1 &= 0x3ffffff;
    uint32_t g2 = h2 + c;
    c = g2 >> 26;
    g2 &= 0x3ffffff;
    uint32_t g3 = h3 + c;
    c = g3 >> 26;
    g3 &= 0x3ffffff;
    uint32_t g4 = h4 + c - (1u << 26);
    const uint32_t mask = (g4 >> 31) - 1u; /* all ones when h >= p: take g */
    h0 = (h0 & ~mask) | (g0 & mask);
    h1 = (h1 & ~mask) | (g1 & mask);
    h2 = (h2 & ~mask) | (g2 & mask);
    h3 = (h3 & ~mask) | (g3 & mask);
    h4 = (h4 & ~mask) | (g4 & mask);
    /* h + s mod 2^128 */
    const uint64_t f0 = ((h0) | (h1 << 26)) + (uint64_t)ld_le32(key + 16);
    const uint64_t f1 = ((h1 >> 6) | (h2 << 20)) + (uint64_t)ld_le32(key + 20) + (f0 >> 32);
    const uint64_t f2 = ((h2 >> 12) | (h3 << 14)) + (uint64_t)ld_le32(key + 24) + (f1 >> 32);
    const uint64_t f3 = ((h3 >> 18) | (h4 << 8)) + (uint64_t)ld_le32(key + 28) + (f2 >> 32);
    st_le32(tag, (uint32_t)f0);
    st_le32(tag + 4, (uint32_t)f1);
    st_le32(tag + 8, (uint32_t)f2);
    st_le32(tag + 12, (uint32_t)f3);
}

/* RFC 8439 §2.6 + §2.8: poly key = first 32 B of block 0; ct = pt XOR
 * keystream from block 1; tag = Poly1305(aad || pad16 || ct || pad16 ||
 * le64(aad_len) || le64(ct_len)). */
static void aead_tag(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                     const uint8_t *ct, size_t ct_len, uint8_t tag[16]) {
    uint8_t blk0[64];
    orc_chacha20_block(key, 0, nonce, blk0);
    const size_t pa = (aad_len + 15) & ~(size_t)15, pc = (ct_len + 15) & ~(size_t)15;
    const size_t mlen = pa + pc + 16;
    uint8_t stackbuf[2048];
    uint8_t *m = mlen <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(mlen);
    memset(m, 0, mlen);
    if (aad_len) memcpy(m, aad, aad_len);
    if (ct_len) memcpy(m + pa, ct, ct_len);
    st_le64(m + pa + pc, aad_len);
    st_le64(m + pa + pc + 8, ct_len);
    orc_poly1305(blk0, m, mlen, tag);
    if (m != stackbuf) free(m);
}

void orc_aead_encrypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                      const uint8_t *pt, size_t len, uint8_t *ct, uint8_t tag[16]) {
    orc_chacha20_xor(key, 1, nonce, pt, ct, len);
    aead_tag(key, nonce, aad, aad_len, ct, len, tag);
}

int orc_aead_decrypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                     const uint8_t *ct, size_t len, const uint8_t tag[16], uint8_t *pt) {
    uint8_t t[16];
    aead_tag(key, nonce, aad, aad_len, ct, len, t);
    uint32_t diff = 0;
    for (int i = 0; i < 16; i++) diff |= (uint32_t)(t[i] ^ tag[i]);
    if (diff) {
        memset(pt, 0, len); /* libsodium's decrypt zeroes the message on a bad tag */
        return -1;
    }
    orc_chacha20_xor(key, 1, nonce, ct, pt, len);
    return 0;
}

/* WireGuard nonce of a data message (proto/proto.cpp:505-506, 563-564):
 * 4 zero bytes, then the 64-bit counter little-endian. */
static void wg_nonce(uint64_t counter, uint8_t nonce[12]) {
    memset(nonce, 0, 4);
    st_le64(nonce + 4, counter);
}

/* Peer::encrypt (proto/proto.cpp:544-583) for one packet: out = DataHeader
 * {type 4, receiver_index, counter} || ChaCha20-Poly1305(pad16(pt)) || tag.
 * Returns the message size (16 + round_up(len, 16) + 16). */
size_t orc_wg_encrypt(const uint8_t key[32], uint32_t receiver_index, uint64_t counter, const uint8_t *pt, size_t len,
                      uint8_t *out) {
    const size_t padded = (len + 15) & ~(size_t)15;
    st_le32(out, 4u); /* MessageType::Data, message_type_and_zeroes */
    st_le32(out + 4, receiver_index);
    st_le64(out + 8, counter);
    uint8_t nonce[12];
    wg_nonce(counter, nonce);
    uint8_t *c = out + 16;
    if (len) memmove(c, pt, len);
    memset(c + len, 0, padded - len); /* :568-572 */
    orc_aead_encrypt(key, nonce, NULL, 0, c, padded, c, c + padded);
    return 16 + padded + 16;
}

/* Peer::decrypt (proto/proto.cpp:496-523) for one message: 0 and the
 * plaintext (msg_len - 32 bytes) in out, or -1 (rejected: shorter than the
 * header, counter past RejectAfterMessages, or a tag that does not verify —
 * out zeroed for a bad tag, untouched otherwise).  The replay window
 * (session->replay.try_advance, :519-520) is the caller's. */
int orc_wg_decrypt(const uint8_t key[32], const uint8_t *msg, size_t msg_len, uint8_t *out) {
    if (msg_len < 16)
        return -1;
    const uint64_t counter = (uint64_t)ld_le32(msg + 8) | ((uint64_t)ld_le32(msg + 12) << 32);
    if (counter > ORC_REJECT_AFTER_MESSAGES)
        return -1;
    if (msg_len < 32) /* crypto_aead_..._decrypt: clen < ABYTES */
        return -1;
    uint8_t nonce[12];
    wg_nonce(counter, nonce);
    const size_t clen = msg_len - 32;
    return orc_aead_decrypt(key, nonce, NULL, 0, msg + 16, clen, msg + 16 + clen, out);
}

/* Batches shaped like the reference's loops: encap encrypts every segment of
 * a PacketBatch into consecutive messages (worker/encap.cpp:136-141, counter
 * encrypt_nonce++ per call); decap decrypts every message of a GRO batch
 * (worker/decap_ref.cpp:78-86).  Uniform segments, the last may be short. */
void orc_wg_encrypt_batch(const uint8_t key[32], uint32_t receiver_index, uint64_t counter0, const uint8_t *in,
                          uint64_t total_len, uint32_t segment_size, uint8_t *out) {
    const uint64_t n = (total_len + segment_size - 1) / segment_size;
    const size_t stride = 16 + (((size_t)segment_size + 15) & ~(size_t)15) + 16;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t off = i * segment_size;
        const size_t len = total_len - off < segment_size ? (size_t)(total_len - off) : segment_size;
        orc_wg_encrypt(key, receiver_index, counter0 + i, in + off, len, out + i * stride);
    }
}

void orc_wg_decrypt_batch(const uint8_t key[32], const uint8_t *in, uint64_t total_len, uint32_t segment_size,
                          uint8_t *out, int8_t *status) {
    const uint64_t n = (total_len + segment_size - 1) / segment_size;
    const size_t ostride = segment_size > 32 ? segment_size - 32 : 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t off = i * segment_size;
        const size_t len = total_len - off < segment_size ? (size_t)(total_len - off) : segment_size;
        status[i] = (int8_t)orc_wg_decrypt(key, in + off, len, out + i * ostride);
    }
}

/* The two batch drivers over host threads (disjoint packet ranges): the CPU
 * baseline of bench.py's f4 workload. */
typedef struct {
    const uint8_t *key;
    uint32_t rx;
    uint64_t c0;
    const uint8_t *in;
    uint64_t total_len;
    uint32_t seg;
    uint8_t *out;
    int8_t *status;
    int dec;
    uint64_t lo, hi;
} aead_job;

static void *aead_job_run(void *arg) {
    aead_job *j = (aead_job *)arg;
    const size_t stride = 16 + (((size_t)j->seg + 15) & ~(size_t)15) + 16;
    const size_t ostride = j->seg > 32 ? j->seg - 32 : 0;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const uint64_t off = i * j->seg;
        const size_t len = j->total_len - off < j->seg ? (size_t)(j->total_len - off) : j->seg;
        if (j->dec)
            j->status[i] = (int8_t)orc_wg_decrypt(j->key, j->in + off, len, j->out + i * ostride);
        else
            orc_wg_encrypt(j->key, j->rx, j->c0 + i, j->in + off, len, j->out + i * stride);
    }
    return NULL;
}

static void aead_parallel(aead_job proto, uint64_t n, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if ((uint64_t)threads > n) threads = n ? (int)n : 1;
    pthread_t tid[256];
    aead_job jobs[256];
    const int spawn = threads > 1 || orc_pin_single();
    for (int t = 0; t < threads; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        if (!spawn)
            aead_job_run(&jobs[t]);
        else {
            orc_spawn(&tid[t], t, aead_job_run, &jobs[t]);
        }
    }
    if (spawn)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
}

void orc_wg_encrypt_batch_mt(const uint8_t key[32], uint32_t receiver_index, uint64_t counter0, const uint8_t *in,
                             uint64_t total_len, uint32_t segment_size, uint8_t *out, int threads) {
    aead_job j = {key, receiver_index, counter0, in, total_len, segment_size, out, NULL, 0, 0, 0};
    aead_parallel(j, (total_len + segment_size - 1) / segment_size, threads);
}

void orc_wg_decrypt_batch_mt(const uint8_t key[32], const uint8_t *in, uint64_t total_len, uint32_t segment_size,
                             uint8_t *out, int8_t *status, int threads) {
    aead_job j = {key, 0, 0, in, total_len, segment_size, out, status, 1, 0, 0};
    aead_parallel(j, (total_len + segment_size - 1) / segment_size, threads);
}
