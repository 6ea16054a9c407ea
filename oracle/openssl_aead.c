/*
 * openssl_aead.c — the data-message AEAD batch (Peer::encrypt per segment,
 * reference proto/proto.cpp:544-583, worker/encap.cpp:136-141) over the
 * system OpenSSL's EVP_chacha20_poly1305: an optimised, independent RFC 8439
 * implementation of the same class as the reference's libsodium (which is
 * not installed here).  TEST INFRASTRUCTURE ONLY: bench.py's f4 CPU
 * comparator and an extra checker in tests/; never part of the product.
 */
#include "orc_pin.h"
#include <openssl/crypto.h>
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

static void st_le32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

typedef struct {
    const uint8_t *key;
    uint32_t rx;
    uint64_t c0;
    const uint8_t *in;
    uint64_t total;
    uint32_t seg;
    uint8_t *out;
    uint64_t lo, hi;
    int rc;
    int slot;
} job;

/* Worker t of a call fetches the cipher in library context t: the default
 * context's provider objects are shared by every thread, and their reference
 * counts and locks made 16 workers on two sockets scale 3x over one (round
 * 6, profiles/r06_aead_bench.json).  The contexts are made once and kept
 * (loading a provider per call per worker cost a visible part of a call);
 * worker t of one call is the only user of slot t, and calls come one at a
 * time from bench.py's thread. */
#define OSS_SLOTS 256
static struct {
    OSSL_LIB_CTX *lc;
    EVP_CIPHER *c;
} g_slot[OSS_SLOTS];

static EVP_CIPHER *slot_cipher(int t) {
    if (t < 0 || t >= OSS_SLOTS)
        return NULL;
    if (!g_slot[t].c) {
        if (!g_slot[t].lc)
            g_slot[t].lc = OSSL_LIB_CTX_new();
        if (g_slot[t].lc)
            g_slot[t].c = EVP_CIPHER_fetch(g_slot[t].lc, "ChaCha20-Poly1305", NULL);
    }
    return g_slot[t].c;
}

static void *run(void *arg) {
    job *j = (job *)arg;
    EVP_CIPHER *cipher = slot_cipher(j->slot);
    EVP_CIPHER_CTX *ctx = EVP_CIPHER_CTX_new();
    const size_t stride = 16 + (((size_t)j->seg + 15) & ~(size_t)15) + 16;
    j->rc = ctx && cipher && EVP_EncryptInit_ex(ctx, cipher, NULL, j->key, NULL) == 1 ? 0 : -1;
    for (uint64_t i = j->lo; i < j->hi && !j->rc; i++) {
        const uint64_t off = i * j->seg;
        const size_t len = j->total - off < j->seg ? (size_t)(j->total - off) : j->seg;
        const size_t padded = (len + 15) & ~(size_t)15;
        const uint64_t counter = j->c0 + i;
        uint8_t *o = j->out + i * stride;
        st_le32(o, 4u);
        st_le32(o + 4, j->rx);
        st_le32(o + 8, (uint32_t)counter);
        st_le32(o + 12, (uint32_t)(counter >> 32));
        uint8_t nonce[12] = {0};
        memcpy(nonce + 4, o + 8, 8);
        memcpy(o + 16, j->in + off, len);
        memset(o + 16 + len, 0, padded - len);
        int n = 0;
        if (EVP_EncryptInit_ex(ctx, NULL, NULL, NULL, nonce) != 1 ||
            (padded && EVP_EncryptUpdate(ctx, o + 16, &n, o + 16, (int)padded) != 1) ||
            EVP_EncryptFinal_ex(ctx, o + 16 + padded, &n) != 1 ||
            EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, o + 16 + padded) != 1)
            j->rc = -1;
    }
    EVP_CIPHER_CTX_free(ctx);
    return NULL;
}

/* 0, or -1 if OpenSSL failed; same output layout as orc_wg_encrypt_batch. */
int oss_wg_encrypt_batch(const uint8_t key[32], uint32_t rx, uint64_t c0, const uint8_t *in, uint64_t total,
                         uint32_t seg, uint8_t *out, int threads) {
    const uint64_t n = (total + seg - 1) / seg;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if ((uint64_t)threads > n) threads = n ? (int)n : 1;
    const int spawn = threads > 1 || orc_pin_single();
    pthread_t tid[256];
    job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job){key, rx, c0, in, total, seg, out, n * (uint64_t)t / (uint64_t)threads,
                        n * (uint64_t)(t + 1) / (uint64_t)threads, 0, t};
        if (!spawn)
            run(&jobs[t]);
        else {
            orc_spawn(&tid[t], t, run, &jobs[t]);
        }
    }
    int rc = 0;
    for (int t = 0; t < threads; t++) {
        if (spawn)
            pthread_join(tid[t], NULL);
        rc |= jobs[t].rc;
    }
    return rc;
}

typedef struct {
    const uint8_t *key;
    const uint8_t *in;
    uint64_t total;
    uint32_t seg;
    uint8_t *out;
    int8_t *status;
    uint64_t lo, hi;
    int rc;
    int slot;
} djob;

/* Peer::decrypt (proto/proto.cpp:496-523) per message of a GRO batch: the
 * header / counter checks, then EVP decrypt with the tag; a failed message
 * gets status -1 (plaintext zeroed on a bad tag, as libsodium leaves it). */
static void *drun(void *arg) {
    djob *j = (djob *)arg;
    EVP_CIPHER *cipher = slot_cipher(j->slot);
    EVP_CIPHER_CTX *ctx = EVP_CIPHER_CTX_new();
    const uint64_t ostride = j->seg > 32 ? j->seg - 32 : 0;
    j->rc = ctx && cipher && EVP_DecryptInit_ex(ctx, cipher, NULL, j->key, NULL) == 1 ? 0 : -1;
    for (uint64_t i = j->lo; i < j->hi && !j->rc; i++) {
        const uint64_t off = i * j->seg;
        const size_t len = j->total - off < j->seg ? (size_t)(j->total - off) : j->seg;
        const uint8_t *m = j->in + off;
        uint8_t *o = j->out + i * ostride;
        uint64_t counter = 0;
        if (len >= 16)
            for (int b = 7; b >= 0; b--) counter = (counter << 8) | m[8 + b];
        if (len < 32 || counter > UINT64_MAX - (1ull << 13)) {
            j->status[i] = -1;
            continue;
        }
        uint8_t nonce[12] = {0};
        memcpy(nonce + 4, m + 8, 8);
        const size_t clen = len - 32;
        int n = 0, ok = EVP_DecryptInit_ex(ctx, NULL, NULL, NULL, nonce) == 1 &&
                        EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_SET_TAG, 16, (void *)(m + 16 + clen)) == 1 &&
                        (!clen || EVP_DecryptUpdate(ctx, o, &n, m + 16, (int)clen) == 1) &&
                        EVP_DecryptFinal_ex(ctx, o + n, &n) == 1;
        if (!ok)
            memset(o, 0, clen);
        j->status[i] = ok ? 0 : -1;
    }
    EVP_CIPHER_CTX_free(ctx);
    return NULL;
}

/* 0, or -1 if OpenSSL could not be set up; plaintext i at out + i * (seg - 32). */
int oss_wg_decrypt_batch(const uint8_t key[32], const uint8_t *in, uint64_t total, uint32_t seg, uint8_t *out,
                         int8_t *status, int threads) {
    const uint64_t n = (total + seg - 1) / seg;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    if ((uint64_t)threads > n) threads = n ? (int)n : 1;
    const int spawn = threads > 1 || orc_pin_single();
    pthread_t tid[256];
    djob jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (djob){key, in, total, seg, out, status, n * (uint64_t)t / (uint64_t)threads,
                         n * (uint64_t)(t + 1) / (uint64_t)threads, 0, t};
        if (!spawn)
            drun(&jobs[t]);
        else {
            orc_spawn(&tid[t], t, drun, &jobs[t]);
        }
    }
    int rc = 0;
    for (int t = 0; t < threads; t++) {
        if (spawn)
            pthread_join(tid[t], NULL);
        rc |= jobs[t].rc;
    }
    return rc;
}
