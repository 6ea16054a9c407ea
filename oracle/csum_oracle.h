/*
 * csum_oracle.h — CPU restatement of wireglider's checksum hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X engine in wireglider_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product path never does.
 *
 * Every function cites the reference (dinhngtu/wireglider @ 2024-11-01,
 * paths relative to the reference root) that it restates.  Pinning: the
 * byte-sum/fold arithmetic is pinned against golden vectors produced by
 * compiling the reference's own test oracle (tests/checksum_tests.hpp:11-48)
 * in place (see oracle/Makefile, tests/golden/).  calc_l4_checksum is pinned
 * against the reference's own checksum.cpp:8-36, compiled unchanged where it
 * lies against this repository's drop-in header (its only dependency that is
 * not in the image is the header's boost/fastcsum include; the drop-in header
 * stands in its place as a caller's would) — tests/golden/l4/.
 * worker/offload.cpp needs boost.endian and the un-vendored fastcsum library
 * directly, so it is unbuildable here; the GSO-split restatement is pinned by
 * the reference tests' own assertions (tests/test-offload.cpp:21-171 segment
 * geometry, tests/test-checksum.cpp:53-82 verify-to-zero) and by an
 * independent RFC 768/793 textbook implementation in tests/.  See DESIGN.md
 * §3.
 */
#ifndef WG_CSUM_ORACLE_H
#define WG_CSUM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* tests/checksum_tests.hpp:11-34 (checksum_ref1, the snabb scalar oracle). */
uint16_t orc_checksum_ref1(const uint8_t *data, size_t size);

/* include/netio/checksum.hpp:79-100 — the dynamic-extent nofold sum
 * (fastcsum_nofold_generic64 contract): 64-bit one's-complement accumulation
 * of the native (LE) words of b, pairing relative to b[0], odd tail byte
 * as the low byte, added to `initial` with end-around carry. */
uint64_t orc_nofold(const uint8_t *b, size_t n, uint64_t initial);
/* The two arms of orc_nofold's dispatch (n >= 256 and AVX2: the vector arm,
 * like checksum.hpp:88-91's vec256 branch): the scalar arm on its own, and
 * whether this CPU takes the vector arm. */
uint64_t orc_nofold_scalar(const uint8_t *b, size_t n, uint64_t initial);
int orc_have_avx2(void);

/* fastcsum_fold_complement contract (include/netio/checksum.hpp:127,148):
 * fold 64 -> 16 bits with end-around carry, then one's complement. */
uint16_t orc_fold_complement(uint64_t sum);

/* include/netio/checksum.hpp:146-149 */
uint16_t orc_checksum(const uint8_t *b, size_t n, uint64_t initial);

/* include/netio/checksum.hpp:102-116 (addresses as dynamic spans; the
 * fixed-extent N=4/16 specialisations at :30-58 give the same value). */
uint64_t orc_pseudo_header_nofold(uint8_t proto, const uint8_t *src, const uint8_t *dst,
                                  size_t addrlen, uint16_t l4len);

/* include/netio/checksum.hpp:120-144 */
uint16_t orc_pseudo_header_checksum(uint8_t proto, const uint8_t *src, const uint8_t *dst,
                                    size_t addrlen, uint16_t l4len);

/* checksum.cpp:8-36.  Preconditions as in the reference (unchecked there):
 * len >= 20 (v4) / 40 (v6) and len >= csum_start.  The oracle defines the
 * out-of-contract cases the same way the GPU engine does: bytes past `len`
 * are never read and count as absent. */
uint16_t orc_calc_l4_checksum(const uint8_t *pkt, size_t len, int isv6, int istcp,
                              uint16_t csum_start);

/* Batched drivers (threads > 1 splits the packet range into contiguous
 * slices, one std::thread-equivalent pthread per slice). */

/* PacketBatch layout, include/worker/offload.hpp:19-29 and
 * include/util/packets.hpp:11-47: packet i = base[i*S, min((i+1)*S, total)). */
void orc_l4_uniform(const uint8_t *base, uint64_t total_len, uint32_t segment_size,
                    uint16_t csum_start, uint32_t flags, uint16_t *out, int threads);

/* Descriptor batch (same layout as wg_pkt_desc in include/wireglider_amd.h). */
typedef struct orc_pkt_desc {
    uint64_t offset;
    uint32_t len;
    uint16_t csum_start;
    uint8_t flags; /* bit0 = v6, bit1 = tcp */
    uint8_t reserved;
} orc_pkt_desc;

void orc_l4_desc(const uint8_t *base, const orc_pkt_desc *desc, uint64_t n, uint16_t *out,
                 int threads);

/* checksum(span, 0) per packet of a descriptor batch (IPv4 header checksum
 * use: worker/offload.cpp:71,184, worker/evaluator.cpp:28). */
void orc_checksum_desc(const uint8_t *base, const orc_pkt_desc *desc, uint64_t n,
                       uint16_t *out, int threads);

/* worker/offload.cpp:46-216 — do_tun_gso_split.  `in` is modified in place
 * exactly as the reference modifies it (ip_sum and the L4 checksum field of
 * the prefix are zeroed; GSO_NONE+NEEDS_CSUM fills checksums in place).
 * vnet fields are the native-order virtio_net_hdr members.  Returns 0 on
 * success, negative on a case the reference does not define
 * (-1: gso_size == 0 with payload -> the reference loops forever;
 *  -2: output capacity below the reference's reserve_size assert). */
typedef struct orc_gso_result {
    uint64_t out_len;      /* PacketBatch.data.size() */
    uint64_t segment_size; /* PacketBatch.segment_size */
    uint16_t hdr_len;      /* vnethdr.hdr_len after the call */
    uint8_t isv6;
    uint8_t ecn;
    uint8_t passthrough;   /* 1: data == inbuf (returned unsegmented) */
    uint8_t pad[3];
} orc_gso_result;

typedef struct orc_vnet_hdr {
    uint8_t flags;
    uint8_t gso_type;
    uint16_t hdr_len;
    uint16_t gso_size;
    uint16_t csum_start;
    uint16_t csum_offset;
} orc_vnet_hdr;

int orc_gso_split(uint8_t *in, size_t in_len, orc_vnet_hdr *vnet, uint8_t *out, size_t out_cap,
                  orc_gso_result *res);

/* A batch of super-buffers in the engine's 40-byte descriptor layout
 * (wg_gso_desc): do_tun_gso_split per descriptor on `threads` pthreads
 * (disjoint super-buffer ranges), status per descriptor.  The CPU baseline
 * of BASELINE config 3. */
typedef struct orc_gso_desc {
    uint64_t in_offset, out_offset;
    uint32_t in_len, out_cap;
    orc_vnet_hdr vnet;
    uint16_t reserved[3];
} orc_gso_desc;
void orc_gso_split_desc(uint8_t *in_base, const orc_gso_desc *desc, uint64_t n, uint8_t *out_base, int8_t *status,
                        int threads);

/* Decap verify gates: the checksum-related decisions of
 * evaluate_packet (include/worker/evaluator.hpp:112-149) with fill_fk_ip4 /
 * fill_fk_ip6 (worker/evaluator.cpp:14-58) and the checksum gates of
 * fill_fk_tcp / fill_fk_udp (include/worker/evaluator.hpp:59-65,89-94).
 * The IP family is the version nibble (the decap caller's choice).
 * Verdict bits: */
#define ORC_V_IP_OK 0x01  /* size bounds + fill_fk_ip4/ip6 pass (v4 header checksum == 0) */
#define ORC_V_L4_OK 0x02  /* TCP/UDP length floor and calc_l4_checksum == 0 */
#define ORC_V_TCP 0x04
#define ORC_V_UDP 0x08
#define ORC_V_V6 0x10
uint8_t orc_verify(const uint8_t *pkt, size_t len, uint16_t *l4_out);
void orc_verify_desc(const uint8_t *base, const orc_pkt_desc *desc, uint64_t n, uint8_t *verdict, uint16_t *l4,
                     int threads);

/* GRO finalize: PacketRefBatch::finalize
 * (include/worker/flowkey_ref.hpp:82-117) / OwnedPacketBatch::finalize
 * (include/worker/flowkey_own.hpp:83-115) on one coalesced flow's header
 * buffer, in place.  The NEEDS_CSUM seed is pseudo_header_checksum over the
 * header's source/destination ADDRESSES (complemented fold, as the reference
 * stores it); the reference's call binds the TAddress overload and sums the
 * std::span objects instead, which is pointer-dependent and
 * not reproduced.  Returns 0, or -3 if the geometry is out of contract. */
int orc_gro_finalize(uint8_t *hdr, size_t hdr_len, uint16_t csum_start, uint16_t csum_offset, int isv6,
                     int istcp, uint64_t payload_bytes);

/* Batched form over the wg_gro_desc layout (include/wireglider_amd.h);
 * status written back into each descriptor. */
typedef struct orc_gro_desc {
    uint64_t hdr_offset;
    uint64_t payload_bytes;
    uint16_t hdr_len;
    uint16_t csum_start;
    uint16_t csum_offset;
    uint8_t flags; /* bit0 = v6, bit1 = tcp */
    int8_t status;
} orc_gro_desc;

void orc_gro_finalize_desc(uint8_t *base, orc_gro_desc *desc, uint64_t n, int threads);

/* Timing helper for the cpu_baseline: runs orc_l4_uniform `reps` times and
 * returns elapsed seconds (monotonic clock). */
double orc_time_l4_uniform(const uint8_t *base, uint64_t total_len, uint32_t segment_size,
                           uint16_t csum_start, uint32_t flags, uint16_t *out, int threads,
                           int reps);

/* The CPU baseline's placement evidence: per-worker busy nanoseconds and
 * calls of the persistent pool since the last reset (returns the worker
 * count), and a read-only probe over [base, base + nbytes) (4-KiB blocks, 64-bit
 * word sums) on the same pinned workers. */
void orc_pool_stats_reset(void);
int orc_pool_stats(uint64_t *busy_ns, uint64_t *calls, int max);
uint64_t orc_read_probe(const uint8_t *base, uint64_t nbytes, int threads);
int orc_numa_retouch(uint8_t *buf, uint64_t nbytes, int threads);

#ifdef __cplusplus
}
#endif

/* ---- data-message AEAD, oracle/aead_oracle.c ---------- */
/* RejectAfterMessages (include/proto/proto.hpp:36) */
#define ORC_REJECT_AFTER_MESSAGES (UINT64_MAX - (1ull << 13))
void orc_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]);
void orc_chacha20_xor(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], const uint8_t *in,
                      uint8_t *out, size_t len);
void orc_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]);
void orc_aead_encrypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                      const uint8_t *pt, size_t len, uint8_t *ct, uint8_t tag[16]);
int orc_aead_decrypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                     const uint8_t *ct, size_t len, const uint8_t tag[16], uint8_t *pt);
size_t orc_wg_encrypt(const uint8_t key[32], uint32_t receiver_index, uint64_t counter, const uint8_t *pt, size_t len,
                      uint8_t *out);
int orc_wg_decrypt(const uint8_t key[32], const uint8_t *msg, size_t msg_len, uint8_t *out);
void orc_wg_encrypt_batch(const uint8_t key[32], uint32_t receiver_index, uint64_t counter0, const uint8_t *in,
                          uint64_t total_len, uint32_t segment_size, uint8_t *out);
void orc_wg_decrypt_batch(const uint8_t key[32], const uint8_t *in, uint64_t total_len, uint32_t segment_size,
                          uint8_t *out, int8_t *status);

void orc_wg_encrypt_batch_mt(const uint8_t key[32], uint32_t receiver_index, uint64_t counter0, const uint8_t *in,
                             uint64_t total_len, uint32_t segment_size, uint8_t *out, int threads);
void orc_wg_decrypt_batch_mt(const uint8_t key[32], const uint8_t *in, uint64_t total_len, uint32_t segment_size,
                             uint8_t *out, int8_t *status, int threads);

#endif
