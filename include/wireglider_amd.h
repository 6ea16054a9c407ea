/*
 * wireglider_amd.h — C ABI of the MI355X (gfx950) Internet-checksum engine.
 *
 * This is the drop-in boundary behind wireglider's checksum hot path
 * (reference dinhngtu/wireglider @ 2024-11-01; citations relative to its
 * root).  Every entry point takes plain pointers and sizes; `stream` is a
 * hipStream_t passed as void* (NULL = the legacy default stream).  All
 * packet/descriptor/output pointers are DEVICE pointers (hipMalloc'd, or
 * host memory registered/mapped for the device) unless a name says _host.
 *
 * Ownership follows the reference: every buffer is borrowed
 * from the caller; nothing is allocated per call; entry points are
 * reentrant and may be called from several host threads at once, on their
 * own streams, on hipStreamPerThread, or on the shared NULL stream
 * (tests/test_mt_batch.py: 1-16 threads, every result against the oracle).
 * No process-wide lock is taken per launch.  Launches are asynchronous on
 * `stream`.
 *
 * Error convention: the reference has no error channel (checksum.cpp:8-36
 * returns the checksum only).  Here a negative return is a launch/argument
 * failure and never changes checksum semantics; 0 = launched.
 *
 * Byte order: checksums are returned in native (little-endian) order, as
 * the reference does, so callers memcpy them straight into headers
 * (worker/offload.cpp:72-77,185-186,203-204).
 */
#ifndef WIREGLIDER_AMD_H
#define WIREGLIDER_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history: 1 = rounds 1-3; 2 = round 4's knob set (removed knob names
 * and values are WG_ERR_INVALID from wg_tune_set, their WG_* environment
 * overrides ignored). */
#define WG_ABI_VERSION 2

/* Return codes. */
#define WG_OK 0
#define WG_ERR_INVALID (-1)  /* bad geometry / null pointer / misaligned descriptor array */
#define WG_ERR_NODEV (-2)    /* no HIP device visible */
#define WG_ERR_LAUNCH (-3)   /* hipLaunchKernel / hipGetLastError failed */
#define WG_ERR_RUNTIME (-4)  /* other HIP runtime failure (alloc, copy, sync) */

/* Packet flags (descriptor `flags`, uniform-batch `flags`). */
#define WG_PKT_V6 0x01u  /* IPv6: addresses at byte 8 / 24, 16 B each; else IPv4 at 12 / 16, 4 B */
#define WG_PKT_TCP 0x02u /* pseudo-header proto 6; else 17 (UDP) */

/*
 * One packet of a variable-length batch.  16 bytes, 16-byte aligned array.
 * The packet is dev_base[offset, offset + len), len < 2^32 - 32 (the
 * kernels compute a packet's geometry in 32-bit offsets from its start).
 * Replaces the per-call (span, isv6, istcp, csum_start) arguments of
 * calc_l4_checksum.
 */
typedef struct wg_pkt_desc {
    uint64_t offset;
    uint32_t len;
    uint16_t csum_start;
    uint8_t flags; /* WG_PKT_* */
    uint8_t reserved;
} wg_pkt_desc;

/* ------------------------------------------------------------------------
 * L4 checksum over a packet batch.
 *
 * Per packet this computes exactly
 *     wireglider::calc_l4_checksum(pkt, isv6, istcp, csum_start)
 * (checksum.cpp:8-36): ~fold16(pseudo-header(proto, src, dst,
 * (uint16_t)(len - csum_start)) + sum of LE words of pkt[csum_start:]),
 * with word pairing relative to csum_start and the odd tail byte as the low
 * byte (include/netio/checksum.hpp:30-149).  Generate mode: the caller has
 * zeroed the checksum field, the result is the value to store
 * (worker/offload.cpp:64,149,202-204).  Verify mode: the field holds the
 * received checksum and the result is 0 iff valid
 * (include/worker/evaluator.hpp:64,93).
 *
 * Out-of-contract packets (len < 20/40 or len < csum_start; undefined in
 * the reference) are computed with the missing bytes treated as absent;
 * nothing outside a packet is ever read.
 * ---------------------------------------------------------------------- */

/*
 * Uniform batch = the reference's PacketBatch (include/worker/offload.hpp:19-29,
 * include/util/packets.hpp:11-47): packet i is
 * dev_base[i*segment_size, min((i+1)*segment_size, total_len)), i.e.
 * nr_segments() = ceil(total_len / segment_size) packets, the last one may be
 * short.  dev_out receives nr_segments() uint16 results.
 * Replaces: calc_l4_checksum (include/netio/checksum.hpp:151, checksum.cpp:8)
 * called once per segment by worker/offload.cpp:202 and
 * include/worker/evaluator.hpp:64,93.
 */
int wg_l4csum_uniform(const uint8_t *dev_base, uint64_t total_len, uint32_t segment_size,
                      uint16_t csum_start, uint32_t flags, uint16_t *dev_out, void *stream);

/*
 * Variable batch: n descriptors (dev_desc 16-byte aligned), one result each.
 * Replaces the same per-packet calc_l4_checksum calls for batches whose
 * packets differ in length / family / protocol (decap GRO batches,
 * worker/decap_ref.cpp:53-89 -> include/worker/evaluator.hpp:112-149).
 */
int wg_l4csum_desc(const uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n,
                   uint16_t *dev_out, void *stream);

/*
 * checksum(span, 0) per descriptor (flags and csum_start ignored): the
 * IPv4 header checksum callers, worker/offload.cpp:71,184,
 * worker/evaluator.cpp:28, include/worker/flowkey_ref.hpp:108.
 * Replaces: wireglider::checksum (include/netio/checksum.hpp:146-149).
 */
int wg_checksum_desc(const uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n,
                     uint16_t *dev_out, void *stream);

/* ------------------------------------------------------------------------
 * Decap verify gates, batched: per packet the checksum
 * decisions of evaluate_packet (include/worker/evaluator.hpp:112-149):
 * size bounds (20/40 <= len <= 65535), fill_fk_ip4 (worker/evaluator.cpp:14-40:
 * ihl == 5, len == ip_len, (ip_off & ~IP_DF) == 0, IPv4 header checksum == 0)
 * or fill_fk_ip6 (:42-58: len - 40 == ip6_plen), then for TCP len - ihs > 20
 * and for UDP len - ihs > 8 (include/worker/evaluator.hpp:61,91) and
 * calc_l4_checksum(pkt, isv6, istcp, ihs) == 0 (:64,93).  The family is the
 * version nibble; descriptor csum_start/flags are ignored.  GRO policy after
 * these gates (TCP doff/flag rules, ECN, has_uso) stays with the caller.
 * dev_verdict[i] = WG_VERDICT_* bits; dev_l4 (nullable) = the L4 checksum
 * result when one was computed, else 0.
 * ---------------------------------------------------------------------- */
#define WG_VERDICT_IP_OK 0x01u /* size bounds + IP header gates pass */
#define WG_VERDICT_L4_OK 0x02u /* TCP/UDP length floor and L4 checksum == 0 */
#define WG_VERDICT_TCP 0x04u
#define WG_VERDICT_UDP 0x08u
#define WG_VERDICT_V6 0x10u
int wg_verify_desc(const uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n, uint8_t *dev_verdict,
                   uint16_t *dev_l4, void *stream);

/* The same gates over a uniform PacketBatch (include/worker/offload.hpp:19-29):
 * packet i = dev_base[i*segment_size, min((i+1)*segment_size, total_len)),
 * no descriptors.  This is the decap worker's own shape: a UDP GRO batch has
 * one segment size (worker/decap.cpp:145-151), and its plaintexts lie at
 * stride segment_size - 32 with that (padded) length (worker/decap_ref.cpp:
 * 78-86).  The kernel follows the segment size: <= 64 B (TCP ACK-sized
 * batches) a lane per packet, longer a wave per packet. */
int wg_verify_uniform(const uint8_t *dev_base, uint64_t total_len, uint32_t segment_size, uint8_t *dev_verdict,
                      uint16_t *dev_l4, void *stream);

/* ------------------------------------------------------------------------
 * GSO split (TSO/USO segmentation + per-segment checksum fixup), batched.
 * Per super-buffer this is worker_impl::do_tun_gso_split
 * (worker/offload.cpp:46-216) bit for bit, including its quirks:
 *   - gso_type with VIRTIO_NET_HDR_GSO_ECN set is segmented as TCP for the
 *     header length but fixed up / checksummed as UDP (:55 vs :151);
 *   - a UDP checksum that computes to 0 is stored as 0 (:202-204);
 *   - the input prefix's ip_sum and L4 checksum field are zeroed in place
 *     (:145-149), and GSO_NONE + NEEDS_CSUM packets are checksummed in
 *     place (:56-78).
 * Contract: in_len <= 65,535 for super-buffers that are split or checksummed
 * in place (tun delivers at most 64 KiB; the IP length fields are 16-bit);
 * longer ones get status -3 and are left untouched.
 * ---------------------------------------------------------------------- */

/* Native-order mirror of struct virtio_net_hdr (linux/virtio_net.h). */
typedef struct wg_vnet_hdr {
    uint8_t flags;    /* VIRTIO_NET_HDR_F_NEEDS_CSUM = 1 */
    uint8_t gso_type; /* NONE 0, TCPV4 1, TCPV6 4, UDP_L4 5, | ECN 0x80 */
    uint16_t hdr_len;
    uint16_t gso_size;
    uint16_t csum_start;
    uint16_t csum_offset;
} wg_vnet_hdr;

typedef struct wg_gso_desc {
    uint64_t in_offset;  /* super-buffer (IP header onwards) = dev_in[in_offset, +in_len) */
    uint64_t out_offset; /* its segments are written to dev_out[out_offset, +out_cap) */
    uint32_t in_len;
    uint32_t out_cap;
    wg_vnet_hdr vnet;
    uint16_t reserved[3];
} wg_gso_desc; /* 40 bytes */

typedef struct wg_gso_result {
    uint64_t out_len;      /* PacketBatch.data.size() (== in_len on passthrough) */
    uint32_t segment_size; /* PacketBatch.segment_size */
    uint16_t hdr_len;      /* vnethdr.hdr_len after the call (:110,:114) */
    uint8_t isv6;
    uint8_t ecn;
    int8_t status;       /* 0 ok; -1 gso_size 0 with payload; -2 out_cap < reserve_size; -3 out of contract */
    uint8_t passthrough; /* 1: batch is the (possibly in-place checksummed) input */
    uint8_t pad[6];
} wg_gso_result; /* 24 bytes */

/* Segment n super-buffers.  dev_desc / dev_res are device arrays of n. */
int wg_gso_split(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                 wg_gso_result *dev_res, void *stream);

/* ------------------------------------------------------------------------
 * GRO finalize, batched, in place on each coalesced flow's
 * header buffer: PacketRefBatch::finalize (include/worker/flowkey_ref.hpp:82-117)
 * — UDP len / IPv6 plen / IPv4 total length, IPv4 header checksum, and the
 * NEEDS_CSUM seed pseudo_header_checksum(proto, src, dst, l4len) (the
 * complemented fold, as the reference stores it) over the header's
 * ADDRESSES.  The reference's call sums the std::span objects instead
 * (pointer-dependent) and is not reproduced.
 * status (out): 0, or -3 when the header geometry is out of contract.
 * Writes stay inside each flow's header: the changed fields, plus (IPv4) the
 * unchanged bytes of header bytes [0, 16) rewritten with their own values
 * (the fields go out as two wide stores).
 * ---------------------------------------------------------------------- */
typedef struct wg_gro_desc {
    uint64_t hdr_offset;    /* header buffer = dev_hdrs[hdr_offset, + hdr_len) */
    uint64_t payload_bytes; /* size_bytes() of the coalesced batch */
    uint16_t hdr_len;
    uint16_t csum_start;
    uint16_t csum_offset;
    uint8_t flags; /* WG_PKT_V6 | WG_PKT_TCP */
    int8_t status; /* out */
} wg_gro_desc;      /* 24 bytes */

int wg_gro_finalize(uint8_t *dev_hdrs, wg_gro_desc *dev_desc, uint64_t n, void *stream);

/* ------------------------------------------------------------------------
 * Data-message AEAD, batched: Peer::encrypt / Peer::decrypt
 * (proto/proto.cpp:544-583, 496-523) over crypto_aead_chacha20poly1305_ietf
 * (RFC 8439) for the batches the workers build.  `key` is the session's
 * 32-byte key in HOST memory (passed by value to the kernel).
 *
 * wg_aead_encrypt_batch: every segment of a PacketBatch (dev_in, total_len,
 * segment_size <= 65535; the last segment may be short), as
 * worker/encap.cpp:136-141 calls Peer::encrypt for each: message i =
 * DataHeader {4, receiver_index, counter0 + i} (little-endian) ||
 * ChaCha20-Poly1305(key, nonce = 0^4 || le64(counter), no AAD, plaintext
 * zero-padded to 16) || 16-B tag, written at dev_out + i * stride with
 * stride = 16 + round_up(segment_size, 16) + 16
 * (Peer::expected_encrypt_size, include/proto/proto.hpp:266-269); dev_out
 * 16-byte aligned.  dev_status (nullable): -1 for a packet whose counter is
 * >= RejectAfterMessages (EncryptError::NoSession; nothing written), else 0.
 *
 * wg_aead_decrypt_batch: every message of a batch of equal-size data
 * messages (a UDP GRO batch, worker/decap_ref.cpp:78-86; the last may be
 * short): plaintext i (message length - 32 bytes, the padding included, as
 * the reference's outsize) at dev_out + i * (segment_size - 32);
 * dev_status[i] = 0, or -1 when Peer::decrypt rejects it: shorter than the
 * 16-B header or than header + tag, counter > RejectAfterMessages (plaintext
 * left untouched), or a tag that does not verify (plaintext zeroed, as
 * libsodium does).  The replay window (session->replay.try_advance,
 * proto.cpp:519-520) stays with the caller: it is a sequential per-session
 * state update over the accepted counters.
 * ---------------------------------------------------------------------- */
int wg_aead_encrypt_batch(const uint8_t *dev_in, uint64_t total_len, uint32_t segment_size, const uint8_t key[32],
                          uint32_t receiver_index, uint64_t counter0, uint8_t *dev_out, int8_t *dev_status,
                          void *stream);
int wg_aead_decrypt_batch(const uint8_t *dev_in, uint64_t total_len, uint32_t segment_size, const uint8_t key[32],
                          uint8_t *dev_out, int8_t *dev_status, void *stream);

/* wg_aead_decrypt_verify_batch: wg_aead_decrypt_batch, and in the same pass
 * the decap verify gates of wg_verify_desc over every plaintext as it is
 * produced (Peer::decrypt then evaluate_packet, worker/decap_ref.cpp:81-86,
 * include/worker/evaluator.hpp:112-149), over the plaintext's libsodium
 * length (the padded one, as the reference evaluates it): dev_verdict[i] =
 * WG_VERDICT_* bits and dev_l4[i] = the L4 checksum result, exactly
 * wg_verify_desc's on the plaintext; 0 / 0 for messages with status -1.
 * The plaintext is read from HBM zero times more than decryption needs. */
int wg_aead_decrypt_verify_batch(const uint8_t *dev_in, uint64_t total_len, uint32_t segment_size,
                                 const uint8_t key[32], uint8_t *dev_out, int8_t *dev_status, uint8_t *dev_verdict,
                                 uint16_t *dev_l4, void *stream);

/* Encap: every segment of wg_gso_split's PacketBatches encrypted for ONE peer,
 * super-buffer by super-buffer and segment by segment, with the counters the
 * reference's encap worker would use (worker/encap.cpp:136-141: Peer::encrypt
 * per segment, encrypt_nonce++): counter0 for super-buffer 0's first
 * segment, then consecutive over every message.  No host round trip: the
 * segment counts come from dev_gso_res on the device.
 *   dev_in / dev_seg / dev_desc / dev_gso_res: wg_gso_split's dev_in, dev_out,
 *     dev_desc and dev_res (passthrough batches are read from dev_in);
 *   dev_msg_offset[i]: where super-buffer i's messages go in dev_msgs
 *     (16-B aligned), msg_cap bytes available there (the caller owns this
 *     extent: nothing here can check it on the device); its messages follow each
 *     other at stride 32 + pad16(segment_size), the last one shorter — the
 *     reference's outbuf layout (worker/encap.cpp:131-141,161-168);
 *   max_segments / max_segment_size: bounds over the batch (super-buffers
 *     past them, or whose messages exceed msg_cap, get nmsg 0);
 *   dev_res[i]: counter0, nmsg (0 for GSO errors), msg_bytes = the bytes of
 *     the messages written, i.e. up to the first refused counter (the
 *     reference's outbuf advances over accepted messages only,
 *     worker/encap.cpp:138-140, while encrypt_nonce counts every segment);
 *   dev_work: 4 * (n + 1024) bytes of scratch; dev_total (nullable): messages
 *     in all, i.e. counter0 + *dev_total is the peer's next encrypt_nonce
 *     (0 for n = 0, written on the stream like every other output).
 * n <= 2^20 super-buffers per call and max_segments * n < 2^32 (the counter
 * scan indexes messages in 32 bits; larger calls are WG_ERR_INVALID, never a
 * repeated nonce).  A message whose counter reaches RejectAfterMessages is
 * not written (the reference's encrypt refuses it). */
typedef struct wg_encap_result {
    uint64_t counter0;
    uint32_t nmsg;
    uint32_t msg_bytes;
} wg_encap_result; /* 16 bytes */

int wg_encap_encrypt(const uint8_t *dev_in, const uint8_t *dev_seg, const wg_gso_desc *dev_desc,
                     const wg_gso_result *dev_gso_res, uint64_t n, const uint8_t key[32], uint32_t receiver_index,
                     uint64_t counter0, const uint64_t *dev_msg_offset, uint32_t msg_cap, uint32_t max_segments,
                     uint32_t max_segment_size, uint8_t *dev_msgs, wg_encap_result *dev_res, uint32_t *dev_work,
                     uint64_t *dev_total, void *stream);

/* The whole encap step in one call: wg_gso_split(dev_in, dev_desc, n,
 * dev_out, dev_gso_res) then wg_encap_encrypt over its output, except that
 * the split writes only each segment's HEADER into dev_out (bytes
 * [0, hdr_len) of every segment slot, checksums as always) and the AEAD reads
 * each segment's payload straight from dev_in — the segment payload copy is
 * never materialised.  On return dev_gso_res, dev_res, dev_msgs, dev_total
 * and dev_in's zeroed prefix fields are exactly what the two calls give;
 * dev_out holds the segment headers only.  dev_out must be sized as for
 * wg_gso_split (the headers sit at the segments' offsets).  Arguments and
 * bounds as for the two calls.
 * max_segment_size also picks the AEAD kernel: for 129 <= max_segment_size
 * <= 6,080 the messages are staged in LDS and (knob encap_synth) the AEAD
 * builds the segment headers itself; outside that range every header comes
 * from the headers-only split and lanes store their own blocks — the same
 * bytes, about 12 % slower on config 3's super-buffers.
 * Pass the batch's real largest segment size, not a jumbo bound. */
int wg_encap_batch(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                   wg_gso_result *dev_gso_res, const uint8_t key[32], uint32_t receiver_index, uint64_t counter0,
                   const uint64_t *dev_msg_offset, uint32_t msg_cap, uint32_t max_segments, uint32_t max_segment_size,
                   uint8_t *dev_msgs, wg_encap_result *dev_res, uint32_t *dev_work, uint64_t *dev_total,
                   void *stream);

/* ------------------------------------------------------------------------
 * Host-memory path: the batch starts and ends in host memory
 * (tun read buffers, worker/encap.cpp:74-97; UDP GRO recvmsg buffers,
 * worker/decap.cpp:16-28,90-156).  Synchronous.  The batch is cut into
 * chunks of whole segments (~host_chunk_mb MiB) that flow through a per-thread pipeline of
 * three device slots on three streams (H2D, kernels, D2H): chunk k+1's
 * hipMemcpyAsync H2D runs under chunk k's kernel and chunk k-1's result copy;
 * results gather in a pinned buffer and reach host_out once at the end.
 * host_base may be pageable (the HIP runtime stages it) or pinned
 * (wg_host_alloc: DMA straight from it).  The
 * workspace (streams, events, device slots, pinned results) is per calling
 * thread and per its current device, reused across calls, and freed at thread
 * exit or by wg_host_release().  An error after the first copy was queued
 * drains the streams before returning: no DMA touches the caller's buffers
 * after any host-path call returns.  Rate: PCIe-bound,
 * never the metric.
 * ---------------------------------------------------------------------- */
int wg_l4csum_uniform_host(const uint8_t *host_base, uint64_t total_len, uint32_t segment_size,
                           uint16_t csum_start, uint32_t flags, uint16_t *host_out);

/* The decap worker's step from a UDP GRO batch in host memory
 * (worker/decap.cpp:90-156 recvmsg -> worker/decap_ref.cpp:53-89 decrypt +
 * evaluate_packet): every message of the batch (equal-size data messages at
 * stride segment_size, the last may be short) decrypted, and — when
 * host_verdict / host_l4 are given (both or neither) — run through the f1
 * verify gates in the same pass, exactly as wg_aead_decrypt_verify_batch
 * (wg_aead_decrypt_batch without them).  Plaintext i lands at host_plain +
 * i * (segment_size - 32) (n * (segment_size - 32) bytes); host_status[i],
 * host_verdict[i], host_l4[i] per message.  Bytes of host_plain outside an
 * accepted message's plaintext (rejected messages, the tail of a short last
 * message's slot) are unspecified.  Pipelined like wg_l4csum_uniform_host
 * (chunks of ~host_chunk_mb MiB of messages, H2D / kernel / D2H on three
 * streams); synchronous; pinned buffers (wg_host_alloc) keep the copies
 * asynchronous. */
int wg_decap_host(const uint8_t *host_msgs, uint64_t total_len, uint32_t segment_size, const uint8_t key[32],
                  uint8_t *host_plain, int8_t *host_status, uint8_t *host_verdict, uint16_t *host_l4);

/* The encap worker's step from tun reads in host memory (worker/encap.cpp:
 * 22-170: do_tun_recv -> do_tun_gso_split -> Peer::encrypt per segment):
 * host_desc[i] (wg_gso_desc) describes tun read i at host_in +
 * in_offset (reads in input order, not overlapping; out_cap = the split's
 * output capacity as the reference's outbuf, out_offset ignored: the segment
 * headers stay on the device).  Exactly wg_encap_batch over the whole batch,
 * with the counters running on across chunks on the device: super-buffer i's
 * messages at host_msgs + i * msg_cap (msg_cap a multiple of 16; bytes of
 * host_msgs past msg_bytes are unspecified), host_res[i] its wg_encap_result,
 * host_gso_res[i] (nullable) its wg_gso_result, *next_counter (nullable) =
 * counter0 + every segment's message = the peer's next encrypt_nonce.
 * Chunks of whole super-buffers, ~host_chunk_mb MiB of input each; input
 * prefixes are zeroed on the device copy only. */
int wg_encap_host(const uint8_t *host_in, const wg_gso_desc *host_desc, uint64_t n, const uint8_t key[32],
                  uint32_t receiver_index, uint64_t counter0, uint32_t max_segments, uint32_t max_segment_size,
                  uint32_t msg_cap, uint8_t *host_msgs, wg_encap_result *host_res, wg_gso_result *host_gso_res,
                  uint64_t *next_counter);

/* Free the calling thread's host-path workspace now (it is rebuilt on the
 * next host-path call).  The caller's current device is left as it was.
 * Always WG_OK. */
int wg_host_release(void);

/* Pinned (page-locked) host memory for packet I/O buffers — the reference's
 * per-thread tun / UDP buffers allocated this way are DMA'd by the host path
 * without runtime staging.  wg_host_free(NULL) is a no-op. */
int wg_host_alloc(void **ptr, uint64_t bytes);
int wg_host_free(void *ptr);

/* Per-call placement counters of the drop-in symbol wireglider::calc_l4_checksum
 * (checksum.cpp:8-36, exported by this library): calls answered by the GPU
 * round trip (WG_PERCALL=gpu), calls that fell back to the host because that
 * round trip failed, and calls answered on the host by placement (the
 * default).  Process-wide, since load; any pointer may be NULL.  Always WG_OK. */
int wg_percall_stats(uint64_t *gpu_answered, uint64_t *host_fallback, uint64_t *host_answered);

/* ------------------------------------------------------------------------
 * Synthetic batches (benchmark / test data, written on the device; not part
 * of the reference interface).  Deterministic in `seed` and in the global
 * packet index, so shards generated on different GPUs agree.
 * ---------------------------------------------------------------------- */

/* Fill dev[0, nbytes) with counter-based pseudo-random bytes. */
int wg_synth_fill(uint8_t *dev, uint64_t nbytes, uint64_t seed, uint64_t counter_base,
                  void *stream);

/* Write IPv4/IPv6 + TCP/UDP headers for each descriptor (payload untouched,
 * L4 checksum field zeroed = generate mode, IPv4 header checksum valid).
 * index_base offsets the packet index used to derive header fields. */
int wg_synth_headers(uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n, uint64_t seed,
                     uint64_t index_base, void *stream);

/* Fill descriptors for a uniform-stride batch: packet i at i*stride, length
 * len, family/protocol by `mode`: 0 = all v4/UDP, 1 = v4/v6 x TCP/UDP mixed
 * 50/50 by a hash of (seed, index_base + i) (BASELINE config 5). */
int wg_synth_desc_stride(wg_pkt_desc *dev_desc, uint64_t n, uint64_t stride, uint32_t len,
                         int mode, uint64_t seed, uint64_t index_base, void *stream);

/* Store each packet's result into its L4 checksum field (csum_start +
 * 6 for UDP, +16 for TCP), turning a generate-mode batch into a valid one. */
int wg_store_l4csum(uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n,
                    const uint16_t *dev_csum, void *stream);

/* ------------------------------------------------------------------------
 * Misc.
 * ---------------------------------------------------------------------- */
int wg_abi_version(void);
const char *wg_strerror(int code);
/* HIP device count (0 when no GPU); never throws. */
int wg_device_count(void);

/* Launch-geometry knobs.  Each key is also read once, at the first launch,
 * from the environment as WG_<KEY> (e.g. WG_L4_NT=0); the environment and
 * wg_tune_set accept the same values and ignore / reject (WG_ERR_INVALID)
 * anything else.  Results never depend on them.  (Variants measured and
 * rejected were removed in round 4; DESIGN.md keeps their numbers.)
 *   "l4_blocks"  grid cap of the wave-per-packet L4 kernel (1 .. 2^20)
 *   "l4_nt"      non-temporal packet loads (0, 1)
 *   "l4_small"   descriptor-batch kernel: 5 (default) split roles — groups
 *                of 4 descriptors whose packets are all <= 64 B are summed a
 *                lane per packet, every other group wave-per-packet; 0 =
 *                wave-per-packet for all
 *   "lane_coop"  l4_small = 5's lane role: the small packets' bytes loaded
 *                by the wave together and handed to their lanes through LDS
 *                (1, default) or each lane loading its own (0)
 *   "l4_small_uniform" uniform batches with segment_size <= 64: a lane per
 *                segment (2, default) or the wave-per-packet kernel (0)
 *   "l4_unroll"  descriptor batches: 16-B loads in flight per lane while
 *                streaming a packet's bytes past its first 2 KiB (4, 8)
 *   "l4_coop"    descriptor batches of n <= l4_coop descriptors: a block of
 *                l4_coop_waves waves per packet (few, long packets; 0 never)
 *   "l4_coop_waves" waves sharing one packet in that mode (2, 4, 8, 16)
 *   "gso_blocks" grid cap of the GSO split kernel (1 .. 2^23)
 *   "gso_groups" blocks per super-buffer, consecutive in the flat grid (1 .. 64)
 *   "gso_waves"  waves per GSO block (1, 2, 4, 8)
 *   "gso_split"  further blocks per super-buffer in grid y (1 .. 64)
 *   "gso_spw"    segments per wave step: 0 serial, 1 ping-pong, 2-4 issued together (4)
 *   "encap_spw"  the same for wg_encap_batch's headers-only split (3)
 *   "encap_parts" wg_encap_batch in slices, each split on a side stream under
 *                the previous slice's AEAD (1 = not pipelined, default; 2-8)
 *   "verify_small" wg_verify_desc kernels: 7 (default) = per call, from the
 *                size mix the previous call on the same stream (per thread
 *                for hipStreamPerThread) sampled: the walking kernel (8) on
 *                the stream's first call
 *                and when all 64 sampled packets are <= 64 B, else the
 *                cheaper of the wave kernel (0) and the compacting path (6)
 *                by a cost model; calls under stream capture take a
 *                stateless kernel.  0 = one-shot 4-packet waves; 6 = lane per
 *                descriptor (<= 64 B decoded in the lane, longer ones
 *                appended to per-shard lists) + a wave kernel over the lists;
 *                8 = a wave per 64 descriptors, small packets in lanes, the
 *                long ones walked 4 at a time
 *   "verify_auto_t" the sample threshold of verify_small 7's compacting path (1 .. 64)
 *   "verify_k2min" compacting path: minimum blocks of its wave kernel
 *                (8 .. 65536; the grid follows the expected long packets)
 *   "host_chunk_mb" host-memory pipeline chunk size in MiB (1 .. 4096)
 *   "host_d2h"   host pipeline downloads into pinned memory by a store
 *                kernel (0-7): bit 1 encap messages, bit 2 every decap
 *                plaintext chunk, bit 4 decap plaintext chunks under 24 MiB
 *                (default 5 = bits 1 and 4; 0: the runtime's copies always)
 *   "aead_k"     AEAD kernels: consecutive ChaCha20 blocks per lane (2, 3;
 *                0 = 2 or 3, whichever fills a wave better for the batch)
 *   "aead_stage" AEAD encrypt: each wave assembles its messages in LDS and
 *                writes them out in whole lines (1, default) or every lane
 *                stores its own blocks (0)
 *   "encap_synth" wg_encap_batch: the AEAD builds the headers of segments
 *                whose header fits one 64-B block itself (fields, IPv4 and L4
 *                checksums) and the split skips those super-buffers (1,
 *                default; needs the staged kernel, i.e. the call's
 *                max_segment_size in [129, 6080]), or every segment header
 *                comes from the split (0)
 *   "gso_ablate" GSO A/B variants: 1 = non-temporal payload stores, 32 = no
 *                XCD swizzle (both correct); 0 = the default kernel.
 * Thread-safe: each launch reads one consistent snapshot of the knobs. */
int wg_tune_set(const char *key, uint64_t value);
/* Current value of a wg_tune_set key. */
int wg_tune_get(const char *key, uint64_t *value);

/* Read-roofline probe (benchmark support): streams dev[0, nbytes) with
 * non-temporal 16-B loads and folds the bytes into a sum that is stored to
 * *dev_out only in a case real data never hits.  run_bytes = 0: one-shot
 * waves of `kib_per_wave` (1/2/4/8) contiguous KiB each.  run_bytes in
 * [1, 2048]: the L4 kernel's own issue structure on a uniform batch of
 * run_bytes-byte segments (4 segments per one-shot wave, two 64-lane 16-B
 * loads per segment, all in flight at once), over nbytes / run_bytes whole
 * segments.  Its bandwidth is the measured read ceiling the checksum kernels
 * are compared against. */
int wg_probe_read(const uint8_t *dev, uint64_t nbytes, uint64_t *dev_out, uint32_t kib_per_wave,
                  uint32_t run_bytes, void *stream);

/* Copy-roofline probe: dst[0, nbytes) = src[0, nbytes) by one-shot waves of
 * `kib_per_wave` (1/2/4) KiB, non-temporal loads and stores, or the default
 * cache policy with WG_PROBE_DEFAULT_POLICY or'ed into kib_per_wave; the
 * measured read+write ceiling for the GSO split and encap kernels. */
#define WG_PROBE_DEFAULT_POLICY 0x100u
int wg_probe_copy(const uint8_t *src, uint8_t *dst, uint64_t nbytes, uint32_t kib_per_wave, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* WIREGLIDER_AMD_H */
