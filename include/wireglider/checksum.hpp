// wireglider/checksum.hpp — drop-in replacement for the reference's
// include/netio/checksum.hpp (dinhngtu/wireglider @ 2024-11-01).
//
// Same namespace, names, template parameters and semantics, so the
// reference's callers compile unchanged against it:
//   worker/offload.cpp:71,75,184,202      checksum(), calc_l4_checksum()
//   worker/evaluator.cpp:28               checksum()
//   include/worker/evaluator.hpp:64,93    calc_l4_checksum()
//   include/worker/flowkey_ref.hpp:108-110, flowkey_own.hpp:106-108
//                                         checksum(), pseudo_header_checksum()
//
// Placement: the header-inline pieces stay header-inline and run
// where the caller runs (each is a 20-40 byte fixed-size sum; a device launch
// would cost more than it saves).  calc_l4_checksum — the reference's only
// out-of-line symbol (checksum.cpp:8) — is exported by libwireglider_amd.so;
// a per-call caller gets its answer on the CPU (host::calc_l4_checksum), and
// batch callers use the wireglider::gpu:: entry points below, which take
// whole PacketBatch-shaped batches in device memory to the MI355X through the
// C ABI (include/wireglider_amd.h).
//
// No boost / fastcsum dependency: the nofold and fold primitives are this
// repository's own (clean-room) with the same contract.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <span>

#include "wireglider_amd.h"

namespace wireglider {

namespace checksum_impl {

static inline uint64_t add_eac(uint64_t a, uint64_t b) {
    uint64_t r;
    bool c = __builtin_add_overflow(a, b, &r);
    return r + c;
}

// include/netio/checksum.hpp:20-25
template <typename T>
static inline uint64_t checksum_add(const T val, uint64_t initial) {
    return add_eac(initial, static_cast<uint64_t>(val));
}

template <size_t N>
static inline uint64_t checksum_nofold(std::span<const uint8_t, N> b, uint64_t initial);

// Fixed extents 16/8/4/2/1: include/netio/checksum.hpp:30-77.
template <>
inline uint64_t checksum_nofold(std::span<const uint8_t, 16> b, uint64_t initial) {
    uint64_t lo, hi;
    std::memcpy(&lo, b.data(), 8);
    std::memcpy(&hi, b.data() + 8, 8);
    return add_eac(add_eac(initial, lo), hi);
}

template <>
inline uint64_t checksum_nofold(std::span<const uint8_t, 8> b, uint64_t initial) {
    uint64_t w;
    std::memcpy(&w, b.data(), 8);
    return add_eac(initial, w);
}

template <>
inline uint64_t checksum_nofold(std::span<const uint8_t, 4> b, uint64_t initial) {
    uint32_t w;
    std::memcpy(&w, b.data(), 4);
    return add_eac(initial, w);
}

template <>
inline uint64_t checksum_nofold(std::span<const uint8_t, 2> b, uint64_t initial) {
    uint16_t w;
    std::memcpy(&w, b.data(), 2);
    return add_eac(initial, w);
}

template <>
inline uint64_t checksum_nofold(std::span<const uint8_t, 1> b, uint64_t initial) {
    // Odd byte is the LOW byte on a little-endian host (:69-77).
    return add_eac(initial, static_cast<uint64_t>(b[0]));
}

// Dynamic extent (:79-100): 8-byte native words with end-around carry, then
// a 4/2/1-byte tail; pairing is relative to b[0].
template <>
inline uint64_t checksum_nofold(std::span<const uint8_t, std::dynamic_extent> b, uint64_t initial) {
    const uint8_t *p = b.data();
    size_t n = b.size();
    uint64_t a0 = 0, a1 = 0;
    while (n >= 16) {
        uint64_t w0, w1;
        std::memcpy(&w0, p, 8);
        std::memcpy(&w1, p + 8, 8);
        a0 = add_eac(a0, w0);
        a1 = add_eac(a1, w1);
        p += 16;
        n -= 16;
    }
    uint64_t acc = add_eac(a0, a1);
    if (n >= 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        acc = add_eac(acc, w);
        p += 8;
        n -= 8;
    }
    if (n >= 4) {
        uint32_t w;
        std::memcpy(&w, p, 4);
        acc = add_eac(acc, w);
        p += 4;
        n -= 4;
    }
    if (n >= 2) {
        uint16_t w;
        std::memcpy(&w, p, 2);
        acc = add_eac(acc, w);
        p += 2;
        n -= 2;
    }
    if (n)
        acc = add_eac(acc, *p);
    return add_eac(acc, initial);
}

// The fastcsum_fold_complement contract: 64 -> 16 end-around fold, then ~.
static inline uint16_t fold_complement(uint64_t s) {
    s = (s & 0xffffffffu) + (s >> 32);
    s = (s & 0xffffffffu) + (s >> 32);
    s = (s & 0xffffu) + (s >> 16);
    s = (s & 0xffffu) + (s >> 16);
    s = (s & 0xffffu) + (s >> 16);
    return static_cast<uint16_t>(~s);
}

// include/netio/checksum.hpp:102-116
template <size_t E1, size_t E2>
static inline uint64_t pseudo_header_checksum_nofold(uint8_t proto, std::span<const uint8_t, E1> srcAddr,
                                                     std::span<const uint8_t, E2> dstAddr, uint16_t l4Len) {
    static_assert(E1 > 1 && E2 > 1);
    auto sum = checksum_nofold(srcAddr, 0);
    sum = checksum_nofold(dstAddr, sum);
    const std::array<uint8_t, 4> tail{0, proto, static_cast<uint8_t>(l4Len >> 8),
                                      static_cast<uint8_t>(l4Len & 0xff)};
    return checksum_nofold(std::span<const uint8_t, 4>(tail), sum);
}

}  // namespace checksum_impl

// include/netio/checksum.hpp:120-128
template <size_t E1, size_t E2>
static inline uint16_t pseudo_header_checksum(uint8_t proto, std::span<const uint8_t, E1> srcAddr,
                                              std::span<const uint8_t, E2> dstAddr, uint16_t l4Len) {
    return checksum_impl::fold_complement(
        checksum_impl::pseudo_header_checksum_nofold(proto, srcAddr, dstAddr, l4Len));
}

// include/netio/checksum.hpp:130-144
template <typename TAddress>
static inline uint16_t pseudo_header_checksum(uint8_t proto, const TAddress &srcAddr, const TAddress &dstAddr,
                                              uint16_t l4Len) {
    std::span<const uint8_t, sizeof(TAddress)> s(reinterpret_cast<const uint8_t *>(&srcAddr), sizeof(srcAddr));
    std::span<const uint8_t, sizeof(TAddress)> d(reinterpret_cast<const uint8_t *>(&dstAddr), sizeof(dstAddr));
    return checksum_impl::fold_complement(checksum_impl::pseudo_header_checksum_nofold(proto, s, d, l4Len));
}

// include/netio/checksum.hpp:146-149
static inline uint16_t checksum(std::span<const uint8_t> b, uint64_t initial) {
    return checksum_impl::fold_complement(checksum_impl::checksum_nofold(b, initial));
}

namespace host {

// checksum.cpp:8-36 on the calling CPU: the pseudo-header over the addresses
// (v4 bytes 12-19, v6 8-39; :14-28) with l4Len = (uint16_t)(len - csum_start)
// (:23,33), seeded into checksum(ippkt[csum_start:]) (:35).  Inputs the
// reference leaves undefined (a packet shorter than its addresses, or than
// csum_start) get the GPU kernels' definition: bytes past the packet are
// absent (zero) and the summed region is empty — so host and device agree on
// every input.
inline uint16_t calc_l4_checksum(std::span<const uint8_t> p, bool isv6, bool istcp, uint16_t csum_start) {
    using namespace checksum_impl;
    const uint8_t proto = istcp ? 6 : 17;
    const size_t ao = isv6 ? 8 : 12, al = isv6 ? 16 : 4;
    const uint16_t l4len = static_cast<uint16_t>(p.size() - csum_start);
    const uint8_t *a = p.data() + ao;
    std::array<uint8_t, 32> pad{};
    if (p.size() < ao + 2 * al) {  // out of contract: missing address bytes are absent
        if (p.size() > ao)
            std::memcpy(pad.data(), p.data() + ao, p.size() - ao);
        a = pad.data();
    }
    const uint64_t ph =
        isv6 ? pseudo_header_checksum_nofold(proto, std::span<const uint8_t, 16>(a, 16),
                                             std::span<const uint8_t, 16>(a + 16, 16), l4len)
             : pseudo_header_checksum_nofold(proto, std::span<const uint8_t, 4>(a, 4),
                                             std::span<const uint8_t, 4>(a + 4, 4), l4len);
    const size_t o0 = csum_start < p.size() ? csum_start : p.size();
    return checksum(p.subspan(o0), ph);
}

}  // namespace host

// include/netio/checksum.hpp:151 / checksum.cpp:8 — exported by
// libwireglider_amd.so with the reference's mangled name.  Per-call callers
// (worker/offload.cpp:75,202, include/worker/evaluator.hpp:64,93) use its
// return value immediately, one packet at a time, so it computes on the
// calling CPU (host::calc_l4_checksum above: ~0.1 us for 1500 B, against
// tens of us for a device round trip).  WG_PERCALL=gpu in the environment
// sends each call through the host-memory GPU path instead (tests, latency
// measurement); if that path fails (no device, runtime error) the call is
// answered on the host — never an abort, never a different checksum.  Batches
// go to the GPU through wireglider::gpu:: below.
uint16_t calc_l4_checksum(std::span<const uint8_t> thispkt, bool isv6, bool istcp, uint16_t csum_start);

namespace gpu {

// Batch entry points (device memory, asynchronous on `stream`); thin C++
// views of include/wireglider_amd.h.  Return WG_OK or a WG_ERR_* code.
inline int calc_l4_checksum_batch(std::span<const uint8_t> dev_batch, size_t segment_size, bool isv6,
                                  bool istcp, uint16_t csum_start, uint16_t *dev_out, void *stream = nullptr) {
    return wg_l4csum_uniform(dev_batch.data(), dev_batch.size(), static_cast<uint32_t>(segment_size), csum_start,
                             (isv6 ? WG_PKT_V6 : 0u) | (istcp ? WG_PKT_TCP : 0u), dev_out, stream);
}

inline int calc_l4_checksum_batch(const uint8_t *dev_base, std::span<const wg_pkt_desc> dev_desc,
                                  uint16_t *dev_out, void *stream = nullptr) {
    return wg_l4csum_desc(dev_base, dev_desc.data(), dev_desc.size(), dev_out, stream);
}

inline int checksum_batch(const uint8_t *dev_base, std::span<const wg_pkt_desc> dev_desc, uint16_t *dev_out,
                          void *stream = nullptr) {
    return wg_checksum_desc(dev_base, dev_desc.data(), dev_desc.size(), dev_out, stream);
}

}  // namespace gpu

}  // namespace wireglider
