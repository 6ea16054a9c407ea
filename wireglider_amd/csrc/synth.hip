// synth.hip — deterministic synthetic packet batches, generated on the device.
//
// Benchmark / test data only (BASELINE configs 2-5 use synthetic packets of
// the named shapes).  Every byte is a pure function of (seed, global byte
// counter) and every header field of (seed, global packet index), so a
// shard generated on one GPU equals the same slice generated anywhere else.
#include <hip/hip_runtime.h>

#include "wg_device.hpp"
#include "wireglider_amd.h"

namespace wg {

// Byte at global counter g = byte (g & 7) of splitmix64(key + (g >> 3)).
__global__ __launch_bounds__(256) void synth_fill_kernel(uint8_t *dev, uint64_t nbytes, uint64_t key,
                                                         uint64_t counter_base) {
    const uint64_t nchunks = nbytes >> 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t w0 = counter_base >> 3;  // counter_base is a multiple of 16
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nchunks; t += stride) {
        uint64_t a = splitmix64(key + w0 + 2 * t);
        uint64_t b = splitmix64(key + w0 + 2 * t + 1);
        uint4 v;
        v.x = (uint32_t)a;
        v.y = (uint32_t)(a >> 32);
        v.z = (uint32_t)b;
        v.w = (uint32_t)(b >> 32);
        *reinterpret_cast<uint4 *>(dev + 16 * t) = v;
    }
    // tail bytes
    const uint64_t tail0 = nchunks << 4;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid < (nbytes - tail0)) {
        const uint64_t g = tail0 + tid;
        uint64_t w = splitmix64(key + w0 + (g >> 3));
        dev[g] = (uint8_t)(w >> (8 * (g & 7)));
    }
}

__device__ __forceinline__ void st_be16(uint8_t *p, uint32_t v, uint32_t len, uint32_t off) {
    if (off < len) p[off] = (uint8_t)(v >> 8);
    if (off + 1 < len) p[off + 1] = (uint8_t)v;
}
__device__ __forceinline__ void st_b(uint8_t *p, uint32_t v, uint32_t len, uint32_t off) {
    if (off < len) p[off] = (uint8_t)v;
}

// One thread per packet: IPv4 (IHL = csum_start/4) or IPv6 fixed header,
// then a TCP (doff 5, ACK|PSH) or UDP header at csum_start, checksum field 0.
__global__ __launch_bounds__(256) void synth_headers_kernel(uint8_t *base, const wg_pkt_desc *desc, uint64_t n,
                                                            uint64_t key, uint64_t index_base) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const wg_pkt_desc d = desc[i];
        uint8_t *p = base + d.offset;
        const uint32_t len = d.len, cs = d.csum_start;
        const bool v6 = d.flags & WG_PKT_V6, tcp = d.flags & WG_PKT_TCP;
        const uint64_t h0 = splitmix64(key ^ splitmix64(index_base + i));
        const uint64_t h1 = splitmix64(h0 + 1), h2 = splitmix64(h0 + 2), h3 = splitmix64(h0 + 3),
                       h4 = splitmix64(h0 + 4);
        const uint32_t proto = tcp ? 6u : 17u;
        if (!v6) {
            const uint32_t ihl = (cs >= 20 && cs <= 60 && (cs & 3) == 0) ? cs / 4 : 5;
            st_b(p, 0x40u | ihl, len, 0);
            st_b(p, 0x00, len, 1);
            st_be16(p, len & 0xffffu, len, 2);
            st_be16(p, (uint32_t)h0 & 0xffffu, len, 4);  // id
            st_be16(p, 0x4000u, len, 6);                  // DF
            st_b(p, 64, len, 8);
            st_b(p, proto, len, 9);
            st_be16(p, 0, len, 10);
            for (uint32_t j = 0; j < 4; j++) {
                st_b(p, (uint32_t)(h1 >> (8 * j)), len, 12 + j);
                st_b(p, (uint32_t)(h1 >> (32 + 8 * j)), len, 16 + j);
            }
            for (uint32_t j = 20; j < 4 * ihl; j++) st_b(p, 0x01, len, j);  // NOP options
            // IPv4 header checksum over [0, 4*ihl), stored in native order
            // (worker/offload.cpp:184-186).
            if (4 * ihl <= len) {
                uint64_t s = 0;
                for (uint32_t j = 0; j < 4 * ihl; j += 2) s += (uint32_t)p[j] | ((uint32_t)p[j + 1] << 8);
                const uint32_t c = ~fold16(s) & 0xffffu;
                p[10] = (uint8_t)c;
                p[11] = (uint8_t)(c >> 8);
            }
        } else {
            st_b(p, 0x60, len, 0);
            st_b(p, (uint32_t)(h0 >> 16) & 0x0f, len, 1);
            st_be16(p, (uint32_t)(h0 >> 24) & 0xffffu, len, 2);  // flow label
            st_be16(p, (len - 40) & 0xffffu, len, 4);
            st_b(p, proto, len, 6);
            st_b(p, 64, len, 7);
            for (uint32_t j = 0; j < 8; j++) {
                st_b(p, (uint32_t)(h1 >> (8 * j)), len, 8 + j);
                st_b(p, (uint32_t)(h2 >> (8 * j)), len, 16 + j);
                st_b(p, (uint32_t)(h3 >> (8 * j)), len, 24 + j);
                st_b(p, (uint32_t)(h4 >> (8 * j)), len, 32 + j);
            }
        }
        const uint32_t ports = (uint32_t)(h2 >> 32);
        st_be16(p, ports & 0xffffu, len, cs + 0);
        st_be16(p, ports >> 16, len, cs + 2);
        if (tcp) {
            const uint32_t seq = (uint32_t)h3, ack = (uint32_t)(h3 >> 32);
            st_be16(p, seq >> 16, len, cs + 4);
            st_be16(p, seq & 0xffffu, len, cs + 6);
            st_be16(p, ack >> 16, len, cs + 8);
            st_be16(p, ack & 0xffffu, len, cs + 10);
            st_b(p, 0x50, len, cs + 12);  // doff 5
            st_b(p, 0x18, len, cs + 13);  // ACK|PSH
            st_be16(p, 0xffffu, len, cs + 14);
            st_be16(p, 0, len, cs + 16);  // checksum (generate mode)
            st_be16(p, 0, len, cs + 18);
        } else {
            st_be16(p, (len - cs) & 0xffffu, len, cs + 4);
            st_be16(p, 0, len, cs + 6);  // checksum (generate mode)
        }
    }
}

__global__ __launch_bounds__(256) void synth_desc_stride_kernel(wg_pkt_desc *desc, uint64_t n, uint64_t stride,
                                                                uint32_t len, int mode, uint64_t key,
                                                                uint64_t index_base) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        wg_pkt_desc d;
        d.offset = i * stride;
        d.len = len;
        uint32_t fl = 0;
        if (mode == 1) {
            const uint64_t h = splitmix64(key ^ splitmix64(index_base + i) ^ 0xC0F5ull);
            fl = (uint32_t)(h & 3u);  // bit0 v6, bit1 tcp
        }
        d.csum_start = (fl & WG_PKT_V6) ? 40 : 20;
        d.flags = (uint8_t)fl;
        d.reserved = 0;
        desc[i] = d;
    }
}

__global__ __launch_bounds__(256) void store_l4csum_kernel(uint8_t *base, const wg_pkt_desc *desc, uint64_t n,
                                                           const uint16_t *csum) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) {
        const wg_pkt_desc d = desc[i];
        const uint32_t off = d.csum_start + ((d.flags & WG_PKT_TCP) ? 16u : 6u);
        if (off + 2 <= d.len) {
            base[d.offset + off] = (uint8_t)csum[i];  // native order
            base[d.offset + off + 1] = (uint8_t)(csum[i] >> 8);
        }
    }
}

static unsigned grid_for(uint64_t items) {
    uint64_t b = (items + 255) / 256;
    if (b > 8192) b = 8192;
    if (b < 1) b = 1;
    return (unsigned)b;
}

}  // namespace wg

using namespace wg;

static uint64_t host_seed_key(uint64_t seed) {
    uint64_t x = seed ^ 0x5EEDC0DEull;
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

extern "C" int wg_synth_fill(uint8_t *dev, uint64_t nbytes, uint64_t seed, uint64_t counter_base,
                             void *stream) {
    if (!nbytes) return WG_OK;
    if (!dev || (reinterpret_cast<uintptr_t>(dev) & 15) || (counter_base & 15)) return WG_ERR_INVALID;
    const uint64_t key = host_seed_key(seed);
    unsigned g = grid_for(nbytes >> 4);
    hipLaunchKernelGGL(synth_fill_kernel, dim3(g), dim3(256), 0, static_cast<hipStream_t>(stream), dev, nbytes,
                       key, counter_base);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_synth_headers(uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n, uint64_t seed,
                                uint64_t index_base, void *stream) {
    if (!n) return WG_OK;
    if (!dev_base || !dev_desc) return WG_ERR_INVALID;
    hipLaunchKernelGGL(synth_headers_kernel, dim3(grid_for(n)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       dev_base, dev_desc, n, host_seed_key(seed), index_base);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_synth_desc_stride(wg_pkt_desc *dev_desc, uint64_t n, uint64_t stride, uint32_t len, int mode,
                                    uint64_t seed, uint64_t index_base, void *stream) {
    if (!n) return WG_OK;
    if (!dev_desc || (mode != 0 && mode != 1)) return WG_ERR_INVALID;
    hipLaunchKernelGGL(synth_desc_stride_kernel, dim3(grid_for(n)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), dev_desc, n, stride, len, mode, host_seed_key(seed),
                       index_base);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}

extern "C" int wg_store_l4csum(uint8_t *dev_base, const wg_pkt_desc *dev_desc, uint64_t n,
                               const uint16_t *dev_csum, void *stream) {
    if (!n) return WG_OK;
    if (!dev_base || !dev_desc || !dev_csum) return WG_ERR_INVALID;
    hipLaunchKernelGGL(store_l4csum_kernel, dim3(grid_for(n)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       dev_base, dev_desc, n, dev_csum);
    return hipGetLastError() == hipSuccess ? WG_OK : WG_ERR_LAUNCH;
}
