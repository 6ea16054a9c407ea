// ChaCha20 quarter-round issue-rate probe (timing only, not library code):
// each lane runs kIters double rounds over two interleaved 16-word states
// (the AEAD kernel's block pair), with the 16- and 8-bit rotates done three
// ways:
//   0  v_alignbit_b32 for every rotate (the library's form),
//   1  the 16-bit rotate fused with its XOR as two SDWA word XORs,
//   2  the 16- and 8-bit rotates by v_perm_b32.
// Launches of W waves per SIMD (256 CUs x 4 SIMDs, 256-thread blocks, all
// resident); each wave stamps s_memtime around its loop.  Prints one JSON
// line per (variant, W): median over waves of cycles per quarter round per
// wave, and that / W (the SIMD's cost per quarter round), plus a checksum of
// the final states (equal across variants: same arithmetic).
// build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/chacha_rate tools/exp/chacha_rate.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int kIters = 256;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }

template <int V>
__device__ __forceinline__ uint32_t xr16(uint32_t d, uint32_t a) {  // rotl(d ^ a, 16)
    if constexpr (V == 1) {
        uint32_t o;
        asm volatile(
            "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n\t"
            "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
            : "=&v"(o)
            : "v"(d), "v"(a));
        return o;
    } else if constexpr (V == 2) {
        return __builtin_amdgcn_perm(d ^ a, d ^ a, 0x01000302u);
    } else {
        return rotl(d ^ a, 16);
    }
}
template <int V>
__device__ __forceinline__ uint32_t xr8(uint32_t d, uint32_t a) {  // rotl(d ^ a, 8)
    if constexpr (V == 2)
        return __builtin_amdgcn_perm(d ^ a, d ^ a, 0x02010003u);
    else
        return rotl(d ^ a, 8);
}

#define QR(V, a, b, c, d)                                                                                           \
    a += b; d = xr16<V>(d, a);                                                                                       \
    c += d; b = rotl(b ^ c, 12);                                                                                     \
    a += b; d = xr8<V>(d, a);                                                                                        \
    c += d; b = rotl(b ^ c, 7);

template <int V>
__global__ __launch_bounds__(256) void probe(uint64_t *cyc, uint32_t *sum) {
    uint32_t x[16], y[16];
#pragma unroll
    for (int m = 0; m < 16; m++) {
        x[m] = threadIdx.x * 0x9e3779b9u + m * 0x85ebca6bu + blockIdx.x;
        y[m] = x[m] ^ 0x5bd1e995u;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
        QR(V, x[0], x[4], x[8], x[12]);
        QR(V, y[0], y[4], y[8], y[12]);
        QR(V, x[1], x[5], x[9], x[13]);
        QR(V, y[1], y[5], y[9], y[13]);
        QR(V, x[2], x[6], x[10], x[14]);
        QR(V, y[2], y[6], y[10], y[14]);
        QR(V, x[3], x[7], x[11], x[15]);
        QR(V, y[3], y[7], y[11], y[15]);
        QR(V, x[0], x[5], x[10], x[15]);
        QR(V, y[0], y[5], y[10], y[15]);
        QR(V, x[1], x[6], x[11], x[12]);
        QR(V, y[1], y[6], y[11], y[12]);
        QR(V, x[2], x[7], x[8], x[13]);
        QR(V, y[2], y[7], y[8], y[13]);
        QR(V, x[3], x[4], x[9], x[14]);
        QR(V, y[3], y[4], y[9], y[14]);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int m = 0; m < 16; m++) acc += x[m] * (2u * m + 1u) + y[m];
    atomicAdd(sum, acc);
    if ((threadIdx.x & 63u) == 0)
        cyc[blockIdx.x * 4u + threadIdx.x / 64u] = t1 - t0;
}

template <int V>
static void run(const char *name, int W, uint64_t *d, uint32_t *sum) {
    const int blocks = 256 * W;
    for (int r = 0; r < 2; r++) {
        (void)hipMemset(sum, 0, 4);
        hipLaunchKernelGGL((probe<V>), dim3(blocks), dim3(256), 0, 0, d, sum);
    }
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> h(blocks * 4);
    uint32_t s = 0;
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&s, sum, 4, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double qr = (double)h[h.size() / 2] / (kIters * 16.0);
    printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"wave_cycles_per_qr\": %.2f, \"simd_cycles_per_qr\": %.2f, "
           "\"checksum\": %u}\n",
           name, W, qr, qr / W, s);
}

int main() {
    uint64_t *d;
    uint32_t *sum;
    (void)hipMalloc(&d, 256 * 8 * 4 * 8);
    (void)hipMalloc(&sum, 4);
    for (int W : {1, 2, 3, 4, 8}) {
        run<0>("alignbit", W, d, sum);
        run<1>("sdwa_rot16", W, d, sum);
        run<2>("perm_rot16_rot8", W, d, sum);
    }
    (void)hipFree(d);
    (void)hipFree(sum);
    return 0;
}
