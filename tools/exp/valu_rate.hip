// Issue-rate probe for the VALU operations the AEAD kernel is made of
// (timing only, not library code): each lane runs 8 independent chains of
// one operation for ITERS iterations; the grid is 2048 blocks x 256 threads
// (8 waves / SIMD on 256 CUs).  Prints wave-instructions per cycle per SIMD
// for each operation at the measured clock-free rate (per ns) and the ratio
// to v_add_u32.
// build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/valu_rate tools/exp/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int kIters = 4096;

template <int Op>
__global__ __launch_bounds__(256) void probe(uint32_t *out, uint32_t k) {
    uint32_t x[8];
    uint64_t y[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        x[i] = threadIdx.x * 7u + i;
        y[i] = x[i];
    }
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if constexpr (Op == 0) {  // v_add_u32
                x[i] += x[(i + 1) & 7];
            } else if constexpr (Op == 1) {  // v_mad_u64_u32 (32 x 32 + 64 -> 64)
                y[i] = (uint64_t)(uint32_t)y[i] * k + y[i];
            } else if constexpr (Op == 2) {  // v_mul_lo_u32
                x[i] *= k;
            } else if constexpr (Op == 3) {  // v_mul_hi_u32
                x[i] = __umulhi(x[i], k) ^ k;
            } else if constexpr (Op == 4) {  // v_alignbit_b32 (rotate)
                x[i] = __builtin_amdgcn_alignbit(x[i], x[i], k);
            } else {  // v_mad_u32_u24
                x[i] = __umul24(x[i], k) + x[i];
            }
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += x[i] + (uint32_t)y[i] + (uint32_t)(y[i] >> 32);
    if (s == 0x12345678u)
        out[threadIdx.x] = s;
}

template <int Op>
static float run(uint32_t *d, const char *name, float base) {
    const dim3 g(2048), b(256);
    hipLaunchKernelGGL(probe<Op>, g, b, 0, 0, d, 3u);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(probe<Op>, g, b, 0, 0, d, 3u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double winst = 2048.0 * 4 * kIters * 8;  // wave-instructions of the operation (4 waves / block)
    const double per_ns = winst / (best * 1e6);
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"winst_per_ns\": %.1f, \"vs_add\": %.3f}\n", name, best, per_ns,
           base > 0 ? base / best : 1.0);
    return best;
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 4096);
    const float add = run<0>(d, "v_add_u32", 0);
    run<1>(d, "v_mad_u64_u32", add);
    run<2>(d, "v_mul_lo_u32", add);
    run<3>(d, "v_mul_hi_u32 (+xor)", add);
    run<4>(d, "v_alignbit_b32", add);
    run<5>(d, "v_mul_u32_u24 (+add)", add);
    hipFree(d);
    return 0;
}
