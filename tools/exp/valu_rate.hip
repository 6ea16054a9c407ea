// Issue-rate probe for the VALU operations the AEAD kernel is made of and
// the ones that could replace them (timing only, not library code).
//
// Each lane runs C independent chains of one operation (inline asm, so the
// compiler cannot fold or strength-reduce them) for kIters iterations; each
// wave stamps s_memtime (shader clock) around its loop.  Launches of W waves
// per SIMD (256 CUs x 4 SIMDs, 256-thread blocks, every wave resident at
// once) give:
//   W = 8, C = 8: the SIMD's throughput cost per wave-instruction (cycles),
//   W = 1, C = 8: what one wave alone issues (independent instructions),
//   W = 1, C = 1: the dependent-issue latency of the operation.
// Prints one JSON line per (op, W, C): median over waves of
// cycles / (kIters * C) and, for W > 1, that divided by W (SIMD cost).
// build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/valu_rate tools/exp/valu_rate.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int kIters = 2048;

// one instruction on chain register x (y: a second operand register, s: an SGPR operand)
template <int Op>
__device__ __forceinline__ void op1(uint32_t &x, uint32_t y, uint32_t s, uint64_t &w) {
    if constexpr (Op == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(y));
    else if constexpr (Op == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
    else if constexpr (Op == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x));
    else if constexpr (Op == 3) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(x) : "v"(y));
    else if constexpr (Op == 4) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x) : "s"(s));
    else if constexpr (Op == 5) asm volatile("v_alignbyte_b32 %0, %0, %0, 2" : "+v"(x));
    else if constexpr (Op == 6) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
    else if constexpr (Op == 7) asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
    else if constexpr (Op == 8) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w) : "v"(x), "s"(s) : "vcc");
    else if constexpr (Op == 9) asm volatile("v_lshl_or_b32 %0, %0, 16, %1" : "+v"(x) : "v"(y));
    else if constexpr (Op == 10) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "s"(s));
    else if constexpr (Op == 11) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "s"(s));
    else if constexpr (Op == 12) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x) : "s"(s));
    else if constexpr (Op == 13) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(y) : "vcc");
    else if constexpr (Op == 14) asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(x) : "s"(s));
    else if constexpr (Op == 15) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(y));
    else if constexpr (Op == 16) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "s"(s));
    else if constexpr (Op == 17) asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(x));
    else if constexpr (Op == 18) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(w));
    else if constexpr (Op == 19) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(x) : "v"(y));
}

template <int Op, int C>
__global__ __launch_bounds__(256) void probe(uint64_t *cyc, uint32_t s, uint32_t *sink) {
    uint32_t x[C], y = threadIdx.x * 3u + 1u;
    uint64_t w[C];
#pragma unroll
    for (int i = 0; i < C; i++) {
        x[i] = threadIdx.x * 7u + i;
        w[i] = x[i];
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int i = 0; i < C; i++) op1<Op>(x[i], y, s, w[i]);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < C; i++) acc += x[i] + (uint32_t)w[i];
    if (acc == 0x9e3779b9u)
        sink[threadIdx.x] = acc;
    if ((threadIdx.x & 63u) == 0)
        cyc[blockIdx.x * 4u + threadIdx.x / 64u] = t1 - t0;
}

template <int Op, int C>
static void run(const char *name, int W, uint64_t *d, uint32_t *sink) {
    const int blocks = 256 * W;  // 4 waves per block, one per SIMD
    for (int r = 0; r < 2; r++)  // warm the clock, keep the second
        hipLaunchKernelGGL((probe<Op, C>), dim3(blocks), dim3(256), 0, 0, d, 0x01000302u, sink);
    hipDeviceSynchronize();
    std::vector<uint64_t> h(blocks * 4);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double med = (double)h[h.size() / 2] / (kIters * (double)C);
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"chains\": %d, \"wave_cycles_per_inst\": %.3f, "
           "\"simd_cycles_per_inst\": %.3f}\n",
           name, W, C, med, med / W);
}

template <int Op>
static void sweep(const char *name, uint64_t *d, uint32_t *sink) {
    run<Op, 8>(name, 8, d, sink);
    run<Op, 8>(name, 1, d, sink);
    run<Op, 1>(name, 1, d, sink);
}

int main() {
    uint64_t *d;
    uint32_t *sink;
    hipMalloc(&d, 256 * 8 * 4 * 8);
    hipMalloc(&sink, 4096);
    sweep<0>("v_add_u32", d, sink);
    sweep<1>("v_xor_b32", d, sink);
    sweep<2>("v_alignbit_b32 x,x,16", d, sink);
    sweep<3>("v_alignbit_b32 x,y,16", d, sink);
    sweep<14>("v_alignbit_b32 x,x,s", d, sink);
    sweep<4>("v_perm_b32 x,x,s", d, sink);
    sweep<5>("v_alignbyte_b32 x,x,2", d, sink);
    sweep<6>("v_add3_u32", d, sink);
    sweep<7>("v_xad_u32", d, sink);
    sweep<9>("v_lshl_or_b32", d, sink);
    sweep<17>("v_lshlrev_b32", d, sink);
    sweep<19>("v_bfi_b32", d, sink);
    sweep<15>("v_pk_add_u16", d, sink);
    sweep<13>("v_add_co_u32", d, sink);
    sweep<8>("v_mad_u64_u32", d, sink);
    sweep<10>("v_mul_lo_u32", d, sink);
    sweep<11>("v_mul_hi_u32", d, sink);
    sweep<12>("v_mad_u32_u24", d, sink);
    sweep<16>("v_mul_u32_u24", d, sink);
    sweep<18>("v_fma_f64", d, sink);
    hipFree(d);
    hipFree(sink);
    return 0;
}
