// Experiment (not built into the library): how do the two GSO structures
// tolerate per-segment instruction work?  Copy-only config 3 layout (as
// gso_persist.hip) plus, per segment, the payload sum, a wave reduction and
// K dependent VALU + K SALU filler instructions whose result is stored with
// the header (so nothing is dead code).
//   A3(K)  one-shot blocks, 3 per super-buffer, 4 waves, ping-pong over every 12th segment
//   C(K)   one-shot waves, one segment each, global order
// usage: gso_alu
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_v4u;
typedef __attribute__((address_space(1))) unsigned char g_u8;

constexpr unsigned N = 1u << 18, IN_STRIDE = 65536, OUT_STRIDE = 73216, IN_LEN = 65535, H = 40, G = 1460;
constexpr unsigned NSEG = (IN_LEN - H + G - 1) / G, S = H + G;

struct Seg {
    uintptr_t src, dst, hdr;
    unsigned dl;
};

__device__ __forceinline__ Seg seg_of(uintptr_t in, uintptr_t out, unsigned i) {
    Seg s;
    s.hdr = in;
    s.src = in + H + (uintptr_t)i * G;
    s.dst = out + (uintptr_t)i * S;
    const unsigned rest = IN_LEN - H - i * G;
    s.dl = rest < G ? rest : G;
    return s;
}

struct Front {
    v4u a, c;
    unsigned hb, eb;
};

__device__ __forceinline__ void issue(const Seg &s, unsigned lane, Front &f) {
    const uintptr_t oa = s.dst + H, ob = oa + s.dl;
    const uintptr_t c0 = (oa + 15) & ~(uintptr_t)15, c1 = ob & ~(uintptr_t)15;
    const unsigned nint = c1 > c0 ? (unsigned)((c1 - c0) >> 4) : 0u;
    const uintptr_t base = s.src + (c0 - oa);
    const unsigned last = nint ? nint - 1 : 0u;
    f.a = *(const g_v4u *)(base + 16u * (lane < last ? lane : last));
    f.c = *(const g_v4u *)(base + 16u * (lane + 64 < last ? lane + 64 : last));
    f.hb = *(const g_u8 *)(s.hdr + (lane < H ? lane : 0u));
    const unsigned he = (unsigned)(c0 - oa), ts = (unsigned)(c1 - oa);
    const unsigned off = lane < 16 ? lane : ts + lane - 16;
    const bool ok = lane < 16 ? lane < he : (lane < 32 && off < s.dl);
    f.eb = *(const g_u8 *)(s.src + (ok ? off : 0u));
}

__device__ __forceinline__ unsigned wsum(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    return (unsigned)__builtin_amdgcn_readlane((int)v, 0) + (unsigned)__builtin_amdgcn_readlane((int)v, 16) +
           (unsigned)__builtin_amdgcn_readlane((int)v, 32) + (unsigned)__builtin_amdgcn_readlane((int)v, 48);
}

template <int K>
__device__ __forceinline__ void finish(const Seg &s, unsigned lane, const Front &f, unsigned i) {
    const uintptr_t oa = s.dst + H, ob = oa + s.dl;
    const uintptr_t c0 = (oa + 15) & ~(uintptr_t)15, c1 = ob & ~(uintptr_t)15;
    const unsigned nint = c1 > c0 ? (unsigned)((c1 - c0) >> 4) : 0u;
    unsigned acc = 0;
    if (lane < nint) {
        *(g_v4u *)(c0 + 16u * lane) = f.a;
        acc += f.a.x + f.a.y + f.a.z + f.a.w;
    }
    if (lane + 64 < nint) {
        *(g_v4u *)(c0 + 16u * (lane + 64)) = f.c;
        acc += f.c.x + f.c.y + f.c.z + f.c.w;
    }
    const unsigned he = (unsigned)(c0 - oa), ts = (unsigned)(c1 - oa);
    const unsigned off = lane < 16 ? lane : ts + lane - 16;
    const bool ok = lane < 16 ? lane < he : (lane < 32 && off < s.dl);
    if (ok) *(g_u8 *)(oa + off) = (unsigned char)f.eb;
    unsigned t = wsum(acc);
    unsigned v = acc ^ lane;
#pragma unroll
    for (int k = 0; k < K; k++) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(v) : "v"(lane));
        asm volatile("s_add_u32 %0, %0, %1" : "+s"(t) : "s"(i) : "scc");
    }
    const unsigned b = lane < H ? (f.hb ^ (v & 0) ^ (t & 0xff)) : 0u;
    if (lane < H) *(g_u8 *)(s.dst + lane) = (unsigned char)b;
}

__device__ __forceinline__ unsigned lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ unsigned wave_in_block() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
__device__ __forceinline__ unsigned swz(unsigned bx, unsigned nb) { return (bx & 7u) * (nb >> 3) + (bx >> 3); }

template <int K>
__global__ __launch_bounds__(256) void kA3(const uint8_t *in, uint8_t *out) {
    const unsigned nb = gridDim.x, u = swz(blockIdx.x, nb);
    const unsigned b = u / 3, grp = u - 3 * b;
    const unsigned lane = lane_id();
    const uintptr_t ib = (uintptr_t)in + (uintptr_t)b * IN_STRIDE, ob = (uintptr_t)out + (uintptr_t)b * OUT_STRIDE;
    unsigned i = grp * 4 + wave_in_block();
    Front fa, fb;
    issue(seg_of(ib, ob, i), lane, fa);
    for (;;) {
        const unsigned i1 = i + 12;
        if (i1 < NSEG) issue(seg_of(ib, ob, i1), lane, fb);
        finish<K>(seg_of(ib, ob, i), lane, fa, i);
        if (i1 >= NSEG) break;
        const unsigned i2 = i1 + 12;
        if (i2 < NSEG) issue(seg_of(ib, ob, i2), lane, fa);
        finish<K>(seg_of(ib, ob, i1), lane, fb, i1);
        if (i2 >= NSEG) break;
        i = i2;
    }
}

template <int K>
__global__ __launch_bounds__(256) void kC(const uint8_t *in, uint8_t *out) {
    const unsigned g = swz(blockIdx.x, gridDim.x) * 4u + wave_in_block();
    if (g >= N * NSEG) return;
    const unsigned b = g / NSEG, i = g - b * NSEG;
    Front f;
    const Seg s = seg_of((uintptr_t)in + (uintptr_t)b * IN_STRIDE, (uintptr_t)out + (uintptr_t)b * OUT_STRIDE, i);
    issue(s, lane_id(), f);
    finish<K>(s, lane_id(), f, i);
}

int main() {
    uint8_t *in, *out;
    hipMalloc(&in, (size_t)N * IN_STRIDE);
    hipMalloc(&out, (size_t)N * OUT_STRIDE);
    hipMemset(in, 7, (size_t)N * IN_STRIDE);
    const double bytes = (double)N * IN_LEN + (double)N * (IN_LEN - H + NSEG * H);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const std::string &name, auto launch) {
        for (int w = 0; w < 3; w++) launch();
        float sum = 0;
        for (int r = 0; r < 6; r++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            sum += ms;
        }
        printf("{\"variant\": \"%s\", \"ms_avg\": %.4f, \"TBps_avg\": %.3f}\n", name.c_str(), sum / 6,
               bytes / (sum / 6 * 1e-3) / 1e12);
        fflush(stdout);
    };
    const unsigned nbc = ((N * NSEG + 3) / 4 + 7) & ~7u;
    for (int rep = 0; rep < 2; rep++) {
        run("A3 K=0", [&] { hipLaunchKernelGGL((kA3<0>), dim3(N * 3), dim3(256), 0, 0, in, out); });
        run("C  K=0", [&] { hipLaunchKernelGGL((kC<0>), dim3(nbc), dim3(256), 0, 0, in, out); });
        run("A3 K=40", [&] { hipLaunchKernelGGL((kA3<40>), dim3(N * 3), dim3(256), 0, 0, in, out); });
        run("C  K=40", [&] { hipLaunchKernelGGL((kC<40>), dim3(nbc), dim3(256), 0, 0, in, out); });
        run("A3 K=80", [&] { hipLaunchKernelGGL((kA3<80>), dim3(N * 3), dim3(256), 0, 0, in, out); });
        run("C  K=80", [&] { hipLaunchKernelGGL((kC<80>), dim3(nbc), dim3(256), 0, 0, in, out); });
        run("A3 K=120", [&] { hipLaunchKernelGGL((kA3<120>), dim3(N * 3), dim3(256), 0, 0, in, out); });
        run("C  K=120", [&] { hipLaunchKernelGGL((kC<120>), dim3(nbc), dim3(256), 0, 0, in, out); });
        run("A3 K=160", [&] { hipLaunchKernelGGL((kA3<160>), dim3(N * 3), dim3(256), 0, 0, in, out); });
        run("C  K=160", [&] { hipLaunchKernelGGL((kC<160>), dim3(nbc), dim3(256), 0, 0, in, out); });
    }
    printf("err=%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
