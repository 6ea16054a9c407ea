// Experiment (not built into the library): does the ORDER in which waves walk
// config 3's segments set the copy ceiling?  Copy-only (payload chunks by one
// unaligned 16-B load + one store each, header bytes by byte copies), no
// sums, config 3 layout (262,144 x 65,535 B in at stride 65,536 -> 45
// segments of 1,500 B out at stride 73,216).
//   A  block per super-buffer, 4 waves striding its segments, ping-pong
//      (the shape of the production kernel)
//   B  persistent waves walking segments in GLOBAL order (segment g = w,
//      w + NW, ...): the bytes in flight are one compact window
//   C  one-shot waves, one segment each, in global order
// usage: gso_order [persistent blocks for B]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_v4u;
typedef __attribute__((address_space(1))) unsigned char g_u8;

constexpr unsigned N = 1u << 18, IN_STRIDE = 65536, OUT_STRIDE = 73216, IN_LEN = 65535, H = 40, G = 1460;
constexpr unsigned NSEG = (IN_LEN - H + G - 1) / G, S = H + G;

struct Seg {
    const unsigned char *src;  // payload source
    unsigned char *dst;        // segment start (header)
    const unsigned char *hdr;  // header template
    unsigned dl;               // payload bytes
};

__device__ __forceinline__ Seg seg_of(const unsigned char *in, unsigned char *out, unsigned b, unsigned i) {
    Seg s;
    s.hdr = in + (size_t)b * IN_STRIDE;
    s.src = s.hdr + H + (size_t)i * G;
    s.dst = out + (size_t)b * OUT_STRIDE + (size_t)i * S;
    const unsigned rest = IN_LEN - H - i * G;
    s.dl = rest < G ? rest : G;
    return s;
}

struct Front {
    v4u a, c;
    unsigned hb, eb;
};

// payload chunks destination-aligned: c0 = align16(dst + H); interior k < nint
__device__ __forceinline__ void issue(const Seg &s, unsigned lane, Front &f) {
    const uintptr_t oa = (uintptr_t)s.dst + H, ob = oa + s.dl;
    const uintptr_t c0 = (oa + 15) & ~(uintptr_t)15, c1 = ob & ~(uintptr_t)15;
    const unsigned nint = c1 > c0 ? (unsigned)((c1 - c0) >> 4) : 0u;
    const uintptr_t base = (uintptr_t)s.src + (c0 - oa);
    const unsigned last = nint ? nint - 1 : 0u;
    f.a = *(const g_v4u *)(base + 16u * (lane < last ? lane : last));
    f.c = *(const g_v4u *)(base + 16u * (lane + 64 < last ? lane + 64 : last));
    f.hb = *(const g_u8 *)((uintptr_t)s.hdr + (lane < H ? lane : 0u));
    // head/tail bytes: lanes 0-15 head [oa, c0), 16-31 tail [c1, ob)
    const unsigned he = (unsigned)(c0 - oa), ts = (unsigned)(c1 - oa);
    const unsigned off = lane < 16 ? lane : ts + lane - 16;
    const bool ok = lane < 16 ? lane < he : (lane < 32 && off < s.dl);
    f.eb = *(const g_u8 *)((uintptr_t)s.src + (ok ? off : 0u));
}

__device__ __forceinline__ void finish(const Seg &s, unsigned lane, const Front &f) {
    const uintptr_t oa = (uintptr_t)s.dst + H, ob = oa + s.dl;
    const uintptr_t c0 = (oa + 15) & ~(uintptr_t)15, c1 = ob & ~(uintptr_t)15;
    const unsigned nint = c1 > c0 ? (unsigned)((c1 - c0) >> 4) : 0u;
    if (lane < nint) *(g_v4u *)(c0 + 16u * lane) = f.a;
    if (lane + 64 < nint) *(g_v4u *)(c0 + 16u * (lane + 64)) = f.c;
    if (lane < H) *(g_u8 *)((uintptr_t)s.dst + lane) = (unsigned char)f.hb;
    const unsigned he = (unsigned)(c0 - oa), ts = (unsigned)(c1 - oa);
    const unsigned off = lane < 16 ? lane : ts + lane - 16;
    const bool ok = lane < 16 ? lane < he : (lane < 32 && off < s.dl);
    if (ok) *(g_u8 *)(oa + off) = (unsigned char)f.eb;
}

__device__ __forceinline__ unsigned lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ unsigned wave_in_block() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// A: block per super-buffer (XCD-swizzled), 4 waves, ping-pong over segments w, w+4, ...
__global__ __launch_bounds__(256) void kA(const unsigned char *in, unsigned char *out) {
    const unsigned nb = gridDim.x, bx = blockIdx.x;
    const unsigned b = (bx & 7u) * (nb >> 3) + (bx >> 3);
    const unsigned lane = lane_id(), w = wave_in_block();
    Front fa, fb;
    unsigned i = w;
    issue(seg_of(in, out, b, i), lane, fa);
    for (;;) {
        const unsigned i1 = i + 4;
        if (i1 < NSEG) issue(seg_of(in, out, b, i1), lane, fb);
        finish(seg_of(in, out, b, i), lane, fa);
        if (i1 >= NSEG) break;
        const unsigned i2 = i1 + 4;
        if (i2 < NSEG) issue(seg_of(in, out, b, i2), lane, fa);
        finish(seg_of(in, out, b, i1), lane, fb);
        if (i2 >= NSEG) break;
        i = i2;
    }
}

// B: persistent waves, global segment order g = wave, wave + NW, ..., ping-pong
__global__ __launch_bounds__(256) void kB(const unsigned char *in, unsigned char *out) {
    const unsigned nw = gridDim.x * 4u;
    const unsigned w0 = blockIdx.x * 4u + wave_in_block();
    const unsigned lane = lane_id(), total = N * NSEG;
    Front fa, fb;
    unsigned g = w0;
    if (g >= total) return;
    issue(seg_of(in, out, g / NSEG, g % NSEG), lane, fa);
    for (;;) {
        const unsigned g1 = g + nw;
        if (g1 < total) issue(seg_of(in, out, g1 / NSEG, g1 % NSEG), lane, fb);
        finish(seg_of(in, out, g / NSEG, g % NSEG), lane, fa);
        if (g1 >= total) break;
        const unsigned g2 = g1 + nw;
        if (g2 < total) issue(seg_of(in, out, g2 / NSEG, g2 % NSEG), lane, fa);
        finish(seg_of(in, out, g1 / NSEG, g1 % NSEG), lane, fb);
        if (g2 >= total) break;
        g = g2;
    }
}

// C: one-shot waves, one segment each, global order (XCD-swizzled blocks)
__global__ __launch_bounds__(256) void kC(const unsigned char *in, unsigned char *out) {
    const unsigned nb = gridDim.x, bx = blockIdx.x;
    const unsigned vb = (bx & 7u) * (nb >> 3) + (bx >> 3);
    const unsigned g = vb * 4u + wave_in_block();
    if (g >= N * NSEG) return;
    Front f;
    const Seg s = seg_of(in, out, g / NSEG, g % NSEG);
    issue(s, lane_id(), f);
    finish(s, lane_id(), f);
}

int main(int argc, char **argv) {
    const unsigned pb = argc > 1 ? atoi(argv[1]) : 2048;
    unsigned char *in, *out;
    hipMalloc(&in, (size_t)N * IN_STRIDE);
    hipMalloc(&out, (size_t)N * OUT_STRIDE);
    hipMemset(in, 7, (size_t)N * IN_STRIDE);
    const double bytes = (double)N * IN_LEN + (double)N * (IN_LEN - H + NSEG * H);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, auto launch) {
        for (int w = 0; w < 5; w++) launch();
        float best = 1e9, sum = 0;
        for (int r = 0; r < 10; r++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf("{\"variant\": \"%s\", \"ms_avg\": %.4f, \"ms_best\": %.4f, \"TBps_avg\": %.3f}\n", name, sum / 10, best,
               bytes / (sum / 10 * 1e-3) / 1e12);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; rep++) {
        run("A block per super-buffer", [&] { hipLaunchKernelGGL(kA, dim3(N), dim3(256), 0, 0, in, out); });
        run("B persistent global order", [&] { hipLaunchKernelGGL(kB, dim3(pb), dim3(256), 0, 0, in, out); });
        run("B4 persistent global order 4x", [&] { hipLaunchKernelGGL(kB, dim3(pb * 4), dim3(256), 0, 0, in, out); });
        run("C one-shot global order", [&] {
            const unsigned nb = ((N * NSEG + 3) / 4 + 7) & ~7u;
            hipLaunchKernelGGL(kC, dim3(nb), dim3(256), 0, 0, in, out);
        });
    }
    printf("err=%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
