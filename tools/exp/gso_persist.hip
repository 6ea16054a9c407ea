// Experiment (not built into the library): can PERSISTENT waves that keep one
// continuous segment pipeline across super-buffers reach the one-shot copy
// ceiling?  Copy-only, config 3 layout (as gso_order.hip).  Each unit is
// (super-buffer, group of G x 4 segment slots); a wave walks its slots of
// unit u, then of u + NB, ... with the next segment's loads always in flight
// (also across unit boundaries), the unit's "setup" modelled by one scalar
// load of a 48-B per-super-buffer record whose value feeds the addresses
// (so the dependency the real kernel has is present).
//   A3     one-shot blocks, G = 3 (the production structure)
//   P3/NB  persistent blocks, G = 3, grid NB (XCD-swizzled unit order)
//   C      one-shot waves, one segment each, global order
// usage: gso_persist
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_v4u;
typedef __attribute__((address_space(1))) unsigned char g_u8;

constexpr unsigned N = 1u << 18, IN_STRIDE = 65536, OUT_STRIDE = 73216, IN_LEN = 65535, H = 40, G = 1460;
constexpr unsigned NSEG = (IN_LEN - H + G - 1) / G, S = H + G;

struct Rec {  // per-super-buffer record (models plan + descriptor)
    uint64_t in_off, out_off;
    uint32_t w[8];
};

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

__device__ __forceinline__ void finish(const Seg &s, unsigned lane, const Front &f) {
    const uintptr_t oa = s.dst + H, ob = oa + s.dl;
    const uintptr_t c0 = (oa + 15) & ~(uintptr_t)15, c1 = ob & ~(uintptr_t)15;
    const unsigned nint = c1 > c0 ? (unsigned)((c1 - c0) >> 4) : 0u;
    if (lane < nint) *(g_v4u *)(c0 + 16u * lane) = f.a;
    if (lane + 64 < nint) *(g_v4u *)(c0 + 16u * (lane + 64)) = f.c;
    if (lane < H) *(g_u8 *)(s.dst + lane) = (unsigned char)f.hb;
    const unsigned he = (unsigned)(c0 - oa), ts = (unsigned)(c1 - oa);
    const unsigned off = lane < 16 ? lane : ts + lane - 16;
    const bool ok = lane < 16 ? lane < he : (lane < 32 && off < s.dl);
    if (ok) *(g_u8 *)(oa + off) = (unsigned char)f.eb;
}

__device__ __forceinline__ unsigned lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ unsigned wave_in_block() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
__device__ __forceinline__ unsigned swz(unsigned bx, unsigned nb) { return (bx & 7u) * (nb >> 3) + (bx >> 3); }

// A wave's position in its segment stream: unit u, segment i.
struct Pos {
    unsigned u, i;
    uintptr_t in, out;
};

template <unsigned GR>
__device__ __forceinline__ bool load_unit(const Rec *rec, const uint8_t *inb, uint8_t *outb, unsigned u, unsigned w,
                                          Pos &p) {
    const unsigned b = u / GR;
    const Rec r = rec[b];  // scalar load (uniform address)
    p.u = u;
    p.i = (u - b * GR) * 4u + w;
    p.in = reinterpret_cast<uintptr_t>(inb) + r.in_off;
    p.out = reinterpret_cast<uintptr_t>(outb) + r.out_off;
    return p.i < NSEG;
}

// persistent (or one-shot when NB == units) walk with a continuous ping-pong
template <unsigned GR>
__global__ __launch_bounds__(256) void kP(const Rec *rec, const uint8_t *in, uint8_t *out) {
    const unsigned nb = gridDim.x, units = N * GR;
    const unsigned lane = lane_id(), w = wave_in_block();
    const unsigned k = swz(blockIdx.x, nb);
    Pos cur;
    if (k >= units || !load_unit<GR>(rec, in, out, k, w, cur))
        return;
    Front fa, fb;
    issue(seg_of(cur.in, cur.out, cur.i), lane, fa);
    for (;;) {
        // next position: next slot of this unit, else the next unit
        Pos nx = cur;
        bool ok = true;
        nx.i += GR * 4u;
        if (nx.i >= NSEG) {
            const unsigned u1 = cur.u + nb;
            ok = u1 < units && load_unit<GR>(rec, in, out, u1, w, nx);
        }
        if (ok)
            issue(seg_of(nx.in, nx.out, nx.i), lane, fb);
        finish(seg_of(cur.in, cur.out, cur.i), lane, fa);
        if (!ok)
            break;
        cur = nx;
        fa = fb;
    }
}

__global__ __launch_bounds__(256) void kC(const Rec *rec, const uint8_t *in, uint8_t *out) {
    const unsigned nb = gridDim.x;
    const unsigned g = swz(blockIdx.x, nb) * 4u + wave_in_block();
    if (g >= N * NSEG) return;
    const unsigned b = g / NSEG, i = g - b * NSEG;
    const Rec r = rec[b];
    Front f;
    const Seg s = seg_of(reinterpret_cast<uintptr_t>(in) + r.in_off, reinterpret_cast<uintptr_t>(out) + r.out_off, i);
    issue(s, lane_id(), f);
    finish(s, lane_id(), f);
}

// C without the record load: addresses from the index alone
__global__ __launch_bounds__(256) void kC0(const Rec *, const uint8_t *in, uint8_t *out) {
    const unsigned nb = gridDim.x;
    const unsigned g = swz(blockIdx.x, nb) * 4u + wave_in_block();
    if (g >= N * NSEG) return;
    const unsigned b = g / NSEG, i = g - b * NSEG;
    Front f;
    const Seg s = seg_of(reinterpret_cast<uintptr_t>(in) + (uintptr_t)b * IN_STRIDE,
                         reinterpret_cast<uintptr_t>(out) + (uintptr_t)b * OUT_STRIDE, i);
    issue(s, lane_id(), f);
    finish(s, lane_id(), f);
}

int main() {
    uint8_t *in, *out;
    Rec *rec;
    hipMalloc(&in, (size_t)N * IN_STRIDE);
    hipMalloc(&out, (size_t)N * OUT_STRIDE);
    hipMalloc(&rec, sizeof(Rec) * N);
    hipMemset(in, 7, (size_t)N * IN_STRIDE);
    Rec *h = (Rec *)calloc(N, sizeof(Rec));
    for (unsigned b = 0; b < N; b++) {
        h[b].in_off = (uint64_t)b * IN_STRIDE;
        h[b].out_off = (uint64_t)b * OUT_STRIDE;
    }
    hipMemcpy(rec, h, sizeof(Rec) * N, hipMemcpyHostToDevice);
    const double bytes = (double)N * IN_LEN + (double)N * (IN_LEN - H + NSEG * H);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, auto launch) {
        for (int w = 0; w < 5; w++) launch();
        float sum = 0;
        for (int r = 0; r < 10; r++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            sum += ms;
        }
        printf("{\"variant\": \"%s\", \"ms_avg\": %.4f, \"TBps_avg\": %.3f}\n", name, sum / 10,
               bytes / (sum / 10 * 1e-3) / 1e12);
        fflush(stdout);
    };
    const unsigned nbc = ((N * NSEG + 3) / 4 + 7) & ~7u;
    for (int rep = 0; rep < 2; rep++) {
        run("A3 one-shot blocks G=3", [&] { hipLaunchKernelGGL(kP<3>, dim3(N * 3), dim3(256), 0, 0, rec, in, out); });
        run("A1 one-shot blocks G=1", [&] { hipLaunchKernelGGL(kP<1>, dim3(N), dim3(256), 0, 0, rec, in, out); });
        for (unsigned nbp : {1024u, 1280u, 2048u, 4096u, 16384u})
            run((std::string("P3 persistent G=3 NB=") + std::to_string(nbp)).c_str(),
                [&] { hipLaunchKernelGGL(kP<3>, dim3(nbp), dim3(256), 0, 0, rec, in, out); });
        for (unsigned nbp : {2048u, 4096u})
            run((std::string("P1 persistent G=1 NB=") + std::to_string(nbp)).c_str(),
                [&] { hipLaunchKernelGGL(kP<1>, dim3(nbp), dim3(256), 0, 0, rec, in, out); });
        run("C one-shot per segment (record load)", [&] { hipLaunchKernelGGL(kC, dim3(nbc), dim3(256), 0, 0, rec, in, out); });
        run("C0 one-shot per segment (no record)", [&] { hipLaunchKernelGGL(kC0, dim3(nbc), dim3(256), 0, 0, rec, in, out); });
    }
    printf("err=%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
