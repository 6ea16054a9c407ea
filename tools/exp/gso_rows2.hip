// Experiment (not built into the library): is a ROW-ORDER GSO split worth
// building?  Config 3 geometry (262,144 x 65,535 B super-buffers, H = 40,
// G = 1460, output stride 73,216 B).  One 256-thread block per 4 KiB output
// region (17 per super-buffer), one 16-B output chunk per thread, source
// byte for output offset o in segment s = in + o - s*H.  Variants add the
// real kernel's costs one at a time:
//   R0  copy only (nt loads + stores, XCD swizzle)
//   R1  + a per-super-buffer record (scalar load) feeding the addresses
//   R2  + the chunk staged through LDS (write, barrier, read) before its store
//   R3  + per-segment payload sums: masked chunk sums, per-wave reduction over
//         its <= 2 segments, LDS atomics per block, slot writes (workspace)
//   R4  + the header bytes: the wave whose 1 KiB window holds a segment's
//         header builds it (lane j = byte j, 7 field values by writelane +
//         ds_bpermute) and writes it into the LDS window before the read-back
//   P2  pass 2 alone: thread per segment, reads its 1-2 slots + the record,
//       stores the 2-byte checksum
// usage: gso_rows2 [iters]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_v4u;
typedef __attribute__((address_space(1))) const v4u gc_v4u;

constexpr unsigned N = 1u << 18, IN_STRIDE = 65536, OUT_STRIDE = 73216, IN_LEN = 65535, H = 40, G = 1460;
constexpr unsigned S = H + G, NSEG = (IN_LEN - H + G - 1) / G, OUT_LEN = IN_LEN - H + NSEG * H;
constexpr unsigned ROWS = (OUT_LEN + 4095) / 4096;  // 17
constexpr unsigned SLOTS = 8;                      // partial-sum slots per region

struct Rec {
    uint64_t in_off, out_off;
    uint32_t w[4];
};

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor((int)v, o);
    return v;
}
__device__ __forceinline__ unsigned fold16(unsigned long long x) {
    unsigned long long t = (x & 0xffffffffull) + (x >> 32);
    unsigned u = (unsigned)(t & 0xffff) + (unsigned)((t >> 16) & 0xffff) + (unsigned)(t >> 32);
    u = (u & 0xffff) + (u >> 16);
    return (u & 0xffff) + (u >> 16);
}
extern "C" __device__ int wl_i32(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

__device__ __forceinline__ unsigned wsum_dpp(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    return (unsigned)__builtin_amdgcn_readlane((int)v, 0) + (unsigned)__builtin_amdgcn_readlane((int)v, 16) +
           (unsigned)__builtin_amdgcn_readlane((int)v, 32) + (unsigned)__builtin_amdgcn_readlane((int)v, 48);
}
__device__ __forceinline__ unsigned keep(unsigned p, unsigned lo, unsigned hi) {  // bytes of dword at p in [lo, hi)
    const int a = (int)lo - (int)p, b = (int)hi - (int)p;
    const unsigned mh = b >= 4 ? ~0u : (b <= 0 ? 0u : (1u << (8 * b)) - 1u);
    const unsigned ml = a >= 4 ? ~0u : (a <= 0 ? 0u : (1u << (8 * a)) - 1u);
    return mh & ~ml;
}

// R5: wave-level windows: efficient dword-masked sums, DPP reductions, one
// global atomic per (wave, segment) into a zero-kept slot array (count in
// bits 24+), header built by the wave holding it, wave-local LDS staging.
__global__ __launch_bounds__(256) void rows5(const unsigned char *in, unsigned char *out, const Rec *recs,
                                             unsigned *slots) {
    __shared__ v4u win[256];
    unsigned b = blockIdx.x;
    if (!(gridDim.x & 7u)) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
    const unsigned sb = b / ROWS, row = b % ROWS;
    const Rec r = recs[sb];
    const uintptr_t src = (uintptr_t)in + r.in_off, dst = (uintptr_t)out + r.out_off;
    const unsigned hdr = r.w[0] & 0xffff, gso = r.w[0] >> 16, out_len = r.w[1];
    const unsigned seg = hdr + gso;
    const unsigned t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const unsigned w0 = row * 4096 + wv * 1024;
    if (w0 >= out_len) return;
    const unsigned o = w0 + 16 * lane;
    const bool live = o < out_len;
    const unsigned oc = live ? o : out_len - 16;
    const unsigned shi = (oc + 15) / seg, phi = oc + 15 - shi * seg;
    const unsigned s = phi < hdr && shi ? shi - 1 : shi;
    unsigned sp = oc - s * hdr;
    if (sp + 16 > IN_LEN) sp = IN_LEN - 16;
    v4u v = __builtin_nontemporal_load(reinterpret_cast<gc_v4u *>(src + sp));
    // payload bytes of segment s: positions [hdr, min(seg, out_len - s*seg)) relative to s*seg
    const unsigned pos0 = oc - s * seg;
    const unsigned pend = (out_len - s * seg) < seg ? out_len - s * seg : seg;
    unsigned lo = 0, hi = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const unsigned w = v[d] & keep(pos0 + 4 * d, hdr, pend);
        unsigned c;
        lo = __builtin_addc(lo, w, 0u, &c);
        hi += c;
    }
    unsigned ps = live ? fold16(((unsigned long long)hi << 32) | lo) : 0u;
    // header of the (at most one) segment starting in this window
    const unsigned sh = (w0 + seg - 1) / seg, hs = sh * seg;
    win[t] = v;
    if (hs < w0 + 1024 && hs < out_len) {
        const unsigned pkt = hs + seg <= out_len ? seg : out_len - hs;
        unsigned tbl = 0;
        tbl = (unsigned)wl_i32((int)pkt, 1, (int)tbl);
        tbl = (unsigned)wl_i32((int)(0x1234 + sh), 2, (int)tbl);
        tbl = (unsigned)wl_i32((int)(~(pkt + sh) & 0xffff), 3, (int)tbl);
        tbl = (unsigned)wl_i32((int)(0x55aa0000u + gso * sh), 5, (int)tbl);
        tbl = (unsigned)wl_i32((int)(sh + 1 == NSEG ? 0x19 : 0x10), 7, (int)tbl);
        const unsigned code = lane == 2 || lane == 3 ? 1 : lane == 4 || lane == 5 ? 2 : lane == 10 || lane == 11 ? 3
                              : lane >= 24 && lane < 28 ? 5 : lane == 33 ? 7 : 0;
        const unsigned r0 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(code << 2), (int)tbl);
        const unsigned byte = code ? (r0 >> (8 * (lane & 1))) & 0xff : lane * 7u;
        const unsigned pos = hs + lane - w0;
        __builtin_amdgcn_wave_barrier();
        if (lane < hdr && pos < 1024)
            reinterpret_cast<unsigned char *>(&win[wv * 64])[pos] = (unsigned char)byte;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        v = win[t];
    }
    if (live)
        __builtin_nontemporal_store(v, reinterpret_cast<g_v4u *>(dst + o));
    // per-segment partials: lanes hold segment s0 or s0 + 1
    const unsigned s0 = __builtin_amdgcn_readfirstlane(s);
    const unsigned pa = wsum_dpp(s == s0 ? ps : 0u), pb = wsum_dpp(s != s0 ? ps : 0u);
    if (lane < 2) {
        const unsigned ss = s0 + lane;
        const unsigned add = (1u << 24) + (lane ? pb : pa);
        unsigned *slot = slots + (size_t)sb * 48 + ss;
        const unsigned old = atomicAdd(slot, add);
        if ((old >> 24) == 1u) {  // second contributor: finish (checksum store), keep the slot zeroed
            const unsigned c = ~fold16((old & 0xffffff) + (add & 0xffffff)) & 0xffffu;
            atomicExch(slot, 0u);
            unsigned char *pp = out + r.out_off + (size_t)ss * seg + 36;
            pp[0] = (unsigned char)c;
            pp[1] = (unsigned char)(c >> 8);
        }
    }
}

template <int V>
__global__ __launch_bounds__(256) void rows(const unsigned char *in, unsigned char *out, const Rec *recs,
                                            unsigned *slots) {
    __shared__ v4u win[256];
    __shared__ unsigned ssum[SLOTS];
    unsigned b = blockIdx.x;
    if (!(gridDim.x & 7u)) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
    const unsigned sb = b / ROWS, row = b % ROWS;
    uintptr_t src = (uintptr_t)in + (uintptr_t)sb * IN_STRIDE;
    uintptr_t dst = (uintptr_t)out + (uintptr_t)sb * OUT_STRIDE;
    unsigned hdr = H, gso = G, out_len = OUT_LEN;
    if (V >= 1) {
        const Rec r = recs[sb];
        src = (uintptr_t)in + r.in_off;
        dst = (uintptr_t)out + r.out_off;
        hdr = r.w[0] & 0xffff;
        gso = r.w[0] >> 16;
        out_len = r.w[1];
    }
    const unsigned seg = hdr + gso;
    const unsigned t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    if (V >= 3 && t < SLOTS) ssum[t] = 0;
    const unsigned k = row * 256 + t;
    const unsigned o = 16 * k;
    const bool live = o < out_len;
    const unsigned oc = live ? o : out_len - 16;
    const unsigned shi = (oc + 15) / seg, phi = oc + 15 - shi * seg;
    const unsigned s = phi < hdr && shi ? shi - 1 : shi;
    unsigned sp = oc - s * hdr;
    if (sp + 16 > IN_LEN) sp = IN_LEN - 16;
    v4u v = __builtin_nontemporal_load(reinterpret_cast<gc_v4u *>(src + sp));
    if (V >= 2) {
        win[t] = v;
        if (V >= 4) {
            // this wave's 1 KiB window [w0, w0 + 1024) holds at most one header
            const unsigned w0 = row * 4096 + wv * 1024;
            const unsigned sh = (w0 + seg - 1) / seg;  // first segment starting at or after w0
            const unsigned hs = sh * seg;
            if (hs < w0 + 1024 && hs < out_len) {
                const unsigned pkt = sh + 1 < (out_len + seg - 1) / seg ? seg : out_len - hs;
                unsigned tbl = 0;
                tbl = (unsigned)wl_i32((int)pkt, 1, (int)tbl);
                tbl = (unsigned)wl_i32((int)(0x1234 + sh), 2, (int)tbl);
                tbl = (unsigned)wl_i32((int)(~(pkt + sh) & 0xffff), 3, (int)tbl);
                tbl = (unsigned)wl_i32((int)(0x55aa0000u + gso * sh), 5, (int)tbl);
                tbl = (unsigned)wl_i32((int)(sh + 1 == NSEG ? 0x19 : 0x10), 7, (int)tbl);
                const unsigned code = lane == 2 || lane == 3 ? 1 : lane == 4 || lane == 5 ? 2 : lane == 10 || lane == 11 ? 3
                                      : lane >= 24 && lane < 28 ? 5 : lane == 33 ? 7 : 0;
                const unsigned r0 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(code << 2), (int)tbl);
                const unsigned byte = code ? (r0 >> (8 * (lane & 1))) & 0xff : lane * 7u;
                const unsigned pos = hs + lane - row * 4096;  // position in the block's 4 KiB window
                __syncthreads();
                if (lane < hdr && pos < 4096)
                    reinterpret_cast<unsigned char *>(win)[pos] = (unsigned char)byte;
            } else {
                __syncthreads();
            }
        }
        __syncthreads();
        v = win[t];
    }
    if (V >= 3) {
        // payload bytes of segment s in this chunk: positions >= hdr within s
        const unsigned pos0 = oc - s * seg;  // may exceed seg - 1 only for the header-of-next part
        unsigned sum = 0;
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const unsigned w = v[d];
#pragma unroll
            for (int bb = 0; bb < 4; bb++) {
                const unsigned p = pos0 + 4 * d + bb;
                const bool pay = p >= hdr && p < seg && oc + 4 * d + bb < out_len;
                sum += pay ? ((w >> (8 * bb)) & 0xffu) << (8 * (bb & 1)) : 0u;
            }
        }
        if (!live) sum = 0;
        const unsigned s0 = __builtin_amdgcn_readfirstlane(s);
        const unsigned lo = wave_sum(s == s0 ? sum : 0u), hi = wave_sum(s != s0 ? sum : 0u);
        const unsigned base = row * 4096 / seg;
        if (lane == 0) {
            atomicAdd(&ssum[(s0 - base) & (SLOTS - 1)], lo);
            atomicAdd(&ssum[(s0 + 1 - base) & (SLOTS - 1)], hi);
        }
        __syncthreads();
        if (t < SLOTS) slots[(size_t)b * SLOTS + t] = fold16(ssum[t]);
    }
    if (live)
        __builtin_nontemporal_store(v, reinterpret_cast<g_v4u *>(dst + o));
}

__global__ __launch_bounds__(256) void pass2(unsigned char *out, const Rec *recs, const unsigned *slots) {
    const unsigned long gid = (unsigned long)blockIdx.x * 256 + threadIdx.x;
    const unsigned sb = gid / 48, i = gid % 48;
    if (sb >= N || i >= NSEG) return;
    const Rec r = recs[sb];
    const unsigned seg = (r.w[0] & 0xffff) + (r.w[0] >> 16);
    const unsigned first = i * seg, last = first + seg - 1;
    const unsigned r0 = first / 4096, r1 = last / 4096;
    unsigned t = slots[((size_t)sb * ROWS + r0) * SLOTS + ((i - r0 * 4096 / seg) & (SLOTS - 1))];
    if (r1 != r0 && r1 < ROWS) t += slots[((size_t)sb * ROWS + r1) * SLOTS + ((i - r1 * 4096 / seg) & (SLOTS - 1))];
    const unsigned c = ~fold16(t + r.w[2] + i) & 0xffff;
    unsigned char *p = out + r.out_off + first + 36;
    p[0] = (unsigned char)c;
    p[1] = (unsigned char)(c >> 8);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 10;
    unsigned char *in, *out;
    Rec *recs;
    unsigned *slots;
    hipMalloc(&in, (size_t)N * IN_STRIDE);
    hipMalloc(&out, (size_t)N * OUT_STRIDE);
    hipMalloc(&recs, (size_t)N * sizeof(Rec));
    hipMalloc(&slots, (size_t)N * ROWS * SLOTS * 4);
    hipMemset(in, 1, (size_t)N * IN_STRIDE);
    Rec *h = (Rec *)malloc((size_t)N * sizeof(Rec));
    for (unsigned i = 0; i < N; i++) {
        h[i].in_off = (uint64_t)i * IN_STRIDE;
        h[i].out_off = (uint64_t)i * OUT_STRIDE;
        h[i].w[0] = H | (G << 16);
        h[i].w[1] = OUT_LEN;
        h[i].w[2] = 0x1234;
        h[i].w[3] = 0;
    }
    hipMemcpy(recs, h, (size_t)N * sizeof(Rec), hipMemcpyHostToDevice);
    const double alg = (double)N * (IN_LEN + OUT_LEN);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, unsigned grid, const char *name, double bytes) {
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out, recs, slots);
        hipEventRecord(e0);
        for (int w = 0; w < iters; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out, recs, slots);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms / iters, bytes / (ms / iters * 1e-3) / 1e9);
    };
    for (int rep = 0; rep < 2; rep++) {
        run(rows<0>, N * ROWS, "R0 copy", alg);
        run(rows<1>, N * ROWS, "R1 +record", alg);
        run(rows<2>, N * ROWS, "R2 +LDS stage", alg);
        run(rows<3>, N * ROWS, "R3 +sums/slots", alg);
        run(rows<4>, N * ROWS, "R4 +headers", alg);
        hipMemset(slots, 0, (size_t)N * ROWS * SLOTS * 4);
        run(rows5, N * ROWS, "R5 wave windows, efficient sums, atomic finish", alg);
        auto p2 = [](unsigned char *, unsigned char *o, const Rec *r, unsigned *s) {};
        (void)p2;
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(pass2, dim3(N * 48 / 256), dim3(256), 0, 0, out, recs, slots);
        hipEventRecord(e0);
        for (int w = 0; w < iters; w++) hipLaunchKernelGGL(pass2, dim3(N * 48 / 256), dim3(256), 0, 0, out, recs, slots);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"P2 pass 2\", \"ms\": %.4f}\n", ms / iters);
    }
    printf("err=%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
