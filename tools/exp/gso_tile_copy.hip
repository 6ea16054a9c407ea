// Experiment (not built into the library): the copy ceiling of the row-order
// tile kernel's access shape (gso.hip gso_tile_kernel) on BASELINE config 3
// (262,144 x 65,535 B super-buffers at stride 65,536 -> 45 x 1,500 B
// segments at stride 73,216).  A 256-thread block per tile of K = 8 segments
// (12,000 B), lane t owning chunks t, t + 256, ... (U per lane): every output
// chunk ONE unaligned 16-B load from its payload source, stored whole; the
// header bytes carry whatever that load returned (no headers, no sums).
//   T<U, NT>: U chunks per lane (2, 3 -> K = 5 / 8 segments per tile), NT bit 1
//   non-temporal loads, bit 2 non-temporal stores.
// Prints one JSON line per variant: ms per launch and read + write TB/s.
// usage: gso_tile_copy [iters]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_v4u;
typedef __attribute__((address_space(1))) const v4u gc_v4u;

constexpr unsigned N = 1u << 18, IN_STRIDE = 65536, OUT_STRIDE = 73216, IN_LEN = 65535, H = 40, G = 1460;
constexpr unsigned S = H + G, NSEG = (IN_LEN - H + G - 1) / G, OUT_LEN = IN_LEN - H + NSEG * H;

template <int U, int NT>
__global__ __launch_bounds__(256) void tile_copy(const unsigned char *in, unsigned char *out, unsigned tiles) {
    constexpr unsigned K = (16u * 256u * U - 30u) / S;
    const unsigned ntiles = (NSEG + K - 1) / K;
    unsigned b = blockIdx.x;
    if (!(gridDim.x & 7u)) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
    const unsigned sb = b / tiles, tile = b % tiles;
    if (sb >= N || tile >= ntiles) return;
    const uintptr_t src = (uintptr_t)in + (uintptr_t)sb * IN_STRIDE, dst = (uintptr_t)out + (uintptr_t)sb * OUT_STRIDE;
    const unsigned seg0 = tile * K, Kt = NSEG - seg0 < K ? NSEG - seg0 : K;
    const unsigned tstart = seg0 * S, tend = seg0 + Kt == NSEG ? OUT_LEN : tstart + Kt * S;
    const unsigned c0 = tstart & ~15u, nch = ((tend + 15u) & ~15u) / 16u - c0 / 16u;
    v4u v[U];
#pragma unroll
    for (int k = 0; k < U; k++) {
        const unsigned ck = k * 256u + threadIdx.x;
        const unsigned q = c0 + 16u * (ck < nch ? ck : nch - 1u);
        const unsigned i = q / S;
        unsigned x = q - i * H;
        if (x + 16u > IN_LEN) x = IN_LEN - 16u;
        if (NT & 1) v[k] = __builtin_nontemporal_load(reinterpret_cast<gc_v4u *>(src + x));
        else v[k] = *reinterpret_cast<gc_v4u *>(src + x);
    }
#pragma unroll
    for (int k = 0; k < U; k++) {
        const unsigned ck = k * 256u + threadIdx.x;
        if (ck >= nch) continue;
        g_v4u *p = reinterpret_cast<g_v4u *>(dst + c0 + 16u * ck);
        if (NT & 2) __builtin_nontemporal_store(v[k], p);
        else *p = v[k];
    }
}

// Segment tiles with ONE chunk per lane: a block of B threads per tile of K
// whole segments (K = (16 B - 30) / S).  E bit: chunks in the tile's first /
// last 128-B line stored with the default policy (the neighbouring tiles'
// bytes share those lines), the rest non-temporal.
template <int B, int NT, int E>
__global__ __launch_bounds__(B) void tile1_copy(const unsigned char *in, unsigned char *out, unsigned tiles) {
    constexpr unsigned K = (16u * B - 30u) / S;
    const unsigned ntiles = (NSEG + K - 1) / K;
    unsigned b = blockIdx.x;
    if (!(gridDim.x & 7u)) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
    const unsigned sb = b / tiles, tile = b % tiles;
    if (sb >= N || tile >= ntiles) return;
    const uintptr_t src = (uintptr_t)in + (uintptr_t)sb * IN_STRIDE, dst = (uintptr_t)out + (uintptr_t)sb * OUT_STRIDE;
    const unsigned seg0 = tile * K, Kt = NSEG - seg0 < K ? NSEG - seg0 : K;
    const unsigned tstart = seg0 * S, tend = seg0 + Kt == NSEG ? OUT_LEN : tstart + Kt * S;
    const unsigned c0 = tstart & ~15u, nch = ((tend + 15u) & ~15u) / 16u - c0 / 16u;
    const unsigned ck = threadIdx.x;
    if (ck >= nch) return;
    const unsigned q = c0 + 16u * ck;
    const unsigned i = q / S;
    unsigned x = q - i * H;
    if (x + 16u > IN_LEN) x = IN_LEN - 16u;
    v4u v;
    if (NT & 1) v = __builtin_nontemporal_load(reinterpret_cast<gc_v4u *>(src + x));
    else v = *reinterpret_cast<gc_v4u *>(src + x);
    g_v4u *p = reinterpret_cast<g_v4u *>(dst + q);
    const bool edge = E && ((q >> 7) == (tstart >> 7) || (q >> 7) == ((tend - 1u) >> 7));
    if ((NT & 2) && !edge) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// The production split's shape (gso.hip gso_split_kernel: 3 blocks of 4 waves
// per super-buffer, 4 consecutive segments per wave with all their loads in
// flight, destination-aligned interior chunks, edge and header bytes one per
// lane), copy only.  P: 0 default policy; 1 non-temporal stores for chunks
// whose 128-B line lies inside the segment's interior (edge lines default);
// 2 = 1 + non-temporal loads for those chunks; 3 every chunk non-temporal.
template <int P, int SPW = 4, int BY = 1>
__global__ __launch_bounds__(256) void seg_copy(const unsigned char *in, unsigned char *out) {
    constexpr unsigned GRP = (NSEG + 4 * SPW - 1) / (4 * SPW);  // blocks per super-buffer
    unsigned b = blockIdx.x;
    if (!(gridDim.x & 7u)) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
    const unsigned sb = b / GRP, grp = b % GRP;
    if (sb >= N) return;
    const unsigned lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uintptr_t src = (uintptr_t)in + (uintptr_t)sb * IN_STRIDE, dst = (uintptr_t)out + (uintptr_t)sb * OUT_STRIDE;
    const unsigned s0 = (grp * 4u + wv) * SPW;
    v4u lo[SPW][2];
    unsigned eb[SPW];
#pragma unroll
    for (int k = 0; k < SPW; k++) {
        const unsigned i = s0 + k < NSEG ? s0 + k : NSEG - 1u;
        const unsigned dl = IN_LEN - H - i * G < G ? IN_LEN - H - i * G : G;
        const uintptr_t oa = dst + i * S + H, sa = src + H + i * G;
        const uintptr_t c0 = (oa + 15u) & ~(uintptr_t)15, c1 = (oa + dl) & ~(uintptr_t)15;
        const unsigned nint = c1 > c0 ? (unsigned)((c1 - c0) >> 4) : 0u;
        const uintptr_t base = c0 + (sa - oa);
        const unsigned last = nint ? nint - 1u : 0u;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const unsigned kk = lane + 64u * h < last ? lane + 64u * h : last;
            const uintptr_t a = base + 16u * kk;
            const uintptr_t la = (c0 + 16u * kk) & ~(uintptr_t)127;
            const bool inner = la >= c0 && la + 128u <= c1;
            if ((P == 3) || (P == 2 && inner)) lo[k][h] = __builtin_nontemporal_load(reinterpret_cast<gc_v4u *>(a));
            else lo[k][h] = *reinterpret_cast<gc_v4u *>(a);
        }
        const unsigned he = (unsigned)((c0 < oa + dl ? c0 : oa + dl) - oa), ts = (unsigned)((c1 > c0 ? c1 : c0) - oa);
        const unsigned xt = ts + lane - 16u;
        const unsigned eo = lane < 16u && lane < he ? lane : (lane >= 16u && lane < 32u && xt < dl ? xt : 0xffffffffu);
        eb[k] = eo != 0xffffffffu ? *reinterpret_cast<const unsigned char *>(sa + eo) : 0u;
    }
#pragma unroll
    for (int k = 0; k < SPW; k++) {
        const unsigned i = s0 + k;
        if (i >= NSEG) break;
        const unsigned dl = IN_LEN - H - i * G < G ? IN_LEN - H - i * G : G;
        const uintptr_t seg = dst + i * S, oa = seg + H;
        const uintptr_t c0 = (oa + 15u) & ~(uintptr_t)15, c1 = (oa + dl) & ~(uintptr_t)15;
        const unsigned nint = c1 > c0 ? (unsigned)((c1 - c0) >> 4) : 0u;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const unsigned kk = lane + 64u * h;
            if (kk < nint) {
                const uintptr_t a = c0 + 16u * kk;
                const uintptr_t la = a & ~(uintptr_t)127;
                const bool inner = la >= c0 && la + 128u <= c1;
                if (P == 3 || (P >= 1 && inner)) __builtin_nontemporal_store(lo[k][h], reinterpret_cast<g_v4u *>(a));
                else *reinterpret_cast<g_v4u *>(a) = lo[k][h];
            }
        }
        const unsigned he = (unsigned)((c0 < oa + dl ? c0 : oa + dl) - oa), ts = (unsigned)((c1 > c0 ? c1 : c0) - oa);
        const unsigned xt = ts + lane - 16u;
        const unsigned eo = lane < 16u && lane < he ? lane : (lane >= 16u && lane < 32u && xt < dl ? xt : 0xffffffffu);
        if (BY && eo != 0xffffffffu) *reinterpret_cast<unsigned char *>(oa + eo) = (unsigned char)eb[k];
        if (BY && lane < H) *reinterpret_cast<unsigned char *>(seg + lane) = *reinterpret_cast<const unsigned char *>(src + lane);
    }
}

// Row windows with the split's work added level by level (timing only: the
// header bytes and checksums written are placeholders):
//   V1  + a per-super-buffer record (scalar load) giving the geometry at run
//       time, chunk -> segment by a float reciprocal
//   V2  + each chunk's payload sum (whole chunks: 4 adds; chunks touching a
//       header or a payload end: byte masks), a two-key DPP reduction per
//       wave row, one non-returning global atomic per (wave, segment)
//   V3  + header bytes merged into the header chunks from an LDS image the
//       wave writes (lane j = byte j), header chunks stored default-policy
//   V4  + the atomic returns; the segment's last contributor stores the
//       2-byte checksum field (default policy) and clears its slot
struct XRec {
    unsigned hdr, gso, in_len, pad;
};
__device__ __forceinline__ unsigned xmask16(int lo, int hi) {
    lo = lo < 0 ? 0 : (lo > 16 ? 16 : lo);
    hi = hi < 0 ? 0 : (hi > 16 ? 16 : hi);
    return hi > lo ? ((1u << hi) - 1u) & ~((1u << lo) - 1u) : 0u;
}
__device__ __forceinline__ unsigned xexp(unsigned m16, int d) {
    const unsigned n = (m16 >> (4 * d)) & 15u, x = (n * 0x00204081u) & 0x01010101u;
    return (x << 8) - x;
}
__device__ __forceinline__ unsigned xwsum(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    return (unsigned)__builtin_amdgcn_readlane((int)v, 0) + (unsigned)__builtin_amdgcn_readlane((int)v, 16) +
           (unsigned)__builtin_amdgcn_readlane((int)v, 32) + (unsigned)__builtin_amdgcn_readlane((int)v, 48);
}
template <int V>
__global__ __launch_bounds__(256) void rowk(const unsigned char *in, unsigned char *out, unsigned rows,
                                            const XRec *recs, unsigned long long *slots) {
    __shared__ unsigned char img[4][192];
    unsigned b = blockIdx.x;
    if (!(gridDim.x & 7u)) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
    const unsigned sb = b / rows, row = b % rows;
    if (sb >= N) return;
    const unsigned lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uintptr_t src = (uintptr_t)in + (uintptr_t)sb * IN_STRIDE, dst = (uintptr_t)out + (uintptr_t)sb * OUT_STRIDE;
    const XRec r = recs[sb];
    const unsigned h = r.hdr, gso = r.gso, in_len = r.in_len, seg = h + gso;
    const unsigned nseg = (in_len - h + gso - 1u) / gso, olen = in_len - h + nseg * h;
    const unsigned o = (row * 256u + threadIdx.x) * 16u;
    const bool live = o < olen;
    const unsigned oc = live ? o : olen - 16u;
    const float rs = 1.0f / (float)seg;
    unsigned i = (unsigned)((float)oc * rs);
    i = i * seg > oc ? i - 1u : ((i + 1u) * seg <= oc ? i + 1u : i);
    const unsigned g = i * seg, dl = in_len - h - i * gso < gso ? in_len - h - i * gso : gso;
    const int q = (int)oc;
    const unsigned pm = live ? xmask16((int)(g + h) - q, (int)(g + h + dl) - q) : 0u;
    unsigned x = oc - i * h;
    if (x + 16u > in_len) x = in_len - 16u;
    v4u v = __builtin_nontemporal_load(reinterpret_cast<gc_v4u *>(src + (pm ? x : 0u)));
    unsigned hm = 0, hseg = i;
    if (V >= 3 && V <= 4) {
        hm = xmask16((int)g - q, (int)(g + h) - q);
        if (!hm && i + 1u < nseg) {
            hm = xmask16((int)(g + seg) - q, (int)(g + seg + h) - q);
            hseg = i + 1u;
        }
        // the wave's header image: the first segment starting in its 1 KiB row
        const unsigned w0 = row * 4096u + wv * 1024u;
        const unsigned sh = (w0 + seg - 1u) / seg, hs = sh * seg;
        if (hs < w0 + 1024u && hs < olen && lane < h)
            img[wv][(hs & 15u) + lane] = (unsigned char)(lane * 7u + sh);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (hm && live) {
            const unsigned hs2 = hseg * seg;
            const unsigned off = (hs2 & 15u) + (o - (hs2 & ~15u)) - (hs2 & 15u);
            v4u im = *reinterpret_cast<const v4u *>(&img[wv][off < 176u ? off & ~15u : 0u]);
            v = v4u{(v.x & xexp(pm, 0)) | (im.x & xexp(hm, 0)), (v.y & xexp(pm, 1)) | (im.y & xexp(hm, 1)),
                    (v.z & xexp(pm, 2)) | (im.z & xexp(hm, 2)), (v.w & xexp(pm, 3)) | (im.w & xexp(hm, 3))};
        }
    }
    if (live) {
        g_v4u *pp = reinterpret_cast<g_v4u *>(dst + o);
        if (V >= 3 && V <= 4 && hm) *pp = v;
        else __builtin_nontemporal_store(v, pp);
    }
    if (V == 6) {  // the atomics alone: one non-returning add per (wave, segment), constant values
        const unsigned kf = (unsigned)__builtin_amdgcn_readfirstlane((int)i);
        const unsigned kl = (unsigned)__builtin_amdgcn_readlane((int)i, 63);
        if (lane < 2u && (lane == 0u || kl != kf))
            __hip_atomic_fetch_add(slots + (size_t)sb * 48u + (lane ? kl : kf), (1ull << 48) | 7ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
    if (V >= 2 && V != 6) {
        unsigned lo = 0, hi = 0, c;
        if (pm == 0xffffu) {
            lo = __builtin_addc(lo, v.x, 0u, &c); hi += c;
            lo = __builtin_addc(lo, v.y, 0u, &c); hi += c;
            lo = __builtin_addc(lo, v.z, 0u, &c); hi += c;
            lo = __builtin_addc(lo, v.w, 0u, &c); hi += c;
        } else {
            lo = __builtin_addc(lo, v.x & xexp(pm, 0), 0u, &c); hi += c;
            lo = __builtin_addc(lo, v.y & xexp(pm, 1), 0u, &c); hi += c;
            lo = __builtin_addc(lo, v.z & xexp(pm, 2), 0u, &c); hi += c;
            lo = __builtin_addc(lo, v.w & xexp(pm, 3), 0u, &c); hi += c;
        }
        unsigned t = (lo & 0xffffu) + (lo >> 16) + hi;
        t = (t & 0xffffu) + (t >> 16);
        const unsigned kf = (unsigned)__builtin_amdgcn_readfirstlane((int)i);
        const unsigned kl = (unsigned)__builtin_amdgcn_readlane((int)i, 63);
        const unsigned s0 = xwsum(i == kf ? t : 0u), s1 = xwsum(i == kf ? 0u : t);
        if (lane < 2u && (lane == 0u || kl != kf)) {
            const unsigned k = lane ? kl : kf;
            unsigned long long *slot = slots + (size_t)sb * 48u + k;
            const unsigned long long add = (1ull << 48) | (lane ? s1 : s0);
            if (V == 5) {  // the sums and reductions alone: kept in LDS, no atomic
                reinterpret_cast<unsigned *>(img[wv])[lane] = (unsigned)add;
            } else if (V >= 4) {
                const unsigned long long old = atomicAdd(slot, add);
                if ((old >> 48) == 1ull) {  // placeholder completion rule (2 contributions)
                    *slot = 0ull;
                    const unsigned cs = ~(unsigned)((old + add) & 0xffffu) & 0xffffu;
                    *reinterpret_cast<unsigned short *>(dst + k * seg + 36u) = (unsigned short)cs;
                }
            } else {
                __hip_atomic_fetch_add(slot, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// Row windows (round 2's R0): a block of B threads per B x 16-B output window
// of the super-buffer (segments straddle windows), one chunk per thread.
template <int B, int NT>
__global__ __launch_bounds__(B) void row_copy(const unsigned char *in, unsigned char *out, unsigned rows) {
    unsigned b = blockIdx.x;
    if (!(gridDim.x & 7u)) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
    const unsigned sb = b / rows, row = b % rows;
    if (sb >= N) return;
    const uintptr_t src = (uintptr_t)in + (uintptr_t)sb * IN_STRIDE, dst = (uintptr_t)out + (uintptr_t)sb * OUT_STRIDE;
    const unsigned o = (row * B + threadIdx.x) * 16u;
    if (o >= OUT_LEN) return;
    const unsigned i = o / S;
    unsigned x = o - i * H;
    if (x + 16u > IN_LEN) x = IN_LEN - 16u;
    v4u v;
    if (NT & 1) v = __builtin_nontemporal_load(reinterpret_cast<gc_v4u *>(src + x));
    else v = *reinterpret_cast<gc_v4u *>(src + x);
    g_v4u *p = reinterpret_cast<g_v4u *>(dst + o);
    if (NT & 2) __builtin_nontemporal_store(v, p);
    else *p = v;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20;
    unsigned char *in, *out;
    hipMalloc(&in, (size_t)N * IN_STRIDE);
    hipMalloc(&out, (size_t)N * OUT_STRIDE);
    hipMemset(in, 1, (size_t)N * IN_STRIDE);
    hipMemset(out, 0, (size_t)N * OUT_STRIDE);
    const double alg = (double)N * (IN_LEN + OUT_LEN);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, unsigned tiles, const char *name, unsigned bs = 0) {
        const unsigned grid = N * tiles;
        if (!bs) {  // the block size from the variant's name: T1 kernels carry it in their template
            bs = 256;
            if (strstr(name, "192 threads")) bs = 192;
            if (strstr(name, "512 threads")) bs = 512;
            if (strstr(name, "768 threads")) bs = 768;
        }
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), 0, 0, in, out, tiles);
        hipEventRecord(e0);
        for (int w = 0; w < iters; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(bs), 0, 0, in, out, tiles);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms / iters, alg / (ms / iters * 1e-3) / 1e12);
    };
    auto runrow = [&](auto kern, unsigned B, const char *name) {
        const unsigned rows = (OUT_LEN + 16 * B - 1) / (16 * B);
        const unsigned grid = ((N * rows + 7) / 8) * 8;
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(B), 0, 0, in, out, rows);
        hipEventRecord(e0);
        for (int w = 0; w < iters; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(B), 0, 0, in, out, rows);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms / iters, alg / (ms / iters * 1e-3) / 1e12);
    };
    auto runseg = [&](auto kern, const char *name, unsigned grp = 3, unsigned lds = 0) {
        const unsigned grid = N * grp;
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, in, out);
        hipEventRecord(e0);
        for (int w = 0; w < iters; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, 0, in, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms / iters, alg / (ms / iters * 1e-3) / 1e12);
    };
    XRec *recs;
    unsigned long long *slots;
    hipMalloc(&recs, (size_t)N * sizeof(XRec));
    hipMalloc(&slots, (size_t)N * 48 * 8);
    hipMemset(slots, 0, (size_t)N * 48 * 8);
    {
        XRec *hr = (XRec *)malloc((size_t)N * sizeof(XRec));
        for (unsigned k = 0; k < N; k++) hr[k] = XRec{H, G, IN_LEN, 0};
        hipMemcpy(recs, hr, (size_t)N * sizeof(XRec), hipMemcpyHostToDevice);
        free(hr);
    }
    auto runv = [&](auto kern, const char *name) {
        const unsigned rows = (OUT_LEN + 4095) / 4096;
        const unsigned grid = ((N * rows + 7) / 8) * 8;
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out, rows, recs, slots);
        hipEventRecord(e0);
        for (int w = 0; w < iters; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out, rows, recs, slots);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, ms / iters, alg / (ms / iters * 1e-3) / 1e12);
    };
    if (argc > 2 && !strcmp(argv[2], "rowk")) {
        for (int rep = 0; rep < 2; rep++) {
            runrow(row_copy<256, 3>, 256, "R0 rows 4 KiB blocks nt both");
            runv(rowk<1>, "V1 + record, run-time geometry");
            runv(rowk<2>, "V2 + chunk sums, two-key reduction, atomics");
            runv(rowk<3>, "V3 + header merge from a wave LDS image");
            runv(rowk<4>, "V4 + returning atomics, last contributor stores the checksum");
            runv(rowk<5>, "V5 = V2 without the atomics (sums to LDS)");
            runv(rowk<6>, "V6 = V1 + the atomics alone (no sums)");
        }
        printf("{\"err\": \"%s\"}\n", hipGetErrorString(hipGetLastError()));
        return 0;
    }
    if (argc > 2 && !strcmp(argv[2], "occ")) {  // the split's shape at capped occupancy (dynamic LDS per block)
        for (int rep = 0; rep < 2; rep++) {
            runseg(seg_copy<0>, "S production shape, default policy");
            runseg(seg_copy<0>, "S, 6 blocks per CU (24 KiB LDS each)", 3, 24576);
            runseg(seg_copy<0>, "S, 5 blocks per CU (30 KiB LDS each)", 3, 30720);
            runseg(seg_copy<0>, "S, 4 blocks per CU (40 KiB LDS each)", 3, 40960);
            runseg(seg_copy<0>, "S, 3 blocks per CU (52 KiB LDS each)", 3, 53248);
            runseg(seg_copy<0, 1, 1>, "S1 one segment per wave, default", 12);
            runseg(seg_copy<0, 1, 1>, "S1, 5 blocks per CU", 12, 30720);
            runseg(seg_copy<0, 1, 1>, "S1, 4 blocks per CU", 12, 40960);
            runrow(row_copy<256, 3>, 256, "R0 rows 4 KiB blocks nt both");
        }
        printf("{\"err\": \"%s\"}\n", hipGetErrorString(hipGetLastError()));
        return 0;
    }
    const bool segs_only = argc > 2;
    for (int rep = 0; rep < 2; rep++) {
        runseg(seg_copy<0>, "S production shape, default policy");
        runseg(seg_copy<1>, "S production shape, nt stores on interior lines");
        runseg(seg_copy<2>, "S production shape, nt loads + stores on interior lines");
        runseg(seg_copy<3>, "S production shape, every chunk nt");
        runseg(seg_copy<0, 4, 0>, "S2 no byte stores, default");
        runseg(seg_copy<3, 4, 0>, "S2 no byte stores, every chunk nt");
        runseg(seg_copy<0, 1, 1>, "S1 one segment per wave, default", 12);
        runseg(seg_copy<3, 1, 0>, "S1 one segment per wave, no byte stores, nt", 12);
        runseg(seg_copy<0, 1, 0>, "S1 one segment per wave, no byte stores, default", 12);
        runrow(row_copy<256, 3>, 256, "R0 rows 4 KiB blocks nt both");
        if (segs_only) continue;
        run(tile1_copy<192, 3, 0>, 23, "T1 tiles of 2 segments, 192 threads, 1 chunk each, nt both");
        run(tile1_copy<192, 3, 1>, 23, "T1 192 threads, nt except the tile-edge lines");
        run(tile1_copy<192, 0, 0>, 23, "T1 192 threads, default policy");
        run(tile1_copy<256, 3, 1>, 23, "T1 tiles of 2 segments, 256 threads, nt except edge lines");
        run(tile1_copy<512, 3, 1>, 9, "T1 tiles of 5 segments, 512 threads, nt except edge lines");
        run(tile1_copy<768, 3, 1>, 6, "T1 tiles of 8 segments, 768 threads, nt except edge lines");
        runrow(row_copy<256, 0>, 256, "R0 rows 4 KiB blocks default");
        runrow(row_copy<256, 3>, 256, "R0 rows 4 KiB blocks nt both");
        runrow(row_copy<128, 3>, 128, "R0 rows 2 KiB blocks nt both");
        runrow(row_copy<512, 3>, 512, "R0 rows 8 KiB blocks nt both");
        runrow(row_copy<64, 3>, 64, "R0 rows 1 KiB blocks nt both");
        run(tile_copy<3, 0>, 6, "U3 default policy");
        run(tile_copy<3, 1>, 6, "U3 nt loads");
        run(tile_copy<3, 2>, 6, "U3 nt stores");
        run(tile_copy<3, 3>, 6, "U3 nt both");
        run(tile_copy<2, 0>, 9, "U2 default policy");
        run(tile_copy<4, 0>, 5, "U4 default policy");
    }
    printf("{\"err\": \"%s\"}\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
