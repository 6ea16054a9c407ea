// Experiment (not built into the library): do the byte stores cost the GSO
// split its last ~10 % to a plain copy?  Copy-only, config 3 layout
// (262,144 x 65,535 B in at stride 65,536 -> 45 segments of 1,500 B out at
// stride 73,216), one-shot waves, one segment each, global order:
//   C  header bytes and the <= 15-B payload head / tail by byte stores,
//      interior payload chunks by 16-B stores (the production split's
//      store pattern; tools/exp/gso_order.hip variant C)
//   D  every output byte by ONE aligned 16-B store: the wave of segment i
//      owns the aligned chunks that START in [seg_i, seg_i+1); a chunk mixing
//      header and payload bytes (segment i's header / payload head, or
//      segment i's payload tail + segment i+1's first header bytes) is
//      composed in registers from a payload-aligned and a header-aligned
//      16-B load with a per-byte select; only the super-buffer's last chunk
//      (past its output) uses byte stores.
// Both verified against a host copy of the same layout.  Then, to locate the
// segment-shaped copy's distance to the plain copy probe (same bytes):
//   Cn  C with non-temporal loads and stores
//   Ca  C with each segment's source moved to the destination's 16-B phase
//       (timing only: reads the same number of bytes, aligned alike)
//   Dn  D with non-temporal loads and stores
//   R   region-owning waves with per-segment sums (kR), Rn non-temporal
//   P   plain copy, 4 KiB per one-shot wave, default policy / Pn non-temporal
//       (the bench copy probe's structure), in -> out contiguous
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_v4u;
typedef __attribute__((address_space(1))) unsigned char g_u8;

constexpr unsigned N = 1u << 18, IN_STRIDE = 65536, OUT_STRIDE = 73216, IN_LEN = 65535, H = 40, G = 1460;
constexpr unsigned NSEG = (IN_LEN - H + G - 1) / G, S = H + G;
constexpr unsigned SLACK = 64;  // readable bytes before / after the input (header / payload over-reads in D)

__device__ __forceinline__ unsigned lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ unsigned wave_in_block() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ unsigned seg_dl(unsigned i) {
    const unsigned rest = IN_LEN - H - i * G;
    return rest < G ? rest : G;
}

// C: production store pattern (NT: non-temporal loads / stores; AL: source
// moved to the destination's 16-B phase, timing only)
template <bool NT, bool AL>
__global__ __launch_bounds__(256) void kCt(const unsigned char *in, unsigned char *out) {
    const unsigned nb = gridDim.x, bx = blockIdx.x;
    const unsigned vb = (bx & 7u) * (nb >> 3) + (bx >> 3);
    const unsigned g = vb * 4u + wave_in_block();
    if (g >= N * NSEG) return;
    const unsigned b = g / NSEG, i = g % NSEG, lane = lane_id();
    const unsigned char *hdr = in + (size_t)b * IN_STRIDE;
    unsigned char *dst = out + (size_t)b * OUT_STRIDE + (size_t)i * S;
    const unsigned char *src = hdr + H + (size_t)i * G;
    if constexpr (AL)
        src = hdr + (((size_t)i * G) & ~(size_t)15) + (((uintptr_t)dst + H) & 15u);
    const unsigned dl = seg_dl(i);
    const uintptr_t oa = (uintptr_t)dst + H, ob = oa + dl;
    const uintptr_t c0 = (oa + 15) & ~(uintptr_t)15, c1 = ob & ~(uintptr_t)15;
    const unsigned nint = c1 > c0 ? (unsigned)((c1 - c0) >> 4) : 0u;
    const uintptr_t base = (uintptr_t)src + (c0 - oa);
    const unsigned last = nint ? nint - 1 : 0u;
    v4u a, c;
    if constexpr (NT) {
        a = __builtin_nontemporal_load((const g_v4u *)(base + 16u * (lane < last ? lane : last)));
        c = __builtin_nontemporal_load((const g_v4u *)(base + 16u * (lane + 64 < last ? lane + 64 : last)));
    } else {
        a = *(const g_v4u *)(base + 16u * (lane < last ? lane : last));
        c = *(const g_v4u *)(base + 16u * (lane + 64 < last ? lane + 64 : last));
    }
    const unsigned hb = *(const g_u8 *)((uintptr_t)hdr + (lane < H ? lane : 0u));
    const unsigned he = (unsigned)(c0 - oa), ts = (unsigned)(c1 - oa);
    const unsigned off = lane < 16 ? lane : ts + lane - 16;
    const bool ok = lane < 16 ? lane < he : (lane < 32 && off < dl);
    const unsigned eb = *(const g_u8 *)((uintptr_t)src + (ok ? off : 0u));
    if constexpr (NT) {
        if (lane < nint) __builtin_nontemporal_store(a, (g_v4u *)(c0 + 16u * lane));
        if (lane + 64 < nint) __builtin_nontemporal_store(c, (g_v4u *)(c0 + 16u * (lane + 64)));
    } else {
        if (lane < nint) *(g_v4u *)(c0 + 16u * lane) = a;
        if (lane + 64 < nint) *(g_v4u *)(c0 + 16u * (lane + 64)) = c;
    }
    if (lane < H) *(g_u8 *)((uintptr_t)dst + lane) = (unsigned char)hb;
    if (ok) *(g_u8 *)(oa + off) = (unsigned char)eb;
}

// P: plain copy of nbytes (multiple of 16), 4 KiB per one-shot wave
template <bool NT>
__global__ __launch_bounds__(256) void kP(const unsigned char *in, unsigned char *out, size_t nch) {
    const unsigned nb = gridDim.x, bx = blockIdx.x;
    const size_t vb = (size_t)(bx & 7u) * (nb >> 3) + (bx >> 3);
    const size_t c0 = (vb * 4u + wave_in_block()) * 256u;
    const unsigned lane = lane_id();
    v4u v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const size_t c = c0 + 64u * u + lane;
        const g_v4u *q = (const g_v4u *)(in + 16u * (c < nch ? c : nch - 1));
        v[u] = NT ? __builtin_nontemporal_load(q) : *q;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const size_t c = c0 + 64u * u + lane;
        if (c < nch) {
            g_v4u *q = (g_v4u *)(out + 16u * c);
            if (NT)
                __builtin_nontemporal_store(v[u], q);
            else
                *q = v[u];
        }
    }
}

// select bytes of h where the byte's bit in m (16 bits) is set, else p
__device__ __forceinline__ v4u sel_bytes(v4u p, v4u h, unsigned m) {
    auto dm = [](unsigned m4) {  // 4 mask bits -> byte mask
        return ((m4 & 1u) ? 0xffu : 0u) | ((m4 & 2u) ? 0xff00u : 0u) | ((m4 & 4u) ? 0xff0000u : 0u) |
               ((m4 & 8u) ? 0xff000000u : 0u);
    };
    const unsigned m0 = dm(m & 15u), m1 = dm((m >> 4) & 15u), m2 = dm((m >> 8) & 15u), m3 = dm(m >> 12);
    return v4u{(p.x & ~m0) | (h.x & m0), (p.y & ~m1) | (h.y & m1), (p.z & ~m2) | (h.z & m2), (p.w & ~m3) | (h.w & m3)};
}

// D: every byte by one aligned 16-B store (segment starts are 4-B aligned here:
// S = 1,500 and the super-buffer stride are multiples of 4; the chunk
// composition itself works at any byte offset)
template <bool NT>
__device__ __forceinline__ void d_chunk(const unsigned char *hdr, const unsigned char *src, uintptr_t sd,
                                        unsigned dl, bool lastseg, unsigned k, uintptr_t c0) {
    // chunk k of the segment's ownership range: start cA = c0 + 16k, c0 the first aligned address >= sd
    const uintptr_t cA = c0 + 16u * k;
    const unsigned rel = (unsigned)(cA - sd);          // offset of the chunk start in segment i (>= 0)
    const g_v4u *pq = (const g_v4u *)((uintptr_t)src + rel - H);  // payload-aligned (bytes rel..rel+15 of segment i as payload)
    const v4u P = NT ? __builtin_nontemporal_load(pq) : *pq;
    // header bytes: of segment i when rel < H, else of segment i+1 (at offset rel - S, may be negative)
    // (chunks without header bytes read the template's first chunk: in bounds)
    const int hrel = rel < H ? (int)rel : (rel + 16u > S ? (int)rel - (int)S : 0);
    const v4u Hd = *(const g_v4u *)((intptr_t)hdr + hrel);
    // header byte positions: the first H - rel (segment i's header), the last
    // rel + 16 - S (segment i+1's), as a 16-bit mask
    const unsigned nlo = rel < H ? (H - rel < 16u ? H - rel : 16u) : 0u;
    const unsigned nhi = (!lastseg && rel + 16u > S) ? rel + 16u - S : 0u;
    const unsigned m = ((1u << nlo) - 1u) | (0xffffu & ~((1u << (16u - nhi)) - 1u));
    const v4u v = sel_bytes(P, Hd, m);
    const unsigned end = H + dl;  // bytes of segment i
    if (!lastseg || rel + 16u <= end) {
        if (NT)
            __builtin_nontemporal_store(v, (g_v4u *)cA);
        else
            *(g_v4u *)cA = v;
    } else {  // the super-buffer's last, partial chunk
        const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (unsigned q = 0; q < 16; q++)
            if (rel + q < end) *(g_u8 *)(cA + q) = (unsigned char)(w[q >> 2] >> (8u * (q & 3u)));
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void kD(const unsigned char *in, unsigned char *out) {
    const unsigned nb = gridDim.x, bx = blockIdx.x;
    const unsigned vb = (bx & 7u) * (nb >> 3) + (bx >> 3);
    const unsigned g = vb * 4u + wave_in_block();
    if (g >= N * NSEG) return;
    const unsigned b = g / NSEG, i = g % NSEG, lane = lane_id();
    const unsigned char *hdr = in + (size_t)b * IN_STRIDE;
    const unsigned char *src = hdr + H + (size_t)i * G;
    const uintptr_t sd = (uintptr_t)out + (size_t)b * OUT_STRIDE + (size_t)i * S;
    const unsigned dl = seg_dl(i);
    const bool lastseg = i + 1 == NSEG;
    const uintptr_t c0 = (sd + 15) & ~(uintptr_t)15;                  // first chunk starting in the segment
    const uintptr_t cend = lastseg ? sd + H + dl : sd + S;             // ownership ends (exclusive)
    const unsigned nch = (unsigned)((cend - c0 + 15) >> 4);
    // segment 0 of a super-buffer starts aligned here (OUT_STRIDE % 16 == 0), so no chunk before c0 is ours
    if (lane < nch) d_chunk<NT>(hdr, src, sd, dl, lastseg, lane, c0);
    if (lane + 64 < nch) d_chunk<NT>(hdr, src, sd, dl, lastseg, lane + 64, c0);
}


// R: region-owning waves (the next-step design): wave = one 4-KiB region of a
// super-buffer's output, every byte by an aligned 16-B store (composed as in
// D); the wave that holds a segment's start also loads that segment's whole
// payload and sums it (bytes the neighbouring region's wave loads too: L2),
// the sum stored per segment.
constexpr unsigned RB = 4096, OUT_LEN = (NSEG - 1) * S + H + (IN_LEN - H - (NSEG - 1) * G);
constexpr unsigned NREG = (OUT_LEN + RB - 1) / RB;

__device__ __forceinline__ unsigned wsum64(unsigned v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <bool NT>
__global__ __launch_bounds__(256) void kR(const unsigned char *in, unsigned char *out, unsigned *sums) {
    const unsigned nb = gridDim.x, bx = blockIdx.x;
    const unsigned vb = (bx & 7u) * (nb >> 3) + (bx >> 3);
    const unsigned g = vb * 4u + wave_in_block();
    if (g >= N * NREG) return;
    const unsigned b = g / NREG, r = g % NREG, lane = lane_id();
    const unsigned char *hdr = in + (size_t)b * IN_STRIDE;
    const uintptr_t ob = (uintptr_t)out + (size_t)b * OUT_STRIDE;
    const unsigned R0 = r * RB, R1 = R0 + RB < OUT_LEN ? R0 + RB : OUT_LEN;
#pragma unroll
    for (unsigned u = 0; u < 4; u++) {
        const unsigned off = R0 + 16u * (lane + 64u * u);
        if (off < R1) {
            const unsigned j = off / S, rel = off - j * S;
            const unsigned char *src = hdr + H + (size_t)j * G;
            d_chunk<NT>(hdr, src, ob + (size_t)j * S, seg_dl(j), j + 1 == NSEG, 0, ob + off);
            (void)rel;
        }
    }
    // sums of the segments starting in [R0, R1)
    const unsigned j0 = (R0 + S - 1) / S, j1 = (R1 + S - 1) / S;
    for (unsigned j = j0; j < j1 && j < NSEG; j++) {
        const unsigned char *src = hdr + H + (size_t)j * G;
        const unsigned dl = seg_dl(j), nc = (dl + 15u) / 16u;
        unsigned acc = 0;
        for (unsigned k = lane; k < nc; k += 64) {
            const v4u v = NT ? __builtin_nontemporal_load((const g_v4u *)(src + 16u * k)) : *(const g_v4u *)(src + 16u * k);
            const unsigned nbytes = dl - 16u * k < 16u ? dl - 16u * k : 16u;
            const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (unsigned q = 0; q < 4; q++) {
                const unsigned kb = nbytes > 4u * q ? (nbytes - 4u * q < 4u ? nbytes - 4u * q : 4u) : 0u;
                const unsigned x = w[q] & (unsigned)((1ull << (8u * kb)) - 1ull);
                acc += (x & 0xffffu) + (x >> 16);
            }
        }
        acc = wsum64(acc);
        if (lane == 0) sums[(size_t)b * NSEG + j] = acc;
    }
}

int main(int argc, char **argv) {
    const bool verify = argc > 1 && atoi(argv[1]);
    unsigned char *inb, *out;
    const size_t in_bytes = (size_t)N * IN_STRIDE, out_bytes = (size_t)N * OUT_STRIDE;
    hipMalloc(&inb, in_bytes + 2 * SLACK);
    hipMalloc(&out, out_bytes);
    unsigned *sums;
    hipMalloc(&sums, sizeof(unsigned) * N * NSEG);
    unsigned char *in = inb + SLACK;
    {
        std::vector<unsigned char> h(in_bytes);
        unsigned x = 12345;
        for (size_t k = 0; k < in_bytes; k++) { x = x * 1664525u + 1013904223u; h[k] = (unsigned char)(x >> 24); }
        hipMemcpy(in, h.data(), in_bytes, hipMemcpyHostToDevice);
    }
    const double bytes = (double)N * IN_LEN + (double)N * (IN_LEN - H + NSEG * H);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const unsigned nbk = ((N * NSEG + 3) / 4 + 7) & ~7u;
    auto check = [&](const char *name) {
        if (!verify) return;
        std::vector<unsigned char> hi(in_bytes), ho(out_bytes);
        hipMemcpy(hi.data(), in, in_bytes, hipMemcpyDeviceToHost);
        hipMemcpy(ho.data(), out, out_bytes, hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (unsigned b = 0; b < N; b += 97)
            for (unsigned i = 0; i < NSEG; i++) {
                const unsigned char *hh = &hi[(size_t)b * IN_STRIDE];
                const unsigned char *o = &ho[(size_t)b * OUT_STRIDE + (size_t)i * S];
                const unsigned dl = IN_LEN - H - i * G < G ? IN_LEN - H - i * G : G;
                bad += memcmp(o, hh, H) != 0;
                bad += memcmp(o + H, hh + H + (size_t)i * G, dl) != 0;
            }
        printf("{\"verify\": \"%s\", \"bad_segments\": %zu}\n", name, bad);
    };
    auto run = [&](const char *name, auto launch, double nbytes = 0) {
        if (nbytes == 0) nbytes = bytes;
        hipMemset(out, 0, out_bytes);
        for (int w = 0; w < 3; w++) launch();
        check(name);
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
               nbytes / (sum / 10 * 1e-3) / 1e12);
        fflush(stdout);
    };
    for (int rep = 0; rep < 3; rep++) {
        run("C byte stores for header + edges", [&] { hipLaunchKernelGGL((kCt<false, false>), dim3(nbk), dim3(256), 0, 0, in, out); });
        run("D aligned 16-B stores only", [&] { hipLaunchKernelGGL(kD<false>, dim3(nbk), dim3(256), 0, 0, in, out); });
        run("Dn D non-temporal", [&] { hipLaunchKernelGGL(kD<true>, dim3(nbk), dim3(256), 0, 0, in, out); });
        const unsigned rbk = ((N * NREG + 3) / 4 + 7) & ~7u;
        run("R region waves + segment sums", [&] { hipLaunchKernelGGL(kR<false>, dim3(rbk), dim3(256), 0, 0, in, out, sums); });
        run("Rn R non-temporal", [&] { hipLaunchKernelGGL(kR<true>, dim3(rbk), dim3(256), 0, 0, in, out, sums); });
        if (!verify) {
            run("Cn C non-temporal", [&] { hipLaunchKernelGGL((kCt<true, false>), dim3(nbk), dim3(256), 0, 0, in, out); });
            run("Ca C source in the destination's 16-B phase", [&] { hipLaunchKernelGGL((kCt<false, true>), dim3(nbk), dim3(256), 0, 0, in, out); });
            // the whole input copied (2 x 17.18 GB moved; C moves 34.84 GB)
            const size_t nch = in_bytes / 16;
            const unsigned pbk = (unsigned)(((nch + 1023) / 1024 + 7) & ~(size_t)7);
            run("P plain copy 4 KiB/wave", [&] { hipLaunchKernelGGL(kP<false>, dim3(pbk), dim3(256), 0, 0, in, out, nch); },
                2.0 * in_bytes);
            run("Pn plain copy 4 KiB/wave non-temporal", [&] { hipLaunchKernelGGL(kP<true>, dim3(pbk), dim3(256), 0, 0, in, out, nch); },
                2.0 * in_bytes);
        }
    }
    printf("err=%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
