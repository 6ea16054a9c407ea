// Experiment (not built into the library): a GSO split with the whole
// super-buffer staged in LDS.  Config 3 geometry (262,144 x 65,535 B
// super-buffers at a 65,536-B input stride, H = 40, G = 1460, 45 segments,
// output stride 73,216 B).  One block per super-buffer:
//   phase 1  the input (4,096 aligned 16-B chunks) -> LDS by global_load_lds
//            (16 B per lane, no VGPRs), one barrier;
//   phase 2  (variant >= 1) per-segment payload sums from LDS, a wave per
//            segment, the 40-B header (template + checksum) into an LDS
//            header area; barrier;
//   phase 3  the output written in ROW order: thread t stores 16-B output
//            chunks t, t + 256, ...; a chunk inside one segment's payload is
//            two 8-B-aligned ds_read_b64 (source offset o - 40 s is a
//            multiple of 8), chunks with header bytes or a segment boundary
//            go byte by byte.
// Variants: 0 copy only (header = input bytes [0, 40)), 1 + sums + header
// area.  Also a plain read+write copy probe over the same byte counts.
// usage: gso_lds [iters]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

constexpr unsigned N = 1u << 18, IN_STRIDE = 65536, OUT_STRIDE = 73216, IN_LEN = 65535, H = 40, G = 1460;
constexpr unsigned S = H + G, NSEG = (IN_LEN - H + G - 1) / G, OUT_LEN = IN_LEN - H + NSEG * H;
constexpr unsigned IN_CHUNKS = (IN_LEN + 15) / 16, OUT_CHUNKS = (OUT_LEN + 15) / 16;
constexpr unsigned HDR_OFF = IN_CHUNKS * 16;  // header area in LDS (bytes)

#define CHECK(x)                                                                                                       \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                  \
            exit(1);                                                                                                   \
        }                                                                                                              \
    } while (0)

__device__ __forceinline__ unsigned fold16(unsigned long long x) {
    unsigned long long t = (x & 0xffffffffull) + (x >> 32);
    unsigned u = (unsigned)(t & 0xffff) + (unsigned)((t >> 16) & 0xffff) + (unsigned)(t >> 32);
    u = (u & 0xffff) + (u >> 16);
    return (u & 0xffff) + (u >> 16);
}
__device__ __forceinline__ unsigned wsum_dpp(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    return (unsigned)__builtin_amdgcn_readlane((int)v, 0) + (unsigned)__builtin_amdgcn_readlane((int)v, 16) +
           (unsigned)__builtin_amdgcn_readlane((int)v, 32) + (unsigned)__builtin_amdgcn_readlane((int)v, 48);
}

template <int V, int W>
__global__ __launch_bounds__(64 * W) void gso_lds(const unsigned char *in, unsigned char *out) {
    __shared__ v4u lds[IN_CHUNKS + (NSEG * H + 15) / 16];
    unsigned char *lb = reinterpret_cast<unsigned char *>(lds);
    unsigned b = blockIdx.x;
    if (!(gridDim.x & 7u)) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
    const unsigned char *src = in + (size_t)b * IN_STRIDE;
    unsigned char *dst = out + (size_t)b * OUT_STRIDE;
    const unsigned t = threadIdx.x, lane = t & 63u, w = t >> 6;
    // phase 1: 64 wave-instructions of 1 KiB
    for (unsigned k = w; k < IN_CHUNKS / 64; k += W)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src + (k * 64 + lane) * 16),
                                         (__attribute__((address_space(3))) void *)(&lds[k * 64]), 16, 0,
                                         0);
    __syncthreads();
    if (V >= 1) {
        // phase 2: wave per segment: payload sum (dword aligned here), header
        for (unsigned s = w; s < NSEG; s += W) {
            const unsigned p0 = H + s * G, p1 = p0 + G < IN_LEN ? p0 + G : IN_LEN;
            const unsigned nd = (p1 - p0) / 4;
            unsigned long long acc = 0;
            for (unsigned d = lane; d < nd; d += 64) acc += *reinterpret_cast<const unsigned *>(lb + p0 + 4 * d);
            const unsigned tailb = (p1 - p0) & 3u;
            if (lane == 0 && tailb) {
                unsigned v = 0;
                for (unsigned j = 0; j < tailb; j++) v |= (unsigned)lb[p0 + 4 * nd + j] << (8 * j);
                acc += v;
            }
            const unsigned sum = fold16(wsum_dpp(fold16(acc)));
            // header: template dwords with the checksum in bytes 36-37
            if (lane < H / 4) {
                unsigned hv = *reinterpret_cast<const unsigned *>(lb + 4 * lane);
                if (lane == 9)
                    hv = (hv & 0xffff0000u) | (~sum & 0xffffu);
                *reinterpret_cast<unsigned *>(lb + HDR_OFF + s * H + 4 * lane) = hv;
            }
        }
        __syncthreads();
    }
    // phase 3: row-order output
    for (unsigned c = t; c < OUT_CHUNKS; c += 64 * W) {
        const unsigned o0 = 16 * c, s0 = o0 / S, r0 = o0 - s0 * S;
        v4u v;
        if (r0 >= H && r0 + 16 <= S && o0 + 16 <= OUT_LEN) {
            const unsigned p = o0 - H * s0;  // multiple of 8
            const v2u a = *reinterpret_cast<const v2u *>(lb + p), bb = *reinterpret_cast<const v2u *>(lb + p + 8);
            v = v4u{a.x, a.y, bb.x, bb.y};
        } else {
            unsigned d[4] = {0, 0, 0, 0};
            for (unsigned j = 0; j < 16; j++) {
                const unsigned o = o0 + j;
                if (o >= OUT_LEN)
                    break;
                const unsigned s = o / S, r = o - s * S;
                const unsigned by = r < H ? (V >= 1 ? lb[HDR_OFF + s * H + r] : lb[r]) : lb[o - H * s];
                d[j >> 2] |= by << (8 * (j & 3));
            }
            v = v4u{d[0], d[1], d[2], d[3]};
        }
        *reinterpret_cast<__attribute__((address_space(1))) v4u *>(reinterpret_cast<uintptr_t>(dst) + o0) = v;
    }
}

__global__ __launch_bounds__(256) void copy_probe(const v4u *in, v4u *out, size_t nin, size_t nout) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t k = i; k < nout; k += stride) out[k] = in[k < nin ? k : k - nin];
}

template <int V, int W>
static float run(const unsigned char *din, unsigned char *dout, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((gso_lds<V, W>), dim3(N), dim3(64 * W), 0, 0, din, dout);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; i++) hipLaunchKernelGGL((gso_lds<V, W>), dim3(N), dim3(64 * W), 0, 0, din, dout);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 10;
    const size_t in_bytes = (size_t)N * IN_STRIDE, out_bytes = (size_t)N * OUT_STRIDE;
    unsigned char *din, *dout;
    CHECK(hipMalloc(&din, in_bytes));
    CHECK(hipMalloc(&dout, out_bytes));
    {
        std::vector<unsigned char> h(in_bytes / 64);
        for (size_t i = 0; i < h.size(); i++) h[i] = (unsigned char)(i * 2654435761u >> 13);
        for (int k = 0; k < 64; k++) CHECK(hipMemcpy(din + k * h.size(), h.data(), h.size(), hipMemcpyHostToDevice));
    }
    const double alg = (double)N * (IN_LEN + OUT_LEN);
    // correctness of variant 0 on a few super-buffers (copy semantics)
    hipLaunchKernelGGL((gso_lds<0, 4>), dim3(N), dim3(256), 0, 0, din, dout);
    CHECK(hipDeviceSynchronize());
    {
        std::vector<unsigned char> hi(IN_STRIDE), ho(OUT_STRIDE);
        int bad = 0;
        for (unsigned sb : {0u, 1u, 777u, N - 1}) {
            CHECK(hipMemcpy(hi.data(), din + (size_t)sb * IN_STRIDE, IN_STRIDE, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(ho.data(), dout + (size_t)sb * OUT_STRIDE, OUT_STRIDE, hipMemcpyDeviceToHost));
            for (unsigned o = 0; o < OUT_LEN; o++) {
                const unsigned s = o / S, r = o - s * S;
                const unsigned char e = r < H ? hi[r] : hi[o - H * s];
                bad += ho[o] != e;
            }
        }
        printf("{\"check_v0_bad_bytes\": %d}\n", bad);
    }
    float t;
    t = run<0, 4>(din, dout, iters);
    printf("{\"variant\": \"V0 copy, 4 waves\", \"ms\": %.4f, \"TBps\": %.3f}\n", t, alg / (t * 1e-3) / 1e12);
    t = run<0, 8>(din, dout, iters);
    printf("{\"variant\": \"V0 copy, 8 waves\", \"ms\": %.4f, \"TBps\": %.3f}\n", t, alg / (t * 1e-3) / 1e12);
    t = run<1, 4>(din, dout, iters);
    printf("{\"variant\": \"V1 + sums + header area, 4 waves\", \"ms\": %.4f, \"TBps\": %.3f}\n", t,
           alg / (t * 1e-3) / 1e12);
    t = run<1, 8>(din, dout, iters);
    printf("{\"variant\": \"V1 + sums + header area, 8 waves\", \"ms\": %.4f, \"TBps\": %.3f}\n", t,
           alg / (t * 1e-3) / 1e12);
    t = run<0, 4>(din, dout, iters);
    printf("{\"variant\": \"V0 copy, 4 waves (again)\", \"ms\": %.4f, \"TBps\": %.3f}\n", t, alg / (t * 1e-3) / 1e12);
    {
        const size_t nin = (size_t)N * IN_LEN / 16, nout = (size_t)N * OUT_LEN / 16;
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        hipLaunchKernelGGL(copy_probe, dim3(1 << 16), dim3(256), 0, 0, (const v4u *)din, (v4u *)dout, nin, nout);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < iters; i++)
            hipLaunchKernelGGL(copy_probe, dim3(1 << 16), dim3(256), 0, 0, (const v4u *)din, (v4u *)dout, nin, nout);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        CHECK(hipEventElapsedTime(&t, e0, e1));
        t /= iters;
        printf("{\"variant\": \"plain copy probe (same read + write bytes)\", \"ms\": %.4f, \"TBps\": %.3f}\n", t,
               alg / (t * 1e-3) / 1e12);
    }
    return 0;
}
