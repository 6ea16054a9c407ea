// Small-packet load shapes (timing only, not library code).  The lane paths
// give each lane one 64-B packet: four 16-B loads per lane whose 64 lanes
// touch 64 different 64-B pieces per instruction (an array-of-structs
// pattern).  This probe reads n contiguous 64-B packets, sums each packet's
// words and stores one uint16 per packet, three ways:
//   aos:   lane l loads packet l's 4 chunks (the library's lane shape);
//   coal:  instruction k of a wave loads bytes [k*1024, +1024) of the wave's
//          4 KiB, lane l chunk l (fully coalesced), and the 4 lanes of a
//          packet combine their sums with two cross-lane xors;
//   lds:   the coalesced loads written to LDS (80-B rows: conflict-free), then
//          each lane reads its own packet back (a transpose).
// Each shape with the default cache policy and non-temporal loads; 1 M and
// 16 M packets; back to back (one event pair around 50 launches) and isolated
// (an event pair and a sync per launch).  Prints one JSON line per case.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -o tools/exp/bin/aos_probe tools/exp/aos_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u g_v4u;

template <bool kNT>
__device__ __forceinline__ v4u ld(uintptr_t a) {
    if constexpr (kNT)
        return __builtin_nontemporal_load(reinterpret_cast<g_v4u *>(a));
    else
        return *reinterpret_cast<g_v4u *>(a);
}

__device__ __forceinline__ uint64_t sum4(v4u v) { return (uint64_t)v.x + v.y + v.z + v.w; }

__device__ __forceinline__ uint16_t fold(uint64_t s) {
    s = (s & 0xffffffffu) + (s >> 32);
    s = (s & 0xffffu) + (s >> 16);
    s = (s & 0xffffu) + (s >> 16);
    s = (s & 0xffffu) + (s >> 16);
    return (uint16_t)~s;
}

__device__ __forceinline__ uint32_t wave_index() {
    const uint32_t nb = gridDim.x;
    const uint32_t b = (nb & 7u) ? blockIdx.x : (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
    return b * 4u + (threadIdx.x >> 6);
}

template <bool kNT>
__global__ __launch_bounds__(256) void k_aos(const uint8_t *base, uint64_t n, uint16_t *out) {
    const uint64_t p = (uint64_t)wave_index() * 64u + (threadIdx.x & 63u);
    if (p >= n)
        return;
    const uintptr_t a = reinterpret_cast<uintptr_t>(base) + p * 64u;
    v4u v[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        v[k] = ld<kNT>(a + 16u * k);
    out[p] = fold(sum4(v[0]) + sum4(v[1]) + sum4(v[2]) + sum4(v[3]));
}

template <bool kNT>
__global__ __launch_bounds__(256) void k_coal(const uint8_t *base, uint64_t n, uint16_t *out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t w = wave_index();
    if (w * 64u >= n)
        return;  // n is a multiple of 64 here
    const uintptr_t a = reinterpret_cast<uintptr_t>(base) + w * 4096u + lane * 16u;
    v4u v[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        v[k] = ld<kNT>(a + 1024u * k);
    uint64_t s[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint64_t x = sum4(v[k]);
        x += __shfl_xor(x, 1);
        x += __shfl_xor(x, 2);
        s[k] = x;
    }
    // lane l holds packet k*16 + l/4's sum in s[k]; lane with l%4 == k stores it
    const uint32_t c = lane & 3u;
    const uint64_t mine = c == 0 ? s[0] : c == 1 ? s[1] : c == 2 ? s[2] : s[3];
    out[w * 64u + c * 16u + (lane >> 2)] = fold(mine);
}

template <bool kNT>
__global__ __launch_bounds__(256) void k_lds(const uint8_t *base, uint64_t n, uint16_t *out) {
    __shared__ v4u rows[4][64 * 5];  // 64 packets x 80 B per wave
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t w = wave_index();
    if (w * 64u >= n)
        return;
    const uintptr_t a = reinterpret_cast<uintptr_t>(base) + w * 4096u + lane * 16u;
    v4u v[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        v[k] = ld<kNT>(a + 1024u * k);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t pk = k * 16u + (lane >> 2), ch = lane & 3u;
        rows[wv][pk * 5u + ch] = v[k];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
        s += sum4(rows[wv][lane * 5u + k]);
    out[w * 64u + lane] = fold(s);
}

template <typename K>
static void run(const char *name, K kern, const uint8_t *d, uint64_t n, uint16_t *o, hipEvent_t e0, hipEvent_t e1,
                std::vector<uint16_t> &ref) {
    const uint64_t waves = n / 64u;
    uint64_t blocks = (waves + 3) / 4;
    if (blocks >= 8)
        blocks = (blocks + 7) & ~7ull;
    for (int i = 0; i < 20; i++)
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, 0, d, n, o);
    (void)hipDeviceSynchronize();
    // results against the aos shape (the first case run)
    std::vector<uint16_t> got(n);
    (void)hipMemcpy(got.data(), o, n * 2, hipMemcpyDeviceToHost);
    bool same = true;
    if (ref.empty())
        ref = got;
    else
        same = got == ref;
    float b2b[3], iso[3];
    for (int r = 0; r < 3; r++) {
        (void)hipEventRecord(e0);
        for (int i = 0; i < 50; i++)
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, 0, d, n, o);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        b2b[r] = ms / 50;
        std::vector<float> t;
        for (int i = 0; i < 20; i++) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, 0, d, n, o);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        iso[r] = t[t.size() / 2];
    }
    std::sort(b2b, b2b + 3);
    std::sort(iso, iso + 3);
    const double bytes = n * 66.0;
    printf("{\"shape\": \"%s\", \"packets\": %llu, \"b2b_us\": %.2f, \"b2b_TBps\": %.3f, \"isolated_us\": %.2f, "
           "\"isolated_TBps\": %.3f, \"same_results\": %s}\n",
           name, (unsigned long long)n, b2b[1] * 1e3, bytes / (b2b[1] * 1e9), iso[1] * 1e3, bytes / (iso[1] * 1e9),
           same ? "true" : "false");
    fflush(stdout);
}

int main() {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (uint64_t n : {1ull << 20, 1ull << 24}) {
        uint8_t *d;
        uint16_t *o;
        if (hipMalloc(&d, n * 64) != hipSuccess || hipMalloc(&o, n * 2) != hipSuccess)
            return 1;
        std::vector<uint32_t> h(n * 16);
        uint64_t x = 0x9e3779b97f4a7c15ull;
        for (auto &w : h) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            w = (uint32_t)x;
        }
        (void)hipMemcpy(d, h.data(), n * 64, hipMemcpyHostToDevice);
        std::vector<uint16_t> ref;
        for (int rep = 0; rep < 2; rep++) {
            run("aos", k_aos<false>, d, n, o, e0, e1, ref);
            run("aos_nt", k_aos<true>, d, n, o, e0, e1, ref);
            run("coal", k_coal<false>, d, n, o, e0, e1, ref);
            run("coal_nt", k_coal<true>, d, n, o, e0, e1, ref);
            run("lds", k_lds<false>, d, n, o, e0, e1, ref);
            run("lds_nt", k_lds<true>, d, n, o, e0, e1, ref);
        }
        (void)hipFree(d);
        (void)hipFree(o);
    }
    return 0;
}
