// Experiment: cost of unaligned 16-byte global loads on gfx950 (copy with a
// source misaligned by `mis` bytes, destination aligned) vs an aligned copy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u g_v4u;

template <int U>
__global__ __launch_bounds__(256) void copy_k(const unsigned char *src, unsigned char *dst, size_t nchunks) {
    size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x);
    size_t stride = (size_t)gridDim.x * 256;
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        size_t c = base + u * stride;
        if (c < nchunks) v[u] = *reinterpret_cast<const g_v4u *>((uintptr_t)(src + 16 * c));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        size_t c = base + u * stride;
        if (c < nchunks) *reinterpret_cast<g_v4u *>((uintptr_t)(dst + 16 * c)) = v[u];
    }
}

int main(int argc, char **argv) {
    size_t bytes = (size_t)4 << 30;
    unsigned char *src, *dst;
    hipMalloc(&src, bytes + 64);
    hipMalloc(&dst, bytes + 64);
    hipMemset(src, 0, bytes + 64);
    std::vector<unsigned char> h(1 << 20);
    for (size_t i = 0; i < h.size(); i++) h[i] = (unsigned char)(i * 7 + 3);
    hipMemcpy(src, h.data(), h.size(), hipMemcpyHostToDevice);
    size_t nchunks = bytes / 16;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int mis : {0, 1, 3, 4, 8, 12, 0}) {
        unsigned blocks = (unsigned)((nchunks / 4 + 255) / 256);
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL((copy_k<4>), dim3(blocks), dim3(256), 0, 0, src + mis, dst, nchunks);
        hipEventRecord(e0);
        const int it = 10;
        for (int w = 0; w < it; w++) hipLaunchKernelGGL((copy_k<4>), dim3(blocks), dim3(256), 0, 0, src + mis, dst, nchunks);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned char> o(4096);
        hipMemcpy(o.data(), dst, o.size(), hipMemcpyDeviceToHost);
        bool ok = memcmp(o.data(), h.data() + mis, o.size()) == 0;
        printf("{\"mis\": %d, \"ms\": %.4f, \"GBps_rw\": %.1f, \"ok\": %s}\n", mis, ms / it,
               2.0 * bytes / (ms / it * 1e-3) / 1e9, ok ? "true" : "false");
    }
    hipError_t err = hipGetLastError();
    printf("err=%s\n", hipGetErrorString(err));
    return 0;
}
