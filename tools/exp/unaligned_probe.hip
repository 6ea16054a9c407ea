// Read-stream probe (timing only, not library code): 16-B loads over a
// 16 GiB buffer at a byte offset of 0, 4, 8 or 12 from 16-B alignment (the
// GSO split's interior chunks are destination-aligned, so their source
// loads sit at (hdr_len + i * gso) mod 16), same grid and unroll as the read
// probe.  Prints TB/s per offset.
// build: hipcc --offload-arch=gfx950 -O3 -o gpurun_out/unaligned_probe tools/exp/unaligned_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void rd(const uint8_t *base, uint64_t chunks, uint32_t off, uint32_t *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t nt = (uint64_t)gridDim.x * 256;
    v4u acc = {0, 0, 0, 0};
    for (uint64_t c = tid; c < chunks; c += 4 * nt) {
        v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t k = c + u * nt < chunks ? c + u * nt : c;
            v[u] = *reinterpret_cast<const __attribute__((address_space(1))) v4u *>(reinterpret_cast<uintptr_t>(base) + off + 16 * k);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) acc ^= v[u];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u)
        out[0] = 1;
}

int main() {
    const uint64_t bytes = 16ull << 30;
    uint8_t *d;
    uint32_t *o;
    if (hipMalloc(&d, bytes + 64) != hipSuccess || hipMalloc(&o, 64) != hipSuccess)
        return 1;
    (void)hipMemset(d, 1, bytes + 64);
    const uint64_t chunks = bytes / 16;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
        for (uint32_t off : {0u, 4u, 8u, 12u, 1u}) {
            float best = 1e30f;
            for (int r = 0; r < 4; r++) {
                (void)hipEventRecord(e0);
                hipLaunchKernelGGL(rd, dim3(256 * 8 * 4), dim3(256), 0, 0, d, chunks, off, o);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            printf("{\"offset\": %u, \"ms\": %.3f, \"TBps\": %.3f}\n", off, best, bytes / (best * 1e9));
        }
    }
    (void)hipFree(d);
    (void)hipFree(o);
    return 0;
}
