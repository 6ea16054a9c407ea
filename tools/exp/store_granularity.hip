// store_granularity.hip — what a partial store into a 64-B header slot costs
// the memory side (GRO finalize's write pattern).
//
// 4,194,304 slots of 64 B (the bench's GRO layout), one thread per slot, each
// variant storing a fixed byte pattern into every slot.  Run under
// rocprofv3 --pmc WRITE_SIZE (and FETCH_SIZE) with --kernel-trace: the
// per-dispatch WRITE_SIZE / slots is the memory-side write cost of the
// pattern.  Patterns (byte ranges within the slot):
//   0 w2      [2,4)                          one 16-bit field
//   1 w4      [24,28)                        one dword (udp len + seed)
//   2 w16     [0,16)                         one 16-B store
//   3 v4tcp   [0,16) + [36,38)               gro_wide, IPv4/TCP
//   4 v4udp   [0,16) + [24,28)               gro_wide, IPv4/UDP
//   5 narrow  [2,4) + [10,12) + [36,38)      gro_wide = 0, IPv4/TCP
//   6 full    [0,64)                         whole slot (4 x 16 B)
// Build: hipcc -O3 --offload-arch=gfx950 -o store_granularity store_granularity.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u gv4u;
typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) unsigned short gu16;

template <int V>
__global__ __launch_bounds__(256) void pattern_kernel(unsigned char *slots, unsigned long n, unsigned v) {
    const unsigned long i = (unsigned long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    const unsigned long a = reinterpret_cast<unsigned long>(slots) + 64ul * i;
    const v4u q = v4u{v, v + 1, v + 2, v + 3};
    if (V == 0) *reinterpret_cast<gu16 *>(a + 2) = (unsigned short)v;
    if (V == 1) *reinterpret_cast<gu32 *>(a + 24) = v;
    if (V == 2 || V == 3 || V == 4) *reinterpret_cast<gv4u *>(a) = q;
    if (V == 3) *reinterpret_cast<gu16 *>(a + 36) = (unsigned short)v;
    if (V == 4) *reinterpret_cast<gu32 *>(a + 24) = v;
    if (V == 5) {
        *reinterpret_cast<gu16 *>(a + 2) = (unsigned short)v;
        *reinterpret_cast<gu16 *>(a + 10) = (unsigned short)v;
        *reinterpret_cast<gu16 *>(a + 36) = (unsigned short)v;
    }
    if (V == 6)
        for (int k = 0; k < 4; k++) *reinterpret_cast<gv4u *>(a + 16 * k) = q;
}

int main(int argc, char **argv) {
    const unsigned long n = 1ul << 22;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    unsigned char *d = nullptr;
    if (hipMalloc(&d, 64 * n) != hipSuccess) return 1;
    hipMemset(d, 0, 64 * n);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"w2", "w4", "w16", "v4tcp", "v4udp", "narrow", "full"};
    const dim3 g((unsigned)(n / 256)), b(256);
    for (int v = 0; v < 7; v++) {
        auto launch = [&](unsigned x) {
            switch (v) {
            case 0: hipLaunchKernelGGL(pattern_kernel<0>, g, b, 0, 0, d, n, x); break;
            case 1: hipLaunchKernelGGL(pattern_kernel<1>, g, b, 0, 0, d, n, x); break;
            case 2: hipLaunchKernelGGL(pattern_kernel<2>, g, b, 0, 0, d, n, x); break;
            case 3: hipLaunchKernelGGL(pattern_kernel<3>, g, b, 0, 0, d, n, x); break;
            case 4: hipLaunchKernelGGL(pattern_kernel<4>, g, b, 0, 0, d, n, x); break;
            case 5: hipLaunchKernelGGL(pattern_kernel<5>, g, b, 0, 0, d, n, x); break;
            default: hipLaunchKernelGGL(pattern_kernel<6>, g, b, 0, 0, d, n, x); break;
            }
        };
        for (int r = 0; r < 5; r++) launch(r);
        hipEventRecord(e0, 0);
        for (int r = 0; r < reps; r++) launch(100 + r);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"pattern\": \"%s\", \"us_per_launch\": %.2f, \"slots\": %lu}\n", names[v], 1000.0 * ms / reps, n);
    }
    hipFree(d);
    return 0;
}
