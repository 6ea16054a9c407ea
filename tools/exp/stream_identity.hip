// stream_identity.hip — what identifies a HIP stream to a library that keeps
// per-stream scratch (wg_verify_desc's compacting path).
//
//  1. create / destroy streams in a loop: do handle values come back, and
//     does hipStreamGetId ever repeat?
//  2. hipStreamDestroy with a ~20 ms kernel pending: does it block?
//  3. four threads: hipStreamGetId of hipStreamPerThread, NULL and
//     hipStreamLegacy (per-thread streams distinct per thread?)
//  4. host cost per call of hipStreamGetId, hipEventRecord,
//     hipStreamWaitEvent (same stream / another stream), hipEventQuery.
//
// Build: hipcc -O2 --offload-arch=gfx950 -std=c++20 stream_identity.hip -o bin/stream_identity -lpthread
//   (-DNO_GETID: without hipStreamGetId, to run against PyTorch's bundled
//   ROCm 7.0 runtime via LD_LIBRARY_PATH: ids print as 0)
//  5. a thread that launches a 20 ms kernel on hipStreamPerThread and exits:
//     does its exit wait for the kernel (join time)?
//  6. hipStreamGetId on a destroyed (not reused) handle
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

// bounded spin on the 100 MHz real-time counter (ticks), one wave
__global__ void spin(uint64_t ticks, uint32_t *out) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t k = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks && k < 200000000u) k++;
    if (threadIdx.x == 0) out[0] = k;
}

__global__ void tiny(uint32_t *out) {
    if (threadIdx.x == 0) out[1] += 1;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#ifdef NO_GETID
static hipError_t get_id(hipStream_t, unsigned long long *id) {
    *id = 0;
    return hipSuccess;
}
#else
static hipError_t get_id(hipStream_t s, unsigned long long *id) { return hipStreamGetId(s, id); }
#endif

int main() {
    CK(hipSetDevice(0));
    uint32_t *d = nullptr;
    CK(hipMalloc(&d, 64));
    CK(hipMemset(d, 0, 64));
    CK(hipDeviceSynchronize());

    // 1. churn
    {
        std::set<void *> handles;
        std::set<unsigned long long> ids;
        int reused_handle = 0, reused_id = 0;
        for (int i = 0; i < 300; i++) {
            hipStream_t s;
            CK(hipStreamCreate(&s));
            unsigned long long id = 0;
            const hipError_t e = get_id(s, &id);
            if (e != hipSuccess) {
                std::printf("churn: hipStreamGetId -> %s\n", hipGetErrorString(e));
                break;
            }
            reused_handle += !handles.insert((void *)s).second;
            reused_id += !ids.insert(id).second;
            if (i < 4) std::printf("churn %d: handle %p id %llu\n", i, (void *)s, id);
            hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
            CK(hipStreamDestroy(s));
        }
        std::printf("churn: 300 streams, distinct handles %zu (reused %d), distinct ids %zu (reused %d)\n",
                    handles.size(), reused_handle, ids.size(), reused_id);
    }
    CK(hipDeviceSynchronize());

    // 2. destroy with work pending
    {
        hipStream_t s;
        CK(hipStreamCreate(&s));
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 2000000ull /* 20 ms */, d);
        const double t0 = now_us();
        CK(hipStreamDestroy(s));
        const double t1 = now_us();
        CK(hipDeviceSynchronize());
        const double t2 = now_us();
        std::printf("destroy with a 20 ms kernel pending: destroy took %.1f us, then device sync %.1f us\n", t1 - t0,
                    t2 - t1);
        // handle reuse right after a pending destroy
        hipStream_t a, b;
        CK(hipStreamCreate(&a));
        unsigned long long ia = 0, ib = 0;
        CK(get_id(a, &ia));
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, a, 2000000ull, d);
        void *ha = (void *)a;
        CK(hipStreamDestroy(a));
        CK(hipStreamCreate(&b));
        CK(get_id(b, &ib));
        std::printf("create right after destroy(pending): old %p id %llu, new %p id %llu, same handle %d\n", ha, ia,
                    (void *)b, ib, ha == (void *)b);
        CK(hipStreamDestroy(b));
        CK(hipDeviceSynchronize());
    }

    // 3. special handles from several threads
    {
        std::mutex mu;
        std::vector<std::thread> th;
        for (int t = 0; t < 4; t++)
            th.emplace_back([t, &mu, d] {
                CK(hipSetDevice(0));
                unsigned long long ipt = 0, inull = 0, ileg = 0;
                const hipError_t e1 = get_id(hipStreamPerThread, &ipt);
                const hipError_t e2 = get_id(nullptr, &inull);
                const hipError_t e3 = get_id(hipStreamLegacy, &ileg);
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, hipStreamPerThread, d);
                CK(hipStreamSynchronize(hipStreamPerThread));
                std::lock_guard<std::mutex> g(mu);
                std::printf("thread %d: perthread id %llu (%s), NULL id %llu (%s), legacy id %llu (%s)\n", t, ipt,
                            hipGetErrorString(e1), inull, hipGetErrorString(e2), ileg, hipGetErrorString(e3));
            });
        for (auto &x : th) x.join();
    }

    // 5. per-thread stream at thread exit
    {
        const double t0 = now_us();
        std::thread th([d] {
            CK(hipSetDevice(0));
            hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, hipStreamPerThread, 2000000ull, d);
        });
        th.join();
        const double t1 = now_us();
        CK(hipDeviceSynchronize());
        const double t2 = now_us();
        std::printf("thread exit with a 20 ms kernel pending on hipStreamPerThread: join %.1f us, then device sync %.1f us\n",
                    t1 - t0, t2 - t1);
    }
#ifndef NO_GETID
    // 6. id query on a destroyed handle (nothing created since)
    {
        hipStream_t s;
        CK(hipStreamCreate(&s));
        unsigned long long id0 = 0, id1 = 0;
        CK(get_id(s, &id0));
        CK(hipStreamDestroy(s));
        const hipError_t e = get_id(s, &id1);
        (void)hipGetLastError();
        std::printf("hipStreamGetId on a destroyed handle: %s (id before %llu, after %llu)\n", hipGetErrorString(e), id0,
                    id1);
    }
#endif

    // 4. host costs
    {
        hipStream_t s, s2;
        CK(hipStreamCreate(&s));
        CK(hipStreamCreate(&s2));
        hipEvent_t ev;
        CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        const int N = 20000;
        unsigned long long id = 0;
        double t0 = now_us();
        for (int i = 0; i < N; i++) CK(get_id(s, &id));
        double t1 = now_us();
        std::printf("hipStreamGetId: %.3f us/call\n", (t1 - t0) / N);
        int dev = 0;
        t0 = now_us();
        for (int i = 0; i < N; i++) CK(hipGetDevice(&dev));
        t1 = now_us();
        std::printf("hipGetDevice: %.3f us/call\n", (t1 - t0) / N);
        hipStreamCaptureStatus cs;
        t0 = now_us();
        for (int i = 0; i < N; i++) CK(hipStreamIsCapturing(s, &cs));
        t1 = now_us();
        std::printf("hipStreamIsCapturing: %.3f us/call\n", (t1 - t0) / N);
        // launches alone vs launches + record + wait(same stream)
        for (int rep = 0; rep < 2; rep++) {
            CK(hipDeviceSynchronize());
            t0 = now_us();
            for (int i = 0; i < N; i++) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
            t1 = now_us();
            CK(hipStreamSynchronize(s));
            const double t2 = now_us();
            std::printf("launch only: %.3f us/launch host, %.3f us/launch incl. drain\n", (t1 - t0) / N, (t2 - t0) / N);
            CK(hipDeviceSynchronize());
            t0 = now_us();
            for (int i = 0; i < N; i++) {
                CK(hipStreamWaitEvent(s, ev, 0));
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
                CK(hipEventRecord(ev, s));
            }
            t1 = now_us();
            CK(hipStreamSynchronize(s));
            const double t3 = now_us();
            std::printf("wait(same stream) + launch + record: %.3f us/iter host, %.3f us incl. drain\n",
                        (t1 - t0) / N, (t3 - t0) / N);
            CK(hipDeviceSynchronize());
            t0 = now_us();
            for (int i = 0; i < N; i++) {
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
                CK(hipEventRecord(ev, s));
            }
            t1 = now_us();
            CK(hipStreamSynchronize(s));
            const double t4 = now_us();
            std::printf("launch + record: %.3f us/iter host, %.3f us incl. drain\n", (t1 - t0) / N, (t4 - t0) / N);
            CK(hipDeviceSynchronize());
            t0 = now_us();
            for (int i = 0; i < N; i++) (void)hipEventQuery(ev);
            t1 = now_us();
            std::printf("hipEventQuery (complete): %.3f us/call\n", (t1 - t0) / N);
            t0 = now_us();
            for (int i = 0; i < N; i++) {
                CK(hipStreamWaitEvent(s2, ev, 0));
                hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s2, d);
            }
            t1 = now_us();
            CK(hipStreamSynchronize(s2));
            const double t5 = now_us();
            std::printf("wait(other stream, event complete) + launch: %.3f us/iter host, %.3f incl. drain\n",
                        (t1 - t0) / N, (t5 - t0) / N);
        }
    }
    CK(hipDeviceSynchronize());
    std::printf("done\n");
    return 0;
}
