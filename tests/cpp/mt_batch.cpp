// mt_batch.cpp — TEST HARNESS (not product): several host threads calling the
// batch entry points of libwireglider_amd.so at once, each on its own stream
// (wireglider's threading model: one worker thread per tun queue,
// wireglider.cpp:117-151; each worker calls the checksum path for its own
// batches, worker/offload.cpp:202, include/worker/evaluator.hpp:64,93).
//
// Inputs and expected outputs come from tests/test_mt_batch.py (the oracle,
// written as raw files into <dir>); this program only calls the C ABI and
// compares bytes.
//
//   mt_batch <dir> conform <threads> <iters> <own|perthread|legacy|churn>
//       every call's outputs (refilled with a sentinel on the stream before
//       the call) compared with the expected files; JSON with mismatch counts
//   mt_batch <dir> rate <threads> <calls> [small]
//       per entry point, every thread enqueues <calls> calls back to back on
//       its own stream: host calls/s per thread, plus the HIP runtime's own
//       floor (an empty kernel launched the same way); `small`: 64-packet
//       batches (2 super-buffers for the split), so the device keeps up and
//       the figure is the host launch path, not the queues' back-pressure
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <barrier>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "wireglider_amd.h"

namespace {

#define CK(x)                                                                                              \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) {                                                                            \
            std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
            std::exit(2);                                                                                  \
        }                                                                                                  \
    } while (0)

std::vector<uint8_t> load(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        std::fprintf(stderr, "missing %s\n", path.c_str());
        std::exit(2);
    }
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

struct Dev {
    void *p = nullptr;
    size_t n = 0;
};

Dev upload(const std::vector<uint8_t> &h) {
    Dev d;
    d.n = h.size();
    CK(hipMalloc(&d.p, std::max<size_t>(d.n, 16)));
    if (d.n)
        CK(hipMemcpy(d.p, h.data(), d.n, hipMemcpyHostToDevice));
    return d;
}

// One input set, shared read-only by every thread (GSO input excepted: the
// split zeroes fields of its input in place, so each thread has a copy).
struct Inputs {
    std::string dir;
    const char *vkinds[3] = {"small", "long", "mixed"};
    Dev vbuf[3], vdesc[3];
    std::vector<uint8_t> vverdict[3], vl4[3];
    uint64_t vn[3];
    Dev l4d_buf, l4d_desc;
    std::vector<uint8_t> l4d_out;
    uint64_t l4d_n;
    Dev l4u_buf;
    std::vector<uint8_t> l4u_out;
    uint32_t l4u_seg = 0, l4u_cs = 0, l4u_flags = 0;
    std::vector<uint8_t> plain_out;               // wg_checksum_desc over the l4d batch
    std::vector<uint8_t> vu_verdict, vu_l4;       // wg_verify_uniform over the l4u batch
    std::vector<uint8_t> aead_out, aead_key;      // wg_aead_encrypt_batch over the l4u batch
    uint32_t aead_rx = 0;
    uint64_t aead_c0 = 0;
    std::vector<uint8_t> gso_in, gso_out, gso_in_after, gso_status;
    Dev gso_desc;
    uint64_t gso_n;

    void read(const std::string &d) {
        dir = d;
        for (int k = 0; k < 3; k++) {
            const std::string b = dir + "/verify_" + vkinds[k];
            vbuf[k] = upload(load(b + ".buf"));
            vdesc[k] = upload(load(b + ".desc"));
            vverdict[k] = load(b + ".verdict");
            vl4[k] = load(b + ".l4");
            vn[k] = vverdict[k].size();
        }
        l4d_buf = upload(load(dir + "/l4d.buf"));
        l4d_desc = upload(load(dir + "/l4d.desc"));
        l4d_out = load(dir + "/l4d.out");
        l4d_n = l4d_out.size() / 2;
        l4u_buf = upload(load(dir + "/l4u.buf"));
        l4u_out = load(dir + "/l4u.out");
        std::ifstream pf(dir + "/params.txt");
        pf >> l4u_seg >> l4u_cs >> l4u_flags >> aead_rx >> aead_c0;
        plain_out = load(dir + "/l4d.plain");
        vu_verdict = load(dir + "/l4u.verdict");
        vu_l4 = load(dir + "/l4u.l4");
        aead_out = load(dir + "/aead.out");
        aead_key = load(dir + "/aead.key");
        gso_in = load(dir + "/gso.in");
        gso_out = load(dir + "/gso.out");
        gso_in_after = load(dir + "/gso.in_after");
        gso_status = load(dir + "/gso.status");
        gso_desc = upload(load(dir + "/gso.desc"));
        gso_n = gso_status.size();
    }
};

constexpr uint8_t kSentinel = 0xA5;

// A thread's outputs (device) and its host copies.
struct Outs {
    Dev verdict, l4, l4d, l4u, gso_in, gso_out, gso_res, plain, vuv, vul, aout, ast;
    std::vector<uint8_t> h;
    void make(const Inputs &in) {
        uint64_t vmax = std::max({in.vn[0], in.vn[1], in.vn[2]});
        verdict = upload(std::vector<uint8_t>(vmax, 0));
        l4 = upload(std::vector<uint8_t>(2 * vmax, 0));
        l4d = upload(std::vector<uint8_t>(in.l4d_out.size(), 0));
        l4u = upload(std::vector<uint8_t>(in.l4u_out.size(), 0));
        gso_in = upload(in.gso_in);
        gso_out = upload(std::vector<uint8_t>(in.gso_out.size(), kSentinel));
        gso_res = upload(std::vector<uint8_t>(in.gso_n * sizeof(wg_gso_result), 0));
        plain = upload(std::vector<uint8_t>(in.plain_out.size(), 0));
        vuv = upload(std::vector<uint8_t>(in.vu_verdict.size(), 0));
        vul = upload(std::vector<uint8_t>(in.vu_l4.size(), 0));
        aout = upload(std::vector<uint8_t>(in.aead_out.size(), 0));
        ast = upload(std::vector<uint8_t>(in.vu_verdict.size(), 0));
    }
    void release() {
        for (Dev *d : {&verdict, &l4, &l4d, &l4u, &gso_in, &gso_out, &gso_res, &plain, &vuv, &vul, &aout, &ast})
            CK(hipFree(d->p));
    }
};

bool same(const void *dev, const std::vector<uint8_t> &exp, hipStream_t st, std::vector<uint8_t> &h) {
    h.resize(exp.size());
    if (exp.empty())
        return true;
    CK(hipMemcpyAsync(h.data(), dev, exp.size(), hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    return std::memcmp(h.data(), exp.data(), exp.size()) == 0;
}

enum Op { kVerify, kL4Desc, kL4Uniform, kGso, kChecksum, kVerifyUniform, kAead, kNumOps };
const char *op_name[kNumOps] = {"wg_verify_desc", "wg_l4csum_desc",        "wg_l4csum_uniform",    "wg_gso_split",
                                "wg_checksum_desc", "wg_verify_uniform", "wg_aead_encrypt_batch"};

// Each thread's verify kinds, phase-shifted per thread: runs of mixed batches
// (the default per-call choice reaches the compacting path after two mixed
// samples) between all-small and all-long ones.
const int kVerifyPattern[] = {2, 2, 2, 0, 1, 2, 2, 0, 0, 1, 1, 2, 2, 2};
constexpr int kPat = sizeof(kVerifyPattern) / sizeof(kVerifyPattern[0]);

// small: the first 64 packets / segments (2 super-buffers for the split), so
// a call's device time stays below its host time (rate mode)
int call(Op op, const Inputs &in, Outs &o, int vk, hipStream_t st, bool small = false) {
    const auto cut = [small](uint64_t n, uint64_t k) { return small && n > k ? k : n; };
    switch (op) {
    case kVerify:
        return wg_verify_desc(static_cast<const uint8_t *>(in.vbuf[vk].p), static_cast<const wg_pkt_desc *>(in.vdesc[vk].p),
                              cut(in.vn[vk], 64), static_cast<uint8_t *>(o.verdict.p), static_cast<uint16_t *>(o.l4.p), st);
    case kL4Desc:
        return wg_l4csum_desc(static_cast<const uint8_t *>(in.l4d_buf.p), static_cast<const wg_pkt_desc *>(in.l4d_desc.p),
                              cut(in.l4d_n, 64), static_cast<uint16_t *>(o.l4d.p), st);
    case kL4Uniform:
        return wg_l4csum_uniform(static_cast<const uint8_t *>(in.l4u_buf.p), cut(in.l4u_buf.n, 64ull * in.l4u_seg),
                                 in.l4u_seg, (uint16_t)in.l4u_cs, in.l4u_flags, static_cast<uint16_t *>(o.l4u.p), st);
    case kGso:
        return wg_gso_split(static_cast<uint8_t *>(o.gso_in.p), static_cast<const wg_gso_desc *>(in.gso_desc.p),
                            cut(in.gso_n, 2), static_cast<uint8_t *>(o.gso_out.p), static_cast<wg_gso_result *>(o.gso_res.p),
                            st);
    case kChecksum:
        return wg_checksum_desc(static_cast<const uint8_t *>(in.l4d_buf.p), static_cast<const wg_pkt_desc *>(in.l4d_desc.p),
                                cut(in.l4d_n, 64), static_cast<uint16_t *>(o.plain.p), st);
    case kVerifyUniform:
        return wg_verify_uniform(static_cast<const uint8_t *>(in.l4u_buf.p), cut(in.l4u_buf.n, 64ull * in.l4u_seg),
                                 in.l4u_seg, static_cast<uint8_t *>(o.vuv.p), static_cast<uint16_t *>(o.vul.p), st);
    case kAead:
        return wg_aead_encrypt_batch(static_cast<const uint8_t *>(in.l4u_buf.p), cut(in.l4u_buf.n, 64ull * in.l4u_seg),
                                     in.l4u_seg, in.aead_key.data(), in.aead_rx, in.aead_c0,
                                     static_cast<uint8_t *>(o.aout.p), static_cast<int8_t *>(o.ast.p), st);
    default:
        return WG_ERR_INVALID;
    }
}

void refill(Op op, const Inputs &in, Outs &o, int vk, hipStream_t st) {
    switch (op) {
    case kVerify:
        CK(hipMemsetAsync(o.verdict.p, kSentinel, in.vn[vk], st));
        CK(hipMemsetAsync(o.l4.p, kSentinel, 2 * in.vn[vk], st));
        break;
    case kL4Desc: CK(hipMemsetAsync(o.l4d.p, kSentinel, o.l4d.n, st)); break;
    case kL4Uniform: CK(hipMemsetAsync(o.l4u.p, kSentinel, o.l4u.n, st)); break;
    case kGso:
        CK(hipMemsetAsync(o.gso_out.p, kSentinel, o.gso_out.n, st));
        CK(hipMemsetAsync(o.gso_res.p, 0xff, o.gso_res.n, st));
        break;
    case kChecksum: CK(hipMemsetAsync(o.plain.p, kSentinel, o.plain.n, st)); break;
    case kVerifyUniform:
        CK(hipMemsetAsync(o.vuv.p, kSentinel, o.vuv.n, st));
        CK(hipMemsetAsync(o.vul.p, kSentinel, o.vul.n, st));
        break;
    case kAead:
        CK(hipMemsetAsync(o.aout.p, kSentinel, o.aout.n, st));
        CK(hipMemsetAsync(o.ast.p, kSentinel, o.ast.n, st));
        break;
    default: break;
    }
}

// Compare op's outputs; returns true when every byte matches.
bool check(Op op, const Inputs &in, Outs &o, int vk, hipStream_t st) {
    switch (op) {
    case kVerify:
        return same(o.verdict.p, in.vverdict[vk], st, o.h) && same(o.l4.p, in.vl4[vk], st, o.h);
    case kL4Desc: return same(o.l4d.p, in.l4d_out, st, o.h);
    case kL4Uniform: return same(o.l4u.p, in.l4u_out, st, o.h);
    case kGso: {
        if (!same(o.gso_out.p, in.gso_out, st, o.h) || !same(o.gso_in.p, in.gso_in_after, st, o.h))
            return false;
        std::vector<uint8_t> r(in.gso_n * sizeof(wg_gso_result));
        CK(hipMemcpyAsync(r.data(), o.gso_res.p, r.size(), hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        for (uint64_t i = 0; i < in.gso_n; i++)
            if ((int8_t)r[i * sizeof(wg_gso_result) + offsetof(wg_gso_result, status)] != (int8_t)in.gso_status[i])
                return false;
        return true;
    }
    case kChecksum: return same(o.plain.p, in.plain_out, st, o.h);
    case kVerifyUniform: return same(o.vuv.p, in.vu_verdict, st, o.h) && same(o.vul.p, in.vu_l4, st, o.h);
    case kAead: {
        // messages equal the oracle's; every status 0
        if (!same(o.aout.p, in.aead_out, st, o.h))
            return false;
        const std::vector<uint8_t> zeros(in.vu_verdict.size(), 0);
        return same(o.ast.p, zeros, st, o.h);
    }
    default: return false;
    }
}

int conform(const Inputs &in, int threads, int iters, const std::string &mode) {
    std::vector<std::array<std::atomic<int>, kNumOps>> bad(threads), calls(threads);
    for (auto &a : bad) for (auto &x : a) x = 0;
    for (auto &a : calls) for (auto &x : a) x = 0;
    std::atomic<int> errors{0};
    std::barrier sync_point(threads);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        th.emplace_back([&, t] {
            CK(hipSetDevice(0));
            Outs o;
            o.make(in);
            hipStream_t own = nullptr;
            if (mode == "own")
                CK(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
            hipStream_t st = mode == "perthread" ? hipStreamPerThread : mode == "legacy" ? nullptr : own;
            CK(hipDeviceSynchronize());
            sync_point.arrive_and_wait();
            if (mode == "churn") {
                // verify only: a fresh stream per call, destroyed right after the
                // launch (its work still pending), so a later stream may get the
                // same handle while earlier work runs; every call has its own
                // outputs, checked after the loop
                std::vector<Dev> v(iters), l(iters);
                std::vector<int> kind(iters);
                for (int i = 0; i < iters; i++) {
                    const int vk = kVerifyPattern[(i + 3 * t) % kPat];
                    kind[i] = vk;
                    v[i] = upload(std::vector<uint8_t>(in.vn[vk], kSentinel));
                    l[i] = upload(std::vector<uint8_t>(2 * in.vn[vk], kSentinel));
                }
                CK(hipDeviceSynchronize());
                for (int i = 0; i < iters; i++) {
                    hipStream_t s;
                    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                    const int vk = kind[i];
                    const int rc = wg_verify_desc(static_cast<const uint8_t *>(in.vbuf[vk].p),
                                                  static_cast<const wg_pkt_desc *>(in.vdesc[vk].p), in.vn[vk],
                                                  static_cast<uint8_t *>(v[i].p), static_cast<uint16_t *>(l[i].p), s);
                    if (rc != WG_OK)
                        errors++;
                    calls[t][kVerify]++;
                    CK(hipStreamDestroy(s));
                }
                CK(hipDeviceSynchronize());
                for (int i = 0; i < iters; i++) {
                    if (!same(v[i].p, in.vverdict[kind[i]], nullptr, o.h) || !same(l[i].p, in.vl4[kind[i]], nullptr, o.h))
                        bad[t][kVerify]++;
                    CK(hipFree(v[i].p));
                    CK(hipFree(l[i].p));
                }
            } else {
                for (int i = 0; i < iters; i++) {
                    for (int k = 0; k < kNumOps; k++) {
                        const Op op = (Op)((k + t + i) % kNumOps);
                        const int vk = kVerifyPattern[(i + 3 * t) % kPat];
                        refill(op, in, o, vk, st);
                        if (call(op, in, o, vk, st) != WG_OK)
                            errors++;
                        calls[t][op]++;
                        if (!check(op, in, o, vk, st))
                            bad[t][op]++;
                    }
                }
            }
            if (own)
                CK(hipStreamDestroy(own));
            o.release();
        });
    }
    for (auto &x : th) x.join();
    int total_bad = 0;
    std::printf("{\"mode\": \"conform\", \"stream\": \"%s\", \"threads\": %d, \"iters\": %d, \"errors\": %d, \"ops\": {",
                mode.c_str(), threads, iters, errors.load());
    for (int op = 0; op < kNumOps; op++) {
        int b = 0, c = 0;
        for (int t = 0; t < threads; t++) {
            b += bad[t][op];
            c += calls[t][op];
        }
        total_bad += b;
        std::printf("%s\"%s\": {\"calls\": %d, \"mismatched\": %d}", op ? ", " : "", op_name[op], c, b);
    }
    std::printf("}, \"mismatched\": %d}\n", total_bad);
    return total_bad == 0 && errors == 0 ? 0 : 1;
}

__global__ void empty_kernel(uint32_t *p) {
    if (p && threadIdx.x == 1024)
        *p = 0;
}

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int rate(const Inputs &in, int threads, int ncalls, bool small) {
    std::printf("{\"mode\": \"rate\", \"batches\": \"%s\", \"threads\": %d, \"calls_per_thread\": %d, \"ops\": {",
                small ? "small (64 packets / 64 segments / 2 super-buffers)" : "full", threads, ncalls);
    for (int op = 0; op <= kNumOps; op++) {  // kNumOps: the runtime's empty-kernel floor
        std::vector<double> enq(threads), done(threads);
        std::barrier sync_point(threads);
        std::vector<std::thread> th;
        std::atomic<int> errors{0};
        for (int t = 0; t < threads; t++) {
            th.emplace_back([&, t] {
                CK(hipSetDevice(0));
                Outs o;
                o.make(in);
                hipStream_t st;
                CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
                // untimed: the stream's first calls (verify state, code objects)
                for (int i = 0; i < 8; i++) {
                    if (op == kNumOps)
                        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr);
                    else if (call((Op)op, in, o, 2, st, small) != WG_OK)
                        errors++;
                }
                CK(hipStreamSynchronize(st));
                sync_point.arrive_and_wait();
                const double t0 = now_s();
                for (int i = 0; i < ncalls; i++) {
                    if (op == kNumOps)
                        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr);
                    else if (call((Op)op, in, o, 2, st, small) != WG_OK)
                        errors++;
                }
                const double t1 = now_s();
                CK(hipStreamSynchronize(st));
                const double t2 = now_s();
                enq[t] = ncalls / (t1 - t0);
                done[t] = ncalls / (t2 - t0);
                CK(hipStreamDestroy(st));
                o.release();
            });
        }
        for (auto &x : th) x.join();
        std::sort(enq.begin(), enq.end());
        std::sort(done.begin(), done.end());
        std::printf("%s\"%s\": {\"enqueue_calls_per_s_per_thread\": {\"median\": %.0f, \"min\": %.0f, \"max\": %.0f}, "
                    "\"completed_calls_per_s_per_thread\": {\"median\": %.0f, \"min\": %.0f}, \"errors\": %d}",
                    op ? ", " : "", op == kNumOps ? "runtime_empty_kernel" : op_name[op], enq[threads / 2], enq[0],
                    enq[threads - 1], done[threads / 2], done[0], errors.load());
    }
    std::printf("}}\n");
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s <dir> conform <threads> <iters> <own|perthread|legacy|churn> | rate <threads> <calls>\n",
                     argv[0]);
        return 2;
    }
    CK(hipSetDevice(0));
    Inputs in;
    in.read(argv[1]);
    const std::string mode = argv[2];
    const int threads = std::atoi(argv[3]);
    if (threads < 1 || threads > 64)
        return 2;
    int rc = 2;
    if (mode == "conform" && argc >= 6)
        rc = conform(in, threads, std::atoi(argv[4]), argv[5]);
    else if (mode == "rate")
        rc = rate(in, threads, std::atoi(argv[4]), argc >= 6 && std::string(argv[5]) == "small");
    CK(hipDeviceSynchronize());
    return rc;
}
