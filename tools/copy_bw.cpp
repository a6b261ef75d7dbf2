// Host <-> device copy rates on the GPU box, for the host-buffer pipeline
// (DESIGN.md §2.1): pageable vs pinned hipMemcpyAsync and host memcpy into
// pinned staging with 1..8 threads, at the 1,024-gate batch's sizes.
//   hipcc -O2 -o tools/bin/copy_bw tools/copy_bw.cpp -lpthread && tools/bin/copy_bw
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));    \
            return 1;                                                       \
        }                                                                   \
    } while (0)

int main() {
    const size_t in_bytes = 2 * 1024 * 701 * 4, out_bytes = 1024 * 701 * 4;
    std::vector<char> src(in_bytes, 1), dst(out_bytes, 0);
    char *pin_in = nullptr, *pin_out = nullptr, *dev = nullptr;
    CK(hipHostMalloc((void **)&pin_in, in_bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void **)&pin_out, out_bytes, hipHostMallocDefault));
    CK(hipMalloc((void **)&dev, in_bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto rate = [](size_t b, double t) { return b / t / 1e9; };
    for (int rep = 0; rep < 3; rep++) {
        double t0 = now();
        CK(hipMemcpyAsync(dev, src.data(), in_bytes, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        double t1 = now();
        CK(hipMemcpyAsync(dev, pin_in, in_bytes, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        double t2 = now();
        CK(hipMemcpyAsync(dst.data(), dev, out_bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        double t3 = now();
        CK(hipMemcpyAsync(pin_out, dev, out_bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        double t4 = now();
        std::printf("H2D %.1f MB: pageable %.3f ms (%.1f GB/s), pinned %.3f ms (%.1f GB/s); D2H %.1f MB: pageable %.3f ms "
                    "(%.1f GB/s), pinned %.3f ms (%.1f GB/s)\n",
                    in_bytes / 1e6, (t1 - t0) * 1e3, rate(in_bytes, t1 - t0), (t2 - t1) * 1e3, rate(in_bytes, t2 - t1),
                    out_bytes / 1e6, (t3 - t2) * 1e3, rate(out_bytes, t3 - t2), (t4 - t3) * 1e3, rate(out_bytes, t4 - t3));
    }
    for (int th : {1, 2, 4, 8}) {
        double best = 1e9;
        for (int rep = 0; rep < 5; rep++) {
            double t0 = now();
            std::vector<std::thread> v;
            for (int k = 0; k < th; k++)
                v.emplace_back([&, k] {
                    const size_t a = in_bytes * k / th, b = in_bytes * (k + 1) / th;
                    std::memcpy(pin_in + a, src.data() + a, b - a);
                });
            for (auto &x : v) x.join();
            best = std::min(best, now() - t0);
        }
        std::printf("memcpy pageable -> pinned %.1f MB, %d thread(s): %.3f ms (%.1f GB/s)\n", in_bytes / 1e6, th, best * 1e3,
                    rate(in_bytes, best));
    }
    // pipelined: 4 chunks, memcpy chunk k then its H2D, on one thread
    {
        double t0 = now();
        const size_t c = in_bytes / 4;
        for (int k = 0; k < 4; k++) {
            std::memcpy(pin_in + k * c, src.data() + k * c, c);
            CK(hipMemcpyAsync(dev + k * c, pin_in + k * c, c, hipMemcpyHostToDevice, s));
        }
        CK(hipStreamSynchronize(s));
        std::printf("staged H2D in 4 chunks, 1 thread: %.3f ms\n", (now() - t0) * 1e3);
    }
    // concurrent pageable H2D / D2H: T host threads, each its own stream and slice
    {
        std::vector<hipStream_t> ss(8);
        for (auto &x : ss) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        std::vector<char> back(in_bytes);
        for (int th : {1, 2, 4, 8}) {
            double best_h = 1e9, best_d = 1e9;
            for (int rep = 0; rep < 5; rep++) {
                for (int dir = 0; dir < 2; dir++) {
                    double t0 = now();
                    std::vector<std::thread> v;
                    for (int k = 0; k < th; k++)
                        v.emplace_back([&, k] {
                            const size_t a = in_bytes * k / th, b = in_bytes * (k + 1) / th;
                            if (dir == 0)
                                (void)hipMemcpyAsync(dev + a, src.data() + a, b - a, hipMemcpyHostToDevice, ss[k]);
                            else
                                (void)hipMemcpyAsync(back.data() + a, dev + a, b - a, hipMemcpyDeviceToHost, ss[k]);
                            (void)hipStreamSynchronize(ss[k]);
                        });
                    for (auto &x : v) x.join();
                    (dir == 0 ? best_h : best_d) = std::min(dir == 0 ? best_h : best_d, now() - t0);
                }
            }
            std::printf("concurrent pageable %.1f MB, %d thread(s)/stream(s): H2D %.3f ms (%.1f GB/s), D2H %.3f ms (%.1f GB/s)\n",
                        in_bytes / 1e6, th, best_h * 1e3, rate(in_bytes, best_h), best_d * 1e3, rate(in_bytes, best_d));
        }
    }
    // Round 6: the multi-device host path's per-shard copies.  T host
    // threads, each one shard of 1,024 gates (H2D a + b, 2 x 2.87 MB; D2H out, 2.87 MB) on its own
    // stream and its own caller buffers, three ways: pageable hipMemcpyAsync from the caller's
    // buffer; pinned staging (host memcpy into the shard's own pinned arena, then the DMA; the
    // library's TFHE_OPT_HOST_STAGING = 1); hipHostRegister of the caller's slice for the call
    // (register, DMA, unregister).  One device here, so the DMAs of all shards share one link:
    // per-shard wall time at T threads is an upper bound on what T distinct devices would see.
    {
        const size_t a_bytes = 1024 * 701 * 4;
        const int T = 8;
        std::vector<std::vector<char>> ca(T, std::vector<char>(a_bytes, 1)), cb(T, std::vector<char>(a_bytes, 2)),
            co(T, std::vector<char>(a_bytes, 0));
        std::vector<char *> pin(T), pout(T), dv(T);
        std::vector<hipStream_t> ss(T);
        for (int k = 0; k < T; k++) {
            CK(hipHostMalloc((void **)&pin[k], 2 * a_bytes, hipHostMallocDefault));
            CK(hipHostMalloc((void **)&pout[k], a_bytes, hipHostMallocDefault));
            CK(hipMalloc((void **)&dv[k], 3 * a_bytes));
            CK(hipStreamCreateWithFlags(&ss[k], hipStreamNonBlocking));
        }
        const char *names[3] = {"pageable", "pinned staging", "hipHostRegister"};
        for (int th : {1, 2, 4, 8}) {
            for (int mode = 0; mode < 3; mode++) {
                std::vector<double> walls;
                for (int rep = 0; rep < 7; rep++) {
                    double t0 = now();
                    std::vector<std::thread> v;
                    for (int k = 0; k < th; k++)
                        v.emplace_back([&, k] {
                            char *d = dv[k];
                            if (mode == 0) {
                                (void)hipMemcpyAsync(d, ca[k].data(), a_bytes, hipMemcpyHostToDevice, ss[k]);
                                (void)hipMemcpyAsync(d + a_bytes, cb[k].data(), a_bytes, hipMemcpyHostToDevice, ss[k]);
                                (void)hipMemcpyAsync(co[k].data(), d + 2 * a_bytes, a_bytes, hipMemcpyDeviceToHost, ss[k]);
                                (void)hipStreamSynchronize(ss[k]);
                            } else if (mode == 1) {
                                std::memcpy(pin[k], ca[k].data(), a_bytes);
                                (void)hipMemcpyAsync(d, pin[k], a_bytes, hipMemcpyHostToDevice, ss[k]);
                                std::memcpy(pin[k] + a_bytes, cb[k].data(), a_bytes);
                                (void)hipMemcpyAsync(d + a_bytes, pin[k] + a_bytes, a_bytes, hipMemcpyHostToDevice, ss[k]);
                                (void)hipMemcpyAsync(pout[k], d + 2 * a_bytes, a_bytes, hipMemcpyDeviceToHost, ss[k]);
                                (void)hipStreamSynchronize(ss[k]);
                                std::memcpy(co[k].data(), pout[k], a_bytes);
                            } else {
                                (void)hipHostRegister(ca[k].data(), a_bytes, hipHostRegisterDefault);
                                (void)hipHostRegister(cb[k].data(), a_bytes, hipHostRegisterDefault);
                                (void)hipHostRegister(co[k].data(), a_bytes, hipHostRegisterDefault);
                                (void)hipMemcpyAsync(d, ca[k].data(), a_bytes, hipMemcpyHostToDevice, ss[k]);
                                (void)hipMemcpyAsync(d + a_bytes, cb[k].data(), a_bytes, hipMemcpyHostToDevice, ss[k]);
                                (void)hipMemcpyAsync(co[k].data(), d + 2 * a_bytes, a_bytes, hipMemcpyDeviceToHost, ss[k]);
                                (void)hipStreamSynchronize(ss[k]);
                                (void)hipHostUnregister(ca[k].data());
                                (void)hipHostUnregister(cb[k].data());
                                (void)hipHostUnregister(co[k].data());
                            }
                        });
                    for (auto &x : v) x.join();
                    walls.push_back(now() - t0);
                }
                std::sort(walls.begin(), walls.end());
                const double med = walls[walls.size() / 2], bytes = 3.0 * a_bytes * th;
                std::printf("shards %d x 1,024 gates (8.6 MB each), %-15s: median %.3f ms (min %.3f), %.1f GB/s total\n",
                            th, names[mode], med * 1e3, walls[0] * 1e3, bytes / med / 1e9);
            }
        }
    }
    return 0;
}
