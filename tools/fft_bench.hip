// Development micro-benchmark: throughput of the device FFT building blocks
// (fft512_x2 / fft512<1>) at one wave per SIMD, registers only in/out.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Izig-tfhe_amd/csrc -o tools/bin/fft_bench tools/fft_bench.hip
#include "../zig-tfhe_amd/csrc/tfhe_device.hpp"
#include <cstdio>
using namespace tfhe;

// three transforms interleaved through one exchange buffer (program-order reuse)
template <bool INV, class TW>
DEV void fft512_x3(C2 (*d)[8], C2 *xb, const TW &T, int t) {
    C2 wb_[7], wc_[7];
    passA<INV>(d[0], T.a);
    ex1_write(d[0], xb, t);
    wave_sync();
    passA<INV>(d[1], T.a);
    ex1_read(d[0], xb, t);
    ex1_write(d[1], xb, t);
    wave_sync();
    passA<INV>(d[2], T.a);
    ex1_read(d[1], xb, t);
    ex1_write(d[2], xb, t);
    wave_sync();
    T.pass_b(wb_, t);
    passBC<INV>(d[0], wb_);
    ex1_read(d[2], xb, t);
    ex2_write(d[0], xb, t);
    wave_sync();
    passBC<INV>(d[1], wb_);
    ex2_read(d[0], xb, t);
    ex2_write(d[1], xb, t);
    wave_sync();
    passBC<INV>(d[2], wb_);
    ex2_read(d[1], xb, t);
    ex2_write(d[2], xb, t);
    wave_sync();
    T.pass_c(wc_, t);
    passBC<INV>(d[0], wc_);
    ex2_read(d[2], xb, t);
    wave_sync();
    passBC<INV>(d[1], wc_);
    passBC<INV>(d[2], wc_);
}

template <int MODE, int W = 1>
__global__ __launch_bounds__(256 * W, 1) void k_bench(DevTables TT, double *out, int iters) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[8192 + 8192 + 4 * W * 16384];
    C2 *s_tw = reinterpret_cast<C2 *>(smem);
    C2 *s_twist = reinterpret_cast<C2 *>(smem + 8192);
    const int tid = threadIdx.x, t = tid & 63, w = tid >> 6;
    C2 *xb = reinterpret_cast<C2 *>(smem + 16384 + w * 16384);
    for (int x = tid; x < 511; x += 256 * W) s_tw[x] = TT.tw[x];
    for (int x = tid; x < 512; x += 256 * W) s_twist[x] = TT.twist[x];
    __syncthreads();
    LdsTw T;
    T.init(s_tw, TT);
    C2 d[3][8];
    for (int q = 0; q < 8; q++) {
        d[0][q] = c2(t * 0.001 + q, q * 0.5);
        d[1][q] = c2(t * 0.002 - q, q * 0.25);
        d[2][q] = c2(t * 0.003 - q, q * 0.125);
    }
    for (int it = 0; it < iters; it++) {
        if (MODE == 0) fft512_x2<false, true>(d, xb, T, t);
        if (MODE == 4) fft512_x3<false>(d, xb, T, t);
        if (MODE == 1) { fft512<1, false>(d, xb, T, t); fft512<1, false>(d + 1, xb, T, t); }
        if (MODE == 2) { C2 w[7]; T.pass_b(w, t); passA<false>(d[0], T.a); passA<false>(d[1], T.a); passBC<false>(d[0], w); passBC<false>(d[1], w); passBC<false>(d[0], w); passBC<false>(d[1], w); }
        if (MODE == 3) { passA<false>(d[0], T.a); passA<false>(d[1], T.a); ex1_write(d[0], xb, t); ex1_write(d[1], xb + 512, t); wave_sync(); ex1_read(d[0], xb, t); ex1_read(d[1], xb + 512, t); wave_sync();}
    }
    double s = 0;
    for (int q = 0; q < 8; q++) s += d[0][q].x + d[1][q].y + d[2][q].x;
    out[blockIdx.x * 256 * W + tid] = s;
}

int main() {
    C2 *tw, *twist; double *out;
    hipMalloc(&tw, 512 * 16); hipMalloc(&twist, 512 * 16); hipMalloc(&out, 2048 * 256 * 8);
    std::vector<C2> h(512);
    for (int k = 0; k < 512; k++) h[k] = {cos(k * 0.01), -sin(k * 0.01)};
    hipMemcpy(tw, h.data(), 512 * 16, hipMemcpyHostToDevice);
    hipMemcpy(twist, h.data(), 512 * 16, hipMemcpyHostToDevice);
    DevTables T{twist, tw, {h[2], h[4], h[5], h[6]}};
    const int iters = 2000, blocks = 256;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const char *nm[5] = {"fft512_x2 (pair, one buffer)", "2 x fft512<1>", "passes only, no exchange", "passA + exchange only", "fft512_x3 (triple, one buffer)"};
    for (int rep = 0; rep < 2; rep++)
    for (int m = 0; m < 5; m++) {
        hipEventRecord(a);
        if (m == 0) hipLaunchKernelGGL(k_bench<0>, dim3(blocks), dim3(256), 0, 0, T, out, iters);
        if (m == 1) hipLaunchKernelGGL(k_bench<1>, dim3(blocks), dim3(256), 0, 0, T, out, iters);
        if (m == 2) hipLaunchKernelGGL(k_bench<2>, dim3(blocks), dim3(256), 0, 0, T, out, iters);
        if (m == 3) hipLaunchKernelGGL(k_bench<3>, dim3(blocks), dim3(256), 0, 0, T, out, iters);
        if (m == 4) hipLaunchKernelGGL(k_bench<4>, dim3(blocks), dim3(256), 0, 0, T, out, iters);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        // cycles per FFT per wave at 2.4 GHz (each iteration = 2 FFTs per wave)
        if (rep) printf("%-32s %8.3f ms  %7.0f cycles per FFT per wave  %6.1f ns per FFT per SIMD\n", nm[m], ms,
                        ms * 1e-3 * 2.4e9 / (iters * (m == 4 ? 3.0 : 2.0)), ms * 1e6 / (iters * (m == 4 ? 3.0 : 2.0)));
    }
    // two waves per SIMD (8 waves per CU, wave-private exchange buffers): SIMD throughput
    for (int rep = 0; rep < 2; rep++)
    for (int m = 0; m < 3; m++) {
        hipEventRecord(a);
        if (m == 0) hipLaunchKernelGGL((k_bench<0, 2>), dim3(blocks), dim3(512), 0, 0, T, out, iters);
        if (m == 1) hipLaunchKernelGGL((k_bench<1, 2>), dim3(blocks), dim3(512), 0, 0, T, out, iters);
        if (m == 2) hipLaunchKernelGGL((k_bench<2, 2>), dim3(blocks), dim3(512), 0, 0, T, out, iters);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (rep) printf("2 waves/SIMD: %-32s %8.3f ms  %6.1f ns per FFT per SIMD\n", nm[m], ms, ms * 1e6 / (iters * 2.0 * 2));
    }
    return 0;
}
