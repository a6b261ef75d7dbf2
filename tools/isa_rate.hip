// Development micro-benchmark: issue rate of the VALU instructions the
// blind-rotation kernel uses, as a function of waves per SIMD (1, 2, 4) and of
// independent chains per wave (4, 8, 16).  Event-timed over all 256 CUs; prints
// ns per wave-instruction per SIMD (lower = better) and, since round 6, the core
// clock the waves held (s_memtime over s_memrealtime at 100 MHz, as the clock probe)
// and cycles per wave-instruction per SIMD, which do not depend on that clock.
// Each configuration runs 8 warm launches first (the clock ramps over ~40 ms).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-value -o tools/bin/isa_rate tools/isa_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP, int C>
__device__ __forceinline__ void body(double (&a)[16], const double (&b)[16], unsigned (&u)[16], double sc) {
#pragma unroll
    for (int i = 0; i < C; i++) {
        if constexpr (OP == 0) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
        if constexpr (OP == 1) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
        if constexpr (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 15]));
        if constexpr (OP == 3) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(a[i]) : "v"(u[i]));
        if constexpr (OP == 4) {  // f64 add + u32 add alternating
            asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(u[(i + 1) & 15]));
        }
        if constexpr (OP == 5) asm volatile("v_trunc_f64 %0, %0" : "+v"(a[i]));
        if constexpr (OP == 6) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b[i]), "v"(b[(i + 1) & 15]));
        if constexpr (OP == 7) asm volatile("v_fmac_f64 %0, %1, %2" : "+v"(a[i]) : "v"(b[i]), "v"(b[(i + 1) & 15]));
        if constexpr (OP == 8) asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(a[i]) : "v"(b[i]));
        if constexpr (OP == 9) {  // fma with a lane-uniform (SGPR) multiplier, as the pass-A twiddles
            asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b[i]), "s"(sc));
        }
        if constexpr (OP == 10) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[i]) : "s"(sc));
    }
}
static const char *NAMES[] = {"v_add_f64", "v_mul_f64", "v_add_u32", "v_cvt_f64_i32", "add_f64+add_u32", "v_trunc_f64",
                              "v_fma_f64", "v_fmac_f64", "v_fma_f64 a*a+c", "v_fma_f64 sgpr", "v_add_f64 sgpr"};

template <int OP, int C>
__global__ void k_rate(double *out, int iters, double sc, unsigned long long *clk) {
    double a[16], b[16];
    unsigned u[16];
    for (int i = 0; i < 16; i++) {
        a[i] = threadIdx.x * 0.5 + i;
        b[i] = 1.0 + i * 1e-3;
        u[i] = threadIdx.x + i;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < iters; k++) {
        body<OP, C>(a, b, u, sc);
        body<OP, C>(a, b, u, sc);
        body<OP, C>(a, b, u, sc);
        body<OP, C>(a, b, u, sc);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {  // per wave: core-clock and 100 MHz ticks of its loop
        atomicAdd(clk, t1 - t0);
        atomicAdd(clk + 1, r1 - r0);
    }
    double s = 0;
    for (int i = 0; i < 16; i++) s += a[i] + u[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP, int C>
void run(double *out, unsigned long long *clk, int wps) {
    const int iters = 16000 / C, blocks = 256, threads = 256 * wps;
    for (int w = 0; w < 8; w++)  // warm launches: the clock settles
        hipLaunchKernelGGL((k_rate<OP, C>), dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001, clk);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e9;
    double ghz = 0;
    for (int r = 0; r < 3; r++) {
        hipMemset(clk, 0, 2 * sizeof(unsigned long long));
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_rate<OP, C>), dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c[2];
        hipMemcpy(c, clk, sizeof c, hipMemcpyDeviceToHost);
        if (ms < best) best = ms, ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 0;
    }
    const double ninst = (double)iters * 4 * C * (OP == 4 ? 2 : 1) * wps;  // per SIMD
    printf("%-16s chains %2d waves/SIMD %d  %.3f ms  %.3f ns/inst/SIMD  clock %.3f GHz  %.2f cycles/inst/SIMD\n",
           NAMES[OP], C, wps, best, best * 1e6 / ninst, ghz, best * 1e6 / ninst * ghz);
}

template <int OP>
void run_op(double *out, unsigned long long *clk) {
    run<OP, 4>(out, clk, 1);
    run<OP, 8>(out, clk, 1);
    run<OP, 16>(out, clk, 1);
    run<OP, 8>(out, clk, 2);
    run<OP, 16>(out, clk, 2);
    run<OP, 8>(out, clk, 4);
}

int main() {
    double *out;
    unsigned long long *clk;
    hipMalloc(&out, 256 * 1024 * sizeof(double));
    hipMalloc(&clk, 2 * sizeof(unsigned long long));
    run_op<0>(out, clk);
    run_op<1>(out, clk);
    run_op<2>(out, clk);
    run_op<3>(out, clk);
    run_op<4>(out, clk);
    run_op<5>(out, clk);
    run_op<6>(out, clk);
    run_op<7>(out, clk);
    run_op<8>(out, clk);
    run_op<9>(out, clk);
    run_op<10>(out, clk);
    hipDeviceSynchronize();
    return 0;
}
