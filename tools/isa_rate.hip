// Development micro-benchmark: issue rate of the VALU instructions the
// blind-rotation kernel uses, as a function of waves per SIMD (1, 2, 4) and of
// independent chains per wave (4, 8, 16).  Event-timed over all 256 CUs; prints
// ns per wave-instruction per SIMD (lower = better).
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
__global__ void k_rate(double *out, int iters, double sc) {
    double a[16], b[16];
    unsigned u[16];
    for (int i = 0; i < 16; i++) {
        a[i] = threadIdx.x * 0.5 + i;
        b[i] = 1.0 + i * 1e-3;
        u[i] = threadIdx.x + i;
    }
    for (int k = 0; k < iters; k++) {
        body<OP, C>(a, b, u, sc);
        body<OP, C>(a, b, u, sc);
        body<OP, C>(a, b, u, sc);
        body<OP, C>(a, b, u, sc);
    }
    double s = 0;
    for (int i = 0; i < 16; i++) s += a[i] + u[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP, int C>
void run(double *out, int wps) {
    const int iters = 16000 / C, blocks = 256, threads = 256 * wps;
    hipLaunchKernelGGL((k_rate<OP, C>), dim3(blocks), dim3(threads), 0, 0, out, 10, 1.0000001);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e9;
    for (int r = 0; r < 3; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_rate<OP, C>), dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0000001);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double ninst = (double)iters * 4 * C * (OP == 4 ? 2 : 1) * wps;  // per SIMD
    printf("%-16s chains %2d waves/SIMD %d  %.3f ms  %.3f ns/inst/SIMD\n", NAMES[OP], C, wps, best,
           best * 1e6 / ninst);
}

template <int OP>
void run_op(double *out) {
    run<OP, 4>(out, 1);
    run<OP, 8>(out, 1);
    run<OP, 16>(out, 1);
    run<OP, 8>(out, 2);
    run<OP, 16>(out, 2);
    run<OP, 8>(out, 4);
}

int main() {
    double *out;
    hipMalloc(&out, 256 * 1024 * sizeof(double));
    run_op<0>(out);
    run_op<1>(out);
    run_op<2>(out);
    run_op<3>(out);
    run_op<4>(out);
    run_op<5>(out);
    run_op<6>(out);
    run_op<7>(out);
    run_op<8>(out);
    run_op<9>(out);
    run_op<10>(out);
    hipDeviceSynchronize();
    return 0;
}
