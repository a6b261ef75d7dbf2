// Development tool: per-phase s_memtime breakdown of the blind-rotation kernel
// on a 1024-gate 128-bit batch with random operands (timing only, no parity).
//   (round 4's -DTFHE_SPIN_STATS poll count and the duo form's phases: profiles/r04_spin_stats.txt,
//   DESIGN.md §4.3d; the duo form now lives in tools/ab/)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DTFHE_PHASE_PROF \
//         -Izig-tfhe_amd/csrc -o tools/bin/phase_prof tools/phase_prof.hip
// With -DTFHE_PHASE_PROF=2 (-o tools/bin/clock_probe) it is the clock probe instead: no phase
// marks, each wave's core-clock and 100 MHz tick deltas over its step loop, six launches.
#include "../zig-tfhe_amd/csrc/tfhe_kernels.hip"
#include "../zig-tfhe_amd/csrc/tfhe_kernels_whole.hip"
#include "ab/tfhe_ab_assist_dev.hip"  // "devN": the A/B copy of the assist form, VAR N

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using namespace tfhe;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char **argv) {
    const size_t B = argc > 1 ? atoi(argv[1]) : 1024;
    KParams P{700, 1024, 3, 6, 2, 9, 0x82080000u};
    std::vector<double> bk((size_t)P.n * 2 * P.L * 2 * 1024);
    srand(1);
    for (auto &x : bk) x = (rand() / (double)RAND_MAX - 0.5) * 1e6;
    std::vector<uint32_t> in((size_t)B * (P.n + 1)), tv(2048, 0x20000000u);
    for (auto &x : in) x = (uint32_t)rand() * 2654435761u;
    std::vector<C2> tw(512), twist(512);
    for (int k = 0; k < 512; k++) {
        twist[k] = {cos(k * (M_PI / 1024)), sin(k * (M_PI / 1024))};
        tw[k] = {cos(k * 0.01), -sin(k * 0.01)};
    }
    double *d_bk; uint32_t *d_in, *d_tv, *d_out; C2 *d_tw, *d_twist;
    CK(hipMalloc(&d_bk, bk.size() * 8));
    CK(hipMalloc(&d_in, in.size() * 4));
    CK(hipMalloc(&d_tv, 2048 * 4));
    CK(hipMalloc(&d_out, B * 2048 * 4));
    CK(hipMalloc(&d_tw, 512 * 16));
    CK(hipMalloc(&d_twist, 512 * 16));
    CK(hipMemcpy(d_bk, bk.data(), bk.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_in, in.data(), in.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tv, tv.data(), 2048 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_tw, tw.data(), 512 * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_twist, twist.data(), 512 * 16, hipMemcpyHostToDevice));
    DevTables T{d_twist, d_tw, {tw[2], tw[4], tw[5], tw[6]}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
#if TFHE_PHASE_PROF == 2
    const int reps = 6;  // the clock settles over the first launches
#else
    const int reps = 2;
#endif
    for (int rep = 0; rep < reps; rep++) {
        unsigned long long z[128] = {0};
#ifdef TFHE_PHASE_PROF
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), z, sizeof z));
#endif
        CK(hipEventRecord(e0));
        LaunchOpts O;  // form from argv[2]: "wide" = latency form, else the whole form
        const char *form = argc > 2 ? argv[2] : "whole";
        O.br_form = form[0] == 'w' && form[1] == 'i' ? 3 : 1;
        const bool assist = O.br_form == 1;  // L = 3 fused: the whole form with loader assist
        const bool dev = form[0] == 'd';
        const bool rc = std::string(form) == "widerc";  // the latency form with row counters (A/B form 30)
        if (rc)
            CK(ab_launch_wide_rc(P, T, nullptr, d_in, nullptr, nullptr, d_tv, (const double2 *)d_bk, d_out, BR_OUT_LV1, B,
                                 0, nullptr));
        else if (dev)
            CK(ab_launch_assist_dev(atoi(form + 3), dim3((unsigned)((B + 3) / 4)), dim3(512), 0, P, T, nullptr, d_in,
                                    nullptr, nullptr, d_tv, (const double2 *)d_bk, d_out, BR_OUT_LV1, B, nullptr));
        else
            CK(launch_blind_rotate(P, T, nullptr, d_in, nullptr, nullptr, d_tv, d_bk, d_out, BR_OUT_LV1, B, 0, O));
        CK(hipEventRecord(e1));
        CK(hipDeviceSynchronize());
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned long long c[128] = {0};
#ifdef TFHE_PHASE_PROF
        CK(hipMemcpyFromSymbol(c, HIP_SYMBOL(g_phase_cycles), sizeof c));
#endif
#if TFHE_PHASE_PROF == 2
        {  // clock probe: [off] core-clock ticks, [off + 1] waves, [off + 2] 100 MHz ticks, per wave group
            double ticks = 0, waves = 0, real = 0;
            for (int off = 0; off + 2 < 128; off += 8)
                if (c[off + 1]) ticks += c[off], waves += c[off + 1], real += c[off + 2];
            printf("rep %d: %.3f ms (%zu gates, %s); clock probe over %.0f waves: mean wave span %.3f ms "
                   "(s_memrealtime, 100 MHz), core clock %.4f GHz (s_memtime / s_memrealtime)\n",
                   rep, ms, B, form, waves, real / waves / 1e5, ticks / real * 0.1);
            continue;
        }
#endif
        if (O.br_form == 3) {  // latency form: per wave, per phase (ticks per step per gate)
            const char *wn0[16] = {"fwd(other)", "barrier1", "sum", "barrier2", "inverse(other)", "barrier3", "tail", "-",
                                   "row: gather", "row: digits+twist", "row: fft", "row: terms", "inv: fft", "inv: untwist+add", "row: prefetch issue", "-"};
            const char *wnrc[16] = {"fwd(other)", "-", "inv: row waits+sum", "-", "inv: operands", "barrier", "tail", "-",
                                    "row: gather", "row: digits+twist", "row: fft", "row: terms+count", "inv: fft", "inv: untwist+add", "row: prefetch, wait", "-"};
            const char **wn = rc ? wnrc : wn0;
            printf("rep %d: %.3f ms (%zu gates); s_memtime ticks per step, per wave:\n", rep, ms, B);
            for (int k = 0; k < 16; k++) {
                if (k == 6 || k == 7 || k > 14) continue;
                printf("  %-20s", wn[k]);
                for (int w = 0; w < 8; w++) printf(" %8.1f", c[w * 16 + k] / (double)B / P.n);
                printf("\n");
            }
            continue;
        }
        if (dev) {  // gates [0, 10), loaders [16, 24), per wave-step
            const char *gn[10] = {"gate: gather+tmp", "gate: pair0 digits+fft", "gate: pub waits", "gate: macs",
                                  "gate: tB wait+tbx", "gate: pairs1-2 digits+fft", "gate: fb hand-off", "gate: inverse a+store",
                                  "gate: r5 wait", "gate: r5 spectrum read"};
            const char *ln[8] = {"loader: vmcnt+pub", "loader: fb wait", "loader: inverse b", "loader: acc_b+gather+tB",
                                 "loader: refill wait+issue+r5 digits", "loader: tail", "loader: tb_read wait", "loader: row-5 fft+store"};
            double tot = 0;
            for (int k = 0; k < 10; k++) tot += c[k];
            printf("rep %d: %.3f ms (%zu gates, %s); s_memtime ticks per wave-step:\n", rep, ms, B, form);
            for (int k = 0; k < 10; k++) printf("  %-36s %9.1f  %5.1f%%\n", gn[k], c[k] / (double)B / P.n, 100.0 * c[k] / tot);
            printf("  %-36s %9.1f\n", "gate total", tot / B / P.n);
            for (int k = 0; k < 8; k++) printf("  %-36s %9.1f\n", ln[k], c[16 + k] / (double)B / P.n);
            continue;
        }
        if (assist) {  // gates [0, 8), loaders [8, 14), per wave-step
            const char *gn[8] = {"gate: gather+tmp", "gate: pair0 digits+fft", "gate: pub waits", "gate: macs",
                                 "gate: tB wait+tbx", "gate: pairs1-2 digits+fft", "gate: fb hand-off", "gate: inverse a+store"};
            const char *ln[6] = {"loader: vmcnt+pub", "loader: fb wait", "loader: inverse b", "loader: acc_b+gather+tB",
                                 "loader: refill wait+issue", "loader: tail"};
            double tot = 0;
            for (int k = 0; k < 8; k++) tot += c[k];
            printf("rep %d: %.3f ms (%zu gates, assist form); s_memtime ticks per wave-step:\n", rep, ms, B);
            for (int k = 0; k < 8; k++) printf("  %-26s %9.1f  %5.1f%%\n", gn[k], c[k] / (double)B / P.n, 100.0 * c[k] / tot);
            printf("  %-26s %9.1f\n", "gate total", tot / B / P.n);
            for (int k = 0; k < 6; k++) printf("  %-26s %9.1f\n", ln[k], c[8 + k] / (double)B / P.n);
            continue;
        }
        const char *nm[8] = {"tmp", "fwd-fft(pairs)", "slot wait", "mac", "counter add", "inverse+add", "tail", "dma-issue"};
        double tot = 0;
        for (int k = 0; k < 8; k++) tot += c[k];  // whole form: [k], loaders [8 + q]
        printf("rep %d: %.3f ms; cycles per wave-step (s_memtime ticks):\n", rep, ms);
        for (int k = 0; k < 8; k++)
            printf("  %-16s %10.1f  %5.1f%%\n", nm[k], c[k] / (double)B / P.n, 100.0 * c[k] / tot);
        printf("  total            %10.1f\n", tot / B / P.n);
        {  // loader waves (one per gate wave)
            const char *ln[3] = {"loader: DMA landing", "loader: wait gates", "loader: issue"};
            for (int k = 0; k < 3; k++) printf("  %-22s %10.1f\n", ln[k], c[8 + k] / (double)B / P.n);
        }
    }
    return 0;
}
