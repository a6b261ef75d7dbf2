// Lane maps of v_mfma_i32_32x32x32_i8 on gfx950, checked with exact integer
// data against candidate maps (the key-switch GEMM).
//   hipcc --offload-arch=gfx950 -O2 -o tools/bin/mfma_i8_probe tools/mfma_i8_probe.hip && tools/bin/mfma_i8_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k_probe(const int8_t *a, const int8_t *b, int *d) {
    const int l = threadIdx.x;
    v4i af, bf;
    for (int w = 0; w < 4; w++) {
        int x = 0, y = 0;
        for (int e = 0; e < 4; e++) {
            x |= (int)(uint8_t)a[l * 16 + w * 4 + e] << (8 * e);
            y |= (int)(uint8_t)b[l * 16 + w * 4 + e] << (8 * e);
        }
        af[w] = x;
        bf[w] = y;
    }
    v16i c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, bf, c, 0, 0, 0);
    for (int r = 0; r < 16; r++) d[l * 16 + r] = c[r];
}

int main() {
    int8_t ha[64 * 16], hb[64 * 16];
    srand(7);
    for (int i = 0; i < 64 * 16; i++) {
        ha[i] = (int8_t)(rand() % 255 - 127);
        hb[i] = (int8_t)(rand() % 255 - 127);
    }
    int8_t *da, *db;
    int *dd;
    (void)hipMalloc(&da, sizeof ha);
    (void)hipMalloc(&db, sizeof hb);
    (void)hipMalloc(&dd, 64 * 16 * 4);
    (void)hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, da, db, dd);
    int hd[64 * 16];
    (void)hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
    // candidate k maps for lane l (r = l & 31, h = l >> 5), element e < 16
    auto kmap = [](int cand, int h, int e) {
        switch (cand) {
        case 0: return 16 * h + e;                          // contiguous halves
        case 1: return e < 8 ? 8 * h + e : 16 + 8 * h + e - 8;  // two K=16 steps
        case 2: return 2 * e + h;                           // interleaved
        default: return 4 * (e / 4) * 2 + 4 * h + e % 4;    // 4-byte groups interleaved
        }
    };
    for (int ca = 0; ca < 4; ca++)
        for (int cb = 0; cb < 4; cb++) {
            int A[32][32], B[32][32];
            for (int l = 0; l < 64; l++)
                for (int e = 0; e < 16; e++) {
                    A[l & 31][kmap(ca, l >> 5, e)] = ha[l * 16 + e];
                    B[kmap(cb, l >> 5, e)][l & 31] = hb[l * 16 + e];
                }
            int bad = 0;
            for (int l = 0; l < 64; l++)
                for (int reg = 0; reg < 16; reg++) {
                    const int col = l & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5);
                    int s = 0;
                    for (int k = 0; k < 32; k++) s += A[row][k] * B[k][col];
                    bad += s != hd[l * 16 + reg];
                }
            std::printf("A map %d, B map %d: %d of 1024 outputs differ%s\n", ca, cb, bad, bad ? "" : "  <== match");
        }
    return 0;
}
