// Probe: operand lane layout of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3,
// unit block scales) on gfx950. Tries candidate (lane, byte) -> k maps and
// reports which one reproduces a host fp32 reference exactly.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void mm(const v8i* a, const v8i* b, v4f* c) {
  v4f acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[threadIdx.x], b[threadIdx.x], acc, 0, 0, 0, 127, 0, 127);
  c[threadIdx.x] = acc;
}

static int kmap(int cand, int l, int j) {
  int g = l >> 4;
  switch (cand) {
    case 0: return 32 * g + j;
    case 1: return 16 * g + (j & 15) + 64 * (j >> 4);
    case 2: return 8 * g + (j & 7) + 32 * (j >> 3);
    case 3: return 4 * g + (j & 3) + 16 * (j >> 2);
    default: return -1;
  }
}

int main() {
  const unsigned char enc[5] = {0x00, 0x30, 0x38, 0x40, 0xB8};  // 0, .5, 1, 2, -1 (e4m3fn)
  const float val[5] = {0.f, 0.5f, 1.f, 2.f, -1.f};
  srand(1);
  static int A[16][128], B[128][16];
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 128; ++k) A[i][k] = rand() % 5;
  for (int k = 0; k < 128; ++k) for (int n = 0; n < 16; ++n) B[k][n] = rand() % 5;
  float ref[16][16];
  for (int i = 0; i < 16; ++i) for (int n = 0; n < 16; ++n) {
    float s = 0; for (int k = 0; k < 128; ++k) s += val[A[i][k]] * val[B[k][n]]; ref[i][n] = s; }
  v8i *da, *db; v4f* dc;
  hipMalloc(&da, 64 * 32); hipMalloc(&db, 64 * 32); hipMalloc(&dc, 64 * 16);
  for (int cand = 0; cand < 4; ++cand) {
    unsigned char ha[64][32], hb[64][32];
    for (int l = 0; l < 64; ++l) for (int j = 0; j < 32; ++j) {
      int k = kmap(cand, l, j);
      ha[l][j] = enc[A[l & 15][k]];
      hb[l][j] = enc[B[k][l & 15]];
    }
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, da, db, dc);
    float hc[64][4];
    hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
      int row = 4 * (l >> 4) + r, col = l & 15;
      if (hc[l][r] != ref[row][col]) ++bad;
    }
    printf("candidate %d: %s (%d/256 mismatches)\n", cand, bad ? "no" : "MATCH", bad);
  }
  return 0;
}
