// Layout probe for v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 operands and unit (E8M0 127)
// scales: which k does byte j of lane l's 32-byte A/B fragment hold? Exact small-integer data;
// prints the max error of each hypothesis (0 = that layout is right).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void mm(const v8i* a, const v8i* b, float* d) {
  v16f c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[threadIdx.x], b[threadIdx.x], c, 0, 0, 0, 127,
                                                       0, 127);
  const int l = threadIdx.x;
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
    d[row * 32 + col] = c[r];
  }
}

static uint8_t e4m3(int v) {  // small integers -4..4
  static const uint8_t pos[5] = {0x00, 0x38, 0x40, 0x44, 0x48};
  return v < 0 ? (uint8_t)(0x80 | pos[-v]) : pos[v];
}
static int kmap(int hyp, int h, int j) {
  switch (hyp) {
    case 0: return 32 * h + j;
    case 1: return 8 * h + (j & 7) + 16 * (j >> 3);
    case 2: return 16 * h + (j & 15) + 32 * (j >> 4);
    default: return 4 * h + (j & 3) + 8 * (j >> 2);
  }
}

int main() {
  int A[32][64], B[64][32];
  float ref[32][32];
  srand(7);
  for (int i = 0; i < 32; ++i)
    for (int k = 0; k < 64; ++k) A[i][k] = rand() % 9 - 4;
  for (int k = 0; k < 64; ++k)
    for (int j = 0; j < 32; ++j) B[k][j] = rand() % 9 - 4;
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      int s = 0;
      for (int k = 0; k < 64; ++k) s += A[i][k] * B[k][j];
      ref[i][j] = (float)s;
    }
  v8i *da, *db;
  float* dd;
  hipMalloc(&da, 64 * 32);
  hipMalloc(&db, 64 * 32);
  hipMalloc(&dd, 32 * 32 * 4);
  for (int hyp = 0; hyp < 4; ++hyp) {
    uint8_t fa[64][32], fb[64][32];
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        const int k = kmap(hyp, l >> 5, j);
        fa[l][j] = e4m3(A[l & 31][k]);
        fb[l][j] = e4m3(B[k][l & 31]);
      }
    hipMemcpy(da, fa, sizeof(fa), hipMemcpyHostToDevice);
    hipMemcpy(db, fb, sizeof(fb), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, da, db, dd);
    float out[32][32];
    hipMemcpy(out, dd, sizeof(out), hipMemcpyDeviceToHost);
    double err = 0;
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) err = fmax(err, fabs(out[i][j] - ref[i][j]));
    printf("hypothesis %d max_err %g\n", hyp, err);
  }
  return 0;
}
