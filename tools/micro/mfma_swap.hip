// Is v_mfma_f32_16x16x32_bf16(b, a) the transpose of (a, b), bit for bit?  (operand K layout)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const __bf16* a, const __bf16* b, float* d1, float* d2) {
  const int l = threadIdx.x;
  bf16x8 av, bv;
  for (int e = 0; e < 8; ++e) { av[e] = a[l * 8 + e]; bv[e] = b[l * 8 + e]; }
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, z, 0, 0, 0);
  f32x4 y = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv, av, z, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {   // lane l: D[4(l/16) + r][l % 16]
    d1[(4 * (l / 16) + r) * 16 + l % 16] = x[r];
    d2[(4 * (l / 16) + r) * 16 + l % 16] = y[r];
  }
}
int main() {
  __bf16 ha[512], hb[512];
  srand(1);
  for (int i = 0; i < 512; ++i) { ha[i] = (__bf16)((rand() % 2001 - 1000) / 997.f); hb[i] = (__bf16)((rand() % 2001 - 1000) / 991.f); }
  __bf16 *a, *b; float *d1, *d2;
  hipMalloc(&a, 1024); hipMalloc(&b, 1024); hipMalloc(&d1, 1024); hipMalloc(&d2, 1024);
  hipMemcpy(a, ha, 1024, hipMemcpyHostToDevice); hipMemcpy(b, hb, 1024, hipMemcpyHostToDevice);
  k<<<1, 64>>>(a, b, d1, d2);
  float h1[256], h2[256];
  hipMemcpy(h1, d1, 1024, hipMemcpyDeviceToHost); hipMemcpy(h2, d2, 1024, hipMemcpyDeviceToHost);
  int bad = 0; double mx = 0;
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
    if (h1[i * 16 + j] != h2[j * 16 + i]) ++bad;
    double df = fabs(h1[i * 16 + j] - h2[j * 16 + i]); if (df > mx) mx = df;
  }
  // reference for the assumed layout: A[i][k] = a[(k/8*16 + i)*8 + k%8], B[k][j] = b[(k/8*16 + j)*8 + k%8]
  int bad_ref = 0;
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
    double s = 0; for (int kk = 0; kk < 32; ++kk) s += (double)(float)ha[((kk / 8) * 16 + i) * 8 + kk % 8] * (double)(float)hb[((kk / 8) * 16 + j) * 8 + kk % 8];
    if (fabs(s - h1[i * 16 + j]) > 1e-3) ++bad_ref;
  }
  printf("swap-transpose mismatches %d (max diff %g); layout-model mismatches %d\n", bad, mx, bad_ref);
  return 0;
}
