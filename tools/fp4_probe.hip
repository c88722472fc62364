// fp4_probe.hip — pin the gfx950 v_mfma_scale_f32_16x16x128_f8f6f4 operand layout with FP4
// (e2m1) operands on exact integer data, before the ACL uses it.
//   A: 16 x 128 in {-1, 0, +1} (ternary rule weights), B: 128 x 16 in {0, 1} (key bits).
//   Hypothesis: lane l holds A[row l & 15][k = 32 (l >> 4) + j] and B[k = 32 (l >> 4) + j][col l & 15]
//   for j = 0..31, element j in nibble j of the first 4 VGPRs (low nibble first); C/D: lane l holds
//   rows 4 (l >> 4) + r, col l & 15 (the shape's standard map).  Scales 2^0 (E8M0 127).
// Prints mismatches for both nibble orders; exact data, so 0 means the layout is right.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t fp4(int v) { return v == 0 ? 0x0u : (v > 0 ? 0x2u : 0xAu); }

template <int ORDER>
__global__ void probe(const int8_t* A, const int8_t* B, float* C) {
  const int l = threadIdx.x;
  v8i a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < 32; ++j) {
    const int k = 32 * (l >> 4) + j;
    const int nib = ORDER == 0 ? j : (j ^ 1);  // ORDER 1: high nibble first within a byte
    a[nib >> 3] |= (int)(fp4(A[(l & 15) * 128 + k]) << (4 * (nib & 7)));
    b[nib >> 3] |= (int)(fp4(B[k * 16 + (l & 15)]) << (4 * (nib & 7)));
  }
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 4, 4, 0, 0x7F7F7F7F, 0, 0x7F7F7F7F);
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);    \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

int main() {
  int8_t hA[16 * 128], hB[128 * 16];
  srand(7);
  for (int i = 0; i < 16 * 128; ++i) hA[i] = (int8_t)(rand() % 3 - 1);
  for (int i = 0; i < 128 * 16; ++i) hB[i] = (int8_t)(rand() & 1);
  float ref[256];
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      int s = 0;
      for (int k = 0; k < 128; ++k) s += hA[m * 128 + k] * hB[k * 16 + n];
      ref[m * 16 + n] = (float)s;
    }
  int8_t *dA, *dB;
  float* dC;
  CK(hipMalloc(&dA, sizeof hA));
  CK(hipMalloc(&dB, sizeof hB));
  CK(hipMalloc(&dC, 256 * sizeof(float)));
  CK(hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice));
  for (int order = 0; order < 2; ++order) {
    CK(hipMemset(dC, 0, 256 * sizeof(float)));
    if (order == 0) probe<0><<<1, 64>>>(dA, dB, dC);
    else probe<1><<<1, 64>>>(dA, dB, dC);
    CK(hipDeviceSynchronize());
    float h[256];
    CK(hipMemcpy(h, dC, sizeof h, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += h[i] != ref[i];
    std::printf("{\"order\": %d, \"mismatches\": %d, \"c00\": %.1f, \"ref00\": %.1f, \"c5_9\": %.1f, \"ref5_9\": %.1f}\n",
                order, bad, h[0], ref[0], h[5 * 16 + 9], ref[5 * 16 + 9]);
  }
  return 0;
}
