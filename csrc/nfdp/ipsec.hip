// IPsec ESP (AES-GCM) kernels: one lane per packet, AES T-table + S-box + GHASH 8-bit reduction
// constants staged in LDS (3.3 KB per workgroup); per-SA round keys and GHASH tables are read
// through the vector L1 (a batch usually touches few SAs).  See ipsec.h for the frame layout.
#include <hip/hip_runtime.h>

#include "host.h"
#include "ipsec.h"

namespace nfdp {

constexpr int kEspBlock = 256;
// Both held to 4 waves / SIMD (<= 128 VGPRs, no spills); profiles/r2_s25_esp_ab.txt, r2_s26_esp_ab.txt

template <bool ENC>
__global__ __launch_bounds__(kEspBlock, 4) void esp_kernel(EspBatch a, const uint32_t* te0_g, const uint8_t* sbox_g,
                                                        const uint64_t* rem_g) {
  __shared__ uint32_t te0[NFDP_ESP_TTABLES4 ? 1024 : 256];
  __shared__ uint8_t sbox[256];
  __shared__ uint64_t rem[256];
  for (int k = threadIdx.x; k < (NFDP_ESP_TTABLES4 ? 1024 : 256); k += kEspBlock) te0[k] = te0_g[k];
  sbox[threadIdx.x] = sbox_g[threadIdx.x];
  rem[threadIdx.x] = rem_g[threadIdx.x];
  __syncthreads();
  const EspTables tb{te0, sbox, rem};
  for (uint32_t i = blockIdx.x * kEspBlock + threadIdx.x; i < a.n; i += gridDim.x * kEspBlock) {
    if constexpr (ENC) esp_encrypt_one(tb, a, i);
    else esp_decrypt_one(tb, a, i);
  }
}

hipError_t launch_esp(const EspBatch& a, bool enc, const uint32_t* te0, const uint8_t* sbox, const uint64_t* rem,
                      int num_cus, hipStream_t s) {
  if (!a.in || !a.out || !a.in_len || !a.out_len || !a.status || !a.sa || !te0 || !sbox || !rem)
    return hipErrorInvalidValue;
  if (enc && !a.seq) return hipErrorInvalidValue;
  if (!enc && (!a.out_sa || !a.out_seq)) return hipErrorInvalidValue;
  if ((a.in_stride & 15u) || (a.out_stride & 15u) || a.in_stride < 64u || a.out_stride < 128u) return hipErrorInvalidValue;
  if (a.spd && ((a.spd_mask + 1) & a.spd_mask)) return hipErrorInvalidValue;
  if (a.rxsa && ((a.rxsa_mask + 1) & a.rxsa_mask)) return hipErrorInvalidValue;
  if (a.n == 0) return hipSuccess;
  const uint32_t blocks = (a.n + kEspBlock - 1) / kEspBlock;
  const uint32_t grid = blocks < (uint32_t)num_cus * 8u ? blocks : (uint32_t)num_cus * 8u;
  if (enc) hipLaunchKernelGGL(esp_kernel<true>, dim3(grid), dim3(kEspBlock), 0, s, a, te0, sbox, rem);
  else hipLaunchKernelGGL(esp_kernel<false>, dim3(grid), dim3(kEspBlock), 0, s, a, te0, sbox, rem);
  return hipGetLastError();
}

}  // namespace nfdp
