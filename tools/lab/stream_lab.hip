// Weight-stream read-pattern lab for the decode GEMV (round 4): how fast can 8 waves per workgroup
// read an [N, K] bf16 matrix once, by access pattern?
//   P0: the GEMV's MFMA-fragment pattern: one wave-instruction = 16 rows x 64 B (lane l: row l & 15,
//       16 B at 8 (l >> 4)), 16 such loads in flight per wave, k-steps round-robin over the waves
//   P1: one wave-instruction = 1 KB contiguous of one row (lane l: 16 B at 16 l), each wave
//       streams whole rows, 16 loads in flight
//   P2: P0 with non-temporal loads
// The values are summed into registers (kept live), so nothing is elided.
// Build: hipcc --offload-arch=gfx950 -O3 -o stream_lab tools/lab/stream_lab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef unsigned short u16;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

template <int P>
__global__ __launch_bounds__(512) void stream_k(const u16* __restrict__ W, int64_t N, int64_t K, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  u32x4 acc = {0, 0, 0, 0};
  if (P == 0 || P == 2) {
    const int64_t n0 = (int64_t)blockIdx.x * 16;
    const u16* row = W + (n0 + (lane & 15)) * K + 8 * (lane >> 4);
    const int64_t nk = K / 32;
    for (int64_t j0 = 0; j0 * 8 < nk; j0 += 16) {
      u32x4 v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int64_t ks = (j0 + i) * 8 + wave;
        const u32x4* ptr = reinterpret_cast<const u32x4*>(row + (ks < nk ? ks : 0) * 32);
        v[i] = P == 2 ? __builtin_nontemporal_load(ptr) : *ptr;
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= v[i];
    }
  } else {
    // 16 rows per workgroup, 2 rows per wave, 1 KB per instruction
    const int64_t n0 = (int64_t)blockIdx.x * 16 + wave * 2;
    for (int r = 0; r < 2; ++r) {
      const u16* row = W + (n0 + r) * K + 8 * lane;
      for (int64_t c0 = 0; c0 < K; c0 += 512 * 16) {
        u32x4 v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int64_t c = c0 + 512 * i;
          v[i] = *reinterpret_cast<const u32x4*>(row + (c < K ? c : 0));
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) acc ^= v[i];
      }
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[threadIdx.x] = 1.f;
}

int main() {
  const int64_t shapes[][2] = {{12288, 4096}, {4096, 4096}, {22016, 4096}, {4096, 11008}, {32064, 4096}};
  u16* W;
  float* out;
  hipMalloc(&W, (size_t)32064 * 11008 * 2);
  hipMalloc(&out, 4096);
  hipMemset(W, 1, (size_t)32064 * 11008 * 2);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (auto& sh : shapes) {
    const int64_t N = sh[0], K = sh[1];
    for (int P = 0; P < 3; ++P) {
      auto run = [&]() {
        if (P == 0) stream_k<0><<<N / 16, 512>>>(W, N, K, out);
        else if (P == 1) stream_k<1><<<N / 16, 512>>>(W, N, K, out);
        else stream_k<2><<<N / 16, 512>>>(W, N, K, out);
      };
      for (int i = 0; i < 3; ++i) run();
      hipEventRecord(a);
      const int it = 50;
      for (int i = 0; i < it; ++i) run();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double us = ms * 1e3 / it;
      printf("N %6ld K %6ld P%d  %8.2f us  %7.1f GB/s\n", (long)N, (long)K, P, us, N * K * 2 / us / 1e3);
    }
  }
  return 0;
}
