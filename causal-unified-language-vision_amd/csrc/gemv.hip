// Weight-streaming product for the decode step (reference
// cullavo/arch_cullavo.py:605-636, every Linear of the cached forward at one token per sequence):
// Y[M, N] = X[M, K] W[N, K]^T with M = B <= 16 rows. The work is reading W once (2 N K bytes;
// 13.2 GB per 7B decode step): HBM-bound, nothing to tile for reuse. gemm.hip dispatches here for
// a_layout = b_layout = 0 and M <= 16 (cullavo_gemm_plan tile 14).
//
// gfx950 design: one workgroup per 16 weight rows, 8 waves splitting K into contiguous ranges.
// Per 32-deep k-step a wave loads its W fragment straight from HBM into the MFMA A-operand layout
// (lane l: row n0 + (l & 15), 8 k at 8 (l >> 4): 16 B per lane, 16 rows x 64 B per instruction)
// and the matching X fragment (B-operand, row b = l & 15, zero for b >= M; X is tiny and stays
// in L2), then one v_mfma_f32_16x16x32_bf16 accumulates C^T[n][b]. Loads go out in batches of 16
// k-steps (16 KiB of W in flight per wave, 128 KiB per CU) before any MFMA consumes them. The
// eight K-range partials are summed through LDS in a fixed wave order (deterministic) and the
// full GEMM epilogue (bias, LoRA addend, activation, residual, beta; store4 of gemm_common.h)
// writes C.
#include "gemm_common.h"

namespace {
using namespace cvgemm;

constexpr int kGemvWaves = 8;
constexpr int kGemvBatch = 16;  // k-steps per load batch

template <int CT>
__global__ __launch_bounds__(512, 1) void gemv_k(GemmArgs p) {
  __shared__ f32x4 red[kGemvWaves][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n0 = (int64_t)blockIdx.x * 16;
  const int64_t nk = cdiv(p.K, 32);
  const int64_t per = cdiv(nk, kGemvWaves);
  const int64_t kb = wave * per, ke = min(nk, kb + per);
  const int r = lane & 15, g = lane >> 4;
  const u16* wrow = p.B + min(n0 + r, p.N - 1) * p.ldb + 8 * g;
  const bool xrow = r < p.M;
  const u16* xp = p.A + (xrow ? r : 0) * p.lda + 8 * g;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t k0 = kb; k0 < ke; k0 += kGemvBatch) {
    frag8 w[kGemvBatch], x[kGemvBatch];
#pragma unroll
    for (int i = 0; i < kGemvBatch; ++i) {
      const int64_t k = (k0 + i) * 32 + 8 * g;  // this lane's first k of step k0 + i
      const bool in = k0 + i < ke && k < p.K;
      const int64_t off = in ? (k0 + i) * 32 : 0;
      w[i] = in ? __builtin_bit_cast(frag8, *reinterpret_cast<const u16x8*>(wrow + off)) : frag8{};
      x[i] = (in && xrow) ? __builtin_bit_cast(frag8, *reinterpret_cast<const u16x8*>(xp + off)) : frag8{};
    }
#pragma unroll
    for (int i = 0; i < kGemvBatch; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[i], x[i], acc, 0, 0, 0);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0) {
    f32x4 s = red[0][lane];
#pragma unroll
    for (int w2 = 1; w2 < kGemvWaves; ++w2) s += red[w2][lane];
    store4<CT>(p, s, r, n0 + 4 * g);
  }
}

}  // namespace

int cvgemm_launch_gemv(const cvgemm::GemmArgs& p, bool f32, hipStream_t s) {
  const unsigned grid = (unsigned)cdiv(p.N, 16);
  if (f32) gemv_k<CULLAVO_DT_F32><<<grid, 64 * kGemvWaves, 0, s>>>(p);
  else gemv_k<CULLAVO_DT_BF16><<<grid, 64 * kGemvWaves, 0, s>>>(p);
  return cullavo_check_launch("gemv");
}
