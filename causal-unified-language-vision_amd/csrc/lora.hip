// LoRA adapters' input gradient with dropout, one launch per adapter group (SURVEY.md §8(f) row 1;
// reference cullavo/load_cullavo.py:94-112: peft LoraLayer, result = base(x) + lora_B(lora_A(
// dropout(x))) * scaling, and its autograd backward through the per-module nn.Dropout).
//
// For a group of n modules sharing the input x (q|k|v: 3, gate|up: 2, o: 1) the adapters add
//     dx += mask_m(t, f) / (1 - p) * (du_m A_m)[t][f]        m = 0 .. n-1, in order,
// with du_m = scaling * dy_m B_m [M, 64] and A_m [64, N] (lora_A.weight). Launched per module
// (cullavo_gemm_ex: layouts (0,1), K = 64, drop_operand 3, beta 1) each product re-reads and
// re-writes dx [M, N] and rehashes its mask; the group's modules are one pass here: each
// workgroup stages the n (du_m, A_m) K-tiles by LDS-DMA at once, keeps its dx values in registers
// and applies the modules in order with the epilogue arithmetic of the per-module product
// (gemm_common.h store8 with alpha = beta = 1: v = alpha acc, v = ms != 0 ? v ms : 0,
// v += beta old, rounded to bf16 after every module) on the same MFMA chain (tile_mfma, one
// 64-deep K-tile from zero) -- bitwise the per-module launches.
#include "gemm_common.h"

namespace {
using namespace cvgemm;

constexpr int LD_M = 64, LD_N = 256;                      // tokens x features per workgroup
constexpr int LD_TA = LD_M * BK * 2, LD_TB = LD_N * BK * 2;  // one module: 8 KiB du, 32 KiB A
constexpr int LD_STAGE = LD_TA + LD_TB;

struct LoraDxArgs {
  const u16* du;   // [M, ld_du]: module m's du in columns m*64 .. m*64+63
  int64_t ld_du;
  const u16* a;    // [n*64, ld_a]: lora_A weights stacked (module m in rows m*64 ..)
  int64_t ld_a;
  u16* dx;         // [M, ld_dx], accumulated in place
  int64_t ld_dx;
  int64_t M, N;
  int tiles_n;
  uint32_t thr;    // dropout threshold (16-bit), as cullavo_gemm_ex derives it from p
  float scale;     // 1 / (1 - p)
  float alpha, beta;
  uint64_t seed[3];
};

template <int NMOD>
__global__ __launch_bounds__(512, 1) void lora_dx_k(LoraDxArgs a) {
  constexpr int TMW = LD_M / 32, TN = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int64_t m0 = (int64_t)(blockIdx.x / a.tiles_n) * LD_M;
  const int64_t n0 = (int64_t)(blockIdx.x % a.tiles_n) * LD_N;
  const __amdgpu_buffer_rsrc_t rdu = make_rsrc(a.du, ((a.M - 1) * a.ld_du + NMOD * 64) * 2);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.a, ((NMOD * 64 - 1) * a.ld_a + a.N) * 2);
#pragma unroll
  for (int m = 0; m < NMOD; ++m) {
    dma_tile<0, LD_M, 8>(rdu, a.ld_du, m0, a.M, m * 64, NMOD * 64, smem + m * LD_STAGE, wave, lane);
    dma_tile<1, LD_N, 8>(ra, a.ld_a, n0, a.N, m * 64, NMOD * 64, smem + m * LD_STAGE + LD_TA, wave, lane);
  }
  // this lane's dx values, in the MFMA output layout (token row, 4 consecutive features)
  float ov[TMW][TN][4];
#pragma unroll
  for (int tm = 0; tm < TMW; ++tm) {
    const int64_t t = m0 + wm * (LD_M / 2) + tm * 16 + (lane & 15);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int64_t f = n0 + wn * (LD_N / 4) + tn * 16 + (lane >> 4) * 4;
      u16x4 o{};
      if (t < a.M && f < a.N) o = *reinterpret_cast<const u16x4*>(a.dx + t * a.ld_dx + f);
#pragma unroll
      for (int j = 0; j < 4; ++j) ov[tm][tn][j] = bf2f(o[j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int m = 0; m < NMOD; ++m) {
    f32x4 acc[TMW][TN];
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    tile_mfma<0, 1, LD_M, LD_N, TMW, TN>(smem + m * LD_STAGE, wm, wn, lane, acc);
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm) {
      const int64_t t = m0 + wm * (LD_M / 2) + tm * 16 + (lane & 15);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int64_t f = n0 + wn * (LD_N / 4) + tn * 16 + (lane >> 4) * 4;
        float ms[4];
        drop_scales<4>(a.seed[m], a.thr, a.scale, t, f, ms);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = acc[tm][tn][j] * a.alpha;
          v = ms[j] != 0.f ? v * ms[j] : 0.f;
          v += a.beta * ov[tm][tn][j];
          ov[tm][tn][j] = round_bf(v);
        }
      }
    }
  }
#pragma unroll
  for (int tm = 0; tm < TMW; ++tm) {
    const int64_t t = m0 + wm * (LD_M / 2) + tm * 16 + (lane & 15);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int64_t f = n0 + wn * (LD_N / 4) + tn * 16 + (lane >> 4) * 4;
      if (t < a.M && f < a.N) {
        u16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(ov[tm][tn][j]);
        *reinterpret_cast<u16x4*>(a.dx + t * a.ld_dx + f) = o;
      }
    }
  }
}

template <int NMOD>
int launch_lora_dx(const LoraDxArgs& a, hipStream_t s) {
  const int smem = NMOD * LD_STAGE;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lora_dx_k<NMOD>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int64_t blocks = cdiv(a.M, LD_M) * a.tiles_n;
  lora_dx_k<NMOD><<<(unsigned)blocks, 512, smem, s>>>(a);
  return cullavo_check_launch("lora_dx");
}

}  // namespace

extern "C" int cullavo_lora_dx(int n_mod, int64_t M, int64_t N, const void* du, int64_t ld_du, const void* a_stack,
                               int64_t ld_a, void* dx, int64_t ld_dx, float drop_p, uint64_t seed0, uint64_t seed1,
                               uint64_t seed2, void* stream) {
  CV_REQUIRE(n_mod >= 1 && n_mod <= 3, CULLAVO_EINVAL, "lora_dx: 1 to 3 modules");
  CV_REQUIRE(M > 0 && N > 0 && N % 8 == 0, CULLAVO_EINVAL, "lora_dx: M > 0, N > 0 and N % 8 == 0");
  CV_REQUIRE(ld_du >= n_mod * 64 && ld_du % 8 == 0 && ld_a >= N && ld_a % 8 == 0 && ld_dx >= N && ld_dx % 4 == 0,
             CULLAVO_EINVAL, "lora_dx: leading dimensions (multiples of 8; ld_dx of 4)");
  CV_REQUIRE(drop_p >= 0.f && drop_p < 1.f, CULLAVO_EINVAL, "lora_dx: 0 <= drop_p < 1");
  CV_REQUIRE(du != nullptr && a_stack != nullptr && dx != nullptr, CULLAVO_EINVAL, "lora_dx: null operand");
  LoraDxArgs a{};
  a.du = (const u16*)du;
  a.ld_du = ld_du;
  a.a = (const u16*)a_stack;
  a.ld_a = ld_a;
  a.dx = (u16*)dx;
  a.ld_dx = ld_dx;
  a.M = M;
  a.N = N;
  a.tiles_n = (int)cdiv(N, LD_N);
  // cullavo_gemm_ex's derivation (gemm.hip), so the masks are the per-module launches' masks
  a.thr = (uint32_t)(drop_p * 65536.0f + 0.5f);
  a.scale = 1.f / (1.f - drop_p);
  a.alpha = 1.f;
  a.beta = 1.f;
  a.seed[0] = seed0;
  a.seed[1] = seed1;
  a.seed[2] = seed2;
  hipStream_t s = CV_STREAM(stream);
  if (n_mod == 1) return launch_lora_dx<1>(a, s);
  if (n_mod == 2) return launch_lora_dx<2>(a, s);
  return launch_lora_dx<3>(a, s);
}
