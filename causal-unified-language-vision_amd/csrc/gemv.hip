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

#include <cstdlib>

namespace {
using namespace cvgemm;

constexpr int kGemvWaves = 8;
constexpr int kGemvBatch = 16;  // W fragment loads per batch
// the default variant (cvgemm_launch_gemv's switch): contiguous K ranges, 8-load batches at two
// workgroups per CU -- 10-15 % faster than 16-load batches at one workgroup per CU on the 7B
// decode products (profiles/r04/decode/gemv_variants.txt)
constexpr int kGemvDefault = 4;

// Decode-row input transforms fused into the X fragment loads (cullavo_decode_linear): XF 0 none;
// 1 RMSNorm (x: the residual stream h [M, K]; each workgroup recomputes the M row statistics with
// rmsnorm_fwd_k's exact arithmetic, norms.hip, then x = bf16(w * bf16(h * rstd)) per element); 2
// SwiGLU (x: gate | up [M, 2K]; x = bf16(bf16(silu(g)) * u) as swiglu_fwd_k, elementwise.hip).
// Either way the values are bitwise those of the unfused kernels, without their launches.
DEV float gemv_silu(float x) { return x / (1.f + __expf(-x)); }

struct GemvArgs {
  GemmArgs g;
  const u16* xf_w;  // RMSNorm weight [K]
  float xf_eps;
};

template <int XF>
DEV frag8 gemv_xfrag(const GemvArgs& a, const u16* xp, int64_t off, int64_t k, const u16* xs_row) {
  if (XF == 1) return __builtin_bit_cast(frag8, *reinterpret_cast<const u16x8*>(xs_row + k));  // normalised, LDS
  const u16x8 xv = *reinterpret_cast<const u16x8*>(xp + off);
  if (XF == 0) return __builtin_bit_cast(frag8, xv);
  u16x8 o;
  {
    const u16x8 uv = *reinterpret_cast<const u16x8*>(xp + off + a.g.K);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(round_bf(gemv_silu(bf2f(xv[j]))) * bf2f(uv[j]));
  }
  return __builtin_bit_cast(frag8, o);
}

// ORDER 0: each wave a contiguous K range; ORDER 1: k-steps dealt round-robin over the 8 waves
// (at any moment a workgroup reads one contiguous 512-B run per weight row); RB: 16-row blocks per
// workgroup (each wave computes all of them over its k-steps). Measured alike on the 7B decode
// step (ORDER 0 / 1: 4.14 / 4.16 ms per token; RB 2: 4.66-4.79, profiles/r04/decode/); what
// mattered was occupancy (NBW below).
// NBW: W fragment loads per batch and wave. 16 keeps 151 VGPRs (one workgroup per CU: every
// workgroup's load ramp and reduction are exposed); 8 fits 2 workgroups per CU (86 VGPRs) and
// 4 fits 4, so one workgroup's ramp / reduction runs under the others' streams.
// NW: waves per workgroup (K split NW ways); 16 for the N = 4096 products, whose 256 workgroups
// are one per CU whatever the occupancy allows
// OT: output transform. 0 none; 1 SwiGLU of the product (cullavo_decode_linear transform 3): B
// holds 2N rows (gate rows [0, N), up rows [N, 2N), the fused gate|up weight) and the workgroup's
// 16 MFMA rows are 8 gate rows and the matching 8 up rows, so each lane pair (l, l + 32) holds
// g and u of one output: y = bf16(bf16(silu(g)) * u) with g, u first rounded to bf16 as the
// unfused product stores them -- bitwise swiglu_fwd_k of that product, without its launch or the
// [M, 2N] round trip.
// WNT: the weight fragments by non-temporal loads (read once per step; cullavo_gemv_set_nt)
template <int CT, int ORDER, int RB, int XF, int NBW = kGemvBatch, int NW = kGemvWaves, int OT = 0, bool WNT = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NBW >= 16 ? 2 : (NBW >= 8 || XF == 1) ? 4 : 8))) void gemv_k(GemvArgs a) {
  static_assert(OT == 0 || RB == 1, "SwiGLU pairing: one 16-row block per workgroup");
  const GemmArgs& p = a.g;
  __shared__ f32x4 red[NW][RB][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n0 = (int64_t)blockIdx.x * (OT == 1 ? 8 : 16 * RB);
  const int64_t nk = cdiv(p.K, 32);
  const int64_t per = cdiv(nk, NW);
  const int r = lane & 15, g = lane >> 4;
  const u16* wrow[RB];
  if constexpr (OT == 1) {
    wrow[0] = p.B + (min(n0 + (r & 7), p.N - 1) + (r >= 8 ? p.N : 0)) * p.ldb + 8 * g;
  } else {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) wrow[rb] = p.B + min(n0 + 16 * rb + r, p.N - 1) * p.ldb + 8 * g;
  }
  const bool xrow = r < p.M;
  const u16* xp = p.A + (xrow ? r : 0) * p.lda + 8 * g;
  // XF 1: the M normalised rows [M][K + 8] in LDS (dynamic; row pad 16 B: the fragment reads of
  // rows r and r + 1 fall on different banks)
  extern __shared__ __attribute__((aligned(16))) u16 xs[];
  const int64_t xs_ld = p.K + 8;
  const u16* xs_row = xs + (xrow ? r : 0) * xs_ld;
  f32x4 acc[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int NB = NBW / RB;  // k-steps per batch (W loads per batch stay NBW)
  // XF 1: the first XR 16-B chunks of the raw rows per thread and the norm weight chunk of the first
  // one, loaded ahead of the weight batch so the normalisation waits on them alone
  constexpr int XR = XF == 1 ? 2 : 1;
  __shared__ float xrs[XF == 1 ? 16 : 1];
  u16x8 xpre[XR], wpre{};
  int64_t wcol = -1;
  if constexpr (XF == 1) {
    const int64_t cpr = p.K / 8, Q = p.M * cpr;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int64_t q = threadIdx.x + (int64_t)(64 * NW) * i;
      xpre[i] = u16x8{};
      if (q < Q) {
        const int64_t row = q / cpr, col = (q - row * cpr) * 8;
        xpre[i] = *reinterpret_cast<const u16x8*>(p.A + row * p.lda + col);
      }
    }
    if ((int64_t)threadIdx.x < Q) {
      wcol = ((int64_t)threadIdx.x % cpr) * 8;
      wpre = *reinterpret_cast<const u16x8*>(a.xf_w + wcol);
    }
  }
  for (int64_t j0 = 0; j0 < per; j0 += NB) {
    frag8 w[NB][RB], x[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int64_t ks = ORDER == 0 ? wave * per + j0 + i : (j0 + i) * NW + wave;
      const int64_t kend = ORDER == 0 ? min(nk, (int64_t)(wave + 1) * per) : nk;
      const int64_t k = ks * 32 + 8 * g;  // this lane's first k of the step
      const bool in = j0 + i < per && ks < kend && k < p.K;
      const int64_t off = in ? ks * 32 : 0;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
        w[i][rb] = in ? __builtin_bit_cast(frag8, WNT ? __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wrow[rb] + off))
                                                      : *reinterpret_cast<const u16x8*>(wrow[rb] + off))
                      : frag8{};
    }
    if (XF == 1 && j0 == 0) {
      // RMSNorm of the M rows, after the first batch of weight loads is in flight, by every thread of
      // the workgroup (round 4/5 ran one wave per row through 8 dependent load rounds: ~10 us per
      // launch): (1) the raw rows into LDS (the first XR chunks per thread were loaded before the
      // weight batch), (2) wave w < M sums row w's squares in rmsnorm_fwd_k's order (lane: chunks c,
      // then elements j; norms.hip) from LDS, (3) every thread normalises its chunks in place,
      // y = bf16(w * bf16(x * rstd)). Barriers wait on the LDS only (the weight loads stay in flight).
      const int64_t cpr = p.K / 8, Q = p.M * cpr;
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        const int64_t q = threadIdx.x + (int64_t)(64 * NW) * i;
        if (q < Q) {
          const int64_t row = q / cpr, col = (q - row * cpr) * 8;
          *reinterpret_cast<u16x8*>(xs + row * xs_ld + col) = xpre[i];
        }
      }
      for (int64_t q = threadIdx.x + (int64_t)(64 * NW) * XR; q < Q; q += 64 * NW) {
        const int64_t row = q / cpr, col = (q - row * cpr) * 8;
        *reinterpret_cast<u16x8*>(xs + row * xs_ld + col) = *reinterpret_cast<const u16x8*>(p.A + row * p.lda + col);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      for (int row = wave; row < p.M; row += NW) {
        float ss = 0.f;
        for (int c = 0; c * 512 < p.K; ++c) {
          const int col = c * 512 + lane * 8;
          if (col < p.K) {
            const u16x8 xv = *reinterpret_cast<const u16x8*>(xs + row * xs_ld + col);
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += bf2f(xv[j]) * bf2f(xv[j]);
          }
        }
        ss = wave_sum(ss);
        if (lane == 0) xrs[row] = rsqrtf(ss / (float)p.K + a.xf_eps);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      for (int64_t q = threadIdx.x; q < Q; q += 64 * NW) {
        const int64_t row = q / cpr, col = (q - row * cpr) * 8;
        const u16x8 wv = col == wcol ? wpre : *reinterpret_cast<const u16x8*>(a.xf_w + col);
        const u16x8 xv = *reinterpret_cast<const u16x8*>(xs + row * xs_ld + col);
        const float rr = xrs[row];
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(wv[j]) * round_bf(bf2f(xv[j]) * rr));
        *reinterpret_cast<u16x8*>(xs + row * xs_ld + col) = o;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int64_t ks = ORDER == 0 ? wave * per + j0 + i : (j0 + i) * NW + wave;
      const int64_t kend = ORDER == 0 ? min(nk, (int64_t)(wave + 1) * per) : nk;
      const int64_t k = ks * 32 + 8 * g;
      const bool in = j0 + i < per && ks < kend && k < p.K;
      const int64_t off = in ? ks * 32 : 0;
      x[i] = (in && xrow) ? gemv_xfrag<XF>(a, xp, off, k, xs_row) : frag8{};
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[i][rb], x[i], acc[rb], 0, 0, 0);
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) red[wave][rb][lane] = acc[rb];
  __syncthreads();
  if (wave < RB) {
    f32x4 s = red[0][wave][lane];
#pragma unroll
    for (int w2 = 1; w2 < NW; ++w2) s += red[w2][wave][lane];
    if constexpr (OT == 1) {
      // lanes 0-31 hold g of outputs n0 + 4 (lane >> 4) + j, lanes 32-63 the matching u
      f32x4 u;
#pragma unroll
      for (int j = 0; j < 4; ++j) u[j] = __shfl_xor(s[j], 32);
      if (g < 2 && r < p.M) {
        u16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(round_bf(gemv_silu(round_bf(s[j]))) * round_bf(u[j]));
        *reinterpret_cast<u16x4*>(reinterpret_cast<u16*>(p.C) + r * p.ldc + n0 + 4 * g) = o;
      }
    } else {
      store4<CT>(p, s, r, n0 + 16 * wave + 4 * g);
    }
  }
}

int g_gemv_nt = 0;  // non-temporal weight loads (cullavo_gemv_set_nt)

}  // namespace

// non-temporal weight loads in the decode GEMV on (1) / off (0); returns the previous setting
extern "C" int cullavo_gemv_set_nt(int on) {
  const int prev = g_gemv_nt;
  g_gemv_nt = on & 1;
  return prev;
}

int cvgemm_launch_gemv(const cvgemm::GemmArgs& p, bool f32, hipStream_t s) {
  // lab switch (CULLAVO_GEMV: 0 contiguous K ranges, 1 round-robin k-steps, 2 / 3 = 0 / 1 with
  // 32 rows per workgroup, 4 / 5 = 0 / 1 with 8-load batches at 2 workgroups per CU, 6 / 7 = 0 / 1
  // with 4-load batches at 4 workgroups per CU), read once per process
  static const int venv = getenv("CULLAVO_GEMV") ? atoi(getenv("CULLAVO_GEMV")) : -1;
  // default: 8-load batches; 4-load batches (four workgroups per CU) for the long-K products
  // (down: 20.9 vs 21.9 us at batch 1, 22.5 vs 24.6 at batch 8, gemv_variants.txt)
  // 16 waves per workgroup with 4-load batches (variant 8) for the widest products (gate|up,
  // lm_head: 34.5 vs 35.5 us and 45.2 vs 46.8 at batch 1, profiles/r04/decode/gemv_variants16.txt);
  // lab variant 9: 16 waves with 8-load batches (slower)
  const int v = venv >= 0 ? venv : (p.K >= 8192 ? 6 : p.N > 16384 ? 8 : kGemvDefault);
  const int rb = (v == 2 || v == 3) ? 2 : 1;
  const unsigned grid = (unsigned)cdiv(p.N, 16 * rb);
  GemvArgs a{};
  a.g = p;
#define GV(O, R, NBW)                                                                                         \
  if (f32) gemv_k<CULLAVO_DT_F32, O, R, 0, NBW><<<grid, 64 * kGemvWaves, 0, s>>>(a);                            \
  else if (g_gemv_nt) gemv_k<CULLAVO_DT_BF16, O, R, 0, NBW, kGemvWaves, 0, true><<<grid, 64 * kGemvWaves, 0, s>>>(a); \
  else gemv_k<CULLAVO_DT_BF16, O, R, 0, NBW><<<grid, 64 * kGemvWaves, 0, s>>>(a);
#define GV16(NBW)                                                                                     \
  if (f32) gemv_k<CULLAVO_DT_F32, 0, 1, 0, NBW, 16><<<grid, 64 * 16, 0, s>>>(a);                        \
  else if (g_gemv_nt) gemv_k<CULLAVO_DT_BF16, 0, 1, 0, NBW, 16, 0, true><<<grid, 64 * 16, 0, s>>>(a);   \
  else gemv_k<CULLAVO_DT_BF16, 0, 1, 0, NBW, 16><<<grid, 64 * 16, 0, s>>>(a);
  if (v == 0) { GV(0, 1, 16) } else if (v == 1) { GV(1, 1, 16) } else if (v == 2) { GV(0, 2, 16) }
  else if (v == 3) { GV(1, 2, 16) } else if (v == 4) { GV(0, 1, 8) } else if (v == 5) { GV(1, 1, 8) }
  else if (v == 6) { GV(0, 1, 4) } else if (v == 7) { GV(1, 1, 4) } else if (v == 8) { GV16(4) } else { GV16(8) }
#undef GV16
#undef GV
  return cullavo_check_launch("gemv");
}

extern "C" int cullavo_decode_linear(int x_transform, int64_t M, int64_t N, int64_t K, const void* x, int64_t ldx,
                                     const void* norm_w, float eps, const void* W, int64_t ldw, void* y,
                                     int64_t ldy, const void* residual, int64_t ldr, void* stream) {
  CV_REQUIRE(x_transform >= 0 && x_transform <= 4, CULLAVO_EINVAL, "decode_linear: transform 0 to 4");
  const int xf = (x_transform == 1 || x_transform == 4) ? 1 : x_transform == 2 ? 2 : 0;
  const bool ot = x_transform == 3 || x_transform == 4;
  CV_REQUIRE(!ot || residual == nullptr, CULLAVO_EINVAL, "decode_linear: the SwiGLU output takes no residual");
  CV_REQUIRE(M >= 1 && M <= 16 && N > 0 && K > 0, CULLAVO_EINVAL, "decode_linear: 1 <= M <= 16 rows, N, K > 0");
  CV_REQUIRE(N % 8 == 0 && K % 8 == 0 && ldx % 8 == 0 && ldw % 8 == 0 && ldy % 8 == 0 &&
                 (residual == nullptr || ldr % 8 == 0),
             CULLAVO_EINVAL, "decode_linear: sizes and strides must be multiples of 8");
  CV_REQUIRE(ldw >= K && ldy >= N && ldx >= (xf == 2 ? 2 * K : K) && (residual == nullptr || ldr >= N),
             CULLAVO_EINVAL, "decode_linear: leading dimension too small");
  // the normalised rows live in LDS: M (K + 8) bf16 <= 64 KiB (M <= 7 at K = 4096)
  CV_REQUIRE(xf != 1 || (norm_w != nullptr && M * (K + 8) * 2 <= 65536), CULLAVO_EINVAL,
             "decode_linear: RMSNorm needs its weight and M * (K + 8) * 2 <= 65536");
  hipStream_t s = CV_STREAM(stream);
  GemvArgs a{};
  GemmArgs& p = a.g;
  p.A = (const u16*)x;
  p.B = (const u16*)W;
  p.C = y;
  p.residual = (const u16*)residual;
  p.M = M; p.N = N; p.K = K; p.lda = ldx; p.ldb = ldw; p.ldc = ldy; p.ldr = ldr;
  p.alpha = 1.f;
  p.beta = 0.f;
  p.act = CULLAVO_ACT_NONE;
  a.xf_w = (const u16*)norm_w;
  a.xf_eps = eps;
  const unsigned grid = (unsigned)cdiv(N, ot ? 8 : 16);
  const size_t smem = xf == 1 ? (size_t)M * (K + 8) * 2 : 0;
  // the shapes' variants as cvgemm_launch_gemv picks them: 16 waves x 4-load batches for the widest
  // products, 4-load batches for K >= 8192, else 8-load batches (SwiGLU output: the 2N-row product)
  const int64_t wrows = ot ? 2 * N : N;
  const int v = K >= 8192 ? 6 : wrows > 16384 ? 8 : kGemvDefault;
#define DL1(XF, OT, NT)                                                                                           \
  if (v == 8) gemv_k<CULLAVO_DT_BF16, 0, 1, XF, 4, 16, OT, NT><<<grid, 64 * 16, smem, s>>>(a);                   \
  else if (v == 6) gemv_k<CULLAVO_DT_BF16, 0, 1, XF, 4, kGemvWaves, OT, NT><<<grid, 64 * kGemvWaves, smem, s>>>(a); \
  else gemv_k<CULLAVO_DT_BF16, 0, 1, XF, 8, kGemvWaves, OT, NT><<<grid, 64 * kGemvWaves, smem, s>>>(a);
#define DL(XF, OT) \
  if (g_gemv_nt) { DL1(XF, OT, true) } else { DL1(XF, OT, false) }
  if (x_transform == 0) { DL(0, 0) } else if (x_transform == 1) { DL(1, 0) } else if (x_transform == 2) { DL(2, 0) }
  else if (x_transform == 3) { DL(0, 1) } else { DL(1, 1) }
#undef DL
#undef DL1
  return cullavo_check_launch("decode_linear");
}
