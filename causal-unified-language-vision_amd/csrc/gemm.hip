// bf16 MFMA GEMM with fused epilogues for every Linear of the CuLLaVO step (forward, dX, dW).
//
// gfx950 design:
//  * 256-thread workgroup (4 waves, 2x2), 128x128 output tile, BK = 64, v_mfma_f32_16x16x32_bf16.
//  * Operands staged global -> VGPR -> LDS (double-buffered, one barrier per K step); the
//    next K tile's global loads are issued before the current tile's MFMAs.
//  * Either operand may be K-contiguous (row fragments via ds_read_b128 from an XOR-swizzled
//    [rows][64] image) or M/N-contiguous (column fragments via ds_read_b64_tr_b16 from a
//    swizzled [64][rows] image): forward Y = X W^T, dX = dY W and dW = dY^T X all run without
//    materialised transposes.
//  * MFMA operands are swapped (A-slot <- weight/N fragment, B-slot <- activation/M fragment)
//    so each lane ends with 4 consecutive output columns of one row: 8-byte bf16 stores.
//  * XCD-aware, grouped tile order: consecutive tiles of one XCD share A/B panels in its L2.
// Epilogue order mirrors the reference's bf16 module chain (see cullavo_capi.h).
#include "gemm_common.h"

#include <map>
#include <mutex>

// the decode-step weight-streaming product (M <= 16, forward layouts) lives in gemv.hip
int cvgemm_launch_gemv(const cvgemm::GemmArgs& p, bool f32, hipStream_t s);

namespace {
using namespace cvgemm;

template <int AL, int BL, int CT, int DROP = 0>
__global__ __launch_bounds__(256, 2) void gemm_k(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#define sA(i) (smem + 2 * (i) * kTileBytes)
#define sB(i) (smem + 2 * (i) * kTileBytes + kTileBytes)

  // tile order: XCD-contiguous chunks, then groups of 8 M-tiles sweeping N
  const int nwg = p.tiles_m * p.tiles_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP_M = 8;
  const int per_group = GROUP_M * p.tiles_n;
  const int group = lid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(p.tiles_m - first_m, GROUP_M);
  const int tm_idx = first_m + (lid % per_group) % gsize;
  const int tn_idx = (lid % per_group) / gsize;
  const int64_t m0 = (int64_t)tm_idx * BM, n0 = (int64_t)tn_idx * BN;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // split-K (blockIdx.y): this block's K-tile range; one split covers all of K
  const int nk_all = (int)cdiv(p.K, BK);
  const int kt0 = p.part ? (int)blockIdx.y * p.kt_per : 0;
  const int nk = p.part ? min(nk_all - kt0, p.kt_per) : nk_all;
  const int64_t kb = (int64_t)kt0 * BK;
  u16x8 ra[4], rb[4];
  load_tile<AL>(p.A, p.lda, m0, p.M, kb, p.K, ra);
  load_tile<BL>(p.B, p.ldb, n0, p.N, kb, p.K, rb);
  if (DROP == 1) drop_tile<AL>(p, m0, kb, ra);
  if (DROP == 2) drop_tile<BL>(p, n0, kb, rb);
  store_tile<AL>(sA(0), ra);
  store_tile<BL>(sB(0), rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    const int64_t k1 = kb + (int64_t)(kt + 1) * BK;
    if (more) {
      load_tile<AL>(p.A, p.lda, m0, p.M, k1, p.K, ra);
      load_tile<BL>(p.B, p.ldb, n0, p.N, k1, p.K, rb);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      frag8 fa[4], fb[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) fa[t] = read_frag<AL>(sA(cur), wm * 64 + t * 16, ks, lane);
#pragma unroll
      for (int t = 0; t < 4; ++t) fb[t] = read_frag<BL>(sB(cur), wn * 64 + t * 16, ks, lane);
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < 4; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[tn], fa[tm], acc[tm][tn], 0, 0, 0);
    }
    if (more) {
      if (DROP == 1) drop_tile<AL>(p, m0, k1, ra);
      if (DROP == 2) drop_tile<BL>(p, n0, k1, rb);
      store_tile<AL>(sA(cur ^ 1), ra);
      store_tile<BL>(sB(cur ^ 1), rb);
    }
    __syncthreads();
  }

  // ---- epilogue: lane holds C[m][n .. n+3] (split-K: raw f32 partials, reduced later) --------
#pragma unroll
  for (int tm = 0; tm < 4; ++tm) {
    const int64_t m = m0 + wm * 64 + tm * 16 + (lane & 15);
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) {
      const int64_t n = n0 + wn * 64 + tn * 16 + (lane >> 4) * 4;
      if (p.part) {
        if (m < p.M && n < p.N)
          *reinterpret_cast<f32x4*>(p.part + ((int64_t)blockIdx.y * p.M + m) * p.N + n) = acc[tm][tn];
      } else {
        store4<CT>(p, acc[tm][tn], m, n);
      }
    }
  }
}

// split-K reduction: fixed split order (deterministic), then the full epilogue of store4
template <int CT>
__global__ __launch_bounds__(256) void splitk_reduce_k(GemmArgs p, int splits) {
  const int64_t nq = p.N / 4, total = p.M * nq;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / nq, n = (i % nq) * 4;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < splits; ++s) acc += *reinterpret_cast<const f32x4*>(p.part + ((int64_t)s * p.M + m) * p.N + n);
    store4<CT>(p, acc, m, n);
  }
}

// LDR selects which waves stage the next K-tile: 0 = all eight (each wave issues its share of
// LDS-DMA pieces before its MFMAs, so both waves of a SIMD stall on DMA issue together);
// 1 = waves 0-3 only, 2 = waves 4-7 only (one loader per SIMD: its DMA issue runs beside the
// partner wave's MFMAs instead of beside nothing). Data-parallel blocks: one whole tile each,
// the sk_dp tiles of the grid.
// Fused LoRA up-projection (round 4; the reference recipe's peft adapters, cullavo/load_cullavo.py:
// 94-112): after the main K loop each lane rounds its base outputs v = round(alpha*acc + bias) into
// packed bf16 registers, the tile's u rows (this N-tile's module block, 64 wide) and lora_B rows
// are staged by LDS-DMA into the now idle stage 0, one 64-deep MFMA K-tile computes u B^T into the
// freed accumulators, and acc := v + round(scale * u B^T): the addend of the unfused path, never
// written to or read back from HBM. The epilogue then runs with alpha 1 and no bias (applied).
template <int BM2, int BN, int TMW, int TN>
DEV void lora_fuse(GemmArgs& p, f32x4 (&acc)[TMW][TN], char* smem, int staged, int64_t m0, int64_t n0, int wave,
                   int wm, int wn, int lane) {
  constexpr int WN_COLS = BN / 4;
  if (staged < 0) {  // not staged by the main loop (its fallback path): stage now
    lora_stage<BM2, BN>(p, m0, n0, smem, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    smem += staged;  // staged by the last K-tile's iteration, waited for and barriered by the loop
  }
  // one 16-row group at a time: the lora_B fragments (TN x 2) and the bias stay in registers, the
  // group's rounded base outputs (TN x 2 packed registers) live only while its u B^T is formed, so
  // the 288-row tile fits the 256 registers without spilling
  frag8 fb[TN][2];
  float bv[TN][4];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fb[tn][ks] = read_frag<0>(smem + BM2 * BK * 2, wn * WN_COLS + tn * 16, ks, lane);
    const int64_t n = n0 + wn * WN_COLS + tn * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[tn][j] = 0.f;
    if (p.bias && n < p.N) {
      const u16x4 b4 = *reinterpret_cast<const u16x4*>(p.bias + n);
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[tn][j] = bf2f(b4[j]);
    }
  }
#pragma unroll
  for (int tm = 0; tm < TMW; ++tm) {
    uint32_t base[TN][2];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      u16 h[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) h[j] = f2bf(acc[tm][tn][j] * p.alpha + bv[tn][j]);
      base[tn][0] = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
      base[tn][1] = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
      acc[tm][tn] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const frag8 fa = read_frag<0>(smem, wm * (BM2 / 2) + tm * 16, ks, lane);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[tn][ks], fa, acc[tm][tn], 0, 0, 0);
    }
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const float bb[4] = {bf2f((u16)(base[tn][0] & 0xFFFF)), bf2f((u16)(base[tn][0] >> 16)),
                           bf2f((u16)(base[tn][1] & 0xFFFF)), bf2f((u16)(base[tn][1] >> 16))};
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[tm][tn][j] = bb[j] + round_bf(acc[tm][tn][j] * p.lora_scale);
    }
  }
  __syncthreads();  // every wave's fragment reads of the staged tiles before the epilogue reuses smem
  p.alpha = 1.f;
  p.bias = nullptr;
}

// EPI > 0: the direct epilogue (direct_epilogue, lean case EPI - 1) instead of the LDS-staged one,
// chosen by the host per product (launch256_lean)
template <int AL, int BL, int CT, int BMT, int BN, int LDR = 0, bool LORA = false, bool SWG = false, int EPI = 0>
__global__ __launch_bounds__(512, 1) void gemm256_k(GemmArgs p) {
  constexpr int BM2 = BMT;  // 256 or 192 (192 only with a K-contiguous A)
  constexpr int WN_COLS = BN / 4;     // per-wave N extent (4 waves across N)
  constexpr int TN = WN_COLS / 16;    // 16-col MFMA tiles per wave
  constexpr int TMW = BM2 / 32;       // 16-row MFMA tiles per wave (BM/2 rows)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int lid = xcd_remap(blockIdx.x, p.sk_dp);
  int64_t m0, n0;
  tile_origin<BM2, BN>(p, lid, m0, n0);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  const int64_t a_bytes = AL == 0 ? ((p.M - 1) * p.lda + p.K) * 2 : ((p.K - 1) * p.lda + p.M) * 2;
  const int64_t b_bytes = BL == 0 ? ((p.N - 1) * p.ldb + p.K) * 2 : ((p.K - 1) * p.ldb + p.N) * 2;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, b_bytes);

  f32x4 acc[TMW][TN];
  const int nk_all = (int)cdiv(p.K, BK);
  if (p.part) {  // split-K (blockIdx.y = split): raw f32 partials, reduced in split order afterwards
    const int kb = (int)blockIdx.y * p.kt_per;
    tile_k_range<AL, BL, BM2, BN, LDR, TMW, TN>(p, ra, rb, m0, n0, kb, min(nk_all, kb + p.kt_per), smem, wave, lane,
                                                acc);
    float* part = p.part + (int64_t)blockIdx.y * p.M * p.N;
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm) {
      const int64_t m = m0 + wm * (BM2 / 2) + tm * 16 + (lane & 15);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int64_t n = n0 + wn * WN_COLS + tn * 16 + (lane >> 4) * 4;
        if (m < p.M && n < p.N) *reinterpret_cast<f32x4*>(part + m * p.N + n) = acc[tm][tn];
      }
    }
    return;
  }
  const int staged = tile_k_range<AL, BL, BM2, BN, LDR, TMW, TN, LORA>(p, ra, rb, m0, n0, 0, nk_all, smem, wave,
                                                                       lane, acc);
  if constexpr (LORA) lora_fuse<BM2, BN, TMW, TN>(p, acc, smem, staged, m0, n0, wave, wm, wn, lane);

  if constexpr (EPI > 0 && BN == 256) {
    const __amdgpu_buffer_rsrc_t rc = make_rsrc((const u16*)p.C, ((p.M - 1) * p.ldc + p.N) * 2);
    direct_epilogue<EPI - 1, TMW>(p, acc, rc, m0 + wm * (BM2 / 2), n0 + wn * WN_COLS, lane);
    return;
  }
  if constexpr (SWG) {  // launched only with act 3, the LDS epilogue on and a bf16 C (launch256_swiglu)
    lds_epilogue_swiglu<CT, BM2, TMW, TN>(p, acc, smem, m0, n0, wm, wn, lane);
    return;
  }
  if constexpr (BN == 256) {
    if (p.epi_lds) {
      lds_epilogue<CT, BM2, TMW, TN>(p, acc, smem, m0, n0, wm, wn, lane);
      return;
    }
  }
#pragma unroll
  for (int tm = 0; tm < TMW; ++tm) {
    const int64_t m = m0 + wm * (BM2 / 2) + tm * 16 + (lane & 15);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int64_t n = n0 + wn * WN_COLS + tn * 16 + (lane >> 4) * 4;
      store4<CT>(p, acc[tm][tn], m, n);
    }
  }
}



int num_cus();
// ---- persistent 256x256 forward kernel (round 5) ---------------------------------------------
// Layout (0,0), bf16 C, no split-K / LoRA: one 512-thread block per CU walks the tiles of the grid in
// the data-parallel kernel's lock-step round order (tile t, t + gridDim, ...; the same XCD remap and
// group order), the same LDS-DMA K-loop (waves 0-3 load), the next tile's first K-tile issued under
// the current tile's last MFMAs, and the LDS epilogue in four 64-row passes through the stage the
// last K-tile freed (64 KiB), each 8-column group written by lds_store_item (the lean paths of
// lds_epilogue and store8 otherwise: the same values as gemm256_k). Lab record:
// tools/lab/gemm256p_lab.hip, profiles/r05/gemm/persistent_lab.txt and epilogue/.
struct PTile { int tm, tn; };
DEV PTile ptile(const GemmArgs& p, int lid) {  // tile_origin's order by value selects
  const bool by_n = p.group_m < 0;
  const int g = by_n ? -p.group_m : p.group_m;
  const int major = by_n ? p.tiles_n : p.tiles_m;
  const int minor = by_n ? p.tiles_m : p.tiles_n;
  const int per_group = g * minor;
  const int group = lid / per_group;
  const int first = group * g;
  const int gsize = min(major - first, g);
  const int in = lid - group * per_group;
  const int a = first + in % gsize, b = in / gsize;
  return by_n ? PTile{b, a} : PTile{a, b};
}

DEV void praw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

constexpr int P_TA = 256 * BK * 2, P_STAGE = 2 * P_TA;  // 32 KiB A + 32 KiB B per stage

template <int Q, int MODE>
DEV void p_epi_pass(const GemmArgs& p, f32x4 (&acc)[8][4], char* ep, int64_t m0, int64_t n0, int wm, int wn, int el) {
  const int elane = el & 63;
  if (wm == (Q >> 1)) {
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4)
#pragma unroll
      for (int tn = 0; tn < 4; ++tn) {
        const int r = t4 * 16 + (elane & 15);
        const int c = wn * 16 + tn * 4 + (elane >> 4);
        *reinterpret_cast<f32x4*>(ep + r * 1024 + ((c ^ (r & 15)) << 4)) = acc[(Q & 1) * 4 + t4][tn];
      }
  }
  praw_barrier();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = el + 512 * i;
    const int r = idx >> 5, pr = idx & 31;
    const int sw = (pr >> 3) & 1;
    const int c0 = 2 * pr + sw, c1 = 2 * pr + 1 - sw;
    const char* rowp = ep + r * 1024;
    const f32x4 x0 = *reinterpret_cast<const f32x4*>(rowp + ((c0 ^ (r & 15)) << 4));
    const f32x4 x1 = *reinterpret_cast<const f32x4*>(rowp + ((c1 ^ (r & 15)) << 4));
    const f32x4 lo = sw ? x1 : x0, hi = sw ? x0 : x1;
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = lo[j]; v[4 + j] = hi[j]; }
    lds_store_item<CULLAVO_DT_BF16>(p, v, m0 + Q * 64 + r, n0 + pr * 8, MODE);
  }
  praw_barrier();
}

// MODE: lds_epi_mode's case, fixed per instantiation (a runtime mode per 8-column group kept every
// path's code in the epilogue and measured slower than the data-parallel kernel)
template <int MODE>
__global__ __launch_bounds__(512, 1) void gemm256p_k(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool loader = wave < 4;
  const int lw = wave & 3;
  const int tiles = p.tiles_m * p.tiles_n;
  const int nk = (int)cdiv(p.K, BK);
  int t = blockIdx.x;
  if (t >= tiles) return;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, ((p.M - 1) * p.lda + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, ((p.N - 1) * p.ldb + p.K) * 2);
  PTile xy = ptile(p, xcd_remap(t, p.sk_dp));
  int64_t m0 = (int64_t)xy.tm * 256, n0 = (int64_t)xy.tn * 256;
  if (loader) {
    dma_tile<0, 256, 4>(ra, p.lda, m0, p.M, 0, p.K, smem, lw, lane);
    dma_tile<0, 256, 4>(rb, p.ldb, n0, p.N, 0, p.K, smem + P_TA, lw, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  praw_barrier();
  int s = 0;
  f32x4 acc[8][4];
  for (;;) {
    const int t1 = t + (int)gridDim.x;
    const bool has_next = t1 < tiles;
    const PTile xy1 = ptile(p, xcd_remap(has_next ? t1 : t, p.sk_dp));
    const int64_t m1 = (int64_t)xy1.tm * 256, n1 = (int64_t)xy1.tn * 256;
    unsigned va[dma_per<256, 4>()], vb[dma_per<256, 4>()];
    dma_prep<0, 256, 4>(p.lda, m0, p.M, lw, lane, va);
    dma_prep<0, 256, 4>(p.ldb, n0, p.N, lw, lane, vb);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      char* cur = smem + ((s + kt) & 1) * P_STAGE;
      char* nxt = smem + ((s + kt + 1) & 1) * P_STAGE;
      if (loader) {
        if (kt + 1 < nk) {
          const int64_t k1 = (int64_t)(kt + 1) * BK;
          dma_issue<256, 4>(ra, va, dma_soff<0>(k1, p.lda), nxt, lw);
          dma_issue<256, 4>(rb, vb, dma_soff<0>(k1, p.ldb), nxt + P_TA, lw);
        } else if (has_next) {  // the next tile's first K-tile under this tile's last MFMAs
          dma_tile<0, 256, 4>(ra, p.lda, m1, p.M, 0, p.K, nxt, lw, lane);
          dma_tile<0, 256, 4>(rb, p.ldb, n1, p.N, 0, p.K, nxt + P_TA, lw, lane);
        }
      }
      tile_mfma<0, 0, 256, 256, 8, 4>(cur, wm, wn, lane, acc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      praw_barrier();
    }
    char* ep = smem + ((s + nk - 1) & 1) * P_STAGE;  // the last K-tile's stage, free after the barrier
    // per-lane epilogue indices behind an opaque copy (hoisted out of the tile loop they would stay
    // live across the K-loop and spill)
    int el = (int)threadIdx.x;
    asm volatile("" : "+v"(el));
    p_epi_pass<0, MODE>(p, acc, ep, m0, n0, wm, wn, el);
    p_epi_pass<1, MODE>(p, acc, ep, m0, n0, wm, wn, el);
    p_epi_pass<2, MODE>(p, acc, ep, m0, n0, wm, wn, el);
    p_epi_pass<3, MODE>(p, acc, ep, m0, n0, wm, wn, el);
    if (!has_next) break;
    s = (s + nk) & 1;
    t = t1;
    m0 = m1;
    n0 = n1;
  }
}

// ---- persistent forward kernel with the direct epilogue (round 6) ------------------------------
// gemm256p_k's tile walk and K-loop, with (a) the epilogue written straight from the accumulators by
// direct_epilogue (permlane16-widened 16-B buffer stores, no LDS round trip, no barrier), (b) the next
// tile's K-tile 1 issued by the loader waves BEFORE those stores (into the stage this tile's last
// K-tile freed), so the stores drain under the next tile's K-tile 0 (the loaders' first wait is a
// counted vmcnt(2 TMW): every wave issues exactly 16 buffer stores), and (c) the per-piece DMA
// offsets as one lane base + a scalar row stride behind an opaque copy (rows past M land past the
// buffer's num_records), which keeps 16 offset registers out of the K-loop. Lab:
// tools/lab/gemm_hc_lab.hip variant 2 (profiles/r06/gemm/hc_lab.txt): ViT K = 1024 products +5-9 %,
// gate|up / lm_head +2-3 % over gemm256p_k.
DEV unsigned dma_base0(int64_t ld, int64_t idx0, int lw, int lane) {
  const int row = lw * 8 + (lane >> 3);
  const int chunk = (lane & 7) ^ ((row >> 1) & 7);  // the same for every piece (+32 rows)
  return (unsigned)(((idx0 + row) * ld + chunk * 8) * 2);
}

template <int NP = 8>
DEV void dma_issue_stride(__amdgpu_buffer_rsrc_t rsrc, unsigned base, unsigned step, int soff, char* lds, int lw) {
  unsigned off = base;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + (lw + 4 * i) * 1024), 16, off, soff, 0, 0);
    off += step;
    asm volatile("" : "+v"(off));  // no precomputed per-piece offsets live across the K-loop
  }
}

// BMT: 256 or 288 rows (the 288-row tile of the N = 4096 / long-K forward products: 36 A pieces, nine
// per loader wave)
template <int MODE, int BMT>
__global__ __launch_bounds__(512, 1) void gemm256pd_k(GemmArgs p) {
  constexpr int TMW = BMT / 32, NPA = BMT / 32;  // MFMA rows per wave; A pieces per loader wave
  constexpr int TA = BMT * BK * 2, STAGE = TA + 256 * BK * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool loader = wave < 4;
  const int lw = wave & 3;
  const int tiles = p.tiles_m * p.tiles_n;
  const int nk = (int)cdiv(p.K, BK);
  int t = blockIdx.x;
  if (t >= tiles) return;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, ((p.M - 1) * p.lda + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, ((p.N - 1) * p.ldb + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rc = make_rsrc((const u16*)p.C, ((p.M - 1) * p.ldc + p.N) * 2);
  const unsigned step_a = (unsigned)(32 * p.lda * 2), step_b = (unsigned)(32 * p.ldb * 2);
  PTile xy = ptile(p, xcd_remap(t, p.sk_dp));
  int64_t m0 = (int64_t)xy.tm * BMT, n0 = (int64_t)xy.tn * 256;
  if (loader) {
    dma_issue_stride<NPA>(ra, dma_base0(p.lda, m0, lw, lane), step_a, 0, smem, lw);
    dma_issue_stride(rb, dma_base0(p.ldb, n0, lw, lane), step_b, 0, smem + TA, lw);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  praw_barrier();
  int s = 0;
  bool k1_early = false;  // this tile's K-tile 1 went out before the previous tile's stores
  f32x4 acc[TMW][4];
  for (;;) {
    const int t1 = t + (int)gridDim.x;
    const bool has_next = t1 < tiles;
    const PTile xy1 = ptile(p, xcd_remap(has_next ? t1 : t, p.sk_dp));
    const int64_t m1 = (int64_t)xy1.tm * BMT, n1 = (int64_t)xy1.tn * 256;
    unsigned ba = dma_base0(p.lda, m0, lw, lane), bb = dma_base0(p.ldb, n0, lw, lane);
    asm volatile("" : "+v"(ba), "+v"(bb));
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      char* cur = smem + ((s + kt) & 1) * STAGE;
      char* nxt = smem + ((s + kt + 1) & 1) * STAGE;
      if (loader && !(kt == 0 && k1_early)) {
        if (kt + 1 < nk) {
          const int64_t k1 = (int64_t)(kt + 1) * BK;
          dma_issue_stride<NPA>(ra, ba, step_a, dma_soff<0>(k1, p.lda), nxt, lw);
          dma_issue_stride(rb, bb, step_b, dma_soff<0>(k1, p.ldb), nxt + TA, lw);
        } else if (has_next) {  // the next tile's first K-tile under this tile's last MFMAs
          unsigned b1a = dma_base0(p.lda, m1, lw, lane), b1b = dma_base0(p.ldb, n1, lw, lane);
          asm volatile("" : "+v"(b1a), "+v"(b1b));
          dma_issue_stride<NPA>(ra, b1a, step_a, 0, nxt, lw);
          dma_issue_stride(rb, b1b, step_b, 0, nxt + TA, lw);
        }
      }
      tile_mfma<0, 0, BMT, 256, TMW, 4>(cur, wm, wn, lane, acc);
      // loaders: K-tile 0 after an early K-tile 1 leaves the previous tile's 2 TMW stores (issued
      // after that DMA) in flight; otherwise everything the wave issued has landed. The other waves
      // issue no vector-memory op in the K-loop: they never wait, so their epilogue stores drain
      // under it
      if (loader) {
        if (kt == 0 && k1_early) {
          if constexpr (TMW == 9) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      praw_barrier();
    }
    // every wave is past the last K-tile's barrier: its stage is free for the next tile's K-tile 1
    k1_early = has_next && nk > 1;
    if (k1_early && loader) {
      char* st1 = smem + ((s + nk + 1) & 1) * STAGE;
      unsigned b1a = dma_base0(p.lda, m1, lw, lane), b1b = dma_base0(p.ldb, n1, lw, lane);
      asm volatile("" : "+v"(b1a), "+v"(b1b));
      dma_issue_stride<NPA>(ra, b1a, step_a, dma_soff<0>(BK, p.lda), st1, lw);
      dma_issue_stride(rb, b1b, step_b, dma_soff<0>(BK, p.ldb), st1 + TA, lw);
    }
    direct_epilogue<MODE, TMW>(p, acc, rc, m0 + wm * (BMT / 2), n0 + wn * 64, lane);
    if (!has_next) break;
    s = (s + nk) & 1;
    t = t1;
    m0 = m1;
    n0 = n1;
  }
}

int g_persist = 1;  // cullavo_gemm_set_epilogue bit 5 turns the persistent forward kernel off (A/B)

template <int MODE>
int launch256p_m(GemmArgs p, hipStream_t s) {
  const int smem = 2 * P_STAGE;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm256p_k<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  p.tiles_m = (int)cdiv(p.M, 256);
  p.tiles_n = (int)cdiv(p.N, 256);
  p.sk_dp = p.tiles_m * p.tiles_n;
  const int grid = std::min(p.sk_dp, num_cus());
  gemm256p_k<MODE><<<(unsigned)grid, 512, smem, s>>>(p);
  return cullavo_check_launch("gemm256 persistent");
}

template <int MODE, int BMT = 256>
int launch256pd_m(GemmArgs p, hipStream_t s) {
  const int smem = 2 * (BMT * BK * 2 + 256 * BK * 2);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm256pd_k<MODE, BMT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              smem);
    attr_set = true;
  }
  p.tiles_m = (int)cdiv(p.M, BMT);
  p.tiles_n = (int)cdiv(p.N, 256);
  p.sk_dp = p.tiles_m * p.tiles_n;
  const int grid = std::min(p.sk_dp, num_cus());
  gemm256pd_k<MODE, BMT><<<(unsigned)grid, 512, smem, s>>>(p);
  return cullavo_check_launch("gemm256 persistent direct");
}

// the lean epilogue case of a product (lds_epi_mode's 0 plain, 1 bias / residual, 2 activation), or
// -1 (the general path); on the host, the same conditions
int lean_mode(const GemmArgs& p) {
  const bool lean = p.act == CULLAVO_ACT_NONE && p.preact == nullptr && p.addend == nullptr && p.beta == 0.f &&
                    p.drop_mode != 3 && !p.nt_store;
  if (lean && p.bias == nullptr && p.residual == nullptr && !(p.epi_lds & 8)) return 0;
  if (lean && !(p.epi_lds & 4) && !(p.bias == nullptr && p.residual == nullptr)) return 1;
  if (p.act != CULLAVO_ACT_NONE && p.act != CULLAVO_ACT_SWIGLU_BWD && p.preact == nullptr && p.addend == nullptr &&
      p.residual == nullptr && p.beta == 0.f && p.drop_mode != 3 && !p.nt_store && !(p.epi_lds & 16))
    return 2;
  return -1;
}

// C (the direct epilogue's stores) and the residual (its loads) addressable by one buffer descriptor each
bool c_fits_rsrc(const GemmArgs& p) {
  return ((p.M - 1) * p.ldc + p.N) * 2 < (int64_t)kOOB &&
         (p.residual == nullptr || ((p.M - 1) * p.ldr + p.N) * 2 < (int64_t)kOOB);
}

// the persistent 288-row direct kernel for a lean (0,0) product; -1: not eligible. Always at K < 2048
// or N <= 2048 (the ViT's products: K = 1024 on 288-row tiles since round 6, fc2 N = 1024): fc1 / o
// 920 / 825 -> 940 / 880 TF/s with the plan's 288-row M-split; ViT step 2481 (round 5's plan) ->
// 2488 (288 rows at short K) -> 2496 img/s (and fc2 persistent), alternating on one box
// (profiles/r06/gemm/vit288_ab.txt). Otherwise opt-in (cullavo_gemm_set_epilogue bit 8): on one box
// (tools/epi_ab.py, profiles/r06/gemm/epi_ab.txt) it beat the data-parallel 288-row direct kernel on
// gate|up (1349 vs 1340 TF/s) but lost on q|k|v, o and down (1358 / 1284 / 1305 vs 1390 / 1317 / 1314)
int launch288pd(const GemmArgs& p, hipStream_t s) {
  if (!(p.epi_lds & 256) && p.K >= 2048 && p.N > 2048) return -1;
  if (p.part != nullptr || !p.epi_lds || (p.epi_lds & (128 | 32)) || !p.dma_pre || !c_fits_rsrc(p)) return -1;
  const int mode = lean_mode(p);
  if (mode == 0) return launch256pd_m<0, 288>(p, s);
  if (mode == 1) return launch256pd_m<1, 288>(p, s);
  if (mode == 2) return launch256pd_m<2, 288>(p, s);
  return -1;
}

// the persistent kernel for the lean epilogue cases (plain, bias / residual, activation); -1: none.
// cullavo_gemm_set_epilogue bit 7 keeps the LDS-staged epilogue (gemm256p_k) for A/B
int launch256p(const GemmArgs& p, hipStream_t s) {
  const int mode = lean_mode(p);
  if (mode < 0) return -1;
  if (!(p.epi_lds & 128) && c_fits_rsrc(p)) {
    if (mode == 0) return launch256pd_m<0>(p, s);
    if (mode == 1) return launch256pd_m<1>(p, s);
    return launch256pd_m<2>(p, s);
  }
  if (mode == 0) return launch256p_m<0>(p, s);
  if (mode == 1) return launch256p_m<1>(p, s);
  return launch256p_m<2>(p, s);
}

// Split-K plan for the register-staged kernel: products whose 128x128 tile grid cannot fill
// the 256 CUs but whose K is long (the LoRA adapter GEMMs: N or M = r = 64, K = tokens or
// features) are cut into K chunks of >= 4 K-tiles, enough of them for ~512 workgroups.
int g_splitk_blocks = 512;  // target blocks of a split-K launch (cullavo_gemm_set_splitk_target)

// Split-K plan for the 8-wave 256x256 kernel: products whose 256x256 grid fills at most a
// quarter of the CUs while K is long (the ViT's fc2 at 4 images: 2308 x 1024 x 4096; the
// projector's weight gradients at 8 images: K = 4608): the K-tiles are cut into equal chunks of
// >= 8 so tiles x splits is about one round of the 256 CUs; f32 partials [splits][M][N] are
// reduced in split order (deterministic) by splitk_reduce_k with the full epilogue. Measured
// (tools/small_gemm_bench.py, profiles/r03/small_gemm.txt): at K = 1024 the partials' round trip
// costs more than the idle CUs (2308 x 3072 x 1024: 223 split vs 514 TF/s unsplit), at K >= 4096
// the split wins (4096 x 1024 x 4608 dW: 652 vs 492). Both M and N >= 256 (else the 256-wide
// tile is mostly padding: the register-staged 128x128 split below takes those).
int num_cus();

// Split over K when the 256x256 grid covers at most half the CUs and K is long (>= 32 K-tiles):
// e.g. the ViT's fc2 at 8 images (4616 x 1024 x 4096: 76 tiles -> 3 splits, 228 blocks).
int splitk256_plan(int64_t M, int64_t N, int64_t K, int* kt_per) {
  const int64_t tiles = cdiv(M, 256) * cdiv(N, 256), nk = cdiv(K, BK);
  if (M < 256 || N < 256 || tiles * 2 > num_cus() || nk < 32) return 1;
  int64_t s = std::min<int64_t>(num_cus() / tiles, nk / 8);
  if (s < 2) return 1;
  const int64_t per = cdiv(nk, s);
  s = cdiv(nk, per);
  if (kt_per) *kt_per = (int)per;
  return (int)s;
}

int splitk_plan(int64_t M, int64_t N, int64_t K, int* kt_per) {
  const int64_t tiles = cdiv(M, BM) * cdiv(N, BN), nk = cdiv(K, BK);
  if (tiles >= 384 || nk < 8) return 1;
  int64_t s = std::min<int64_t>(std::max<int64_t>(g_splitk_blocks / tiles, 2), std::min<int64_t>(nk / 4, 32));
  if (s < 2) return 1;
  const int64_t per = cdiv(nk, s);
  s = cdiv(nk, per);
  if (kt_per) *kt_per = (int)per;
  return (int)s;
}

template <int AL, int BL, int CT, int DROP = 0>
int launch(const GemmArgs& p, hipStream_t s) {
  const int smem = 4 * kTileBytes;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_k<AL, BL, CT, DROP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              smem);
    attr_set = true;
  }
  if (p.part) {
    const int splits = (int)cdiv(cdiv(p.K, BK), p.kt_per);
    gemm_k<AL, BL, CT, DROP><<<dim3(p.tiles_m * p.tiles_n, splits), 256, smem, s>>>(p);
    const int64_t work = p.M * (p.N / 4);
    const int g = (int)std::min<int64_t>(cdiv(work, 256), 4096);
    splitk_reduce_k<CT><<<g, 256, 0, s>>>(p, splits);
    return cullavo_check_launch("gemm splitk");
  }
  gemm_k<AL, BL, CT, DROP><<<p.tiles_m * p.tiles_n, 256, smem, s>>>(p);
  return cullavo_check_launch("gemm");
}


int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    n = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  return n;
}


template <int AL, int BL, int CT, int BM2, int BN2, bool LORA = false, bool SWG = false, int EPI = 0>
int launch256(GemmArgs p, hipStream_t s) {
  // two K-tile stages; the LDS-staged epilogue needs BM2/2 f32 rows of 1 KiB (288 rows: 144 KiB)
  const int smem = std::max(2 * (BM2 * BK * 2 + BN2 * BK * 2), BN2 == 256 && EPI == 0 ? BM2 / 2 * 1024 : 0);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm256_k<AL, BL, CT, BM2, BN2, 1, LORA, SWG, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  p.tiles_m = (int)cdiv(p.M, BM2);
  p.tiles_n = (int)cdiv(p.N, BN2);
  const int64_t tiles = (int64_t)p.tiles_m * p.tiles_n, nk = cdiv(p.K, BK);
  p.sk_dp = (int)tiles;
  if (p.part) {  // split-K over the 8-wave kernel (small grids, splitk256_plan), then the reduce
    const int splits = (int)cdiv(nk, p.kt_per);
    gemm256_k<AL, BL, CT, BM2, BN2, 1, LORA, SWG, EPI><<<dim3((unsigned)tiles, splits), 512, smem, s>>>(p);
    const int64_t work = p.M * (p.N / 4);
    splitk_reduce_k<CT><<<(int)std::min<int64_t>(cdiv(work, 256), 4096), 256, 0, s>>>(p, splits);
    return cullavo_check_launch("gemm256 split-K");
  }
  gemm256_k<AL, BL, CT, BM2, BN2, 1, LORA, SWG, EPI><<<(unsigned)tiles, 512, smem, s>>>(p);
  return cullavo_check_launch("gemm256");
}

// the data-parallel 8-wave kernel with the direct epilogue for the lean plain (EPI 1) and bias /
// residual (EPI 2) cases of the step's 7B shapes (forward / dX at 288 rows, dX / dW at 256 rows); -1
// when the product is not one of them (the LDS-staged general epilogue then runs)
template <int AL, int BL, int BM2>
int launch256_lean(const GemmArgs& p, hipStream_t s) {
  if (p.part != nullptr || !p.epi_lds || (p.epi_lds & 128) || !c_fits_rsrc(p)) return -1;
  const int mode = lean_mode(p);
  if (mode == 0) return launch256<AL, BL, CULLAVO_DT_BF16, BM2, 256, false, false, 1>(p, s);
  if (mode == 1) return launch256<AL, BL, CULLAVO_DT_BF16, BM2, 256, false, false, 2>(p, s);
  return -1;
}

// Kernel-shape choice. Time model = FLOPs / (per-tile rate of the shape) x (whole rounds of
// tiles over the 256 CUs / exact rounds): the 8-wave kernels run one 512-thread block per CU,
// so a grid of 544 tiles takes 3 rounds for 2.125 rounds of work. Per-tile rates (TFLOP/s,
// measured on MI355X with tools/gemm_bench.py): 256x256 ~1300, 192x256
// ~1150 (A K-contiguous only; the 256-row tile reads 14 % less LDS per MFMA), 128x128 4-wave
// (2 blocks/CU, 512 slots) ~840.
// Measured slower and moved out of the library in round 5 (sources in tools/lab/ and git history,
// records under profiles/): the 8-phase / ping-pong kernels (round-1 modes 4/5 and round-4 modes
// 12/13/15/16: +3-7 % on big-N forward products, -10-25 % on dX, dW and N = 4096;
// profiles/r01/gemm_8phase.md, profiles/r04/gemm/), the BK=32 4-stage kernel (mode 8, slower on every
// step shape, profiles/r02/gemm_lab.md), the stream-K tail (-5-43 %, profiles/r02/streamk_bench.log),
// the all-waves-loading alternatives (modes 6/7/11, profiles/r03/ldr/), the L2 prefetch of K-tile
// kt+2 (-5-12 %, profiles/r03/prefetch/) and the 256x128 tile (mode 1, never chosen).
// kT288x256 (round 3): 288-row tiles for a K-contiguous A (9 MFMA rows per wave, 36 A pieces
// over the 4 loader waves). The per-K-tile overhead (barrier, DMA issue, fragment-read latency)
// is roughly fixed, so a taller tile amortises it over more MFMAs, and M = 8704 = 30.2 x 288
// makes the N = 4096 products (every dX, o and down forward) 496 tiles = 1.94 rounds instead of
// 736 192-row tiles = 2.88 rounds.
// Round 5 tried a 4-wave 256x256 kernel (one wave per SIMD, AGPR accumulators, register- or
// LDS-DMA-staged, with and without a stream-K head): equal or slower on every step shape, kept
// in tools/lab/gemm4w_r5.hip with its ablations (profiles/r05/gemm/).
enum { kT128 = 0, kT256x256 = 2, kT192x256 = 3, kT288x256 = 10 };
// plan rates of tile modes 2, 3, 10 (cullavo_gemm_set_tile_rate)
double g_tile_rate[3] = {1300.0, 1150.0, 1360.0};
// M-tail split (round 5): when M is just past a multiple of a tile's height, its last M-tile row
// is mostly padding and can cost a whole extra round (the ViT's M = 64 x 577 = 36928 = 144 x 256
// + 64: fc1 at 256x256 is 2,320 tiles = 9.06 rounds -> 10; fc2 / o at 288x256 are 516 tiles =
// 2.02 rounds -> 3). The plan then runs rows [0, m_main) (m_main = a multiple of the tile height)
// on that tile and the remaining rows as a second, thin product (128x128 tiles, split over K
// when the caller gives the workspace), if that is estimated faster: g_msplit 2 (the default since
// round 6) on any estimated gain, 1 only on >= 5 % (round 5's rule, which left fc1 unsplit: its
// estimate is 3 %; split, fc1 runs 902 -> 928 TF/s and the ViT step 2505 -> 2518 img/s,
// profiles/r06/gemm/msplit_eager_ab.txt).
int g_msplit = 2;
// 288-row tiles at K < 2048 (round 6, with the persistent 288-row direct kernel: launch288pd);
// cullavo_gemm_set_epilogue bit 9 restores the round-3 exclusion below
int g_short288 = 1;
// the thin product's time: its split-K launch + reduce cost 16-19 us at the ViT shapes (64 rows:
// profiles/r05/vit/vit_kernel_trace.txt), so a split pays only where it saves more than that --
// fc2 (K = 4096: 3 -> 2 rounds of 288-row tiles), not fc1 / o (K = 1024)
double rem_seconds(int64_t rows, int64_t N, int64_t K) { return 2.0 * rows * N * K / 150e12 + 16e-6; }

// a round split's tail (round 6): when its 256x256 grid fits half the CUs and K is long, the tail rows
// run split over K on the 8-wave kernel (splitk256_plan): its rounds at K / s plus the f32 partials'
// write + reduce; otherwise the thin product of rem_seconds
double tail_seconds(int64_t rows, int64_t N, int64_t K) {
  int per = 0;
  const int s = splitk256_plan(rows, N, K, &per);
  if (s > 1) {
    const int64_t tiles = cdiv(rows, 256) * cdiv(N, 256);
    const double t_tile = 2.0 * 256 * 256 * (double)per * BK * 256 / (g_tile_rate[0] * 1e12);
    const double reduce = (double)rows * N * 4 * s * 2 / 5e12 + 10e-6;
    return (double)cdiv(tiles * s, num_cus()) * t_tile + reduce;
  }
  return rem_seconds(rows, N, K);
}

int choose_tile(int64_t M, int64_t N, int64_t K, int a_layout, int force, int64_t* m_main = nullptr) {
  if (m_main) *m_main = 0;
  if (force >= 0) return force;
  struct C { int id; int64_t bm, bn, slots; double rate; };
  const C cands[4] = {{kT128, 128, 128, 512, 840.0}, {kT256x256, 256, 256, 256, g_tile_rate[0]},
                      {kT192x256, 192, 256, 256, g_tile_rate[1]}, {kT288x256, 288, 256, 256, g_tile_rate[2]}};
  // time = whole rounds of tiles x one round (a tile's FLOPs over the per-CU share of the rate)
  auto seconds = [&](const C& c, int64_t m) {
    const int64_t tiles = cdiv(m, c.bm) * cdiv(N, c.bn);
    return (double)cdiv(tiles, c.slots) * 2.0 * c.bm * c.bn * K * c.slots / (c.rate * 1e12);
  };
  double best = 1e300, best_split = 1e300;
  int bid = kT128, bid_split = kT128;
  int64_t mm_split = 0;
  for (const C& c : cands) {
    if ((c.id == kT192x256 || c.id == kT288x256) && a_layout != 0) continue;
    // round 3: 288 rows only for long K -- with 16 K-tiles (the ViT's K = 1024 products) its larger
    // per-tile prologue and 144 KiB LDS-staged epilogue cost more than the rounds it saved (config 2:
    // fc1 36928x4096x1024 at 815 TF/s against 865 for the 256-row tile); with the direct epilogue
    // and the persistent 288-row kernel (round 6) short K takes it too, unless bit 9
    if (c.id == kT288x256 && K < 2048 && !g_short288) continue;
    if (c.rate <= 0.0) continue;
    const double t = seconds(c, M);
    if (t < best * 0.999) { best = t; bid = c.id; }
    const int64_t mm = M / c.bm * c.bm;
    // the remaining rows run as a product of their own: keep them above the decode-row sizes (a tail
    // of <= 16 rows would reach kernels with an M > 16 requirement, e.g. the fused LoRA up-projection)
    if (m_main && g_msplit && c.id != kT128 && mm > 0 && M - mm > 16) {
      const double ts = seconds(c, mm) + rem_seconds(M - mm, N, K);
      if (ts < best_split * 0.999) { best_split = ts; bid_split = c.id; mm_split = mm; }
    }
    // round split (round 6): when the N-tiles divide the CU slots, the head as whole rounds of tiles
    // and the last partial round's rows as a product of their own, split over K on the 8-wave kernel
    // (tail_seconds): the gate|up weight gradient 22016 x 4096 x 8704 is 5.375 rounds of 256x256
    // tiles -> 5 rounds + 96 tiles at half K
    if (m_main && g_msplit && c.id != kT128) {
      const int64_t tn = cdiv(N, c.bn);
      if (c.slots % tn == 0) {
        const int64_t mpr = c.slots / tn, full = cdiv(M, c.bm) / mpr;
        const int64_t mm2 = full * mpr * c.bm;
        if (full >= 1 && mm2 < M && M - mm2 > 16 && mm2 != mm) {
          const double ts = seconds(c, mm2) + tail_seconds(M - mm2, N, K);
          if (ts < best_split * 0.999) { best_split = ts; bid_split = c.id; mm_split = mm2; }
        }
      }
    }
  }
  if (m_main && best_split < (g_msplit == 2 ? 0.999 : 0.95) * best) {
    *m_main = mm_split;
    return bid_split;
  }
  return bid;
}

}  // namespace

static int g_force_tile = -1;
static int g_gemv = 1;  // cullavo_gemm_set_tile(mode >= 0) forces a tiled kernel for decode rows too
static bool gemv_eligible(int64_t M, int a_layout, int b_layout, bool dropping) {
  return g_gemv && g_force_tile < 0 && M >= 1 && M <= 16 && a_layout == 0 && b_layout == 0 && !dropping;
}
static int g_epi_lds = 1;
static int g_nt_store = 0;
static int g_dma_pre = 1;  // +2.7 % on the 7B step (profiles/r03/dma_ab.md)
// Groups of 4 N-tiles sweeping the M-tiles: measured against groups of 4 M-tiles on every 7B
// step shape in one process (profiles/r02/closing/group_sweep.txt), 1-5 % faster on 13 of 15.
static int g_group_m = -4;

extern "C" int cullavo_gemm_set_splitk_target(int blocks) {
  const int prev = g_splitk_blocks;
  if (blocks >= 64 && blocks <= 8192) g_splitk_blocks = blocks;
  return prev;
}

extern "C" int cullavo_gemm_set_group(int group) {
  const int prev = g_group_m;
  if (group != 0 && group >= -64 && group <= 64) g_group_m = group;
  return prev;
}

extern "C" int cullavo_gemm_set_tile(int mode) {
  const int prev = g_force_tile;
  g_force_tile = (mode == kT128 || mode == kT256x256 || mode == kT192x256 || mode == kT288x256) ? mode : -1;
  return prev;
}

extern "C" int cullavo_gemm_set_tile_rate(int mode, float tflops, float* previous) {
  const int i = mode == kT256x256 ? 0 : mode == kT192x256 ? 1 : mode == kT288x256 ? 2 : -1;
  CV_REQUIRE(i >= 0, CULLAVO_EINVAL, "tile rate: mode must be 2, 3 or 10");
  CV_REQUIRE(i != 0 || tflops > 0.f, CULLAVO_EINVAL, "tile rate: mode 2 cannot be removed");
  if (previous) *previous = (float)g_tile_rate[i];
  g_tile_rate[i] = tflops > 0.f ? (double)tflops : 0.0;
  return CULLAVO_OK;
}

// A/B switch for the precomputed-offset LDS-DMA loop of the 8-wave 256-row kernels
extern "C" int cullavo_gemm_set_dma(int precomputed) {
  const int prev = g_dma_pre;
  g_dma_pre = precomputed & 1;
  return prev;
}

// A/B switch for the LDS-staged epilogue of the 8-wave kernels (1 = on, the default)
extern "C" int cullavo_gemm_set_epilogue(int lds_staged) {
  const int prev = (g_epi_lds & 1) | (g_nt_store << 1) | (g_epi_lds & 508) | (g_short288 ? 0 : 512);
  g_epi_lds = lds_staged & 509;  // bit 0 LDS-staged; bits 2 / 3 / 4 disable its bias-residual / plain /
                                 // activation + SwiGLU-backward paths; bit 5 the persistent forward kernel;
                                 // bit 6 the prefetching SwiGLU-backward instantiation; bit 7 the direct
                                 // (register) epilogue of the lean cases; bit 8 the persistent 288-row
                                 // direct forward kernel (opt-in)
  g_short288 = !((lds_staged >> 9) & 1);  // bit 9: no 288-row tiles at K < 2048 (round 5's plan)
  g_nt_store = (lds_staged >> 1) & 1;
  return prev;
}

extern "C" int cullavo_gemm_plan(int64_t M, int64_t N, int64_t K, int a_layout, int b_layout, int64_t* grid) {
  if (gemv_eligible(M, a_layout, b_layout, false)) {  // 14: the decode GEMV (gemv.hip)
    if (grid) *grid = cdiv(N, 16);
    return 14;
  }
  if (g_force_tile < 0) {  // 9: the 8-wave 256x256 kernel split over K (given its workspace)
    int per = 0;
    const int s = splitk256_plan(M, N, K, &per);
    if (s > 1) {
      if (grid) *grid = cdiv(M, 256) * cdiv(N, 256) * s;
      return 9;
    }
  }
  int64_t mm = 0;
  int tile = choose_tile(M, N, K, a_layout, g_force_tile, &mm);
  if ((tile == kT192x256 || tile == kT288x256) && a_layout != 0) tile = kT256x256;
  const int bm = tile == kT128 ? 128 : tile == kT192x256 ? 192 : tile == kT288x256 ? 288 : 256;  // 2: 256
  const int bn = tile == kT128 ? 128 : 256;
  if (grid) *grid = cdiv(mm > 0 ? mm : M, bm) * cdiv(N, bn);
  (void)b_layout;
  return mm > 0 ? 100 + tile : tile;
}

static int gemm_impl(const cullavo_gemm_desc& d, void* stream, int tile_hint = -1);

// rows [m0, M) of the product d as a product of its own (every row-indexed operand shifted)
static cullavo_gemm_desc rows_from(const cullavo_gemm_desc& d, int64_t m0) {
  cullavo_gemm_desc r = d;
  const int64_t cz = d.c_dtype == CULLAVO_DT_F32 ? 4 : 2;
  r.M = d.M - m0;
  r.A = (const char*)d.A + (d.a_layout == 0 ? m0 * d.lda : m0) * 2;
  r.C = (char*)d.C + m0 * d.ldc * cz;
  if (d.preact) r.preact = (char*)d.preact + m0 * d.ldc * 2;
  if (d.residual) r.residual = (const char*)d.residual + m0 * d.ldr * 2;
  if (d.addend) r.addend = (const char*)d.addend + m0 * d.ld_addend * 2;
  if (d.lora_u) r.lora_u = (const char*)d.lora_u + m0 * d.ld_lora_u * 2;
  return r;
}

// the M-tail split of d (rows of the head product; its tile in *tile), or 0 (choose_tile)
static int64_t msplit_rows(const cullavo_gemm_desc& d, int* tile = nullptr) {
  if (d.f32_operands || (d.drop_operand != 0 && d.drop_p > 0.f) || d.M <= 16 || d.N <= 0 || d.K <= 0) return 0;
  const int64_t a_ext = d.a_layout == 0 ? (d.M - 1) * d.lda + d.K : (d.K - 1) * d.lda + d.M;
  const int64_t b_ext = d.b_layout == 0 ? (d.N - 1) * d.ldb + d.K : (d.K - 1) * d.ldb + d.N;
  if (a_ext * 2 >= (int64_t)kOOB || b_ext * 2 >= (int64_t)kOOB) return 0;  // the kT128 path
  int64_t mm = 0;
  const int t = choose_tile(d.M, d.N, d.K, d.a_layout, g_force_tile, &mm);
  if (tile) *tile = t;
  return mm;
}

static int gemm_impl(const cullavo_gemm_desc& d, void* stream, int tile_hint) {
  const int a_layout = d.a_layout, b_layout = d.b_layout, c_dtype = d.c_dtype, act = d.act;
  const int64_t M = d.M, N = d.N, K = d.K, lda = d.lda, ldb = d.ldb, ldc = d.ldc, ldr = d.ldr;
  const void* residual = d.residual;
  CV_REQUIRE(a_layout == 0 || a_layout == 1, CULLAVO_EINVAL, "a_layout");
  CV_REQUIRE(b_layout == 0 || b_layout == 1, CULLAVO_EINVAL, "b_layout");
  CV_REQUIRE(M >= 0 && N >= 0 && K >= 0, CULLAVO_EINVAL, "negative size");
  CV_REQUIRE(N % 8 == 0, CULLAVO_EINVAL, "N must be a multiple of 8");
  CV_REQUIRE((a_layout == 1 && b_layout == 1) || K % 8 == 0, CULLAVO_EINVAL,
             "K must be a multiple of 8 when an operand is K-contiguous");
  CV_REQUIRE(a_layout == 0 || M % 8 == 0, CULLAVO_EINVAL, "M must be a multiple of 8 for a_layout 1");
  CV_REQUIRE(lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 && (residual == nullptr || ldr % 8 == 0),
             CULLAVO_EINVAL, "leading dimensions must be multiples of 8");
  CV_REQUIRE(lda >= (a_layout == 0 ? K : M) && ldb >= (b_layout == 0 ? K : N) && ldc >= N,
             CULLAVO_EINVAL, "leading dimension too small");
  CV_REQUIRE(c_dtype == CULLAVO_DT_BF16 || c_dtype == CULLAVO_DT_F32, CULLAVO_EUNSUPPORTED, "c_dtype");
  CV_REQUIRE(act >= CULLAVO_ACT_NONE && act <= CULLAVO_ACT_SWIGLU_BWD, CULLAVO_EINVAL, "act");
  if (act == CULLAVO_ACT_SWIGLU_BWD) {
    CV_REQUIRE(c_dtype == CULLAVO_DT_BF16 && !d.f32_operands, CULLAVO_EUNSUPPORTED, "SwiGLU-backward epilogue is bf16 only");
    CV_REQUIRE(residual != nullptr && ldr >= 2 * N && ldc >= 2 * N, CULLAVO_EINVAL,
               "SwiGLU-backward epilogue needs gu (residual) and C of 2N columns");
    CV_REQUIRE(d.bias == nullptr && d.preact == nullptr && d.addend == nullptr && d.drop_operand == 0 &&
               d.beta == 0.f, CULLAVO_EINVAL, "SwiGLU-backward epilogue takes no bias/preact/addend/dropout/beta");
  }
  CV_REQUIRE(d.addend == nullptr || (d.ld_addend % 4 == 0 && d.ld_addend >= N), CULLAVO_EINVAL,
             "ld_addend must be >= N and a multiple of 4");
  CV_REQUIRE(d.drop_operand >= 0 && d.drop_operand <= 3, CULLAVO_EINVAL, "drop_operand");
  CV_REQUIRE(d.drop_operand == 0 || (d.drop_p >= 0.f && d.drop_p < 1.f), CULLAVO_EINVAL, "drop_p must be in [0, 1)");
  CV_REQUIRE(d.drop_operand != 1 || a_layout == 0, CULLAVO_EUNSUPPORTED, "dropout on A needs a_layout 0");
  CV_REQUIRE(d.drop_operand != 2 || b_layout == 1, CULLAVO_EUNSUPPORTED, "dropout on B needs b_layout 1");
  CV_REQUIRE(d.lora_u == nullptr || !d.f32_operands, CULLAVO_EUNSUPPORTED, "fused LoRA: bf16 operands only");
  if (d.f32_operands) return cullavo_gemm_f32_impl(d, CV_STREAM(stream));  // gemm_f32.hip
  if (M == 0 || N == 0) return CULLAVO_OK;
  if (tile_hint < 0 && !gemv_eligible(M, a_layout, b_layout, d.drop_operand != 0 && d.drop_p > 0.f)) {
    int head_tile = 0;
    const int64_t mm = msplit_rows(d, &head_tile);
    if (mm > 0) {  // whole rounds on the planned tile, then the remaining rows (see choose_tile)
      cullavo_gemm_desc head = d;
      head.M = mm;
      head.workspace = nullptr;
      head.workspace_bytes = 0;
      const int rc = gemm_impl(head, stream, head_tile);
      if (rc != CULLAVO_OK) return rc;
      return gemm_impl(rows_from(d, mm), stream, -1);
    }
  }
  const int64_t tm = cdiv(M, BM), tn = cdiv(N, BN);
  CV_REQUIRE(tm * tn < (1ll << 31), CULLAVO_EINVAL, "too many tiles");
  GemmArgs p;
  p.A = (const u16*)d.A; p.B = (const u16*)d.B; p.C = d.C;
  p.bias = (const u16*)d.bias; p.preact = (u16*)d.preact; p.residual = (const u16*)residual;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldr = ldr;
  p.alpha = d.alpha; p.beta = d.beta; p.act = act;
  p.tiles_m = (int)tm; p.tiles_n = (int)tn;
  p.addend = (const u16*)d.addend; p.ld_add = d.ld_addend;
  const bool dropping = d.drop_operand != 0 && d.drop_p > 0.f;
  p.drop_mode = dropping ? d.drop_operand : 0;
  p.drop_thr = (uint32_t)(d.drop_p * 65536.0f + 0.5f);
  p.drop_scale = dropping ? 1.f / (1.f - d.drop_p) : 1.f;
  p.drop_seed = d.drop_seed;
  p.part = nullptr;
  p.kt_per = 0;
  p.sk_dp = 0;
  p.group_m = g_group_m;
  {
    auto a16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    p.epi_lds = a16(d.C) && a16(d.bias) && a16(d.preact) && a16(residual) && a16(d.addend) &&
                        (d.addend == nullptr || d.ld_addend % 8 == 0) && (g_epi_lds & 1)
                    ? g_epi_lds
                    : 0;
  }
  p.nt_store = g_nt_store;
  p.dma_pre = g_dma_pre && (a_layout == 1 || K % BK == 0) && (b_layout == 1 || K % BK == 0);
  p.lora_u = nullptr;
  p.lora_b = nullptr;
  p.ld_lu = 0;
  p.lora_out = 0;
  p.lora_scale = 0.f;
  hipStream_t s = CV_STREAM(stream);
  const bool f32 = c_dtype == CULLAVO_DT_F32;
  const int64_t a_ext = a_layout == 0 ? (M - 1) * lda + K : (K - 1) * lda + M;
  const int64_t b_ext = b_layout == 0 ? (N - 1) * ldb + K : (K - 1) * ldb + N;
  const bool dma_ok = K > 0 && a_ext * 2 < (int64_t)kOOB && b_ext * 2 < (int64_t)kOOB;
  if (d.lora_u != nullptr) {  // the LoRA up-projection fused into the 256x256 kernel (lora_fuse)
    CV_REQUIRE(a_layout == 0 && b_layout == 0 && !f32 && !d.f32_operands && d.lora_b != nullptr &&
                   d.lora_r == 64 && d.lora_out > 0 && d.lora_out % 256 == 0 && N % d.lora_out == 0 &&
                   d.ld_lora_u % 8 == 0 && d.ld_lora_u >= (N / d.lora_out) * 64 && d.addend == nullptr &&
                   d.drop_operand == 0 && d.beta == 0.f && act != CULLAVO_ACT_SWIGLU_BWD && M > 16 && dma_ok,
               CULLAVO_EUNSUPPORTED, "fused LoRA: a_layout = b_layout = 0, bf16, r = 64, module width a multiple of 256 "
                                     "dividing N, no addend / dropout / beta, M > 16");
    p.lora_u = (const u16*)d.lora_u;
    p.ld_lu = d.ld_lora_u;
    p.lora_b = (const u16*)d.lora_b;
    p.lora_out = d.lora_out;
    p.lora_scale = d.lora_scale;
    // the 288-row tile where the plan takes it (the N = 4096 products: 2 rounds instead of 3), at
    // K >= 2048 only: the direct epilogue is not used here (beside the fused LoRA's registers it spills
    // ~100 VGPRs), and with the LDS-staged one short-K 288-row tiles lose (round 3; choose_tile)
    if (choose_tile(M, N, K, 0, g_force_tile) == kT288x256 && (K >= 2048 || g_force_tile == kT288x256))
      return launch256<0, 0, CULLAVO_DT_BF16, 288, 256, true>(p, s);
    return launch256<0, 0, CULLAVO_DT_BF16, 256, 256, true>(p, s);
  }
  // decode rows (M = batch <= 16, Y = X W^T): stream W once through the GEMV kernel (gemv.hip)
  if (gemv_eligible(M, a_layout, b_layout, dropping)) return cvgemm_launch_gemv(p, f32, s);
  bool split256 = false;
  {
    int per = 0, per256 = 0;
    const int s256 = (dma_ok && d.drop_operand != 1 && d.drop_operand != 2) ? splitk256_plan(M, N, K, &per256) : 1;
    const int splits = s256 > 1 ? s256 : splitk_plan(M, N, K, &per);
    const int64_t need = (int64_t)splits * M * N * 4;
    if (splits > 1 && d.workspace != nullptr && d.workspace_bytes >= need && g_force_tile < 0) {
      p.part = (float*)d.workspace;
      p.kt_per = s256 > 1 ? per256 : per;
      split256 = s256 > 1;
    }
  }
  int tile = dma_ok ? (tile_hint >= 0 ? tile_hint : choose_tile(M, N, K, a_layout, g_force_tile)) : kT128;
  // 288-row layout-1 A images do not fit the register budget of the transposed-read kernel
  // (197 VGPRs spilled): the weight-gradient products keep the 256-row tile
  if ((tile == kT192x256 || tile == kT288x256) && a_layout != 0) tile = kT256x256;
  if (p.part) tile = split256 ? kT256x256 : kT128;
  if (p.drop_mode == 1) return f32 ? launch<0, 0, CULLAVO_DT_F32, 1>(p, s) : launch<0, 0, CULLAVO_DT_BF16, 1>(p, s);
  if (p.drop_mode == 2) {
    if (a_layout == 0) return f32 ? launch<0, 1, CULLAVO_DT_F32, 2>(p, s) : launch<0, 1, CULLAVO_DT_BF16, 2>(p, s);
    return f32 ? launch<1, 1, CULLAVO_DT_F32, 2>(p, s) : launch<1, 1, CULLAVO_DT_BF16, 2>(p, s);
  }
  // the SwiGLU-backward dX (act 3, bf16, LDS epilogue on, not split): its own instantiation with the
  // prefetching epilogue (lds_epilogue_swiglu); cullavo_gemm_set_epilogue bit 6 keeps the general path
  if (act == CULLAVO_ACT_SWIGLU_BWD && !f32 && p.epi_lds && p.part == nullptr && !(g_epi_lds & 64) &&
      a_layout == 0 && (tile == kT288x256 || tile == kT256x256)) {
    if (tile == kT288x256)
      return b_layout == 0 ? launch256<0, 0, CULLAVO_DT_BF16, 288, 256, false, true>(p, s)
                           : launch256<0, 1, CULLAVO_DT_BF16, 288, 256, false, true>(p, s);
    return b_layout == 0 ? launch256<0, 0, CULLAVO_DT_BF16, 256, 256, false, true>(p, s)
                         : launch256<0, 1, CULLAVO_DT_BF16, 256, 256, false, true>(p, s);
  }
  if (tile == kT288x256) {  // a_layout 0 (above), one loader wave per SIMD
    if (!f32 && b_layout == 0 && g_persist) {
      const int rc = launch288pd(p, s);
      if (rc != -1) return rc;
    }
    if (!f32) {
      const int rc = b_layout == 0 ? launch256_lean<0, 0, 288>(p, s) : launch256_lean<0, 1, 288>(p, s);
      if (rc != -1) return rc;
    }
    if (b_layout == 0)
      return f32 ? launch256<0, 0, CULLAVO_DT_F32, 288, 256>(p, s) : launch256<0, 0, CULLAVO_DT_BF16, 288, 256>(p, s);
    return f32 ? launch256<0, 1, CULLAVO_DT_F32, 288, 256>(p, s) : launch256<0, 1, CULLAVO_DT_BF16, 288, 256>(p, s);
  }
  if (tile == kT192x256) {
    if (b_layout == 0)
      return f32 ? launch256<0, 0, CULLAVO_DT_F32, 192, 256>(p, s) : launch256<0, 0, CULLAVO_DT_BF16, 192, 256>(p, s);
    return f32 ? launch256<0, 1, CULLAVO_DT_F32, 192, 256>(p, s) : launch256<0, 1, CULLAVO_DT_BF16, 192, 256>(p, s);
  }
  if (tile == kT256x256) {
#define L256(AL, BL) \
  return f32 ? launch256<AL, BL, CULLAVO_DT_F32, 256, 256>(p, s) : launch256<AL, BL, CULLAVO_DT_BF16, 256, 256>(p, s);
    if (a_layout == 0 && b_layout == 0 && !f32 && g_persist && p.part == nullptr && p.epi_lds && p.dma_pre &&
        !(g_epi_lds & 32)) {
      const int rc = launch256p(p, s);
      if (rc != -1) return rc;
    }
    if (!f32 && a_layout == 0) {
      const int rc = b_layout == 1 ? launch256_lean<0, 1, 256>(p, s) : launch256_lean<0, 0, 256>(p, s);
      if (rc != -1) return rc;
    }
    if (!f32 && a_layout == 1 && b_layout == 1) {
      const int rc = launch256_lean<1, 1, 256>(p, s);
      if (rc != -1) return rc;
    }
    if (a_layout == 0 && b_layout == 0) { L256(0, 0) }
    if (a_layout == 0 && b_layout == 1) { L256(0, 1) }
    if (a_layout == 1 && b_layout == 0) { L256(1, 0) }
    L256(1, 1)
#undef L256
  }
  if (a_layout == 0 && b_layout == 0) return f32 ? launch<0, 0, CULLAVO_DT_F32>(p, s) : launch<0, 0, CULLAVO_DT_BF16>(p, s);
  if (a_layout == 0 && b_layout == 1) return f32 ? launch<0, 1, CULLAVO_DT_F32>(p, s) : launch<0, 1, CULLAVO_DT_BF16>(p, s);
  if (a_layout == 1 && b_layout == 0) return f32 ? launch<1, 0, CULLAVO_DT_F32>(p, s) : launch<1, 0, CULLAVO_DT_BF16>(p, s);
  return f32 ? launch<1, 1, CULLAVO_DT_F32>(p, s) : launch<1, 1, CULLAVO_DT_BF16>(p, s);
}

extern "C" int cullavo_gemm(int a_layout, int b_layout, int64_t M, int64_t N, int64_t K, const void* A,
                            int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int c_dtype,
                            float alpha, const void* bias, int act, void* preact, const void* residual,
                            int64_t ldr, float beta, void* stream) {
  cullavo_gemm_desc d{};
  d.a_layout = a_layout; d.b_layout = b_layout; d.M = M; d.N = N; d.K = K;
  d.A = A; d.lda = lda; d.B = B; d.ldb = ldb; d.C = C; d.ldc = ldc; d.c_dtype = c_dtype;
  d.alpha = alpha; d.bias = bias; d.act = act; d.preact = preact; d.residual = residual; d.ldr = ldr;
  d.beta = beta;
  return gemm_impl(d, stream);
}

extern "C" size_t cullavo_gemm_desc_size(void) { return sizeof(cullavo_gemm_desc); }

extern "C" size_t cullavo_gemm_workspace(const cullavo_gemm_desc* d) {
  if (d == nullptr || d->M <= 0 || d->N <= 0 || d->K <= 0 || g_force_tile >= 0) return 0;
  const int64_t mm = msplit_rows(*d);
  if (mm > 0) {  // only the remaining rows' product can be split over K
    const cullavo_gemm_desc r = rows_from(*d, mm);
    return cullavo_gemm_workspace(&r);
  }
  const bool dma_layouts = d->drop_operand != 1 && d->drop_operand != 2;
  const int s256 = dma_layouts ? splitk256_plan(d->M, d->N, d->K, nullptr) : 1;
  const int splits = s256 > 1 ? s256 : splitk_plan(d->M, d->N, d->K, nullptr);
  return splits > 1 ? (size_t)splits * (size_t)d->M * (size_t)d->N * 4 : 0;
}

extern "C" int cullavo_gemm_ex(const cullavo_gemm_desc* desc, void* stream) {
  CV_REQUIRE(desc != nullptr, CULLAVO_EINVAL, "desc");
  return gemm_impl(*desc, stream);
}

// A/B switch for the M-tail split of the automatic plan (1 = on, the default); returns the previous
extern "C" int cullavo_gemm_set_msplit(int on) {
  const int prev = g_msplit;
  g_msplit = on == 2 ? 2 : on ? 1 : 0;
  return prev;
}
