// Lab: a persistent variant of the production 256x256 8-wave GEMM (gemm.hip gemm256_k, the same
// LDS-DMA K-loop helpers of gemm_common.h), one block per CU looping over the tiles of the grid in
// the production's lock-step round order. What it tests: the per-tile fixed cost of the
// non-persistent kernel (prologue DMA + wait, epilogue store burst) -- ~12 us per 256x256 tile,
// 10 % of a K = 4096 tile and ~30 % of a K = 1024 one (profiles/r05/vit/).
//   VAR bit 0: the epilogue's global stores are issued by waves 4-7 only (the loader waves 0-3 never
//              store), and waves 4-7 skip the K-loop's vmcnt(0): their stores drain under the next
//              tile's MFMAs instead of stalling the next tile's first K-tile
//   VAR bit 1: no prefetch of the next tile's first K-tile during the last K-tile (prologue exposed)
//   VAR bit 2: full __syncthreads in the epilogue (the production epilogue's waits)
//   VAR bit 3: ablation: no global stores (the epilogue's LDS round trip and conversion stay)
//   VAR bit 4: ablation: no epilogue at all
//   VAR bits 7/8: the same stagger within each XCD (odd CUs of every XCD late)
//   VAR bits 9/10/11: the epilogue's bf16 stores with cache policy sc1 / nt / sc0 sc1
//   VAR bits 5/6: stagger -- the blocks of XCDs 4-7 start ~8 us (bit 5) / ~16 us (bit 6) late, so the two
//              XCD halves store their epilogues at different times (each XCD keeps its own lock-step)
// Layout (0,0) and (1,1), bf16 out; for tools/lab/gemm_lab.py (v = 1000 + VAR: persistent, layout (0,0)).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC tools/lab/gemm256p_lab.hip \
//     -o tools/lab/bin/libgemm256p_lab.so
#include "../../causal-unified-language-vision_amd/csrc/gemm_common.h"

using namespace cvgemm;

namespace {

constexpr int P_BM = 256, P_BN = 256, P_TMW = 8, P_TN = 4, P_WNC = 64;
constexpr int P_TILE_A = P_BM * BK * 2, P_TILE_B = P_BN * BK * 2, P_STAGE = P_TILE_A + P_TILE_B;  // 64 KiB
constexpr int P_SMEM = 2 * P_STAGE;

// tile lid -> (M-tile, N-tile) indices by value selects (gemm_common.h tile_origin's order; written
// through references inside the persistent loop the compiler merged its two branches into a
// pointer select and kept m0/n0 in scratch)
struct TileXY { int tm, tn; };
DEV TileXY tile_xy(const GemmArgs& p, int lid) {
  const bool by_n = p.group_m < 0;
  const int g = by_n ? -p.group_m : p.group_m;
  const int major = by_n ? p.tiles_n : p.tiles_m;  // the grouped dimension
  const int minor = by_n ? p.tiles_m : p.tiles_n;
  const int per_group = g * minor;
  const int group = lid / per_group;
  const int first = group * g;
  const int gsize = min(major - first, g);
  const int in = lid - group * per_group;
  const int a = first + in % gsize, b = in / gsize;
  return by_n ? TileXY{b, a} : TileXY{a, b};
}

DEV void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int VAR, int Q>
DEV void epi_pass(const GemmArgs& p, f32x4 (&acc)[P_TMW][P_TN], char* ep, int64_t m0, int64_t n0, int wm, int wn,
                  bool loader, int el) {
  const int elane = el & 63;
  if (wm == (Q >> 1)) {
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4)
#pragma unroll
      for (int tn = 0; tn < P_TN; ++tn) {
        const int r = t4 * 16 + (elane & 15);
        const int c = wn * 16 + tn * 4 + (elane >> 4);
        *reinterpret_cast<f32x4*>(ep + r * 1024 + ((c ^ (r & 15)) << 4)) = acc[(Q & 1) * 4 + t4][tn];
      }
  }
  if (VAR & 4) __syncthreads(); else raw_barrier();
  constexpr int NT = (VAR & 1) ? 256 : 512;
  if (!(VAR & 1) || !loader) {
    const int tid = (VAR & 1) ? el - 256 : el;
#pragma unroll
    for (int i = 0; i < 64 * 32 / NT; ++i) {
      const int idx = tid + NT * i;
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
      if (VAR & (512 | 1024 | 2048)) {  // cache-policy variants of the plain bf16 store
        const int64_t mm = m0 + Q * 64 + r, nn = n0 + pr * 8;
        if (mm < p.M && nn < p.N) {
          u16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
          u16* dst = reinterpret_cast<u16*>(p.C) + mm * p.ldc + nn;
          typedef __attribute__((ext_vector_type(4))) unsigned u32x4v;
          const u32x4v d = __builtin_bit_cast(u32x4v, o);
          if (VAR & 512) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(d) : "memory");
          else if (VAR & 1024) __builtin_nontemporal_store(d, reinterpret_cast<u32x4v*>(dst));
          else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(dst), "v"(d) : "memory");
        }
      } else if (VAR & 8) {
        if (v[0] == 12345.f && v[7] == -1.f) store8<CULLAVO_DT_BF16>(p, v, m0 + Q * 64 + r, n0 + pr * 8);
      } else {
        store8<CULLAVO_DT_BF16>(p, v, m0 + Q * 64 + r, n0 + pr * 8);
      }
    }
  }
  if (VAR & 4) __syncthreads(); else raw_barrier();
}

template <int AL, int BL, int VAR>
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
  if ((VAR & 96) && (blockIdx.x & 7) >= 4) {
    const int n = (VAR & 32 ? 2 : 0) + (VAR & 64 ? 4 : 0);
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
  }
  if ((VAR & 384) && ((blockIdx.x >> 3) & 1)) {  // within-XCD stagger: every other CU of each XCD late
    const int n = (VAR & 128 ? 2 : 0) + (VAR & 256 ? 4 : 0);
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
  }

  const int64_t a_bytes = AL == 0 ? ((p.M - 1) * p.lda + p.K) * 2 : ((p.K - 1) * p.lda + p.M) * 2;
  const int64_t b_bytes = BL == 0 ? ((p.N - 1) * p.ldb + p.K) * 2 : ((p.K - 1) * p.ldb + p.N) * 2;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, b_bytes);

  TileXY xy = tile_xy(p, xcd_remap(t, p.sk_dp));
  int64_t m0 = (int64_t)xy.tm * P_BM, n0 = (int64_t)xy.tn * P_BN;
  if (loader) {
    dma_tile<AL, P_BM, 4>(ra, p.lda, m0, p.M, 0, p.K, smem, lw, lane);
    dma_tile<BL, P_BN, 4>(rb, p.ldb, n0, p.N, 0, p.K, smem + P_TILE_A, lw, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  raw_barrier();
  int s = 0;  // stage holding the current tile's first K-tile
  f32x4 acc[P_TMW][P_TN];
  for (;;) {
    const int t1 = t + (int)gridDim.x;
    const bool has_next = t1 < tiles;
    const TileXY xy1 = tile_xy(p, xcd_remap(has_next ? t1 : t, p.sk_dp));
    const int64_t m1 = (int64_t)xy1.tm * P_BM, n1 = (int64_t)xy1.tn * P_BN;
    // per-lane DMA offsets of this tile, loop-invariant in its K-loop (the next tile's first K-tile is
    // issued with inline offsets so these never change inside the loop)
    unsigned va[dma_per<P_BM, 4>()], vb[dma_per<P_BN, 4>()];
    dma_prep<AL, P_BM, 4>(p.lda, m0, p.M, lw, lane, va);
    dma_prep<BL, P_BN, 4>(p.ldb, n0, p.N, lw, lane, vb);
#pragma unroll
    for (int i = 0; i < P_TMW; ++i)
#pragma unroll
      for (int j = 0; j < P_TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      char* cur = smem + ((s + kt) & 1) * P_STAGE;
      char* nxt = smem + ((s + kt + 1) & 1) * P_STAGE;
      if (loader) {
        if (kt + 1 < nk) {
          const int64_t k1 = (int64_t)(kt + 1) * BK;
          dma_issue<P_BM, 4>(ra, va, dma_soff<AL>(k1, p.lda), nxt, lw);
          dma_issue<P_BN, 4>(rb, vb, dma_soff<BL>(k1, p.ldb), nxt + P_TILE_A, lw);
        } else if (!(VAR & 2) && has_next) {  // the next tile's first K-tile under this one's last MFMAs
          dma_tile<AL, P_BM, 4>(ra, p.lda, m1, p.M, 0, p.K, nxt, lw, lane);
          dma_tile<BL, P_BN, 4>(rb, p.ldb, n1, p.N, 0, p.K, nxt + P_TILE_A, lw, lane);
        }
      }
      tile_mfma<AL, BL, P_BM, P_BN, P_TMW, P_TN>(cur, wm, wn, lane, acc);
      if (!(VAR & 1) || loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      raw_barrier();
    }
    char* ep = smem + ((s + nk - 1) & 1) * P_STAGE;  // the last K-tile's stage, free after the barrier
    // per-lane epilogue indices recomputed per tile behind an opaque copy: hoisted out of the tile
    // loop they would stay live across the K-loop and spill
    int el = (int)threadIdx.x;
    asm volatile("" : "+v"(el));
    // epilogue in four 64-row passes through a 64 KiB f32 image (explicit calls: a rolled pass loop
    // would index acc dynamically and put it in scratch)
    if (!(VAR & 16)) {
      epi_pass<VAR, 0>(p, acc, ep, m0, n0, wm, wn, loader, el);
      epi_pass<VAR, 1>(p, acc, ep, m0, n0, wm, wn, loader, el);
      epi_pass<VAR, 2>(p, acc, ep, m0, n0, wm, wn, loader, el);
      epi_pass<VAR, 3>(p, acc, ep, m0, n0, wm, wn, loader, el);
    } else if (acc[0][0][0] == 12345.f) {
      *(float*)p.C = acc[1][1][1];
    }
    if (!has_next) break;
    if (VAR & 2) {  // exposed prologue
      if (loader) {
        dma_tile<AL, P_BM, 4>(ra, p.lda, m1, p.M, 0, p.K, smem + ((s + nk) & 1) * P_STAGE, lw, lane);
        dma_tile<BL, P_BN, 4>(rb, p.ldb, n1, p.N, 0, p.K, smem + ((s + nk) & 1) * P_STAGE + P_TILE_A, lw, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      raw_barrier();
    }
    s = (s + nk) & 1;
    t = t1;
    m0 = m1;
    n0 = n1;
  }
}

template <int AL, int BL, int VAR>
int launch_p(GemmArgs p, hipStream_t st) {
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)gemm256p_k<AL, BL, VAR>, hipFuncAttributeMaxDynamicSharedMemorySize, P_SMEM);
    set = true;
  }
  p.tiles_m = (int)cdiv(p.M, P_BM);
  p.tiles_n = (int)cdiv(p.N, P_BN);
  p.sk_dp = p.tiles_m * p.tiles_n;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = std::min(p.sk_dp, cus);
  gemm256p_k<AL, BL, VAR><<<grid, 512, P_SMEM, st>>>(p);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace

extern "C" int lab_gemm(int v, int64_t M, int64_t N, int64_t K, const void* A, const void* B, void* C, void* stream) {
  GemmArgs p{};
  p.A = (const u16*)A; p.B = (const u16*)B; p.C = C;
  p.M = M; p.N = N; p.K = K; p.lda = K; p.ldb = K; p.ldc = N;
  p.alpha = 1.f; p.act = CULLAVO_ACT_NONE; p.epi_lds = 1; p.group_m = -4; p.dma_pre = 1;
  hipStream_t s = (hipStream_t)stream;
  switch (v) {
#define C(V) case 1000 + V: return launch_p<0, 0, V>(p, s);
    C(0) C(8) C(512) C(1024) C(2048)
#undef C
  }
  return 2;
}
