// Round-6 GEMM lab: the persistent 256x256 forward kernel with the finished tile's C HELD in
// registers (bf16, permlane16-widened to 16-B rows) and stored a few instructions per K-tile under
// the NEXT tile's K-loop, instead of the LDS-staged epilogue that writes the whole 128 KiB tile at
// once between two K-loops (profiles/r05/gemm/persistent_lab.txt: those stores were the per-tile
// fixed cost, +34 % at K = 1024 and +8-10 % at K = 4096 when removed).
//
// Layout (0,0), bf16 C = alpha * A B^T. Variants (lab_gemm v):
//   0   production-like persistent kernel (gemm256p_k<0>'s structure, LDS epilogue in 4 passes)
//   1   held C, all 16 chunk pairs per wave, per-piece DMA offsets (dma_prep, 16 VGPRs)
//   2   held C, DMA offsets as one lane base + scalar piece stride (rows past M land past the buffer)
//   3   as 2, stores issued at the END of the K-tile's MFMAs instead of after the DMA
//   4   as 2, 4 chunks per K-tile (drain over 4 K-tiles instead of 8)
//   5   as 2, 1 chunk per K-tile (drain over 16 K-tiles)
// Built by tools/lab/build_lab.sh; driven by tools/lab/gemm_lab.py --lib tools/lab/so/libgemm_hc.so.
#include "../../causal-unified-language-vision_amd/csrc/gemm_common.h"

using namespace cvgemm;

namespace {

struct PTile { int tm, tn; };
DEV PTile ptile(const GemmArgs& p, int lid) {
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

constexpr int P_TA = 256 * BK * 2, P_STAGE = 2 * P_TA;

// ---- variant 0: the production structure -------------------------------------------------------
template <int Q>
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
    const int64_t m = m0 + Q * 64 + r, n = n0 + pr * 8;
    if (m < p.M && n < p.N) {
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) { o[j] = f2bf(lo[j] * p.alpha); o[4 + j] = f2bf(hi[j] * p.alpha); }
      *reinterpret_cast<u16x8*>(reinterpret_cast<u16*>(p.C) + m * p.ldc + n) = o;
    }
  }
  praw_barrier();
}

__global__ __launch_bounds__(512, 1) void gemm_p0_k(GemmArgs p) {
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
        } else if (has_next) {
          dma_tile<0, 256, 4>(ra, p.lda, m1, p.M, 0, p.K, nxt, lw, lane);
          dma_tile<0, 256, 4>(rb, p.ldb, n1, p.N, 0, p.K, nxt + P_TA, lw, lane);
        }
      }
      tile_mfma<0, 0, 256, 256, 8, 4>(cur, wm, wn, lane, acc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      praw_barrier();
    }
    char* ep = smem + ((s + nk - 1) & 1) * P_STAGE;
    int el = (int)threadIdx.x;
    asm volatile("" : "+v"(el));
    p_epi_pass<0>(p, acc, ep, m0, n0, wm, wn, el);
    p_epi_pass<1>(p, acc, ep, m0, n0, wm, wn, el);
    p_epi_pass<2>(p, acc, ep, m0, n0, wm, wn, el);
    p_epi_pass<3>(p, acc, ep, m0, n0, wm, wn, el);
    if (!has_next) break;
    s = (s + nk) & 1;
    t = t1;
    m0 = m1;
    n0 = n1;
  }
}

// ---- held-C variants -----------------------------------------------------------------------
// A wave's 128 x 64 output block as 16 chunks: chunk j = (tm = j >> 1, pair = j & 1) covers rows
// tm*16 + (lane & 15) and the two 16-column MFMA tiles tn = 2 pair, 2 pair + 1. After packing to
// bf16 (2 dwords per tile and lane) one v_permlane16_swap per dword pair gives each lane 8
// consecutive columns: lane group g = lane >> 4 holds tile 2 pair + (g & 1), columns 8 (g >> 1)..+7.
// So each chunk is ONE 16-B store per lane (16 rows x 2 x 32 B contiguous per instruction).
struct Held {
  u32x4 c[16];
};

DEV unsigned pack2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}

DEV void hold(const GemmArgs& p, const f32x4 (&acc)[8][4], Held& h) {
#pragma unroll
  for (int tm = 0; tm < 8; ++tm)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const f32x4& a = acc[tm][2 * pr];
      const f32x4& b = acc[tm][2 * pr + 1];
      unsigned p0 = pack2(a[0] * p.alpha, a[1] * p.alpha), p1 = pack2(a[2] * p.alpha, a[3] * p.alpha);
      unsigned q0 = pack2(b[0] * p.alpha, b[1] * p.alpha), q1 = pack2(b[2] * p.alpha, b[3] * p.alpha);
      // rows 1, 3 of the first operand <-> rows 0, 2 of the second (16-lane rows)
      const auto r0 = __builtin_amdgcn_permlane16_swap(p0, q0, false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(p1, q1, false, false);
      h.c[tm * 2 + pr] = u32x4{r0[0], r1[0], r0[1], r1[1]};
    }
}

// store chunk J of the held tile (origin hm0, hn0 of the wave's block)
template <int J>
DEV void put(const GemmArgs& p, const Held& h, int64_t hm0, int64_t hn0, int lane) {
  const int tm = J >> 1, pr = J & 1, g = lane >> 4;
  const int64_t m = hm0 + tm * 16 + (lane & 15);
  const int64_t n = hn0 + (2 * pr + (g & 1)) * 16 + (g >> 1) * 8;
  if (m < p.M && n < p.N)
    *reinterpret_cast<u32x4*>(reinterpret_cast<u16*>(p.C) + m * p.ldc + n) = h.c[J];
}

template <int J0, int PER>
DEV void put_range(const GemmArgs& p, const Held& h, int64_t hm0, int64_t hn0, int lane) {
  if constexpr (PER >= 1) put<J0>(p, h, hm0, hn0, lane);
  if constexpr (PER >= 2) put<J0 + 1>(p, h, hm0, hn0, lane);
  if constexpr (PER >= 4) { put<J0 + 2>(p, h, hm0, hn0, lane); put<J0 + 3>(p, h, hm0, hn0, lane); }
}

template <int PER>
DEV void put_step(const GemmArgs& p, const Held& h, int64_t hm0, int64_t hn0, int lane, int k) {
  // k-th group of PER chunks; k uniform (scalar branches), chunk indices compile-time
#define PS(G) \
  if (k == G) { put_range<(G) * PER, PER>(p, h, hm0, hn0, lane); return; }
  PS(0) PS(1) PS(2) PS(3)
  if constexpr (PER <= 2) { PS(4) PS(5) PS(6) PS(7) }
  if constexpr (PER == 1) { PS(8) PS(9) PS(10) PS(11) PS(12) PS(13) PS(14) PS(15) }
#undef PS
}

DEV void put_all_from(const GemmArgs& p, const Held& h, int64_t hm0, int64_t hn0, int lane, int first) {
#define PA(J) if (first <= J) put<J>(p, h, hm0, hn0, lane);
  PA(0) PA(1) PA(2) PA(3) PA(4) PA(5) PA(6) PA(7) PA(8) PA(9) PA(10) PA(11) PA(12) PA(13) PA(14) PA(15)
#undef PA
}

// DMA for a 256-row layout-0 operand with one lane base: piece i of loader wave lw is rows
// (lw + 4 i) * 8 + (lane >> 3), the byte offset base + i * (32 rows * ld * 2) (scalar); rows past M
// land past the buffer's num_records (ld >= K) and read as zero
DEV unsigned dma_base0(int64_t ld, int64_t idx0, int lw, int lane) {
  const int row = lw * 8 + (lane >> 3);
  const int chunk = (lane & 7) ^ ((row >> 1) & 7);  // (row >> 1) & 7 is the same for every piece (+32 rows)
  return (unsigned)(((idx0 + row) * ld + chunk * 8) * 2);
}

// the running offset goes through an empty asm after each step, so the compiler cannot precompute
// (and keep live across the K-loop) the eight per-piece offsets: one VGPR instead of eight
DEV void dma_issue_stride(__amdgpu_buffer_rsrc_t rsrc, unsigned base, unsigned step, int soff, char* lds, int lw) {
  unsigned off = base;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + (lw + 4 * i) * 1024), 16, off, soff, 0, 0);
    off += step;
    asm volatile("" : "+v"(off));
  }
}

// H chunks (0, 8, 16) of the tile's 16 per wave are held and stored PER per K-tile under the next
// tile's K-loop; chunks [H, 16) are stored at the tile's end straight from registers (no LDS round
// trip, no barrier). VAR bits: 1 the next tile's K-tile 1 DMA is issued before those end-of-tile stores
// (they then overlap K-tile 0, counted vmcnt); 2 sc1 stores (written through, dropped from L2);
// 4 ablation: no stores at all (values kept live); 8 per-piece DMA offsets (dma_prep) instead of strided
DEV void put_chunk(const GemmArgs& p, const u32x4& v, int j, int64_t hm0, int64_t hn0, int lane, bool sc1) {
  const int tm = j >> 1, pr = j & 1, g = lane >> 4;
  const int64_t m = hm0 + tm * 16 + (lane & 15);
  const int64_t n = hn0 + (2 * pr + (g & 1)) * 16 + (g >> 1) * 8;
  if (m < p.M && n < p.N) {
    u32x4* dst = reinterpret_cast<u32x4*>(reinterpret_cast<u16*>(p.C) + m * p.ldc + n);
    if (sc1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(v) : "memory");
    else *dst = v;
  }
}

DEV u32x4 pack_chunk(const GemmArgs& p, const f32x4& a, const f32x4& b) {
  unsigned p0 = pack2(a[0] * p.alpha, a[1] * p.alpha), p1 = pack2(a[2] * p.alpha, a[3] * p.alpha);
  unsigned q0 = pack2(b[0] * p.alpha, b[1] * p.alpha), q1 = pack2(b[2] * p.alpha, b[3] * p.alpha);
  const auto r0 = __builtin_amdgcn_permlane16_swap(p0, q0, false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(p1, q1, false, false);
  return u32x4{r0[0], r1[0], r0[1], r1[1]};
}

template <int H>
struct HeldN { u32x4 c[H > 0 ? H : 1]; };

template <int H, int J0>
DEV void put_held2(const GemmArgs& p, const HeldN<H>& h, int64_t hm0, int64_t hn0, int lane, bool sc1) {
  if constexpr (J0 < H) put_chunk(p, h.c[J0], J0, hm0, hn0, lane, sc1);
  if constexpr (J0 + 1 < H) put_chunk(p, h.c[J0 + 1], J0 + 1, hm0, hn0, lane, sc1);
}

template <int H>
DEV void put_held_step(const GemmArgs& p, const HeldN<H>& h, int64_t hm0, int64_t hn0, int lane, int k, bool sc1) {
#define PS(G) if (k == G) { put_held2<H, 2 * (G)>(p, h, hm0, hn0, lane, sc1); return; }
  PS(0) PS(1) PS(2) PS(3) PS(4) PS(5) PS(6) PS(7)
#undef PS
}

template <int H>
DEV void put_held_from(const GemmArgs& p, const HeldN<H>& h, int64_t hm0, int64_t hn0, int lane, int first, bool sc1) {
#define PA(J) if constexpr (J < H) { if (first <= J) put_chunk(p, h.c[J], J, hm0, hn0, lane, sc1); }
  PA(0) PA(1) PA(2) PA(3) PA(4) PA(5) PA(6) PA(7) PA(8) PA(9) PA(10) PA(11) PA(12) PA(13) PA(14) PA(15)
#undef PA
}

template <int H, int VAR>
__global__ __launch_bounds__(512, 1) void gemm_hc_k(GemmArgs p) {
  constexpr bool SC1 = VAR & 2, NOSTORE = VAR & 4, EARLY = VAR & 1, PRE = VAR & 8, NLSKIP = VAR & 16;
  constexpr int GROUPS = H / 2;  // K-tiles that drain the held chunks (2 per K-tile)
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
  const unsigned step_a = (unsigned)(32 * p.lda * 2), step_b = (unsigned)(32 * p.ldb * 2);
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
  HeldN<H> h;
  int64_t hm0 = 0, hn0 = 0;
  bool held = false;
  bool k1_issued = false;  // EARLY: this tile's K-tile 1 DMA went out before the last tile's stores
  int pending = 0;         // EARLY: end-of-tile stores issued after that DMA (the first K-tile's vmcnt)
  for (;;) {
    const int t1 = t + (int)gridDim.x;
    const bool has_next = t1 < tiles;
    const PTile xy1 = ptile(p, xcd_remap(has_next ? t1 : t, p.sk_dp));
    const int64_t m1 = (int64_t)xy1.tm * 256, n1 = (int64_t)xy1.tn * 256;
    unsigned va[dma_per<256, 4>()], vb[dma_per<256, 4>()];
    unsigned ba = 0, bb = 0;
    if constexpr (PRE) {
      dma_prep<0, 256, 4>(p.lda, m0, p.M, lw, lane, va);
      dma_prep<0, 256, 4>(p.ldb, n0, p.N, lw, lane, vb);
    } else {
      ba = dma_base0(p.lda, m0, lw, lane);
      bb = dma_base0(p.ldb, n0, lw, lane);
      asm volatile("" : "+v"(ba), "+v"(bb));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      char* cur = smem + ((s + kt) & 1) * P_STAGE;
      char* nxt = smem + ((s + kt + 1) & 1) * P_STAGE;
      if (loader && !(kt == 0 && k1_issued)) {
        if (kt + 1 < nk) {
          const int64_t k1 = (int64_t)(kt + 1) * BK;
          if constexpr (PRE) {
            dma_issue<256, 4>(ra, va, dma_soff<0>(k1, p.lda), nxt, lw);
            dma_issue<256, 4>(rb, vb, dma_soff<0>(k1, p.ldb), nxt + P_TA, lw);
          } else {
            dma_issue_stride(ra, ba, step_a, dma_soff<0>(k1, p.lda), nxt, lw);
            dma_issue_stride(rb, bb, step_b, dma_soff<0>(k1, p.ldb), nxt + P_TA, lw);
          }
        } else if (has_next) {
          unsigned b1a = dma_base0(p.lda, m1, lw, lane), b1b = dma_base0(p.ldb, n1, lw, lane);
          asm volatile("" : "+v"(b1a), "+v"(b1b));
          dma_issue_stride(ra, b1a, step_a, 0, nxt, lw);
          dma_issue_stride(rb, b1b, step_b, 0, nxt + P_TA, lw);
        }
      }
      const bool storing = H > 0 && !NOSTORE && held && kt < GROUPS;
      if (storing) put_held_step<H>(p, h, hm0, hn0, lane, kt, SC1);
      tile_mfma<0, 0, 256, 256, 8, 4>(cur, wm, wn, lane, acc);
      if (NLSKIP && !loader) {
        // the non-loader waves issue no vector-memory op in the K-loop: their stores drain freely
      } else if (kt == 0 && pending > 0) {  // the end-of-tile stores (after K-tile 1's DMA) may stay in flight
        constexpr int P = 16 - H;
        if (storing) {
          if constexpr (P + 2 == 18) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        } else {
          if constexpr (P == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
        static_assert(H == 0 || H == 8 || H == 16, "H");
      } else if (storing) {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      praw_barrier();
    }
    if (H > 0 && !NOSTORE && held && nk < GROUPS) put_held_from<H>(p, h, hm0, hn0, lane, nk * 2, SC1);
    // this tile: chunks [0, H) held, [H, 16) stored now
    hm0 = m0 + wm * 128;
    hn0 = n0 + wn * 64;
    held = H > 0;
    k1_issued = false;
    pending = 0;
    if constexpr (EARLY) {
      // the next tile's K-tile 1 into the stage this tile's last K-tile freed (all waves are past
      // the loop's final barrier), before the stores below enter the memory pipeline
      if (has_next && nk > 1) {
        if (loader) {
          char* st1 = smem + ((s + nk + 1) & 1) * P_STAGE;  // next tile's K-tile 1 stage
          unsigned b1a = dma_base0(p.lda, m1, lw, lane), b1b = dma_base0(p.ldb, n1, lw, lane);
          asm volatile("" : "+v"(b1a), "+v"(b1b));
          dma_issue_stride(ra, b1a, step_a, dma_soff<0>(BK, p.lda), st1, lw);
          dma_issue_stride(rb, b1b, step_b, dma_soff<0>(BK, p.ldb), st1 + P_TA, lw);
        }
        k1_issued = true;
        pending = 16 - H;
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const u32x4 v = pack_chunk(p, acc[j >> 1][2 * (j & 1)], acc[j >> 1][2 * (j & 1) + 1]);
      if (j < H) {
        if constexpr (H > 0) h.c[j < H ? j : 0] = v;
      } else if constexpr (NOSTORE) {
        asm volatile("" ::"v"(v));
      } else {
        put_chunk(p, v, j, hm0, hn0, lane, SC1);
      }
    }
    if constexpr (NOSTORE && H > 0) {
#pragma unroll
      for (int j = 0; j < H; ++j) asm volatile("" ::"v"(h.c[j]));
    }
    if (!has_next) break;
    s = (s + nk) & 1;
    t = t1;
    m0 = m1;
    n0 = n1;
  }
  if constexpr (H > 0 && !NOSTORE) put_held_from<H>(p, h, hm0, hn0, lane, 0, SC1);
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

template <typename KF>
int launch(KF kern, GemmArgs p, hipStream_t st) {
  const int smem = 2 * P_STAGE;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  p.tiles_m = (int)cdiv(p.M, 256);
  p.tiles_n = (int)cdiv(p.N, 256);
  p.sk_dp = p.tiles_m * p.tiles_n;
  const int grid = std::min(p.sk_dp, num_cus());
  kern<<<(unsigned)grid, 512, smem, st>>>(p);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace

extern "C" int lab_gemm(int v, int64_t M, int64_t N, int64_t K, const void* A, const void* B, void* C, void* stream) {
  if (K % 64 != 0 || N % 8 != 0) return 2;
  GemmArgs p{};
  p.A = (const u16*)A;
  p.B = (const u16*)B;
  p.C = C;
  p.M = M; p.N = N; p.K = K;
  p.lda = K; p.ldb = K; p.ldc = N;
  p.alpha = 1.f;
  p.group_m = -4;
  hipStream_t st = (hipStream_t)stream;
  switch (v) {
    case 0: return launch(gemm_p0_k, p, st);
    // 100 * H/8 + VAR: H = 0 (direct stores only), 8 (half held), 16 (all held)
    case 1: return launch(gemm_hc_k<0, 0>, p, st);
    case 2: return launch(gemm_hc_k<0, 1>, p, st);
    case 3: return launch(gemm_hc_k<0, 2>, p, st);
    case 4: return launch(gemm_hc_k<0, 4>, p, st);
    case 5: return launch(gemm_hc_k<0, 8>, p, st);
    case 6: return launch(gemm_hc_k<0, 3>, p, st);
    case 7: return launch(gemm_hc_k<0, 17>, p, st);   // early DMA + non-loaders never wait
    case 8: return launch(gemm_hc_k<0, 16>, p, st);   // non-loaders never wait
    case 101: return launch(gemm_hc_k<8, 0>, p, st);
    case 102: return launch(gemm_hc_k<8, 1>, p, st);
    case 103: return launch(gemm_hc_k<8, 2>, p, st);
    case 104: return launch(gemm_hc_k<8, 4>, p, st);
    case 201: return launch(gemm_hc_k<16, 0>, p, st);
    default: return 3;
  }
}
