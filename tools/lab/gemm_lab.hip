// GEMM structure lab (not part of the product library): ablation variants of the production
// 2-stage 256-row LDS-DMA kernel for the forward layout (A [M][K], B [N][K], both K-contiguous),
// built as its own small .so so a structural experiment compiles in seconds.
//   python tools/lab/gemm_lab.py   (on the GPU box)
#include "../../causal-unified-language-vision_amd/csrc/common.h"

namespace {

constexpr int BK = 64;
typedef __attribute__((ext_vector_type(8))) __bf16 frag8;
typedef __attribute__((address_space(3))) void lds_void;
constexpr unsigned kOOB = 0x7FFFFFF0u;

enum : int { F_NODMA = 1, F_NOMFMA = 2, F_LDR1 = 4, F_NOEPI = 8, F_SPLITKS = 16, F_STAG = 32, F_SPLIT2 = 64,
             F_NOWAIT = 128, F_NOBAR = 256, F_SPREAD = 512, F_REGS = 1024, F_MIDW = 2048 };

DEV int img0_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

DEV __amdgpu_buffer_rsrc_t make_rsrc(const u16* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <int ROWS, int NW>
DEV void dma_tile0(__amdgpu_buffer_rsrc_t rsrc, int64_t ld, int64_t idx0, int64_t idx_max, int64_t k0, int64_t K,
                   char* lds, int wave, int lane) {
  constexpr int kPieces = ROWS / 8;
#pragma unroll
  for (int i = 0; i < kPieces / NW; ++i) {
    const int pc = wave + NW * i;
    const int row = pc * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    const int64_t gi = idx0 + row, gk = k0 + chunk * 8;
    const unsigned off = (gi < idx_max && gk < K) ? (unsigned)((gi * ld + gk) * 2) : kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + pc * 1024), 16, off, 0, 0, 0);
  }
}

// piece i (0 <= i < ROWS / 8 / NW) of this wave's share of dma_tile0
template <int ROWS, int NW>
DEV void dma_piece0(__amdgpu_buffer_rsrc_t rsrc, int64_t ld, int64_t idx0, int64_t idx_max, int64_t k0, int64_t K,
                    char* lds, int wave, int lane, int i) {
  const int pc = wave + NW * i;
  const int row = pc * 8 + (lane >> 3);
  const int chunk = (lane & 7) ^ ((row >> 1) & 7);
  const int64_t gi = idx0 + row, gk = k0 + chunk * 8;
  const unsigned off = (gi < idx_max && gk < K) ? (unsigned)((gi * ld + gk) * 2) : kOOB;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + pc * 1024), 16, off, 0, 0, 0);
}

DEV frag8 read_frag0(const char* lds, int rbase, int ks, int lane) {
  const int row = rbase + (lane & 15);
  const int c = ks * 4 + (lane >> 4);
  u16x8 v = *reinterpret_cast<const u16x8*>(lds + img0_off(row, c));
  return __builtin_bit_cast(frag8, v);
}

// register staging (F_REGS): the next K-tile is read by plain 16-B buffer loads into VGPRs
// (8 threads per 128-B row segment, coalesced) and written to the same swizzled image with
// ds_write_b128, instead of LDS-DMA pieces
template <int ROWS>
DEV void regs_load0(__amdgpu_buffer_rsrc_t rsrc, int64_t ld, int64_t idx0, int64_t idx_max, int64_t k0, int64_t K,
                    u16x8 (&r)[ROWS / 64]) {
#pragma unroll
  for (int i = 0; i < ROWS / 64; ++i) {
    const int q = threadIdx.x + 512 * i;
    const int row = q >> 3, c = q & 7;
    const int64_t gi = idx0 + row, gk = k0 + c * 8;
    const unsigned off = (gi < idx_max && gk < K) ? (unsigned)((gi * ld + gk) * 2) : kOOB;
    r[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
  }
}
template <int ROWS>
DEV void regs_store0(char* lds, const u16x8 (&r)[ROWS / 64]) {
#pragma unroll
  for (int i = 0; i < ROWS / 64; ++i) {
    const int q = threadIdx.x + 512 * i;
    const int row = q >> 3, c = q & 7;
    *reinterpret_cast<u16x8*>(lds + img0_off(row, c)) = r[i];
  }
}

struct LabArgs {
  const u16* A;
  const u16* B;
  u16* C;
  int64_t M, N, K;
  int tiles_m, tiles_n;
};

// LDS-staged epilogue: per half (wm), the owning waves write f32 acc into a [BM2/2][256] image
// (16-B chunk c of row r at chunk c ^ (r & 15)); then all 512 threads store 8 contiguous
// columns each with one 16-B store (full 512-B rows per 32 lanes).
template <int BM2, int TMW, int TN>
DEV void lds_epilogue(const LabArgs& p, f32x4 (&acc)[TMW][TN], char* smem, int64_t m0, int64_t n0, int wm,
                      int wn, int lane) {
  constexpr int R = BM2 / 2;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (wm == half) {
#pragma unroll
      for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int r = tm * 16 + (lane & 15);
          const int c = wn * 16 + tn * 4 + (lane >> 4);
          *reinterpret_cast<f32x4*>(smem + r * 1024 + ((c ^ (r & 15)) << 4)) = acc[tm][tn];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < R * 32 / 512; ++i) {
      const int idx = threadIdx.x + 512 * i;
      const int r = idx >> 5, pr = idx & 31;
      const int sw = (pr >> 3) & 1;  // odd chunk first for pairs 8-15, 24-31: conflict-free
      const int c0 = 2 * pr + sw, c1 = 2 * pr + 1 - sw;
      const char* rowp = smem + r * 1024;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(rowp + ((c0 ^ (r & 15)) << 4));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(rowp + ((c1 ^ (r & 15)) << 4));
      const f32x4 lo = sw ? x1 : x0, hi = sw ? x0 : x1;
      const int64_t m = m0 + half * R + r, n = n0 + pr * 8;
      if (m < p.M && n < p.N) {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f2bf(lo[j]);
          o[4 + j] = f2bf(hi[j]);
        }
        *reinterpret_cast<u16x8*>(p.C + m * p.N + n) = o;
      }
    }
    __syncthreads();
  }
}

template <int BM2, int FL>
__global__ __launch_bounds__(512, 1) void lab256_k(LabArgs p) {
  constexpr int BN = 256;
  constexpr int TILE_A = BM2 * BK * 2;
  constexpr int TILE_B = BN * BK * 2;
  constexpr int STAGE = TILE_A + TILE_B;
  constexpr int TN = 4;
  constexpr int TMW = BM2 / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nwg = p.tiles_m * p.tiles_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP_M = 4;
  const int per_group = GROUP_M * p.tiles_n;
  const int group = lid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(p.tiles_m - first_m, GROUP_M);
  const int tm_idx = first_m + (lid % per_group) % gsize;
  const int tn_idx = (lid % per_group) / gsize;
  const int64_t m0 = (int64_t)tm_idx * BM2, n0 = (int64_t)tn_idx * BN;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, ((p.M - 1) * p.K + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, ((p.N - 1) * p.K + p.K) * 2);

  f32x4 acc[TMW][TN];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)cdiv(p.K, BK);
  dma_tile0<BM2, 8>(ra, p.K, m0, p.M, 0, p.K, smem, wave, lane);
  dma_tile0<BN, 8>(rb, p.K, n0, p.N, 0, p.K, smem + TILE_A, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    const bool more = kt + 1 < nk;
    char* nxt = smem + ((kt + 1) & 1) * STAGE;
    const int64_t k1 = (int64_t)(kt + 1) * BK;
    if constexpr (FL & (F_STAG | F_SPLIT2)) {
      // issue placement experiments: the rest of the pieces go in before ks = 1
      if (more) {
        if constexpr (FL & F_STAG) {
          if (wave < 4) {
            dma_tile0<BM2, 8>(ra, p.K, m0, p.M, k1, p.K, nxt, wave, lane);
            dma_tile0<BN, 8>(rb, p.K, n0, p.N, k1, p.K, nxt + TILE_A, wave, lane);
          }
        } else {
          if (wave < 4) dma_tile0<BM2, 4>(ra, p.K, m0, p.M, k1, p.K, nxt, wave, lane);
        }
      }
    } else if constexpr (FL & F_REGS) {
    } else if (more && !(FL & F_NODMA) && !(FL & F_SPREAD)) {
      if constexpr (FL & F_LDR1) {
        if (wave < 4) {
          dma_tile0<BM2, 4>(ra, p.K, m0, p.M, k1, p.K, nxt, wave, lane);
          dma_tile0<BN, 4>(rb, p.K, n0, p.N, k1, p.K, nxt + TILE_A, wave, lane);
        }
      } else {
        dma_tile0<BM2, 8>(ra, p.K, m0, p.M, k1, p.K, nxt, wave, lane);
        dma_tile0<BN, 8>(rb, p.K, n0, p.N, k1, p.K, nxt + TILE_A, wave, lane);
      }
    }
    u16x8 rga[BM2 / 64], rgb[BN / 64];
    if constexpr (FL & F_REGS) {
      if (more) {
        regs_load0<BM2>(ra, p.K, m0, p.M, k1, p.K, rga);
        regs_load0<BN>(rb, p.K, n0, p.N, k1, p.K, rgb);
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if constexpr ((FL & F_REGS) && (FL & F_MIDW)) {
        if (ks == 1 && more) {
          regs_store0<BM2>(nxt, rga);
          regs_store0<BN>(nxt + TILE_A, rgb);
        }
      }
      if constexpr (FL & (F_STAG | F_SPLIT2)) {
        if (ks == 1 && more) {
          if constexpr (FL & F_STAG) {
            if (wave >= 4) {
              dma_tile0<BM2, 8>(ra, p.K, m0, p.M, k1, p.K, nxt, wave, lane);
              dma_tile0<BN, 8>(rb, p.K, n0, p.N, k1, p.K, nxt + TILE_A, wave, lane);
            }
          } else {
            if (wave < 4) dma_tile0<BN, 4>(rb, p.K, n0, p.N, k1, p.K, nxt + TILE_A, wave, lane);
          }
        }
      }
      frag8 fb[TN];
#pragma unroll
      for (int t = 0; t < TN; ++t) fb[t] = read_frag0(cur + TILE_A, wn * 64 + t * 16, ks, lane);
#pragma unroll
      for (int tm = 0; tm < TMW; ++tm) {
        const frag8 fa = read_frag0(cur, wm * (BM2 / 2) + tm * 16, ks, lane);
        if constexpr (FL & F_NOMFMA) {
          asm volatile("" ::"v"(fa));
        } else {
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[tn], fa, acc[tm][tn], 0, 0, 0);
        }
        if constexpr ((FL & F_SPREAD) && BM2 == 256) {
          // one of this wave's 8 pieces (4 A + 4 B) after every other tm group of MFMAs
          const int slot = ks * TMW + tm;
          if ((slot & 1) && more) {
            const int pi = slot >> 1;
            __builtin_amdgcn_sched_barrier(0);
            if (pi < 4) dma_piece0<BM2, 8>(ra, p.K, m0, p.M, k1, p.K, nxt, wave, lane, pi);
            else dma_piece0<BN, 8>(rb, p.K, n0, p.N, k1, p.K, nxt + TILE_A, wave, lane, pi - 4);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      if constexpr (FL & F_NOMFMA) {
#pragma unroll
        for (int t = 0; t < TN; ++t) asm volatile("" ::"v"(fb[t]));
      }
    }
    if constexpr ((FL & F_REGS) && !(FL & F_MIDW)) {
      if (more) {
        regs_store0<BM2>(nxt, rga);
        regs_store0<BN>(nxt + TILE_A, rgb);
      }
    }
    if constexpr (!(FL & F_NOWAIT) && !(FL & F_REGS)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (!(FL & F_NOBAR)) __syncthreads();
  }

  if constexpr (FL & F_SPLITKS) {
    lds_epilogue<BM2, TMW, TN>(p, acc, smem, m0, n0, wm, wn, lane);
    return;
  }
#pragma unroll
  for (int tm = 0; tm < TMW; ++tm) {
    const int64_t m = m0 + wm * (BM2 / 2) + tm * 16 + (lane & 15);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int64_t n = n0 + wn * 64 + tn * 16 + (lane >> 4) * 4;
      if (m >= p.M || n >= p.N) continue;
      const f32x4 v = acc[tm][tn];
      if constexpr (FL & F_NOEPI) {
        if (v[0] == 12345.f) p.C[m * p.N + n] = 1;
      } else {
        u16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
        *reinterpret_cast<u16x4*>(p.C + m * p.N + n) = o;
      }
    }
  }
}

template <int BM2, int FL>
int launch(LabArgs p, hipStream_t s) {
  constexpr int smem = 2 * (BM2 * BK * 2 + 256 * BK * 2);
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)lab256_k<BM2, FL>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    set = true;
  }
  p.tiles_m = (int)cdiv(p.M, BM2);
  p.tiles_n = (int)cdiv(p.N, 256);
  lab256_k<BM2, FL><<<p.tiles_m * p.tiles_n, 512, smem, s>>>(p);
  return (int)hipGetLastError();
}

// ============================================================================================
// 4-wave 256x256 kernel: one wave per SIMD, each wave owns a 128x128 output quadrant (256
// accumulator registers), so a K-tile's LDS fragment reads are 128 KiB per CU instead of the
// 8-wave kernel's 192 KiB. The wave's own instruction stream hides latency: the next K-tile's
// LDS-DMA pieces and the ks=1 fragment reads are interleaved with the ks=0 MFMAs
// (sched_group_barrier), so the matrix pipe never waits on an issue burst.
// FL4: 1 = no steady-state DMA (ablation, wrong results), 4 = interleave schedule
// ============================================================================================
template <int FL4>
__global__ __launch_bounds__(256, 1) void lab4_k(LabArgs p) {
  constexpr int TILE = 256 * BK * 2;  // 32 KiB per operand image
  constexpr int STAGE = 2 * TILE;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nwg = p.tiles_m * p.tiles_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP_M = 4;
  const int per_group = GROUP_M * p.tiles_n;
  const int group = lid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(p.tiles_m - first_m, GROUP_M);
  const int tm_idx = first_m + (lid % per_group) % gsize;
  const int tn_idx = (lid % per_group) / gsize;
  const int64_t m0 = (int64_t)tm_idx * 256, n0 = (int64_t)tn_idx * 256;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, ((p.M - 1) * p.K + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, ((p.N - 1) * p.K + p.K) * 2);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)cdiv(p.K, BK);
  dma_tile0<256, 4>(ra, p.K, m0, p.M, 0, p.K, smem, wave, lane);
  dma_tile0<256, 4>(rb, p.K, n0, p.N, 0, p.K, smem + TILE, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt + 1) & 1) * STAGE;
    // the last iteration stages K past the end: the buffer range check zero-fills it into the
    // stage nobody reads again (no branch, so the whole body is one scheduling region)
    const int64_t k1 = (int64_t)(kt + 1) * BK;
    if constexpr (!(FL4 & F_NODMA)) {
      dma_tile0<256, 4>(ra, p.K, m0, p.M, k1, p.K, nxt, wave, lane);
      dma_tile0<256, 4>(rb, p.K, n0, p.N, k1, p.K, nxt + TILE, wave, lane);
    }
    frag8 fa0[8], fb0[8], fa1[8], fb1[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) fb0[t] = read_frag0(cur + TILE, wn * 128 + t * 16, 0, lane);
#pragma unroll
    for (int t = 0; t < 8; ++t) fa0[t] = read_frag0(cur, wm * 128 + t * 16, 0, lane);
#pragma unroll
    for (int t = 0; t < 8; ++t) fb1[t] = read_frag0(cur + TILE, wn * 128 + t * 16, 1, lane);
#pragma unroll
    for (int t = 0; t < 8; ++t) fa1[t] = read_frag0(cur, wm * 128 + t * 16, 1, lane);
#pragma unroll
    for (int tm = 0; tm < 8; ++tm)
#pragma unroll
      for (int tn = 0; tn < 8; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[tn], fa0[tm], acc[tm][tn], 0, 0, 0);
#pragma unroll
    for (int tm = 0; tm < 8; ++tm)
#pragma unroll
      for (int tn = 0; tn < 8; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[tn], fa1[tm], acc[tm][tn], 0, 0, 0);
    if constexpr (FL4 & F_LDR1) {
      // order: ks0 fragments, then per 4 MFMAs one DMA piece and one ks1 fragment read
      __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        if (!(FL4 & F_NODMA)) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // LDS-staged epilogue (2 halves of 128 rows x 256 columns f32)
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (wm == half) {
#pragma unroll
      for (int tm = 0; tm < 8; ++tm)
#pragma unroll
        for (int tn = 0; tn < 8; ++tn) {
          const int r = tm * 16 + (lane & 15);
          const int c = wn * 32 + tn * 4 + (lane >> 4);
          *reinterpret_cast<f32x4*>(smem + r * 1024 + ((c ^ (r & 15)) << 4)) = acc[tm][tn];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 128 * 32 / 256; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx >> 5, pr = idx & 31;
      const int sw = (pr >> 3) & 1;
      const int c0 = 2 * pr + sw, c1 = 2 * pr + 1 - sw;
      const char* rowp = smem + r * 1024;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(rowp + ((c0 ^ (r & 15)) << 4));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(rowp + ((c1 ^ (r & 15)) << 4));
      const f32x4 lo = sw ? x1 : x0, hi = sw ? x0 : x1;
      const int64_t m = m0 + half * 128 + r, n = n0 + pr * 8;
      if (m < p.M && n < p.N) {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f2bf(lo[j]);
          o[4 + j] = f2bf(hi[j]);
        }
        *reinterpret_cast<u16x8*>(p.C + m * p.N + n) = o;
      }
    }
    __syncthreads();
  }
}

template <int FL4>
int launch4(LabArgs p, hipStream_t s) {
  constexpr int smem = 2 * 2 * 256 * BK * 2;
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)lab4_k<FL4>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    set = true;
  }
  p.tiles_m = (int)cdiv(p.M, 256);
  p.tiles_n = (int)cdiv(p.N, 256);
  lab4_k<FL4><<<p.tiles_m * p.tiles_n, 256, smem, s>>>(p);
  return (int)hipGetLastError();
}

// ============================================================================================
// 4-wave 256x256 kernel with cross-K-tile fragment pipelining: each wave (one per SIMD) owns a
// 128x128 quadrant; fragments of the next half K-step are read from LDS while the MFMAs of the
// current half run (two register sets), and the barrier sits between the two halves:
//   read B = ks1(kt) | MFMA A | wait vmcnt(0), lgkmcnt(0), barrier | DMA tile kt+2 -> cur |
//   read A = ks0(kt+1) | MFMA B
// so tile kt+1's DMA had a full K-tile of MFMAs to land and no fragment read sits alone.
// FLP: 1 = no steady-state DMA (ablation, wrong results), 4 = interleave DMA issue with MFMAs
// ============================================================================================
template <int FLP>
__global__ __launch_bounds__(256, 1) void labpipe_k(LabArgs p) {
  constexpr int TILE = 256 * BK * 2;  // 32 KiB per operand image
  constexpr int STAGE = 2 * TILE;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nwg = p.tiles_m * p.tiles_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP_M = 4;
  const int per_group = GROUP_M * p.tiles_n;
  const int group = lid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(p.tiles_m - first_m, GROUP_M);
  const int tm_idx = first_m + (lid % per_group) % gsize;
  const int tn_idx = (lid % per_group) / gsize;
  const int64_t m0 = (int64_t)tm_idx * 256, n0 = (int64_t)tn_idx * 256;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, ((p.M - 1) * p.K + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, ((p.N - 1) * p.K + p.K) * 2);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)cdiv(p.K, BK);
  dma_tile0<256, 4>(ra, p.K, m0, p.M, 0, p.K, smem, wave, lane);
  dma_tile0<256, 4>(rb, p.K, n0, p.N, 0, p.K, smem + TILE, wave, lane);
  dma_tile0<256, 4>(ra, p.K, m0, p.M, BK, p.K, smem + STAGE, wave, lane);
  dma_tile0<256, 4>(rb, p.K, n0, p.N, BK, p.K, smem + STAGE + TILE, wave, lane);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 (16 pieces per wave) landed
  __syncthreads();
  frag8 fa0[8], fb0[8], fa1[8], fb1[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) fb0[t] = read_frag0(smem + TILE, wn * 128 + t * 16, 0, lane);
#pragma unroll
  for (int t = 0; t < 8; ++t) fa0[t] = read_frag0(smem, wm * 128 + t * 16, 0, lane);

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt + 1) & 1) * STAGE;
#pragma unroll
    for (int t = 0; t < 8; ++t) fb1[t] = read_frag0(cur + TILE, wn * 128 + t * 16, 1, lane);
#pragma unroll
    for (int t = 0; t < 8; ++t) fa1[t] = read_frag0(cur, wm * 128 + t * 16, 1, lane);
#pragma unroll
    for (int tm = 0; tm < 8; ++tm)
#pragma unroll
      for (int tn = 0; tn < 8; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[tn], fa0[tm], acc[tm][tn], 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    // tile kt is in registers on every wave: its buffer takes tile kt+2 (zero-filled past K)
    if constexpr (!(FLP & F_NODMA)) {
      const int64_t k2 = (int64_t)(kt + 2) * BK;
      dma_tile0<256, 4>(ra, p.K, m0, p.M, k2, p.K, cur, wave, lane);
      dma_tile0<256, 4>(rb, p.K, n0, p.N, k2, p.K, cur + TILE, wave, lane);
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) fb0[t] = read_frag0(nxt + TILE, wn * 128 + t * 16, 0, lane);
#pragma unroll
    for (int t = 0; t < 8; ++t) fa0[t] = read_frag0(nxt, wm * 128 + t * 16, 0, lane);
#pragma unroll
    for (int tm = 0; tm < 8; ++tm)
#pragma unroll
      for (int tn = 0; tn < 8; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[tn], fa1[tm], acc[tm][tn], 0, 0, 0);
    if constexpr (FLP & F_LDR1) {
      // 16 DMA pieces + 16 fragment reads spread over the 64 MFMAs of the second half
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        if (!(FLP & F_NODMA)) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (wm == half) {
#pragma unroll
      for (int tm = 0; tm < 8; ++tm)
#pragma unroll
        for (int tn = 0; tn < 8; ++tn) {
          const int r = tm * 16 + (lane & 15);
          const int c = wn * 32 + tn * 4 + (lane >> 4);
          *reinterpret_cast<f32x4*>(smem + r * 1024 + ((c ^ (r & 15)) << 4)) = acc[tm][tn];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 128 * 32 / 256; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int r = idx >> 5, pr = idx & 31;
      const int sw = (pr >> 3) & 1;
      const int c0 = 2 * pr + sw, c1 = 2 * pr + 1 - sw;
      const char* rowp = smem + r * 1024;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(rowp + ((c0 ^ (r & 15)) << 4));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(rowp + ((c1 ^ (r & 15)) << 4));
      const f32x4 lo = sw ? x1 : x0, hi = sw ? x0 : x1;
      const int64_t m = m0 + half * 128 + r, n = n0 + pr * 8;
      if (m < p.M && n < p.N) {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f2bf(lo[j]);
          o[4 + j] = f2bf(hi[j]);
        }
        *reinterpret_cast<u16x8*>(p.C + m * p.N + n) = o;
      }
    }
    __syncthreads();
  }
}

template <int FLP>
int launch_pipe(LabArgs p, hipStream_t s) {
  constexpr int smem = 2 * 2 * 256 * BK * 2;
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)labpipe_k<FLP>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    set = true;
  }
  p.tiles_m = (int)cdiv(p.M, 256);
  p.tiles_n = (int)cdiv(p.N, 256);
  labpipe_k<FLP><<<p.tiles_m * p.tiles_n, 256, smem, s>>>(p);
  return (int)hipGetLastError();
}

// ============================================================================================
// 8-wave 256x256 kernel (two waves per SIMD, 128x64 per wave) with the same cross-K-tile
// fragment pipelining as labpipe_k: the reads of one half K-step run under the MFMAs of the other.
// FLQ: 1 = no steady-state DMA (ablation, wrong results), 4 = interleave schedule hints
// ============================================================================================
template <int FLQ>
__global__ __launch_bounds__(512, 1) void labpipe8_k(LabArgs p) {
  constexpr int TILE = 256 * BK * 2;
  constexpr int STAGE = 2 * TILE;
  constexpr int TMW = 8, TN = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nwg = p.tiles_m * p.tiles_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP_M = 4;
  const int per_group = GROUP_M * p.tiles_n;
  const int group = lid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(p.tiles_m - first_m, GROUP_M);
  const int tm_idx = first_m + (lid % per_group) % gsize;
  const int tn_idx = (lid % per_group) / gsize;
  const int64_t m0 = (int64_t)tm_idx * 256, n0 = (int64_t)tn_idx * 256;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, ((p.M - 1) * p.K + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, ((p.N - 1) * p.K + p.K) * 2);

  f32x4 acc[TMW][TN];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)cdiv(p.K, BK);
  dma_tile0<256, 8>(ra, p.K, m0, p.M, 0, p.K, smem, wave, lane);
  dma_tile0<256, 8>(rb, p.K, n0, p.N, 0, p.K, smem + TILE, wave, lane);
  dma_tile0<256, 8>(ra, p.K, m0, p.M, BK, p.K, smem + STAGE, wave, lane);
  dma_tile0<256, 8>(rb, p.K, n0, p.N, BK, p.K, smem + STAGE + TILE, wave, lane);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 (8 pieces per wave) landed
  __syncthreads();
  frag8 fa0[TMW], fb0[TN], fa1[TMW], fb1[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) fb0[t] = read_frag0(smem + TILE, wn * 64 + t * 16, 0, lane);
#pragma unroll
  for (int t = 0; t < TMW; ++t) fa0[t] = read_frag0(smem, wm * 128 + t * 16, 0, lane);

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt + 1) & 1) * STAGE;
#pragma unroll
    for (int t = 0; t < TN; ++t) fb1[t] = read_frag0(cur + TILE, wn * 64 + t * 16, 1, lane);
#pragma unroll
    for (int t = 0; t < TMW; ++t) fa1[t] = read_frag0(cur, wm * 128 + t * 16, 1, lane);
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[tn], fa0[tm], acc[tm][tn], 0, 0, 0);
    if constexpr (FLQ & F_LDR1) {
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (!(FLQ & F_NODMA)) {
      const int64_t k2 = (int64_t)(kt + 2) * BK;
      dma_tile0<256, 8>(ra, p.K, m0, p.M, k2, p.K, cur, wave, lane);
      dma_tile0<256, 8>(rb, p.K, n0, p.N, k2, p.K, cur + TILE, wave, lane);
    }
#pragma unroll
    for (int t = 0; t < TN; ++t) fb0[t] = read_frag0(nxt + TILE, wn * 64 + t * 16, 0, lane);
#pragma unroll
    for (int t = 0; t < TMW; ++t) fa0[t] = read_frag0(nxt, wm * 128 + t * 16, 0, lane);
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[tn], fa1[tm], acc[tm][tn], 0, 0, 0);
    if constexpr (FLQ & F_LDR1) {
      __builtin_amdgcn_sched_group_barrier(0x020, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  lds_epilogue<256, TMW, TN>(p, acc, smem, m0, n0, wm, wn, lane);
}

template <int FLQ>
int launch_pipe8(LabArgs p, hipStream_t s) {
  constexpr int smem = 2 * 2 * 256 * BK * 2;
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)labpipe8_k<FLQ>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    set = true;
  }
  p.tiles_m = (int)cdiv(p.M, 256);
  p.tiles_n = (int)cdiv(p.N, 256);
  labpipe8_k<FLQ><<<p.tiles_m * p.tiles_n, 512, smem, s>>>(p);
  return (int)hipGetLastError();
}

// ============================================================================================
// 8-wave 256x256 kernel with only A staged through LDS (LDS-DMA, 2 stages) and the B fragments
// loaded straight into registers (16-B buffer loads, one K-tile ahead): halves the LDS-DMA
// write traffic, B's 2x-redundant fragment loads hit L2. Tests whether the DMA's LDS writes
// are what separates the DMA-fed kernel from the DMA-free ablation.
// FLD: 1 = no A DMA (ablation, wrong), 2 = no B loads (ablation, wrong)
// ============================================================================================
template <int FLD>
__global__ __launch_bounds__(512, 1) void labdirb_k(LabArgs p) {
  constexpr int TILE = 256 * BK * 2;
  constexpr int TMW = 8, TN = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nwg = p.tiles_m * p.tiles_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP_M = 4;
  const int per_group = GROUP_M * p.tiles_n;
  const int group = lid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(p.tiles_m - first_m, GROUP_M);
  const int tm_idx = first_m + (lid % per_group) % gsize;
  const int tn_idx = (lid % per_group) / gsize;
  const int64_t m0 = (int64_t)tm_idx * 256, n0 = (int64_t)tn_idx * 256;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, ((p.M - 1) * p.K + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, ((p.N - 1) * p.K + p.K) * 2);
  // B fragment t, half-step ks of K-tile kt: row n0 + wn*64 + t*16 + (lane&15), k = kt*64 + ks*32 + 8*(lane>>4)
  unsigned boff[TN];
  bool bok[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int64_t n = n0 + wn * 64 + t * 16 + (lane & 15);
    bok[t] = n < p.N;
    boff[t] = (unsigned)((n * p.K + 8 * (lane >> 4)) * 2);
  }
  auto load_b = [&](u16x8 (&dst)[2][TN], int64_t k0) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int64_t kk = k0 + ks * 32 + 8 * (lane >> 4);
        const unsigned off = (bok[t] && kk < p.K) ? boff[t] + (unsigned)((k0 + ks * 32) * 2) : kOOB;
        dst[ks][t] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0));
      }
  };

  f32x4 acc[TMW][TN];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)cdiv(p.K, BK);
  u16x8 bcur[2][TN], bnxt[2][TN];
  dma_tile0<256, 8>(ra, p.K, m0, p.M, 0, p.K, smem, wave, lane);
  load_b(bcur, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * TILE;
    char* nxt = smem + ((kt + 1) & 1) * TILE;
    const int64_t k1 = (int64_t)(kt + 1) * BK;
    if constexpr (!(FLD & 1)) dma_tile0<256, 8>(ra, p.K, m0, p.M, k1, p.K, nxt, wave, lane);
    if constexpr (!(FLD & 2)) load_b(bnxt, k1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int tm = 0; tm < TMW; ++tm) {
        const frag8 fa = read_frag0(cur, wm * 128 + tm * 16, ks, lane);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(frag8, bcur[ks][tn]), fa,
                                                               acc[tm][tn], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int t = 0; t < TN; ++t) bcur[ks][t] = bnxt[ks][t];
  }
  lds_epilogue<256, TMW, TN>(p, acc, smem, m0, n0, wm, wn, lane);
}

template <int FLD>
int launch_dirb(LabArgs p, hipStream_t s) {
  constexpr int smem = 2 * 256 * BK * 2 > 128 * 1024 ? 2 * 256 * BK * 2 : 128 * 1024;  // epilogue image
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)labdirb_k<FLD>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    set = true;
  }
  p.tiles_m = (int)cdiv(p.M, 256);
  p.tiles_n = (int)cdiv(p.N, 256);
  labdirb_k<FLD><<<p.tiles_m * p.tiles_n, 512, smem, s>>>(p);
  return (int)hipGetLastError();
}

// ============================================================================================
// 8-wave kernel on a 5-slot ring of K-half-tiles (32 k each, A and B: 32 KiB at 256x256),
// one barrier per half-tile, four half-tiles in flight (distance 4): a DMA has ~4x as long
// to land as in the 2-stage loop before its vmcnt.
// slot image: [rows][32 k] bf16, 64-B rows, 16-B chunk c of row r at c ^ ((r >> 2) & 3)
// ============================================================================================
DEV int img_h_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

template <int ROWS, int NW>
DEV void dma_half0(__amdgpu_buffer_rsrc_t rsrc, int64_t ld, int64_t idx0, int64_t idx_max, int64_t k0, int64_t K,
                   char* lds, int wave, int lane) {
  constexpr int kPieces = ROWS / 16;  // 16 rows x 64 B per 1 KiB piece
#pragma unroll
  for (int i = 0; i < kPieces / NW; ++i) {
    const int pc = wave + NW * i;
    const int row = pc * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 2) & 3);
    const int64_t gi = idx0 + row, gk = k0 + chunk * 8;
    const unsigned off = (gi < idx_max && gk < K) ? (unsigned)((gi * ld + gk) * 2) : kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + pc * 1024), 16, off, 0, 0, 0);
  }
}

DEV frag8 read_frag_h(const char* lds, int rbase, int lane) {
  const int row = rbase + (lane & 15);
  u16x8 v = *reinterpret_cast<const u16x8*>(lds + img_h_off(row, lane >> 4));
  return __builtin_bit_cast(frag8, v);
}

template <int P>
DEV void wait_vm() {
  if constexpr (P == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (P == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (P == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if constexpr (P == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else if constexpr (P == 18) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  else if constexpr (P == 21) asm volatile("s_waitcnt vmcnt(21)" ::: "memory");
  else if constexpr (P == 42) asm volatile("s_waitcnt vmcnt(42)" ::: "memory");
  else if constexpr (P == 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  else static_assert(P < 0, "add the count");
}

template <int BM2, int LDRF>
__global__ __launch_bounds__(512, 1) void labring_k(LabArgs p) {
  constexpr int BN = 256, SLOTS = 5, DIST = 4;
  constexpr int HA = BM2 * 64, HB = BN * 64;  // bytes of one half-tile image
  constexpr int SLOT = HA + HB;
  constexpr int TN = 4, TMW = BM2 / 32;
  constexpr int NWL = LDRF ? 4 : 8;                        // loader waves
  constexpr int PPW = (BM2 / 16 + BN / 16) / NWL;          // pieces per loader wave per half-tile
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nwg = p.tiles_m * p.tiles_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  constexpr int GROUP_M = 4;
  const int per_group = GROUP_M * p.tiles_n;
  const int group = lid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(p.tiles_m - first_m, GROUP_M);
  const int tm_idx = first_m + (lid % per_group) % gsize;
  const int tn_idx = (lid % per_group) / gsize;
  const int64_t m0 = (int64_t)tm_idx * BM2, n0 = (int64_t)tn_idx * BN;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool loader = LDRF ? wave < 4 : true;
  const int lw = LDRF ? (wave & 3) : wave;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, ((p.M - 1) * p.K + p.K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, ((p.N - 1) * p.K + p.K) * 2);

  f32x4 acc[TMW][TN];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nh = (int)cdiv(p.K, 32);
  auto stage = [&](int h) {
    char* dst = smem + (h % SLOTS) * SLOT;
    const int64_t k0 = (int64_t)h * 32;
    dma_half0<BM2, NWL>(ra, p.K, m0, p.M, k0, p.K, dst, lw, lane);
    dma_half0<BN, NWL>(rb, p.K, n0, p.N, k0, p.K, dst + HA, lw, lane);
  };
  if (loader) {
#pragma unroll
    for (int h = 0; h < DIST; ++h) stage(h);
    wait_vm<(DIST - 1) * PPW>();
  }
  __builtin_amdgcn_s_barrier();

  for (int h = 0; h < nh; ++h) {
    const char* cur = smem + (h % SLOTS) * SLOT;
    if (loader) stage(h + DIST);  // past K: zero-filled into a free slot
    frag8 fb[TN];
#pragma unroll
    for (int t = 0; t < TN; ++t) fb[t] = read_frag_h(cur + HA, wn * 64 + t * 16, lane);
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm) {
      const frag8 fa = read_frag_h(cur, wm * (BM2 / 2) + tm * 16, lane);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[tn], fa, acc[tm][tn], 0, 0, 0);
    }
    if (loader) wait_vm<(DIST - 1) * PPW>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (loader) wait_vm<0>();
  __syncthreads();
  lds_epilogue<BM2, TMW, TN>(p, acc, smem, m0, n0, wm, wn, lane);
}

template <int BM2, int LDRF>
int launch_ring(LabArgs p, hipStream_t s) {
  constexpr int smem = 5 * (BM2 * 64 + 256 * 64);
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)labring_k<BM2, LDRF>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    set = true;
  }
  p.tiles_m = (int)cdiv(p.M, BM2);
  p.tiles_n = (int)cdiv(p.N, 256);
  labring_k<BM2, LDRF><<<p.tiles_m * p.tiles_n, 512, smem, s>>>(p);
  return (int)hipGetLastError();
}

}  // namespace

void cullavo_set_error(const std::string&) {}
int cullavo_check_launch(const char*) { return 0; }

// variant = BM selector * 100 + flags
extern "C" int lab_gemm(int variant, int64_t M, int64_t N, int64_t K, const void* A, const void* B, void* C,
                        void* stream) {
  LabArgs p{(const u16*)A, (const u16*)B, (u16*)C, M, N, K, 0, 0};
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
#define V(BMV, FLV) \
  case (BMV == 256 ? 0 : 100) + FLV: return launch<BMV, FLV>(p, s);
    V(256, 0) V(256, 1) V(256, 2) V(256, 3) V(256, 4) V(256, 5) V(256, 8) V(256, 9) V(256, 10) V(256, 12)
    V(256, 16) V(256, 20) V(256, 17) V(256, 48) V(256, 80) V(192, 48) V(192, 80)
    V(192, 0) V(192, 1) V(192, 2) V(192, 4) V(192, 8) V(192, 16) V(192, 20)
    V(256, 1040) V(256, 3088) V(192, 1040) V(192, 3088) V(256, 1024) V(256, 128) V(256, 384) V(256, 257) V(256, 144) V(256, 528) V(256, 656) V(256, 912)
#undef V
    case 400: return launch4<0>(p, s);
    case 401: return launch4<1>(p, s);
    case 404: return launch4<4>(p, s);
    case 405: return launch4<5>(p, s);
    case 800: return launch_dirb<0>(p, s);
    case 801: return launch_dirb<1>(p, s);
    case 802: return launch_dirb<2>(p, s);
    case 803: return launch_dirb<3>(p, s);
    case 700: return launch_pipe8<0>(p, s);
    case 701: return launch_pipe8<1>(p, s);
    case 704: return launch_pipe8<4>(p, s);
    case 705: return launch_pipe8<5>(p, s);
    case 600: return launch_pipe<0>(p, s);
    case 601: return launch_pipe<1>(p, s);
    case 604: return launch_pipe<4>(p, s);
    case 605: return launch_pipe<5>(p, s);
    case 500: return launch_ring<256, 0>(p, s);
    case 501: return launch_ring<256, 1>(p, s);
    case 511: return launch_ring<192, 1>(p, s);
    default: return -1;
  }
}
