// 256x256 bf16 GEMM tile with FOUR waves (one per SIMD), each owning a 128x128 output block whose
// 256 f32 accumulators stay in the AGPR half of the register file (inline-asm MFMAs, "+a"), and a
// register-staged global -> LDS pipeline two K-tiles deep (round 5).
//
// Why (profiles/r05/gemm/): on the forward products the PMC of hipBLASLt's 4-wave kernel
// (MT256x256x64, 1 wave per SIMD) shows MFMA busy 0.73-0.80 with waves waiting 7 % of their
// cycles, against 0.59-0.60 and 30 % for the 8-wave LDS-DMA kernel of gemm.hip, whose every K-tile
// ends in vmcnt(0) + a barrier with one tile of prefetch and begins with an exposed fragment-read
// burst. The issue-cost lab (tools/lab/issue_lab.hip) prices the instructions beside MFMAs: with
// one wave per SIMD two ds_read_b128 per 8 MFMAs cost +3.6 % (at two waves per SIMD +13.8 %), a
// ds_write_b128 ~0, one global load ~+9 %: a 128x128-per-wave tile (2 fragment reads per 8 MFMAs
// instead of 3) at one wave per SIMD is the cheaper way to feed the matrix pipes.
//
// Pipeline (BK = 64 = two 32-deep halves, 2 LDS stages of A|B = 128 KiB, 64 staging VGPRs):
//   K-tile kt, half 0: MFMAs on the ks0 fragments of kt (in registers) with, under them, the ks1
//     fragment reads of kt, the LDS writes of tile kt+1 (loaded into registers during kt-1) into
//     the other stage, and the global loads of tile kt+2 (first half of the registers);
//     lgkmcnt(0) + barrier (tile kt+1 visible; stage kt no longer read after this point except
//     by the ks1 fragments already in registers);
//   half 1: MFMAs on the ks1 fragments with, under them, the ks0 fragment reads of tile kt+1 and
//     the global loads of tile kt+2's second half.
//   One barrier per K-tile; no wave ever waits for a fragment read at a half's start, and a
//   global load has a whole K-tile (~2,000 MFMA cycles) before its LDS write needs it.
// Layouts: a K-contiguous operand (layout 0, K % 64 == 0) is staged as [256 rows][64 k] with the
// XOR swizzle of gemm_common.h img0_off and read by ds_read_b128; an M/N-contiguous operand
// (layout 1) as [64 k][256 cols] with img1w_off and read by ds_read_b64_tr_b16 (the builtin:
// with no LDS-DMA in flight hipcc has nothing to alias it with). Rows past M / N and k-rows
// past K read as zeros (buffer range check: the operand's extent or a per-lane out-of-range
// offset). The epilogue stages each half of the tile's rows through the (then idle) 128 KiB
// of LDS as f32 and runs the gemm_common.h store8 chain (bias, preact, activation, LoRA addend,
// residual, beta, SwiGLU backward) on 8 contiguous columns per lane, as the 8-wave kernels do.
#include "gemm_common.h"

namespace {
using namespace cvgemm;

constexpr int T4 = 256;                    // tile rows = tile cols
constexpr int OPB4 = T4 * BK * 2;          // 32 KiB per operand image
constexpr int STAGE4 = 2 * OPB4;           // A | B
constexpr int SMEM4 = 2 * STAGE4;          // 128 KiB (the epilogue's [128][256] f32 image fits)

typedef __attribute__((ext_vector_type(4))) unsigned u32x4v;

// accumulator MFMAs pinned to AGPRs (swapped operands as in gemm.hip: A slot <- N fragment, B slot
// <- M fragment, so lane l ends with C[m = lane & 15][n = 4 (lane >> 4) + j])
DEV void mfma4_acc(f32x4& c, const frag8& nb, const frag8& ma) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(nb), "v"(ma));
}
DEV void mfma4_zero(f32x4& c, const frag8& nb, const frag8& ma) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(nb), "v"(ma));
}

// staging geometry of one operand: 8 loads of 16 B per thread per K-tile.
// layout 0 (K-contiguous, [rows][K]): load i covers rows 32 i + t / 8, 16-B chunk t % 8
// layout 1 ([K][rows]): load i covers k-rows 8 i + t / 32, columns 8 (t % 32) .. +7
template <int L>
struct Stage {
  unsigned voff;  // per-lane byte offset of load 0 at K-tile 0 (kOOBp for rows / columns past the edge)
  int64_t step;   // byte distance between load i and i+1 (scalar)
  int lds[8];     // LDS byte offset of each load's 16 B in the operand image
};

template <int L>
DEV Stage<L> stage_geom(int64_t ld, int64_t idx0, int64_t idx_max, int t) {
  Stage<L> g;
  if (L == 0) {
    const int row = t >> 3, c = t & 7;
    // rows past idx_max lie past the buffer's extent ((idx_max - 1) * ld + K elements): zeros
    g.voff = (unsigned)(((idx0 + row) * ld + c * 8) * 2);
    g.step = 32 * ld * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) g.lds[i] = img0_off(row + 32 * i, c);
  } else {
    const int k = t >> 5, col = (t & 31) * 8;
    g.voff = idx0 + col < idx_max ? (unsigned)((k * ld + idx0 + col) * 2) : kOOBp;
    g.step = 8 * ld * 2;
    const int unit = col >> 4, half = (col >> 3) & 1;
#pragma unroll
    for (int i = 0; i < 8; ++i) g.lds[i] = img1w_off<T4>(k + 8 * i, unit) + half * 16;
  }
  return g;
}

template <int L>
DEV int64_t ktile_soff(int64_t kt, int64_t ld) { return L == 0 ? kt * BK * 2 : kt * BK * ld * 2; }

// fragment of rows rbase.. (16) at K-half ks from an operand image
template <int L>
DEV frag8 frag4(const char* img, int rbase, int ks, int lane) { return read_frag_w<L, T4>(img, rbase, ks, lane); }

DEV void dma_piece(__amdgpu_buffer_rsrc_t rs, char* lds, unsigned vo, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 16, vo, soff, 0, 0);
}

struct Frags4 {
  frag8 a[8];  // M fragments: rows wr*128 + 16 i
  frag8 b[8];  // N fragments: cols wc*128 + 16 j
};

template <int CT>
DEV void epilogue4(const GemmArgs& p, f32x4 (&acc)[8][8], char* smem, int64_t m0, int64_t n0, int wr, int wc, int t,
                   int lane) {
  // epilogue: per row half h, waves (h, 0) and (h, 1) write their f32 block into a [128][256]
  // image (16-B chunk c of row r at c ^ (r & 15)), then all 256 threads run store8 on 8 columns
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wr == h) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = i * 16 + (lane & 15);
          const int c = wc * 32 + j * 4 + (lane >> 4);
          *reinterpret_cast<f32x4*>(smem + r * 1024 + ((c ^ (r & 15)) << 4)) = acc[i][j];
        }
    }
    __syncthreads();
#pragma unroll 4
    for (int it = 0; it < 128 * 32 / 256; ++it) {
      const int idx = t + 256 * it;
      const int r = idx >> 5, pr = idx & 31;
      const int sw = (pr >> 3) & 1;
      const int c0 = 2 * pr + sw, c1 = 2 * pr + 1 - sw;
      const char* rowp = smem + r * 1024;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(rowp + ((c0 ^ (r & 15)) << 4));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(rowp + ((c1 ^ (r & 15)) << 4));
      const f32x4 lo = sw ? x1 : x0, hi = sw ? x0 : x1;
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] = lo[j]; v[4 + j] = hi[j]; }
      store8<CT>(p, v, m0 + h * 128 + r, n0 + pr * 8);
    }
    __syncthreads();
  }
}

// ABL: lab ablations only (tools/lab/gemm4w_lab.hip; results wrong): bit 0 = no in-loop global
// loads, 1 = no in-loop LDS writes, 2 = no barrier, 3 = no in-loop fragment reads, 4 = every
// global load in half 0 right after its register's LDS write, 5 = one global load per row group
// (A in half 0, B in half 1; both results right), 6 = loads kept but the LDS writes take other
// registers (no wait on a load in the loop), 7 = LDS-DMA staging instead of registers (tile kt+2
// DMA'd into stage kt & 1 under half 1 of K-tile kt, waited before the mid-barrier of kt+1)
template <int AL, int BL, int CT, int ABL = 0>
__global__ __launch_bounds__(256, 1) void gemm4w_k(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lid = xcd_remap(blockIdx.x, p.sk_dp);
  int64_t m0, n0;
  tile_origin<T4, T4>(p, lid, m0, n0);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  const int64_t a_bytes = AL == 0 ? ((p.M - 1) * p.lda + p.K) * 2 : ((p.K - 1) * p.lda + p.M) * 2;
  const int64_t b_bytes = BL == 0 ? ((p.N - 1) * p.ldb + p.K) * 2 : ((p.K - 1) * p.ldb + p.N) * 2;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, b_bytes);
  const Stage<AL> ga = stage_geom<AL>(p.lda, m0, p.M, t);
  const Stage<BL> gb = stage_geom<BL>(p.ldb, n0, p.N, t);
  const int nk = (int)cdiv(p.K, BK);

  constexpr bool DMA = (ABL & 128) != 0;
  unsigned dva[dma_per<T4, 4>()], dvb[dma_per<T4, 4>()];
  if constexpr (DMA) {
    dma_prep<AL, T4, 4>(p.lda, m0, p.M, wave, lane, dva);
    dma_prep<BL, T4, 4>(p.ldb, n0, p.N, wave, lane, dvb);
  }
  // LDS-DMA pieces [lo, hi) of tile kt (0-7 A, 8-15 B) into stage
  auto dma = [&](int kt, char* stage, int lo, int hi) {
    const int64_t k0 = (int64_t)kt * BK;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i < lo || i >= hi) continue;
      if (i < 8) dma_piece(ra, stage + (wave + 4 * i) * 1024, dva[i], dma_soff<AL>(k0, p.lda));
      else dma_piece(rb, stage + OPB4 + (wave + 4 * (i - 8)) * 1024, dvb[i - 8], dma_soff<BL>(k0, p.ldb));
    }
  };
  u32x4v st[16];  // [0, 8): A loads, [8, 16): B loads
  auto gload = [&](int kt, int lo, int hi) {
    if constexpr ((ABL & 1) != 0 || DMA) return;
    const int64_t sa = ktile_soff<AL>(kt, p.lda), sb = ktile_soff<BL>(kt, p.ldb);  // uniform
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i < lo || i >= hi) continue;
      if (i < 8) st[i] = __builtin_amdgcn_raw_buffer_load_b128(ra, ga.voff, (int)(sa + i * ga.step), 0);
      else st[i] = __builtin_amdgcn_raw_buffer_load_b128(rb, gb.voff, (int)(sb + (i - 8) * gb.step), 0);
    }
  };
  auto swrite1 = [&](char* stage, int i) {
    if constexpr ((ABL & 2) != 0 || DMA) return;
    if constexpr ((ABL & 64) != 0) {  // lab: write registers that no load feeds (loads kept alive below)
      *reinterpret_cast<u32x4v*>(stage + (i < 8 ? ga.lds[i] : OPB4 + gb.lds[i - 8])) = u32x4v{ga.voff, gb.voff, 1u, 2u};
      return;
    }
    if (i < 8) *reinterpret_cast<u32x4v*>(stage + ga.lds[i]) = st[i];
    else *reinterpret_cast<u32x4v*>(stage + OPB4 + gb.lds[i - 8]) = st[i];
  };
  // the reads issued under row group r of a half: every row of the next half needs all eight N
  // fragments but only its own M fragment, so the N fragments come first (groups 0-3) and the M
  // fragments after them (groups 4-7): the next half's row r waits on reads >= 4 groups old
  auto fread_row = [&](const char* stage, int ks, int r, Frags4& f) {
    if constexpr ((ABL & 8) != 0) return;
    if (r < 4) {
      f.b[2 * r] = frag4<BL>(stage + OPB4, wc * 128 + 2 * r * 16, ks, lane);
      f.b[2 * r + 1] = frag4<BL>(stage + OPB4, wc * 128 + (2 * r + 1) * 16, ks, lane);
    } else {
      f.a[2 * r - 8] = frag4<AL>(stage, wr * 128 + (2 * r - 8) * 16, ks, lane);
      f.a[2 * r - 7] = frag4<AL>(stage, wr * 128 + (2 * r - 7) * 16, ks, lane);
    }
  };

  f32x4 acc[8][8];
  Frags4 F0, F1;

  // prologue: tile 0 -> stage 0, tile 1 into the registers, ks0 fragments of tile 0
  if constexpr (DMA) {
    dma(0, smem, 0, 16);
    dma(1, smem + STAGE4, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  gload(0, 0, 16);
#pragma unroll
  for (int i = 0; i < 16; ++i) swrite1(smem, i);
  gload(1, 0, 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int r = 0; r < 8; ++r) fread_row(smem, 0, r, F0);

  // half 0 of K-tile kt: MFMAs on F0 (ks0 of kt); under them F1 <- ks1 of kt, tile kt+1's LDS
  // writes (registers -> other stage) and tile kt+2's first 8 global loads
  auto half0 = [&](auto first_c, int kt) {
    constexpr bool FIRST = decltype(first_c)::value;
    const char* cur = smem + (kt & 1) * STAGE4;
    char* nxt = smem + ((kt + 1) & 1) * STAGE4;
    // no branches in the stream: past the last K-tile the writes fill a stage nobody reads and the
    // loads read zeros or in-range bytes nobody uses (buffer loads are range-checked)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      fread_row(cur, 1, r, F1);
      swrite1(nxt, 2 * r);
      swrite1(nxt, 2 * r + 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (FIRST) mfma4_zero(acc[r][j], F0.b[j], F0.a[r]);
        else mfma4_acc(acc[r][j], F0.b[j], F0.a[r]);
      }
      if constexpr ((ABL & 16) != 0) gload(kt + 2, 2 * r, 2 * r + 2);  // lab: every load in half 0
      else if constexpr ((ABL & 32) != 0) gload(kt + 2, r, r + 1);     // lab: one load per row group
      else if (r < 4) gload(kt + 2, 2 * r, 2 * r + 2);  // A loads 0..7
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile kt+1 landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr ((ABL & 4) == 0) __builtin_amdgcn_s_barrier();
  };
  // half 1: MFMAs on F1 (ks1 of kt); under them F0 <- ks0 of tile kt+1, tile kt+2's B loads
  auto half1 = [&](int kt) {
    const char* nxt = smem + ((kt + 1) & 1) * STAGE4;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      fread_row(nxt, 0, r, F0);
#pragma unroll
      for (int j = 0; j < 8; ++j) mfma4_acc(acc[r][j], F1.b[j], F1.a[r]);
      if constexpr (DMA) dma(kt + 2, smem + (kt & 1) * STAGE4, 2 * r, 2 * r + 2);
      else if constexpr ((ABL & 32) != 0) gload(kt + 2, 8 + r, 9 + r);
      else if ((ABL & 16) == 0 && r < 4) gload(kt + 2, 8 + 2 * r, 10 + 2 * r);  // B loads 8..15
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  half0(std::true_type{}, 0);
  half1(0);
  for (int kt = 1; kt < nk; ++kt) {
    half0(std::false_type{}, kt);
    half1(kt);
  }
  if constexpr ((ABL & 64) != 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(st[i]));
  }
  // the last MFMAs' results before the epilogue reads the AGPRs (8-pass XDL write -> read)
  asm volatile("s_nop 15\n\ts_nop 7" : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]),
               "+a"(acc[7][4]), "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]));
  __builtin_amdgcn_s_barrier();  // every wave's last fragment reads are done before LDS is reused

  epilogue4<CT>(p, acc, smem, m0, n0, wr, wc, t, lane);
}

// ============================================================================================
// LDS-DMA variant with the stage released in ks halves (gemm4q_k)
// ============================================================================================
// The register-staged kernel above waits on its own global loads before each LDS write
// (ablations, profiles/r05/gemm/gemm4w_ablations.txt: without the loads 1.8 PF/s, with them 1.2);
// LDS-DMA needs no such wait, only a counted vmcnt before the barrier whose readers need the data.
// Each stage holds a K-tile as two 32-deep regions (ks0 | ks1) per operand, and a region is
// DMA'd as soon as nobody reads it any more, two K-halves before it is needed:
//   half 0 of K-tile kt: MFMAs on F0 = ks0(kt); reads F1 <- ks1(kt); DMA ks0(kt+2) -> stage kt&1
//     (its ks0 region was last read under half 1 of kt-1); then wait until ks0(kt+1) (DMA'd under
//     half 0 of kt-1) has landed, barrier;
//   half 1: MFMAs on F1; reads F0 <- ks0(kt+1); DMA ks1(kt+2) -> stage kt&1 (its ks1 region was last
//     read under half 0 of kt); wait until ks1(kt+1) has landed, barrier.
// Every DMA piece is issued a full K-tile before the barrier that publishes it (vmcnt(16): the 16
// pieces of the two younger halves stay in flight).
// Layout-0 regions are [256 rows][32 k] with 64-B rows (16-B chunk c of row r at c ^ ((r >> 2) & 3):
// the 16 rows of a ds_read_b128 lane group on 16 distinct 16-B bank slots); layout-1 regions are k-rows
// 32 ks .. 32 ks + 31 of the [64 k][256] image of the register-staged kernel.
constexpr int REG4 = T4 * 32 * 2;  // 16 KiB: one operand's ks region

DEV int img0q_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// per-lane source offset of the wave's DMA pieces of one operand (piece pc = wave + 4 i, i = 0..3 of
// a region; K-tile 0, ks 0; later pieces / ks / K-tiles through the scalar offset)
template <int L>
DEV unsigned dmaq_voff(int64_t ld, int64_t idx0, int64_t idx_max, int wave, int lane) {
  if (L == 0) {
    const int row = 16 * wave + (lane >> 2);
    const int csrc = (lane & 3) ^ ((row >> 2) & 3);
    return (unsigned)(((idx0 + row) * ld + csrc * 8) * 2);  // rows past idx_max: past the extent
  }
  const int byte = wave * 1024 + lane * 16;  // pieces wave + 4 i: k-rows 2 (wave + 4 i) + byte / 512
  const int k = byte / 512, b = byte % 512;
  const int unit = upos<T4>(b >> 5, k), half = (b >> 4) & 1;
  const int64_t gi = idx0 + unit * 16 + half * 8;
  return gi < idx_max ? (unsigned)((k * ld + gi) * 2) : kOOBp;
}
// scalar offset of piece i of region ks of K-tile kt
template <int L>
DEV int dmaq_soff(int kt, int ks, int i, int64_t ld) {
  if (L == 0) return (int)((int64_t)kt * BK * 2 + ks * 64 + (int64_t)i * 64 * ld * 2);
  return (int)(((int64_t)kt * BK + ks * 32 + i * 8) * ld * 2);
}

// Fragment reads by inline asm: hipcc (ROCm 7.2) cannot tell an LDS read from the LDS-DMA in flight
// into the other region and would wait vmcnt(0) before every compiler-visible one (gemm_common.h
// tr_issue). The reads of a half are consumed only in the next half, after that half's
// lgkmcnt(0) + barrier; fq_tie() then re-defines the registers so that no consumer is hoisted above it.
template <int L>
struct FragQ;
template <>
struct FragQ<0> {
  frag8 v;
  DEV frag8 get() const { return v; }
  DEV void tie() { asm volatile("" : "+v"(v)); }
};
template <>
struct FragQ<1> {
  s16x4 lo, hi;
  DEV frag8 get() const { return tr_join(lo, hi); }
  DEV void tie() { asm volatile("" : "+v"(lo), "+v"(hi)); }
};

DEV void fq_issue(FragQ<0>& f, const char* region, int rbase, int ks, int lane) {
  (void)ks;
  const int row = rbase + (lane & 15), c = lane >> 4;
  asm volatile("ds_read_b128 %0, %1" : "=&v"(f.v) : "v"(lds_addr(region + img0q_off(row, c))) : "memory");
}
DEV void fq_issue(FragQ<1>& f, const char* region, int rbase, int ks, int lane) {
  tr_issue<T4>(region - ks * REG4, rbase, ks, lane, f.lo, f.hi);  // k-rows of the [64][256] image
}

template <int AL, int BL>
struct FragsQ {
  FragQ<AL> a[8];
  FragQ<BL> b[8];
  DEV void tie() {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a[i].tie();
      b[i].tie();
    }
  }
};

template <int AL, int BL, int CT>
__global__ __launch_bounds__(256, 1) void gemm4q_k(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lid = xcd_remap(blockIdx.x, p.sk_dp);
  int64_t m0, n0;
  tile_origin<T4, T4>(p, lid, m0, n0);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t a_bytes = AL == 0 ? ((p.M - 1) * p.lda + p.K) * 2 : ((p.K - 1) * p.lda + p.M) * 2;
  const int64_t b_bytes = BL == 0 ? ((p.N - 1) * p.ldb + p.K) * 2 : ((p.K - 1) * p.ldb + p.N) * 2;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, a_bytes);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, b_bytes);
  const unsigned va = dmaq_voff<AL>(p.lda, m0, p.M, wave, lane);
  const unsigned vb = dmaq_voff<BL>(p.ldb, n0, p.N, wave, lane);
  const int nk = (int)cdiv(p.K, BK);
  // region (ks) of operand op (0 A, 1 B) of stage s
  auto region = [&](int s, int op, int ks) { return smem + s * STAGE4 + op * OPB4 + ks * REG4; };
  // the wave's 8 DMA pieces (4 A, 4 B) of region ks of K-tile kt into stage s; piece j of a
  // region sits at (wave + 4 j) KiB
  auto dma_region = [&](int kt, int ks, int s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dma_piece(ra, region(s, 0, ks) + (wave + 4 * i) * 1024, va, dmaq_soff<AL>(kt, ks, i, p.lda));
      dma_piece(rb, region(s, 1, ks) + (wave + 4 * i) * 1024, vb, dmaq_soff<BL>(kt, ks, i, p.ldb));
    }
  };
  // pieces i of region ks of K-tile kt (one A and one B piece): the DMA spread over a half's row groups
  auto dma_region_piece2 = [&](int kt, int ks, int s, int i) {
    dma_piece(ra, region(s, 0, ks) + (wave + 4 * i) * 1024, va, dmaq_soff<AL>(kt, ks, i, p.lda));
    dma_piece(rb, region(s, 1, ks) + (wave + 4 * i) * 1024, vb, dmaq_soff<BL>(kt, ks, i, p.ldb));
  };
  auto fread_row = [&](int s, int ks, int r, FragsQ<AL, BL>& f) {
    if (r < 4) {
      fq_issue(f.b[2 * r], region(s, 1, ks), wc * 128 + 2 * r * 16, ks, lane);
      fq_issue(f.b[2 * r + 1], region(s, 1, ks), wc * 128 + (2 * r + 1) * 16, ks, lane);
    } else {
      fq_issue(f.a[2 * r - 8], region(s, 0, ks), wr * 128 + (2 * r - 8) * 16, ks, lane);
      fq_issue(f.a[2 * r - 7], region(s, 0, ks), wr * 128 + (2 * r - 7) * 16, ks, lane);
    }
  };
  f32x4 acc[8][8];
  FragsQ<AL, BL> F0, F1;

  // prologue: tiles 0, 1 in stages 0, 1; F0 <- ks0(0); then the ks0 region of stage 0 is free
  dma_region(0, 0, 0);
  dma_region(0, 1, 0);
  dma_region(1, 0, 1);
  dma_region(1, 1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int r = 0; r < 8; ++r) fread_row(0, 0, r, F0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  F0.tie();
  __builtin_amdgcn_s_barrier();

  auto half0 = [&](auto first_c, int kt) {
    constexpr bool FIRST = decltype(first_c)::value;
    const int s = kt & 1;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      fread_row(s, 1, r, F1);
      if (r & 1) dma_region_piece2(kt + 2, 0, s, r >> 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (FIRST) mfma4_zero(acc[r][j], F0.b[j].get(), F0.a[r].get());
        else mfma4_acc(acc[r][j], F0.b[j].get(), F0.a[r].get());
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // ks0(kt+1) landed; ks1(kt+1), ks0(kt+2) may fly
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    F1.tie();
    __builtin_amdgcn_s_barrier();
  };
  auto half1 = [&](int kt) {
    const int s = kt & 1;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      fread_row(s ^ 1, 0, r, F0);
      if (r & 1) dma_region_piece2(kt + 2, 1, s, r >> 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) mfma4_acc(acc[r][j], F1.b[j].get(), F1.a[r].get());
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // ks1(kt+1) landed; ks0(kt+2), ks1(kt+2) may fly
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    F0.tie();
    __builtin_amdgcn_s_barrier();
  };

  half0(std::true_type{}, 0);
  half1(0);
  for (int kt = 1; kt < nk; ++kt) {
    half0(std::false_type{}, kt);
    half1(kt);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_nop 15\n\ts_nop 7" : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]),
               "+a"(acc[7][4]), "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]));
  __builtin_amdgcn_s_barrier();
  epilogue4<CT>(p, acc, smem, m0, n0, wr, wc, t, lane);
}

template <int AL, int BL, int CT>
int launch4w(GemmArgs p, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm4w_k<AL, BL, CT>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM4);
    attr_set = true;
  }
  p.tiles_m = (int)cdiv(p.M, T4);
  p.tiles_n = (int)cdiv(p.N, T4);
  p.sk_dp = p.tiles_m * p.tiles_n;
  gemm4w_k<AL, BL, CT><<<(unsigned)p.sk_dp, 256, SMEM4, s>>>(p);
  return cullavo_check_launch("gemm4w");
}

}  // namespace

// 4-wave kernel (tile mode 4): a_layout/b_layout any of (0,0), (0,1), (1,1), (1,0); a layout-0
// operand needs K % 64 == 0 and the LDS-staged epilogue's alignment (p.epi_lds); the caller checks
bool cvgemm_4w_eligible(const cvgemm::GemmArgs& p, int a_layout, int b_layout) {
  return p.epi_lds && p.part == nullptr && p.lora_u == nullptr && p.drop_mode == 0 &&
         (a_layout == 1 || p.K % cvgemm::BK == 0) && (b_layout == 1 || p.K % cvgemm::BK == 0) && p.K > 0;
}

int cvgemm_launch_4w(const cvgemm::GemmArgs& p, int a_layout, int b_layout, bool f32, hipStream_t s) {
#define L4W(AL, BL) return f32 ? launch4w<AL, BL, CULLAVO_DT_F32>(p, s) : launch4w<AL, BL, CULLAVO_DT_BF16>(p, s);
  if (a_layout == 0 && b_layout == 0) { L4W(0, 0) }
  if (a_layout == 0 && b_layout == 1) { L4W(0, 1) }
  if (a_layout == 1 && b_layout == 0) { L4W(1, 0) }
  L4W(1, 1)
#undef L4W
}
