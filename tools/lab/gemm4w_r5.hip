// LAB KERNEL (round 5; not in the product library): measured equal to or slower than the 8-wave
// production kernels on every 7B step shape (profiles/r05/gemm/gemm4w_lab.txt), so it lives here
// with its ablations; built by tools/lab/gemm4w_lab.hip. A stream-K variant (G persistent blocks
// sharing the K-iterations of the last round, write-through f32 partials, last arriver adds) ran
// 9-22 % slower and is in git history only.
//
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
#include "../../causal-unified-language-vision_amd/csrc/gemm_common.h"

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

// epilogue: per row half h, waves (h, 0) and (h, 1) write their f32 block into a [128][256]
// image (16-B chunk c of row r at c ^ (r & 15)), then all 256 threads take 8 columns each and
// either run the store8 chain (after adding the f32 partial tile part_in, row-major [256][256],
// when given) or, with part_out, store the f32 values row-major write-through (stream-K pieces)
template <int CT>
DEV void epilogue4(const GemmArgs& p, f32x4 (&acc)[8][8], char* smem, int64_t m0, int64_t n0, int wr, int wc, int t,
                   int lane, float* part_out = nullptr, const float* part_in = nullptr) {
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)part_out, (short)0, T4 * T4 * 4, 0x00020000);
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
      f32x4 lo = sw ? x1 : x0, hi = sw ? x0 : x1;
      const int off = (h * 128 + r) * T4 + pr * 8;  // element offset in the row-major partial tile
      if (part_out != nullptr) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, lo), rp, (unsigned)(off * 4), 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, hi), rp, (unsigned)(off * 4 + 16), 0, 16);
        continue;
      }
      if (part_in != nullptr) {
        lo += *reinterpret_cast<const f32x4*>(part_in + off);
        hi += *reinterpret_cast<const f32x4*>(part_in + off + 4);
      }
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] = lo[j]; v[4 + j] = hi[j]; }
      store8<CT>(p, v, m0 + h * 128 + r, n0 + pr * 8);
    }
    __syncthreads();
  }
}

// ABL: lab ablations only (tools/lab/gemm4w_lab.hip; results wrong): 256 no epilogue, 512 one K-tile;
// bit 0 = no in-loop global
// loads, 1 = no in-loop LDS writes, 2 = no barrier, 3 = no in-loop fragment reads, 4 = every
// global load in half 0 right after its register's LDS write, 5 = one global load per row group
// (A in half 0, B in half 1; both results right), 6 = loads kept but the LDS writes take other
// registers (no wait on a load in the loop), 7 = LDS-DMA staging instead of registers (tile kt+2
// DMA'd into stage kt & 1 under half 1 of K-tile kt, waited before the mid-barrier of kt+1)
// K-tiles [kb, ke) of the tile at (m0, n0) into acc (the whole pipeline: prologue, ke - kb
// K-tiles, the AGPR drain and a barrier after which LDS is free)
template <int AL, int BL, int ABL>
DEV void mainloop4(const GemmArgs& p, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int64_t m0, int64_t n0,
                   int kb, int ke, char* smem, f32x4 (&acc)[8][8]) {
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const Stage<AL> ga = stage_geom<AL>(p.lda, m0, p.M, t);
  const Stage<BL> gb = stage_geom<BL>(p.ldb, n0, p.N, t);
  if constexpr ((ABL & 512) != 0) ke = kb + 1;  // lab 512: one K-tile (prologue + epilogue cost)

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

  Frags4 F0, F1;

  // prologue: tile kb -> stage 0, tile kb+1 into the registers, ks0 fragments of tile kb
  if constexpr (DMA) {
    dma(kb, smem, 0, 16);
    dma(kb + 1, smem + STAGE4, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  gload(kb, 0, 16);
#pragma unroll
  for (int i = 0; i < 16; ++i) swrite1(smem, i);
  gload(kb + 1, 0, 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int r = 0; r < 8; ++r) fread_row(smem, 0, r, F0);

  // half 0 of K-tile kt: MFMAs on F0 (ks0 of kt); under them F1 <- ks1 of kt, tile kt+1's LDS
  // writes (registers -> other stage) and tile kt+2's first 8 global loads (stage: (kt - kb) & 1)
  auto half0 = [&](auto first_c, int kt) {
    constexpr bool FIRST = decltype(first_c)::value;
    const char* cur = smem + ((kt - kb) & 1) * STAGE4;
    char* nxt = smem + ((kt - kb + 1) & 1) * STAGE4;
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
    const char* nxt = smem + ((kt - kb + 1) & 1) * STAGE4;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      fread_row(nxt, 0, r, F0);
#pragma unroll
      for (int j = 0; j < 8; ++j) mfma4_acc(acc[r][j], F1.b[j], F1.a[r]);
      if constexpr (DMA) dma(kt + 2, smem + ((kt - kb) & 1) * STAGE4, 2 * r, 2 * r + 2);
      else if constexpr ((ABL & 32) != 0) gload(kt + 2, 8 + r, 9 + r);
      else if ((ABL & 16) == 0 && r < 4) gload(kt + 2, 8 + 2 * r, 10 + 2 * r);  // B loads 8..15
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  half0(std::true_type{}, kb);
  half1(kb);
  for (int kt = kb + 1; kt < ke; ++kt) {
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
}

DEV __amdgpu_buffer_rsrc_t rsrc_a(const GemmArgs& p, int al) {
  return make_rsrc(p.A, al == 0 ? ((p.M - 1) * p.lda + p.K) * 2 : ((p.K - 1) * p.lda + p.M) * 2);
}
DEV __amdgpu_buffer_rsrc_t rsrc_b(const GemmArgs& p, int bl) {
  return make_rsrc(p.B, bl == 0 ? ((p.N - 1) * p.ldb + p.K) * 2 : ((p.K - 1) * p.ldb + p.N) * 2);
}

// one block per tile
template <int AL, int BL, int CT, int ABL = 0>
__global__ __launch_bounds__(256, 1) void gemm4w_k(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lid = xcd_remap(blockIdx.x, p.sk_dp);
  int64_t m0, n0;
  tile_origin<T4, T4>(p, lid, m0, n0);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  f32x4 acc[8][8];
  mainloop4<AL, BL, ABL>(p, rsrc_a(p, AL), rsrc_b(p, BL), m0, n0, 0, (int)cdiv(p.K, BK), smem, acc);
  if constexpr ((ABL & 256) != 0) return;  // lab: no epilogue (the MFMAs are volatile asm)
  epilogue4<CT>(p, acc, smem, m0, n0, wave >> 1, wave & 1, t, lane);
}

template <int AL, int BL, int CT>
int launch4w(GemmArgs p, hipStream_t s) {
  p.tiles_m = (int)cdiv(p.M, T4);
  p.tiles_n = (int)cdiv(p.N, T4);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm4w_k<AL, BL, CT>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM4);
    attr_set = true;
  }
  p.sk_dp = p.tiles_m * p.tiles_n;
  gemm4w_k<AL, BL, CT><<<(unsigned)p.sk_dp, 256, SMEM4, s>>>(p);
  return cullavo_check_launch("gemm4w");
}

}  // namespace

// 4-wave kernel (lab tile mode 4): a_layout/b_layout any of (0,0), (0,1), (1,1), (1,0); a layout-0
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
