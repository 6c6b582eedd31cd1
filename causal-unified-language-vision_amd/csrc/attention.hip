// Flash attention forward/backward for gfx950 (v_mfma_f32_32x32x16_bf16).
//
// Replaces the LM's causal attention (FA2 in the reference: cullavo/load_cullavo.py:72;
// arithmetic of tf:llama/modeling_llama.py:191-214, scale 1/sqrt(128)) and CLIP's non-causal
// attention (tf:clip/modeling_clip.py:280-336, scale 1/8). Tensors are [B, L, H, D] with a
// token stride, i.e. the q/k/v projection outputs are consumed in place.
//
// Forward: a wave owns 32 query rows; the 4 waves of a workgroup share 64-key K/V tiles in
// LDS (double-buffered, register-staged, one barrier per tile). Scores are computed swapped,
// S^T = K Q^T, so every lane owns one query row: the online-softmax row max/sum is 32 register
// ops plus one cross-half shuffle, P^T feeds the P·V MFMA straight from the accumulator
// registers (O^T = V^T P^T) and V^T fragments come from ds_read_b64_tr_b16 transposed reads.
// Backward: kernel A (per 32-key slice per wave: dV = P^T dO, dK = dS^T Q) and kernel B (per
// 32-query slice: dQ = dS K), both recomputing P from the saved log-sum-exp; no atomics, so
// results are bitwise reproducible.
#include "common.h"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 frag8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr float kLog2e = 1.4426950408889634f;

// bijective XCD-aware block remap (as in gemm.hip; cdna_hip_programming.md §5)
DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}
constexpr float kLn2 = 0.6931471805599453f;
constexpr int kVmcnt0 = 0x0F70;  // s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15) (gfx9 encoding)

// bare v_exp_f32: results below 2^-126 flush to zero (softmax weights that small are noise);
// exp2f adds a denormal range fix-up (compare, select, ldexp) around every call
DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// LDS image of a [rows][D] bf16 tile, 16-byte chunk ch of row r. D=128: the dual-use XOR
// image (conflict-free for both the row reads and the tr16 reads, cdna_hip_programming.md
// T10 (b)); D=64: chunk ^ ((r>>1)&7) (row reads conflict-free, tr reads 2-way).
template <int D>
DEV int kv_off(int r, int ch) {
  if (D == 128) return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
  return 128 * r + 16 * (ch ^ ((r >> 1) & 7));
}

// row fragment for a 32x32x16 operand: lane holds T[rbase + (lane&31)][16s + 8h + j]
template <int D>
DEV frag8 row_frag(const char* lds, int rbase, int s, int lane) {
  const int r = rbase + (lane & 31), ch = 2 * s + (lane >> 5);
  return __builtin_bit_cast(frag8, *reinterpret_cast<const u16x8*>(lds + kv_off<D>(r, ch)));
}

// transposed fragment: lane holds T[kb + 8(j>>2) + 4h + (j&3)][d0 + (lane&31)], j = 0..7
// (the k order of an accumulator tile used as the other MFMA operand, guide §3)
template <int D>
DEV frag8 tr_frag(const char* lds, int kb, int d0, int lane) {
  const int h = lane >> 5, i = lane & 15, q = i >> 2, p = i & 3;
  const int dcol = d0 + 16 * ((lane >> 4) & 1);
  const int ch = (dcol >> 3) + (p >> 1);
  const int r0 = kb + 4 * h + q;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + kv_off<D>(r0, ch) + 8 * (p & 1)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + kv_off<D>(r0 + 8, ch) + 8 * (p & 1)));
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(frag8, v);
}

// fragment reads at precomputed LDS addresses (see attn_fwd_k): a row fragment, and a
// transposed fragment from its two ds_read_b64_tr_b16 halves (tr_frag's lo / hi)
// (LDS byte addresses as integers, so a read is one VGPR plus its immediate offset)
typedef __attribute__((address_space(3))) u16x8 lds_u16x8;
DEV unsigned lds_addr(const char* p) { return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p; }
DEV frag8 lds_frag(unsigned a) { return __builtin_bit_cast(frag8, *(const lds_u16x8*)(uintptr_t)a); }
DEV frag8 lds_tr_frag(unsigned lo_a, unsigned hi_a) {
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)lo_a);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)hi_a);
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(frag8, v);
}

// accumulator registers 8s..8s+7 of a 32x32 tile -> bf16 operand fragment
DEV frag8 pack_frag(const f32x16& a, int s) {
  frag8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)a[8 * s + j];
  return f;
}

// Forward tile rows are read with 16-B buffer loads whose range check zero-fills rows past nrows
// (one select per chunk instead of a branch around every load; ~13 % fewer VALU instructions in
// the forward loop, 5-7 % faster forward on the MI355X, tools/attn_bench.py ATTN_STAGE_AB). The buffer covers one (batch, head) slice of the tensor, so
// its byte offsets fit 32 bits unless nrows * ld is very large; then the pointer path runs.
constexpr unsigned kOOB = 0x7FFFFFF0u;

__device__ float g_rescale_thr = 8.f;  // forward's deferred-rescale threshold (cullavo_attn_set_rescale)
// forward staging (cullavo_attn_set_stage): 0 = pointer loads behind a bounds branch, 1 = per-chunk
// range-checked buffer loads, 2 = per-tile descriptor (StageT), 3 = 2 + s_setprio, 4 = LDS-DMA
// (StageDMA, the default since round 3: 138.3 -> 132.0 us on the 7B layer, 153.3 -> 141.9 us on
// the ViT bs-64 layer, alternating on one MI355X, profiles/r03/s3a/attn_bench.txt), 5 = 4 with
// inline-asm fragment groups (131.7 / 141.1 us: within noise of 4, kept as an A/B), 7 = the
// software-pipelined kernel attn_fwd_pipe_k (round 4); -1 (default) = 7 (with its widened O
// stores: 7B layer 151 -> 124-128 us, ViT bs-64 layer 148-154 -> 139-144 us alternating on one
// box, profiles/r04/attn/attn_fwd_ab.txt)
int g_fwd_stage = -1;
// backward staging (cullavo_attn_set_bwd_stage): bit 0 = dK/dV Q / dO by LDS-DMA, bit 1 = the
// dQ-from-dS kernel's K / dS^T by LDS-DMA (else registers, StageT), bit 2 = the 4-stage LDS-DMA
// ring dQ kernel attn_bwd_dq_ring_k (D = 128; round 6, takes precedence over bit 1), bit 3 = the
// blocked dS^T layout (ds_layout). Round 5: with bit 0 the dK/dV kernel reads every fragment by
// inline asm one step ahead of its MFMAs (no vmcnt(0) in front of the reads, the dS^T stores left
// in flight at the tile's end): 7B layer backward 467.5 -> 449.7 us, bitwise equal
// (profiles/r05/attn/attn_bwd_stage_ab.txt), so bit 0 is the default.
//
// ds_layout: the mode-7 dS^T workspace [B H][LkP][LqP] bf16 is stored either row-major (key rows of
// LqP queries: a dQ tile of 64 keys x 128 queries is 64 runs of 256 B, 2 LqP bytes apart) or
// blocked by 128-query column blocks ([B H][LqP / 128][LkP][128]: the same tile is one contiguous
// 16 KiB run). Same bytes, same values; the address is bh st_bh + (q / 128) st_blk + key ldst + q % 128
int g_bwd_stage = 1;

DEV bool buf_ok(int64_t ld, int nrows, int D) { return ((int64_t)nrows * ld + D) * 2 < (int64_t)kOOB; }

DEV __amdgpu_buffer_rsrc_t tile_rsrc(const u16* base, int64_t ld, int nrows, int D) {
  const int64_t bytes = nrows > 0 ? ((int64_t)(nrows - 1) * ld + D) * 2 : 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

DEV u16x8 buf_row_load(__amdgpu_buffer_rsrc_t rs, int64_t ld, int row0, int nrows, int row, int ch) {
  const int gr = row0 + row;
  const unsigned off = gr < nrows ? (unsigned)(gr * (unsigned)ld + ch * 8) * 2u : kOOB;
  return __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}

// global -> registers -> LDS staging of a [ROWS][D] tile of a [L, H, D]-strided tensor
// BUF: buffer loads (attn_fwd_k; measured neutral to slightly slower in the backward kernels)
template <int ROWS, int D, bool BUF = false>
struct Stage {
  static constexpr int kChunks = ROWS * D / 8;
  static constexpr int kPer = kChunks / 256;  // 16-byte chunks per thread
  u16x8 r[kPer];
  DEV void load(const u16* base, int64_t ld, int row0, int nrows) {
    if (BUF && buf_ok(ld, nrows, D)) {
      const __amdgpu_buffer_rsrc_t rs = tile_rsrc(base, ld, nrows, D);
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int q = threadIdx.x + 256 * i;
        r[i] = buf_row_load(rs, ld, row0, nrows, q / (D / 8), q % (D / 8));
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = threadIdx.x + 256 * i;
      const int row = q / (D / 8), ch = q % (D / 8);
      r[i] = (row0 + row < nrows) ? *reinterpret_cast<const u16x8*>(base + (int64_t)(row0 + row) * ld + ch * 8)
                                  : u16x8(0);
    }
  }
  DEV void store(char* lds) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = threadIdx.x + 256 * i;
      const int row = q / (D / 8), ch = q % (D / 8);
      *reinterpret_cast<u16x8*>(lds + kv_off<D>(row, ch)) = r[i];
    }
  }
};

// Per-tile descriptor staging (the forward's default, STAGE 2): the buffer descriptor is rebuilt
// per tile from scalars (base advanced to the tile's first row, num_records covering only the
// rows that exist, so rows past the sequence end read as zeros), every lane keeps ONE
// loop-invariant byte offset, and the i-th chunk's row step (i * rows-per-pass * ld) is the
// instruction's scalar offset: no per-tile VALU address arithmetic, compares or selects (the
// per-chunk form kept 16 v_mul_lo_u32 + range selects in the loop and spilled 62 VGPRs).
template <int ROWS, int D, int NT = 256>
struct StageT {
  static constexpr int kPer = ROWS * D / 8 / NT;  // 16-byte chunks per thread
  static constexpr int kPass = NT / (D / 8);      // rows covered by one pass of NT threads
  static_assert(kPer * NT * 8 == ROWS * D && NT % (D / 8) == 0, "tile must split evenly over the threads");
  u16x8 r[kPer];
  DEV static unsigned lane_off(int64_t ld) {
    return (unsigned)(((int64_t)(threadIdx.x / (D / 8)) * ld + (threadIdx.x % (D / 8)) * 8) * 2);
  }
  DEV void load(const u16* base, int64_t ld, int row0, int nrows, unsigned vo) {
    const int left = min(nrows - row0, ROWS);
    const int bytes = left > 0 ? (int)(((int64_t)(left - 1) * ld + D) * 2) : 0;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)row0 * ld), (short)0, bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < kPer; ++i)
      r[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (int)(i * kPass * ld * 2), 0));
  }
  DEV void store(char* lds) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = threadIdx.x + NT * i;
      *reinterpret_cast<u16x8*>(lds + kv_off<D>(q / (D / 8), q % (D / 8))) = r[i];
    }
  }
};

// LDS-DMA staging of a [ROWS][D] tile (the forward's STAGE 4): buffer_load ... lds writes each
// 1 KiB piece lane-linearly (lane i -> byte 16 i of the piece), so the kv_off XOR image is
// produced by permuting the SOURCE chunk: the lane landing in slot s of image row r loads chunk
// s ^ swizzle(r) (the swizzle is an involution). No staging VGPRs and no ds_write: the data goes
// HBM/L2 -> LDS directly. Pieces are dealt round-robin over NW waves; the per-lane offsets are
// loop-invariant (rows relative to the tile origin, which the per-tile descriptor carries, as in
// StageT: rows past the sequence end fall outside num_records and land as zeros).
typedef __attribute__((address_space(3))) void lds_void_t;
// (a free function: the builtin inside a member function made the host pass drop the kernel
// stubs of every instantiation using it, silently -- undefined symbols at load)
DEV void lds_dma16(__amdgpu_buffer_rsrc_t rs, char* lds, unsigned vo) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds, 16, vo, 0, 0, 0);
}
template <int ROWS, int D, int NW>
struct StageDMA {
  static constexpr int kRP = 1024 / (2 * D);            // image rows per 1 KiB piece
  static constexpr int kPieces = ROWS / kRP;
  static constexpr int kPer = kPieces / NW;             // pieces per wave
  static_assert(kPer * NW == kPieces, "pieces must split evenly over the waves");
  unsigned vo[kPer];
  DEV void prep(int64_t ld, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int pc = wave + NW * i;
      const int r = pc * kRP + lane / (D / 8), s = lane % (D / 8);
      const int sw = D == 128 ? (((r & 3) << 2) | ((r >> 2) & 3)) : ((r >> 1) & 7);
      vo[i] = (unsigned)(((int64_t)r * ld + (s ^ sw) * 8) * 2);
    }
  }
  DEV void issue(const u16* base, int64_t ld, int row0, int nrows, char* lds, int wave) const {
    const int left = min(nrows - row0, ROWS);
    const int bytes = left > 0 ? (int)(((int64_t)(left - 1) * ld + D) * 2) : 0;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)row0 * ld), (short)0, bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < kPer; ++i)
      lds_dma16(rs, lds + (wave + NW * i) * 1024, vo[i]);
  }
};

// StageDMA with one per-lane offset: piece i sits NW * kRP rows (a multiple of 16) below piece 0,
// where the image swizzle (a function of row & 15) repeats, so its source offset is piece 0's
// plus a wave-uniform row step, passed as the instruction's scalar offset (inside the buffer's
// range check like the per-lane part; tests/test_oob_guard.py)
DEV void lds_dma16s(__amdgpu_buffer_rsrc_t rs, char* lds, unsigned vo, int so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds, 16, vo, so, 0, 0);
}
template <int ROWS, int D, int NW>
struct StageDMA1 {
  static constexpr int kRP = 1024 / (2 * D);
  static constexpr int kPer = ROWS / kRP / NW;
  static_assert(kPer * NW * kRP == ROWS && (NW * kRP) % 16 == 0, "pieces must split evenly, 16-row steps");
  unsigned vo;
  DEV void prep(int64_t ld, int wave, int lane) {
    const int r = wave * kRP + lane / (D / 8), s = lane % (D / 8);
    const int sw = D == 128 ? (((r & 3) << 2) | ((r >> 2) & 3)) : ((r >> 1) & 7);
    vo = (unsigned)(((int64_t)r * ld + (s ^ sw) * 8) * 2);
  }
  DEV void issue(const u16* base, int64_t ld, int row0, int nrows, char* lds, int wave) const {
    const int left = min(nrows - row0, ROWS);
    const int bytes = left > 0 ? (int)(((int64_t)(left - 1) * ld + D) * 2) : 0;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)row0 * ld), (short)0, bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < kPer; ++i) lds_dma16s(rs, lds + (wave + NW * i) * 1024, vo, (int)(i * NW * kRP * ld * 2));
  }
};

// row of accumulator register r of a 32x32 tile for lane half h
DEV int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// a transposed fragment from its two ds_read_b64_tr_b16 halves
DEV frag8 tr_join(const s16x4& lo, const s16x4& hi) {
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(frag8, v);
}

// four row fragments by inline-asm ds_read_b128 / four transposed halves by ds_read_b64_tr_b16
// (issued together), and the counted lgkmcnt wait that ties a group's registers before use
DEV void rd4(s16x8& a, s16x8& b, s16x8& c, s16x8& d, unsigned pa, unsigned pb, unsigned pc, unsigned pd) {
  asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7"
               : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
               : "v"(pa), "v"(pb), "v"(pc), "v"(pd)
               : "memory");
}
template <int CNT>
DEV void tie4(s16x8& a, s16x8& b, s16x8& c, s16x8& d) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(CNT) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
DEV void rd4t(s16x4& a, s16x4& b, s16x4& c, s16x4& d, unsigned pa, unsigned pb, unsigned pc, unsigned pd) {
  asm volatile("ds_read_b64_tr_b16 %0, %4\n\tds_read_b64_tr_b16 %1, %5\n\tds_read_b64_tr_b16 %2, %6\n\t"
               "ds_read_b64_tr_b16 %3, %7"
               : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
               : "v"(pa), "v"(pb), "v"(pc), "v"(pd)
               : "memory");
}
template <int CNT>
DEV void tie4t(s16x4& a, s16x4& b, s16x4& c, s16x4& d) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(CNT) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Forward STAGE 5: the P V^T product's V^T fragments through inline-asm ds_read_b64_tr_b16 (one
// group = the ND fragments of one 16-key slice, VB the slice's LDS byte offset as an immediate),
// tied by a counted lgkmcnt wait (CNT = reads allowed to stay in flight: the next group's)
template <int ND, unsigned VB>
DEV void tr_group_issue(s16x4 (&lo)[ND], s16x4 (&hi)[ND], const unsigned (&toff)[ND][2]) {
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
    asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%4\n\tds_read_b64_tr_b16 %1, %3 offset:%4"
                 : "=&v"(lo[dt]), "=&v"(hi[dt])
                 : "v"(toff[dt][0]), "v"(toff[dt][1]), "n"(VB)
                 : "memory");
}
template <int ND, int CNT>
DEV void tr_group_tie(s16x4 (&lo)[ND], s16x4 (&hi)[ND]) {
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(lo[dt]), "+v"(hi[dt]) : "n"(CNT) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// Forward STAGE 5, S = K Q^T: 4 K row fragments (k-steps S0..S0+3 at LDS byte offset OFF from
// each lane's roff) by inline-asm ds_read_b128, tied by a counted lgkmcnt wait
template <int NS, int S0, unsigned OFF>
DEV void k_group_issue(s16x8 (&kf)[4], const unsigned (&roff)[NS]) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=&v"(kf[j]) : "v"(roff[S0 + j]), "n"(OFF) : "memory");
}
template <int CNT>
DEV void k_group_tie(s16x8 (&kf)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3]) : "n"(CNT) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int NS, int S0>
DEV void k_group_mfma(const s16x8 (&kf)[4], const frag8 (&qf)[NS], f32x16& acc) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(frag8, kf[j]), qf[S0 + j], acc, 0, 0, 0);
}
template <int ND>
DEV void tr_group_mfma(const s16x4 (&lo)[ND], const s16x4 (&hi)[ND], const frag8& pf, f32x16 (&o)[ND]) {
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
    const s16x8 v = __builtin_shufflevector(lo[dt], hi[dt], 0, 1, 2, 3, 4, 5, 6, 7);
    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(frag8, v), pf, o[dt], 0, 0, 0);
  }
}

// two V^T fragments (column blocks DT0, DT0 + 1 of a 16-key slice at LDS offset VB) by inline asm,
// tied by a counted lgkmcnt wait: the pipelined forward's P V reads in pairs (fewer registers in
// flight than a whole slice: register pressure made the compiler spill in-flight fragments)
template <int ND, unsigned VB, int DT0>
DEV void tr2_issue(s16x4 (&lo)[2], s16x4 (&hi)[2], const unsigned (&toff)[ND][2]) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
    asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%4\n\tds_read_b64_tr_b16 %1, %3 offset:%4"
                 : "=&v"(lo[j]), "=&v"(hi[j])
                 : "v"(toff[DT0 + j][0]), "v"(toff[DT0 + j][1]), "n"(VB)
                 : "memory");
}
template <int CNT>
DEV void tr2_tie(s16x4 (&lo)[2], s16x4 (&hi)[2]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(lo[0]), "+v"(hi[0]), "+v"(lo[1]), "+v"(hi[1]) : "n"(CNT) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int ND, int DT0>
DEV void tr2_mfma(const s16x4 (&lo)[2], const s16x4 (&hi)[2], const frag8& pf, f32x16 (&o)[ND]) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const s16x8 v = __builtin_shufflevector(lo[j], hi[j], 0, 1, 2, 3, 4, 5, 6, 7);
    o[DT0 + j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(frag8, v), pf, o[DT0 + j], 0, 0, 0);
  }
}

// ============================================================================================
// forward
// ============================================================================================
template <int D, bool CAUSAL, int STAGE, int PRIO = 0>
__global__ __launch_bounds__(256, 2) void attn_fwd_k(const u16* __restrict__ Q, int64_t ldq,
                                                     const u16* __restrict__ K, int64_t ldk,
                                                     const u16* __restrict__ V, int64_t ldv,
                                                     u16* __restrict__ O, int64_t ldo,
                                                     float* __restrict__ LSE, int H, int Lq, int Lk,
                                                     float scale, const int32_t* __restrict__ kv_start) {
  constexpr int KT = 64;                 // keys per tile
  constexpr int TILE = KT * D * 2;       // bytes per K (or V) tile
  constexpr int NS = D / 16;             // k-steps over D
  constexpr int ND = D / 32;             // O^T tiles
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // 1-D grid of (query block, head, batch), XCD-remapped: the query blocks of one (b, h) run
  // on one XCD and share its K/V tiles in L2; heavy causal blocks first within a group
  const int nqb = (Lq + 127) / 128;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qi = lid % nqb, hb = lid / nqb;
  const int qb = CAUSAL ? (nqb - 1 - qi) : qi;
  const int h = hb % H, b = hb / H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hf = lane >> 5;
  const int q = qb * 128 + wave * 32 + (lane & 31);
  const int kstart = kv_start ? kv_start[b] : 0;

  const u16* Qb = Q + (int64_t)b * Lq * ldq + (int64_t)h * D;
  const u16* Kb = K + (int64_t)b * Lk * ldk + (int64_t)h * D;
  const u16* Vb = V + (int64_t)b * Lk * ldv + (int64_t)h * D;

  frag8 qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    u16x8 v = (q < Lq) ? *reinterpret_cast<const u16x8*>(Qb + (int64_t)q * ldq + 16 * s + 8 * hf) : u16x8(0);
    qf[s] = __builtin_bit_cast(frag8, v);
  }

  f32x16 o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) o[i] = f32x16(0.f);
  float m = -INFINITY, l = 0.f;
  const float c = scale * kLog2e;
  const float rescale_thr = g_rescale_thr;

  // live keys of this lane's query: [kstart, khi)
  const int khi = CAUSAL ? min(Lk, q + 1) : Lk;
  const unsigned kspan = (unsigned)max(khi - kstart, 0);
  int kend = Lk;
  if (CAUSAL) kend = min(Lk, qb * 128 + 128);
  const int ntiles = (kend + KT - 1) / KT;
  const int t0 = kstart / KT;

  using St = std::conditional_t<STAGE == 2 || STAGE >= 4, StageT<KT, D>, Stage<KT, D, STAGE == 1>>;
  St sk, sv;
  unsigned vok = 0, vov = 0;
  if constexpr (STAGE == 2) {
    vok = StageT<KT, D>::lane_off(ldk);
    vov = StageT<KT, D>::lane_off(ldv);
  }
  StageDMA<KT, D, 4> dk_, dv_;
  if constexpr (STAGE >= 4) {
    dk_.prep(ldk, __builtin_amdgcn_readfirstlane(wave), lane);
    dv_.prep(ldv, __builtin_amdgcn_readfirstlane(wave), lane);
  }
  // STAGE 4: K and V of the tile at row0 straight into LDS buffer pair i
  auto dma_kv = [&](int row0, int i) {
    const int w = __builtin_amdgcn_readfirstlane(wave);
    dk_.issue(Kb, ldk, row0, Lk, smem + 2 * i * TILE, w);
    dv_.issue(Vb, ldv, row0, Lk, smem + 2 * i * TILE + TILE, w);
  };
  auto load_kv = [&](int row0) {
    if constexpr (STAGE == 2 || STAGE >= 4) {
      sk.load(Kb, ldk, row0, Lk, vok);
      sv.load(Vb, ldv, row0, Lk, vov);
    } else {
      sk.load(Kb, ldk, row0, Lk);
      sv.load(Vb, ldv, row0, Lk);
    }
  };
  // buffer i: K at smem + 2*i*TILE, V right after it
#define bufK(i) (smem + 2 * (i) * TILE)
#define bufV(i) (smem + 2 * (i) * TILE + TILE)
  if (t0 < ntiles) {
    if constexpr (STAGE == 6) {
      dma_kv(t0 * KT, 0);
      dma_kv(t0 * KT, 1);
    } else if constexpr (STAGE >= 4) {
      dma_kv(t0 * KT, 0);
    } else {
      load_kv(t0 * KT);
      sk.store(bufK(0));
      sv.store(bufV(0));
    }
  }
  // vmcnt(0) the compiler can see on every path: the Q fragments are then known to have
  // landed inside the loop, so the in-loop prefetch of the next K/V tile is not waited for
  // before the first MFMA (hipcc otherwise emits vmcnt(0) there: the prefetch is conditional)
  __builtin_amdgcn_s_waitcnt(kVmcnt0);
  __syncthreads();

  // Per-lane LDS offsets of every fragment read, hoisted out of the tile loop: the swizzle of
  // kv_off depends on row & 15 only, so a fragment at row base kb (kb % 16 == 0) sits at the
  // kb = 0 offset plus 2*D*kb (a constant): each read costs one add to the buffer base instead
  // of recomputing the swizzled address.
  // They are absolute LDS addresses in buffer pair 0; the loop body is instantiated once per
  // buffer pair (CUR = 0 / 1, two tiles per trip), so the pair offset 2*CUR*TILE and every
  // fragment's row base are compile-time immediates of the ds_read (no per-tile address adds).
  const unsigned sbase = lds_addr(smem);
  unsigned roff[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) roff[s] = sbase + kv_off<D>(lane & 31, 2 * s + hf);
  unsigned toff[ND][2];
  {
    const int i = lane & 15, qq = i >> 2, p = i & 3;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int ch = ((dt * 32 + 16 * ((lane >> 4) & 1)) >> 3) + (p >> 1);
      toff[dt][0] = sbase + TILE + kv_off<D>(4 * hf + qq, ch) + 8 * (p & 1);
      toff[dt][1] = sbase + TILE + kv_off<D>(4 * hf + qq + 8, ch) + 8 * (p & 1);
    }
  }
  const f32x2 c2 = {c, c};
  auto tile = [&](auto cur_c, int t) {
    constexpr int CUR = decltype(cur_c)::value;
    constexpr unsigned PAIR = 2u * CUR * TILE;
    const bool more = t + 1 < ntiles;
    if constexpr (STAGE == 6) {
      // lab only (cullavo_attn_set_stage(6), WRONG results): no K/V loads after the first tile,
      // every tile computes on the first tile's LDS -- the forward's time without its memory waits
    } else if constexpr (STAGE >= 4) {
      if (more) dma_kv((t + 1) * KT, CUR ^ 1);  // pair CUR^1 was last read before the previous barrier
    } else {
      if (more) load_kv((t + 1) * KT);
    }
    // PRIO (A/B, cullavo_attn_set_stage(3)): the two MFMA blocks at raised wave priority, so the
    // SIMD's other wave (in its softmax) yields the issue slot to the MFMAs (guide T5)
    if constexpr (PRIO) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // S^T = K Q^T for two 32-key halves
    f32x16 st[2];
    if constexpr (STAGE == 5) {
      // K fragments by inline-asm ds_read_b128 in groups of 4, the next group in flight while
      // the current one's MFMAs issue (hipcc otherwise reads each fragment into one register
      // quad right before its MFMA, exposing the LDS latency 16 times per tile)
      st[0] = f32x16(0.f);
      st[1] = f32x16(0.f);
      s16x8 ka[4], kb[4];
      if constexpr (NS == 8) {
        k_group_issue<NS, 0, PAIR>(ka, roff);
        k_group_issue<NS, 4, PAIR>(kb, roff);
        k_group_tie<4>(ka);
        k_group_mfma<NS, 0>(ka, qf, st[0]);
        k_group_issue<NS, 0, PAIR + 32 * 2 * D>(ka, roff);
        k_group_tie<4>(kb);
        k_group_mfma<NS, 4>(kb, qf, st[0]);
        k_group_issue<NS, 4, PAIR + 32 * 2 * D>(kb, roff);
        k_group_tie<4>(ka);
        k_group_mfma<NS, 0>(ka, qf, st[1]);
        k_group_tie<0>(kb);
        k_group_mfma<NS, 4>(kb, qf, st[1]);
      } else {
        k_group_issue<NS, 0, PAIR>(ka, roff);
        k_group_issue<NS, 0, PAIR + 32 * 2 * D>(kb, roff);
        k_group_tie<4>(ka);
        k_group_mfma<NS, 0>(ka, qf, st[0]);
        k_group_tie<0>(kb);
        k_group_mfma<NS, 0>(kb, qf, st[1]);
      }
    } else {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      st[kt] = f32x16(0.f);
#pragma unroll
      for (int s = 0; s < NS; ++s)
        st[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_frag(roff[s] + PAIR + kt * 32 * 2 * D), qf[s], st[kt], 0, 0, 0);
    }
    }
    if constexpr (PRIO) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // mask (boundary tiles only, branch-free), tile max on the raw scores (c > 0)
    const int kbase = t * KT;
    const bool need_mask = (CAUSAL && kbase + KT - 1 > qb * 128) || kbase + KT > Lk || kbase < kstart;
    if (need_mask) {
      // key is live for this lane's query iff kstart <= key < khi: one unsigned compare
      const int koff = kbase + 4 * hf - kstart;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          st[kt][r] = (unsigned)(koff + kt * 32 + acc_row(r, 0)) >= kspan ? -INFINITY : st[kt][r];
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, st[kt][r]);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * c;
    // Deferred rescale (cdna_hip_programming.md T13): the reference max m moves -- and O, l are
    // rescaled by exp2(m_old - m_new) -- only on tiles where some row's max grew by more than
    // g_rescale_thr (log2 units); otherwise P = exp2(s c - m) <= 2^thr against the stale m (f32,
    // and bf16 keeps its relative precision at that scale). LSE = m + log2(l) is exact either
    // way. thr = 0 rescales whenever a max grows: the plain online softmax. Branch-free: alpha = 1
    // on tiles that keep the max (a branch around the O multiplies made hipcc reconcile two O
    // register sets with 64 v_mov_b64 per tile on the common path, more than it skipped).
    const bool grow = __any(tmax > m + rescale_thr);  // wave-uniform
    const float mnew = grow ? fmaxf(m, tmax) : m;
    const float muse = (mnew == -INFINITY) ? 0.f : mnew;
    const float alpha = grow ? fast_exp2(m - muse) : 1.f;
    l *= alpha;
#pragma unroll
    for (int i = 0; i < ND; ++i) o[i] *= alpha;
    m = mnew;
    // P = exp2(s c - m): the scale-and-shift and the row sum two lanes' worth at a time
    // (v_pk_fma_f32 / v_pk_add_f32 on the accumulator's even-aligned register pairs)
    const f32x2 nm2 = {-muse, -muse};
    f32x2 rs2 = {0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const f32x2 x = {st[kt][r], st[kt][r + 1]};
        const f32x2 y = __builtin_elementwise_fma(x, c2, nm2);
        const f32x2 pv = {fast_exp2(y[0]), fast_exp2(y[1])};  // exp2(-inf) = 0 for masked keys
        st[kt][r] = pv[0];
        st[kt][r + 1] = pv[1];
        rs2 += pv;
      }
    float rs = rs2[0] + rs2[1];
    rs += __shfl_xor(rs, 32, 64);
    l += rs;
    // O^T += V^T P^T
    if constexpr (PRIO) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (STAGE == 5) {
      // V^T fragments by inline-asm ds_read_b64_tr_b16 (the builtin carries no memory operand,
      // so hipcc puts vmcnt(0) -- the next tile's in-flight LDS-DMA -- in front of it), in four
      // groups of ND fragments, the next group issued before the current one's MFMAs; a counted
      // lgkmcnt wait ties each group's registers (DS operations complete in order)
      s16x4 lo0[ND], hi0[ND], lo1[ND], hi1[ND];
      tr_group_issue<ND, PAIR + 0 * 2 * D>(lo0, hi0, toff);
      tr_group_issue<ND, PAIR + 16 * 2 * D>(lo1, hi1, toff);
      tr_group_tie<ND, 2 * ND>(lo0, hi0);
      tr_group_mfma<ND>(lo0, hi0, pack_frag(st[0], 0), o);
      tr_group_issue<ND, PAIR + 32 * 2 * D>(lo0, hi0, toff);
      tr_group_tie<ND, 2 * ND>(lo1, hi1);
      tr_group_mfma<ND>(lo1, hi1, pack_frag(st[0], 1), o);
      tr_group_issue<ND, PAIR + 48 * 2 * D>(lo1, hi1, toff);
      tr_group_tie<ND, 2 * ND>(lo0, hi0);
      tr_group_mfma<ND>(lo0, hi0, pack_frag(st[1], 0), o);
      tr_group_tie<ND, 0>(lo1, hi1);
      tr_group_mfma<ND>(lo1, hi1, pack_frag(st[1], 1), o);
    } else {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const frag8 pf = pack_frag(st[kt], s);
        const unsigned vb = PAIR + (kt * 32 + 16 * s) * 2 * D;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lds_tr_frag(toff[dt][0] + vb, toff[dt][1] + vb), pf, o[dt], 0, 0, 0);
      }
    }
    if constexpr (PRIO) {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (STAGE >= 4) {
      // the next pair's DMA has landed in LDS (vmcnt counts LDS-DMA), then every wave's
      // reads of pair CUR are done before anyone overwrites it; the sched_barrier keeps the
      // tile's MFMAs in front of the wait (hipcc otherwise sinks the last ones below it)
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    } else {
      if (more) {
        sk.store(bufK(CUR ^ 1));
        sv.store(bufV(CUR ^ 1));
      }
      __syncthreads();
    }
  };
  for (int t = t0; t < ntiles; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntiles) tile(std::integral_constant<int, 1>{}, t + 1);
  }

  if (q < Lq) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    u16* Ob = O + ((int64_t)b * Lq + q) * ldo + (int64_t)h * D;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        u16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = f2bf(o[dt][rr * 4 + j] * inv);
        *reinterpret_cast<u16x4*>(Ob + dt * 32 + 8 * rr + 4 * hf) = w;
      }
    if (hf == 0) LSE[((int64_t)b * H + h) * Lq + q] = l > 0.f ? (m + log2f(l)) * kLn2 : INFINITY;
  }
}

// ============================================================================================
// forward, software-pipelined (STAGE 7)
// ============================================================================================
// attn_fwd_k runs a tile's three steps in order -- S = K Q^T on the matrix pipe, the softmax on
// the VALU, P V on the matrix pipe -- so inside a wave the matrix pipe idles through the softmax
// and the VALU through both products. Here iteration t runs tile t's softmax in the issue gaps
// of tile t+1's S MFMAs (independent work: S_{t+1} does not need tile t's max) and of tile t's
// first P V MFMAs. K and V have two-slot rings of their own; K runs one tile ahead of V, so at
// iteration t the K tile t+1 and the V tile t are resident and the DMA of K t+2 / V t+1 lands
// under the iteration (one barrier per tile, as before). Every LDS read is inline asm with a
// counted lgkmcnt wait (the fragment group after the current one stays in flight; hipcc puts a
// vmcnt(0) -- the in-flight LDS-DMA -- in front of the builtin transposed read) and each
// softmax chunk is pinned beside its MFMA group by sched_group_barrier. Per element the
// arithmetic is attn_fwd_k's, in the same order: outputs bitwise equal to STAGE 4.
// both wave halves' values of a per-query quantity combined (lane l with lane l ^ 32) by one
// v_permlane32_swap on two registers holding x: afterwards one holds the lower half's values in
// both halves, the other the upper half's. Inline asm, so the two operands are two registers: the
// builtin given the same value twice may get one register for both, and then swaps nothing
// useful (both results read back as the lower half: a doubled row sum). The 2 wait states a VALU
// write needs before the swap reads it are the s_nop (cdna_hip_programming.md, permlane hazard).
DEV void swap_halves(unsigned& a, unsigned& b) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
DEV float swap_max(float x) {
  unsigned a = __builtin_bit_cast(unsigned, x), b = a;
  swap_halves(a, b);
  return fmaxf(__builtin_bit_cast(float, a), __builtin_bit_cast(float, b));
}
DEV float swap_sum(float x) {
  unsigned a = __builtin_bit_cast(unsigned, x), b = a;
  swap_halves(a, b);
  return __builtin_bit_cast(float, a) + __builtin_bit_cast(float, b);
}
// NM MFMAs, each followed by NV VALU instructions (the scheduler's placement of the group's code)
template <int NM, int NV>
DEV void interleave() {
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (NV > 0) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
  }
}
// P = exp2(s c - m) of accumulator registers R0..R0+3 of score tile KT_, the row sum's even /
// odd partials (the pair order of attn_fwd_k's v_pk_add accumulation)
// 2 K row fragments (k-steps S0, S0+1 at LDS byte offset OFF from each lane's roff) by inline-asm
// ds_read_b128, tied by a counted lgkmcnt wait
template <int NS, int S0, unsigned OFF>
DEV void k2_issue(s16x8 (&kf)[2], const unsigned (&roff)[NS]) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=&v"(kf[j]) : "v"(roff[S0 + j]), "n"(OFF) : "memory");
}
template <int CNT>
DEV void k2_tie(s16x8 (&kf)[2]) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(kf[0]), "+v"(kf[1]) : "n"(CNT) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int NS, int S0>
DEV void k2_mfma(const s16x8 (&kf)[2], const frag8 (&qf)[NS], f32x16& acc) {
#pragma unroll
  for (int j = 0; j < 2; ++j)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(frag8, kf[j]), qf[S0 + j], acc, 0, 0, 0);
}
// an empty asm on a value: the code computing it cannot sink below this point, and code reading it
// cannot rise above it (hipcc's instruction selection otherwise gathers a whole softmax next to its
// last consumer, out of the MFMA groups it was written beside)
template <class T>
DEV void pin(T& x) {
  asm volatile("" : "+v"(x));
}
template <int KT_, int R0>
DEV void sm_exp4(f32x16 (&sp)[2], float c, float nm, float& rsE, float& rsO) {
  pin(sp[KT_]);
#pragma unroll
  for (int r = R0; r < R0 + 4; r += 2) {
    const float p0 = fast_exp2(__builtin_fmaf(sp[KT_][r], c, nm));
    const float p1 = fast_exp2(__builtin_fmaf(sp[KT_][r + 1], c, nm));
    sp[KT_][r] = p0;
    sp[KT_][r + 1] = p1;
    rsE += p0;
    rsO += p1;
  }
  pin(sp[KT_]);
  pin(rsE);
  pin(rsO);
}

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_fwd_pipe_k(const u16* __restrict__ Q, int64_t ldq,
                                                          const u16* __restrict__ K, int64_t ldk,
                                                          const u16* __restrict__ V, int64_t ldv,
                                                          u16* __restrict__ O, int64_t ldo,
                                                          float* __restrict__ LSE, int H, int Lq, int Lk,
                                                          float scale, const int32_t* __restrict__ kv_start) {
  constexpr int KT = 64;
  constexpr int TILE = KT * D * 2;
  constexpr int NS = D / 16;  // k-steps over D: 8 (D = 128) or 4 (D = 64)
  constexpr int ND = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // K slots 0, 1 then V slots 0, 1

  const int nqb = (Lq + 127) / 128;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qi = lid % nqb, hb = lid / nqb;
  const int qb = CAUSAL ? (nqb - 1 - qi) : qi;
  const int h = hb % H, b = hb / H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hf = lane >> 5;
  const int q = qb * 128 + wave * 32 + (lane & 31);
  const int kstart = kv_start ? kv_start[b] : 0;

  const u16* Qb = Q + (int64_t)b * Lq * ldq + (int64_t)h * D;
  const u16* Kb = K + (int64_t)b * Lk * ldk + (int64_t)h * D;
  const u16* Vb = V + (int64_t)b * Lk * ldv + (int64_t)h * D;

  frag8 qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    u16x8 v = (q < Lq) ? *reinterpret_cast<const u16x8*>(Qb + (int64_t)q * ldq + 16 * s + 8 * hf) : u16x8(0);
    qf[s] = __builtin_bit_cast(frag8, v);
  }
  f32x16 o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) o[i] = f32x16(0.f);
  float m = -INFINITY, l = 0.f;
  const float c = scale * kLog2e;
  const float rescale_thr = g_rescale_thr;
  const int khi = CAUSAL ? min(Lk, q + 1) : Lk;
  const unsigned kspan = (unsigned)max(khi - kstart, 0);
  int kend = Lk;
  if (CAUSAL) kend = min(Lk, qb * 128 + 128);
  const int ntiles = (kend + KT - 1) / KT;
  const int t0 = kstart / KT;

  StageDMA1<KT, D, 4> dk_, dv_;
  const int w = __builtin_amdgcn_readfirstlane(wave);
  dk_.prep(ldk, w, lane);
  dv_.prep(ldv, w, lane);
  auto dma_k = [&](int t, int slot) { dk_.issue(Kb, ldk, t * KT, Lk, smem + slot * TILE, w); };
  auto dma_v = [&](int t, int slot) { dv_.issue(Vb, ldv, t * KT, Lk, smem + (2 + slot) * TILE, w); };

  const unsigned sbase = lds_addr(smem);
  unsigned roff[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) roff[s] = sbase + kv_off<D>(lane & 31, 2 * s + hf);
  unsigned toff[ND][2];
  {
    const int i = lane & 15, qq = i >> 2, p = i & 3;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int ch = ((dt * 32 + 16 * ((lane >> 4) & 1)) >> 3) + (p >> 1);
      toff[dt][0] = sbase + 2 * TILE + kv_off<D>(4 * hf + qq, ch) + 8 * (p & 1);
      toff[dt][1] = sbase + 2 * TILE + kv_off<D>(4 * hf + qq + 8, ch) + 8 * (p & 1);
    }
  }

  // S = K Q^T of the K tile in slot SLOT, plain (prologue): NS groups of 2 fragments (32-key half
  // G / (NS / 2), k-steps 2 (G % (NS / 2)) + 0, 1), two groups in flight
  auto s_plain = [&](auto slot_c, f32x16 (&st)[2]) {
    constexpr unsigned KO = decltype(slot_c)::value * TILE;
    constexpr int HG = NS / 2;
    constexpr unsigned K1 = 32 * 2 * D;
    s16x8 ka[2], kb[2];
    st[0] = f32x16(0.f);
    st[1] = f32x16(0.f);
    auto grp = [&](auto g_c) {
      constexpr int G = decltype(g_c)::value;
      constexpr int CNT = G + 1 < NS ? 2 : 0;
      if constexpr (G % 2 == 0) {
        k2_tie<CNT>(ka);
        k2_mfma<NS, 2 * (G % HG)>(ka, qf, st[G / HG]);
        if constexpr (G + 2 < NS) k2_issue<NS, 2 * ((G + 2) % HG), KO + ((G + 2) / HG) * K1>(ka, roff);
      } else {
        k2_tie<CNT>(kb);
        k2_mfma<NS, 2 * (G % HG)>(kb, qf, st[G / HG]);
        if constexpr (G + 2 < NS) k2_issue<NS, 2 * ((G + 2) % HG), KO + ((G + 2) / HG) * K1>(kb, roff);
      }
    };
    k2_issue<NS, 0, KO>(ka, roff);
    k2_issue<NS, 2 * (1 % HG), KO + (1 / HG) * K1>(kb, roff);
    grp(std::integral_constant<int, 0>{});
    grp(std::integral_constant<int, 1>{});
    grp(std::integral_constant<int, 2>{});
    grp(std::integral_constant<int, 3>{});
    if constexpr (NS == 8) {
      grp(std::integral_constant<int, 4>{});
      grp(std::integral_constant<int, 5>{});
      grp(std::integral_constant<int, 6>{});
      grp(std::integral_constant<int, 7>{});
    }
  };

  // Tile t's mask, row max and rescale decision, run on its scores before tile t's iteration (at
  // the end of iteration t-1, or after the prologue's S): no control flow (the mask and rescale
  // branches) may sit between an inline-asm LDS read and its counted wait, since the compiler
  // may then copy the read's destination registers before the data has landed
  float muse = 0.f;
  float alpha_p = 1.f;  // the pending rescale of l, folded into the next row-sum add
  auto prep = [&](int t, f32x16 (&sp)[2]) {
    const int kbase = t * KT;
    const bool need_mask = (CAUSAL && kbase + KT - 1 > qb * 128) || kbase + KT > Lk || kbase < kstart;
    if (need_mask) {
      const int koff = kbase + 4 * hf - kstart;
      if (kbase >= kstart) {
        // koff >= 0: key j of the tile is live iff j < kspan - koff (one compare against a
        // constant per score instead of an add and an unsigned compare)
        const int lim = (int)kspan - koff;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) sp[kt][r] = kt * 32 + acc_row(r, 0) < lim ? sp[kt][r] : -INFINITY;
      } else {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            sp[kt][r] = (unsigned)(koff + kt * 32 + acc_row(r, 0)) >= kspan ? -INFINITY : sp[kt][r];
      }
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sp[kt][r]);
    tmax = swap_max(tmax) * c;
    const bool grow = __any(tmax > m + rescale_thr);  // wave-uniform
    const float mnew = grow ? fmaxf(m, tmax) : m;
    muse = (mnew == -INFINITY) ? 0.f : mnew;
    alpha_p = 1.f;
    if (grow) {
      const float alpha = fast_exp2(m - muse);
      alpha_p = alpha;
#pragma unroll
      for (int i = 0; i < ND; ++i) o[i] *= alpha;
    }
    m = mnew;
  };

  // one tile: P of sp (tile t, masked scores in registers, decision taken by prep) beside S of
  // tile t+1 (K slot KS, into sn; NEXT = false on the last tile: no S), then P V of tile t (V slot
  // VS), then prep of tile t+1
  auto tile = [&](auto ks_c, auto vs_c, auto next_c, int t, f32x16 (&sp)[2], f32x16 (&sn)[2]) {
    constexpr unsigned KO = decltype(ks_c)::value * TILE;
    constexpr unsigned VO = decltype(vs_c)::value * TILE;
    constexpr bool NEXT = decltype(next_c)::value;
    if constexpr (NEXT) {
      // V slot VS^1 was last read by tile t-1's P V, K slot KS^1 by tile t's S (both before the
      // previous barrier)
      dma_v(t + 1, decltype(vs_c)::value ^ 1);
      if (t + 2 < ntiles) dma_k(t + 2, decltype(ks_c)::value ^ 1);
    }
    // S of tile t+1 in NS groups of 2 MFMAs (K fragments 2 groups in flight), each group's issue
    // gaps carrying one (D = 128) or two (D = 64) of the P chunks 0-7 of tile t
    s16x8 ka[2], kb[2];
    s16x4 la[2], ha[2], lb[2], hb[2];  // P V fragment pairs, two in flight
    constexpr int PG = ND / 2;           // pairs per 16-key slice
    constexpr int NPV = 4 * PG;          // P V groups
    float rsE = 0.f, rsO = 0.f;
    frag8 pf[4];
    const float nm = -muse;
    constexpr unsigned K1 = 32 * 2 * D;  // second 32-key half of the K tile
    constexpr int HG = NS / 2;           // groups per 32-key half
    // P chunk C: registers 4 (C % 4) .. + 3 of score tile C / 4, the packed fragment when a
    // 16-key slice is complete
    auto chunk = [&](auto c_c) {
      constexpr int C = decltype(c_c)::value;
      constexpr int KT_ = C / 4, R0 = (C % 4) * 4;
      sm_exp4<KT_, R0>(sp, c, nm, rsE, rsO);
      if constexpr (R0 == 4 || R0 == 12) {
        pf[2 * KT_ + R0 / 8] = pack_frag(sp[KT_], R0 / 8);
        pin(pf[2 * KT_ + R0 / 8]);
      }
    };
    constexpr int kFill[8] = {6, 8, 6, 8, 6, 8, 6, 8};
    // group G: its MFMAs, its chunk(s), then the reads two groups ahead (or the first P V reads)
    auto group = [&](auto g_c) {
      constexpr int G = decltype(g_c)::value;
      constexpr int S0 = 2 * (G % HG);
      if constexpr (NEXT) {
        if constexpr (G % 2 == 0) {
          k2_tie<G == NS - 1 ? 4 : 2>(ka);
          k2_mfma<NS, S0>(ka, qf, sn[G / HG]);
        } else {
          k2_tie<G == NS - 1 ? 4 : 2>(kb);
          k2_mfma<NS, S0>(kb, qf, sn[G / HG]);
        }
      }
      constexpr int CPG = 8 / NS;  // chunks per group
      chunk(std::integral_constant<int, G * CPG>{});
      if constexpr (CPG == 2) chunk(std::integral_constant<int, G * CPG + 1>{});
      if constexpr (NEXT) interleave<2, kFill[G * CPG] + (CPG == 2 ? kFill[G * CPG + 1] : 0)>();
      if constexpr (G + 2 < NS) {
        if constexpr (NEXT) {
          constexpr unsigned OFF2 = KO + ((G + 2) / HG) * K1;
          if constexpr (G % 2 == 0) k2_issue<NS, 2 * ((G + 2) % HG), OFF2>(ka, roff);
          else k2_issue<NS, 2 * ((G + 2) % HG), OFF2>(kb, roff);
        }
      } else if constexpr (G == NS - 2) {
        tr2_issue<ND, VO, 0>(la, ha, toff);  // P V group 0
      } else {
        tr2_issue<ND, VO + (1 / PG) * 16 * 2 * D, 2 * (1 % PG)>(lb, hb, toff);  // P V group 1
      }
    };
    if constexpr (NEXT) {
      sn[0] = f32x16(0.f);
      sn[1] = f32x16(0.f);
      k2_issue<NS, 0, KO>(ka, roff);
      k2_issue<NS, 2 * (1 % HG), KO + (1 / HG) * K1>(kb, roff);
    }
    group(std::integral_constant<int, 0>{});
    group(std::integral_constant<int, 1>{});
    group(std::integral_constant<int, 2>{});
    group(std::integral_constant<int, 3>{});
    if constexpr (NS == 8) {
      group(std::integral_constant<int, 4>{});
      group(std::integral_constant<int, 5>{});
      group(std::integral_constant<int, 6>{});
      group(std::integral_constant<int, 7>{});
    }
    // P V in NPV pair groups (slice v / PG, column blocks 2 (v % PG) + 0, 1), one group in flight
    // under the current one's MFMAs; the row sum beside the first
    auto pv = [&](auto v_c) {
      constexpr int V = decltype(v_c)::value;
      constexpr int CNT = V + 1 < NPV ? 4 : 0;
      if constexpr (V % 2 == 0) {
        tr2_tie<CNT>(la, ha);
        tr2_mfma<ND, 2 * (V % PG)>(la, ha, pf[V / PG], o);
      } else {
        tr2_tie<CNT>(lb, hb);
        tr2_mfma<ND, 2 * (V % PG)>(lb, hb, pf[V / PG], o);
      }
      if constexpr (V == 0) {
        float rs = rsE + rsO;
        rs = swap_sum(rs);
        // l = l alpha + rs in one rounding, as attn_fwd_k's contracted l *= alpha; ...; l += rs
        // (alpha = 1 when the max held: an exact add)
        l = __builtin_fmaf(l, alpha_p, rs);
        interleave<2, 2>();
      }
      if constexpr (V + 2 < NPV) {
        constexpr unsigned VB = VO + ((V + 2) / PG) * 16 * 2 * D;
        if constexpr (V % 2 == 0) tr2_issue<ND, VB, 2 * ((V + 2) % PG)>(la, ha, toff);
        else tr2_issue<ND, VB, 2 * ((V + 2) % PG)>(lb, hb, toff);
      }
    };
    pv(std::integral_constant<int, 0>{});
    pv(std::integral_constant<int, 1>{});
    pv(std::integral_constant<int, 2>{});
    pv(std::integral_constant<int, 3>{});
    if constexpr (NPV == 8) {
      pv(std::integral_constant<int, 4>{});
      pv(std::integral_constant<int, 5>{});
      pv(std::integral_constant<int, 6>{});
      pv(std::integral_constant<int, 7>{});
    }
    if constexpr (NEXT) {
      prep(t + 1, sn);
      // K t+2 / V t+1 landed (vmcnt counts LDS-DMA), and every wave's reads of the slots they
      // refill next iteration are done
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  };

  f32x16 sa[2], sb[2];
  if (t0 < ntiles) {
    dma_k(t0, 0);
    dma_v(t0, 0);
    if (t0 + 1 < ntiles) dma_k(t0 + 1, 1);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    __syncthreads();
    s_plain(std::integral_constant<int, 0>{}, sa);
    prep(t0, sa);
    __syncthreads();  // K slot 0 is refilled (tile t0 + 2) by the first iteration
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using NT = std::integral_constant<bool, true>;
    using NF = std::integral_constant<bool, false>;
    // tile t: K slot of tile t+1 = (t - t0 + 1) & 1, V slot of tile t = (t - t0) & 1. Pairs of
    // tiles with a successor in a plain loop, the last one or two after it (a loop with the last
    // tile's variant inside it spilled ~95 VGPRs)
    int t = t0;
    for (; t + 2 < ntiles; t += 2) {
      tile(I1{}, I0{}, NT{}, t, sa, sb);
      tile(I0{}, I1{}, NT{}, t + 1, sb, sa);
    }
    if (t + 1 < ntiles) {
      tile(I1{}, I0{}, NT{}, t, sa, sb);
      tile(I0{}, I1{}, NF{}, t + 1, sb, sa);
    } else {
      tile(I1{}, I0{}, NF{}, t, sa, sb);
    }
  }

  // O rows, widened stores (cdna_hip_programming.md T21): lanes l and l ^ 32 hold the two
  // 4-column halves of each 8-column group of the same row; one v_permlane32_swap per dword of a
  // pair of groups (k, k+1) leaves the lower half-wave with columns 8k..8k+7 and the upper with
  // 8k+8..8k+15, one 16-B store each instead of two 8-B stores. The swaps run on every lane (a
  // lane and its partner hold the same query row, so the row guard is uniform across the pair).
  {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    u16* Ob = O + ((int64_t)b * Lq + q) * ldo + (int64_t)h * D;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int rr = 0; rr < 4; rr += 2) {
        u16x4 wa, wb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          wa[j] = f2bf(o[dt][rr * 4 + j] * inv);
          wb[j] = f2bf(o[dt][(rr + 1) * 4 + j] * inv);
        }
        u32x2 a = __builtin_bit_cast(u32x2, wa), bb = __builtin_bit_cast(u32x2, wb);
        unsigned ax = a[0], ay = a[1], bx = bb[0], by = bb[1];
        swap_halves(ax, bx);
        swap_halves(ay, by);
        if (q < Lq) {
          const u32x4 w4 = {ax, ay, bx, by};
          *reinterpret_cast<u32x4*>(Ob + dt * 32 + 8 * rr + 8 * hf) = w4;
        }
      }
    if (q < Lq && hf == 0) LSE[((int64_t)b * H + h) * Lq + q] = l > 0.f ? (m + log2f(l)) * kLn2 : INFINITY;
  }
}

// ============================================================================================
// backward
// ============================================================================================
// delta[b,h,q] = sum_d dO*O  (f32); one 16-lane group per (token, head) row for D=128
template <int D>
__global__ __launch_bounds__(256) void attn_delta_k(const u16* __restrict__ O, int64_t ldo,
                                                    const u16* __restrict__ dO, int64_t lddo,
                                                    float* __restrict__ delta, int B, int H, int L) {
  constexpr int LPR = D / 8;  // lanes per row
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;  // (b, t, h) row
  const int sub = threadIdx.x % LPR;
  const int64_t nrows = (int64_t)B * L * H;
  float acc = 0.f;
  if (row < nrows) {
    const int hh = (int)(row % H);
    const int64_t bt = row / H;
    float a[8], d[8];
    load8(O + bt * ldo + (int64_t)hh * D + sub * 8, a);
    load8(dO + bt * lddo + (int64_t)hh * D + sub * 8, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * d[j];
  }
#pragma unroll
  for (int o = LPR / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (row < nrows && sub == 0) {
    const int hh = (int)(row % H);
    const int64_t bt = row / H;
    const int64_t bb = bt / L, t = bt % L;
    delta[(bb * H + hh) * L + t] = acc;
  }
}

// Kernel A: dK, dV. A wave owns 32 keys (K, V fragments in registers); the workgroup sweeps
// 32-row query tiles staged in LDS. S = Q K^T and dP = dO V^T keep the key on the lane;
// dV = P^T dO and dK = dS^T Q take P / dS straight from the accumulators (A operand) and
// dO / Q as transposed LDS fragments.
template <int D, bool CAUSAL, int QT>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv_k(
    const u16* __restrict__ Q, int64_t ldq, const u16* __restrict__ K, int64_t ldk,
    const u16* __restrict__ V, int64_t ldv, const u16* __restrict__ dO, int64_t lddo,
    const float* __restrict__ LSE, const float* __restrict__ DELTA, u16* __restrict__ dK,
    int64_t lddk, u16* __restrict__ dV, int64_t lddv, int H, int Lq, int Lk, float scale,
    const int32_t* __restrict__ kv_start) {
  constexpr int NSUB = QT / 32;  // 32-row query sub-tiles per barrier
  constexpr int TILE = QT * D * 2;
  constexpr int NS = D / 16;
  constexpr int ND = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // [buf][Q tile | dO tile | lse(32 f32) | delta(32 f32)]
  constexpr int BUF = 2 * TILE + 2 * QT * 4;

  // 1-D grid of (key block, head, batch), XCD-remapped: the key blocks of one (b, h) share
  // its Q / dO tiles in one XCD's L2
  const int nkb = (Lk + 127) / 128;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = lid % nkb, hb = lid / nkb;
  const int h = hb % H, b = hb / H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hf = lane >> 5;
  const int key = kb * 128 + wave * 32 + (lane & 31);  // this lane's key (operand column)
  const int kstart = kv_start ? kv_start[b] : 0;

  const u16* Qb = Q + (int64_t)b * Lq * ldq + (int64_t)h * D;
  const u16* dOb = dO + (int64_t)b * Lq * lddo + (int64_t)h * D;
  const u16* Kb = K + (int64_t)b * Lk * ldk + (int64_t)h * D;
  const u16* Vb = V + (int64_t)b * Lk * ldv + (int64_t)h * D;
  const float* lseb = LSE + ((int64_t)b * H + h) * Lq;
  const float* delb = DELTA + ((int64_t)b * H + h) * Lq;

  frag8 kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const bool ok = key < Lk;
    kf[s] = __builtin_bit_cast(frag8, ok ? *reinterpret_cast<const u16x8*>(Kb + (int64_t)key * ldk + 16 * s + 8 * hf) : u16x8(0));
    vf[s] = __builtin_bit_cast(frag8, ok ? *reinterpret_cast<const u16x8*>(Vb + (int64_t)key * ldv + 16 * s + 8 * hf) : u16x8(0));
  }
  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) { dk[i] = f32x16(0.f); dv[i] = f32x16(0.f); }
  const float c = scale * kLog2e;

  // query tiles that can see this block's keys
  const int kmin = kb * 128;
  int qt0 = CAUSAL ? (kmin / QT) : 0;
  const int nqt = (Lq + QT - 1) / QT;
  const bool block_live = kmin < Lk && (kmin + 128 > kstart);

  Stage<QT, D> sq, sdo;
  // lse / delta of a query tile (threads 0..2QT-1, one value each): loaded together with the
  // tile's Q / dO prefetch and written to LDS with them (not loaded and waited for at the end)
  float aux = 0.f;
  // the next tile's lse / delta: loaded raw and first used when staged after the tile's compute
  // (arithmetic on the loaded value at load time made the compiler wait for it -- and for the
  // in-flight tile prefetch -- at the top of every tile)
  bool aux_in = false;
  auto load_aux = [&](int qt) {
    if (threadIdx.x < 2 * QT) {
      const int qq = qt * QT + (int)threadIdx.x % QT;
      aux_in = qq < Lq;
      aux = (threadIdx.x < QT ? lseb : delb)[min(qq, Lq - 1)];
    }
  };
  auto store_aux = [&](char* buf) {
    if (threadIdx.x < 2 * QT)
      ((float*)(buf + 2 * TILE))[threadIdx.x] = aux_in ? aux : (threadIdx.x < QT ? INFINITY : 0.f);
  };
  if (block_live && qt0 < nqt) {
    sq.load(Qb, ldq, qt0 * QT, Lq);
    sdo.load(dOb, lddo, qt0 * QT, Lq);
    sq.store(smem);
    sdo.store(smem + TILE);
    load_aux(qt0);
    store_aux(smem);
  }
  __builtin_amdgcn_s_waitcnt(kVmcnt0);  // see attn_fwd_k: keeps hipcc from waiting on the prefetch
  __syncthreads();

  for (int qt = qt0; block_live && qt < nqt; ++qt) {
    const int cur = (qt - qt0) & 1;
    char* buf = smem + cur * BUF;
    char* nbuf = smem + (cur ^ 1) * BUF;
    const bool more = qt + 1 < nqt;
    if (more) {
      sq.load(Qb, ldq, (qt + 1) * QT, Lq);
      sdo.load(dOb, lddo, (qt + 1) * QT, Lq);
      load_aux(qt + 1);
    }
    const float* slse = (const float*)(buf + 2 * TILE);
    const float* sdel = slse + QT;
    // S[q][key], dP[q][key] of the NSUB 32-row sub-tiles (independent MFMA chains)
    f32x16 sacc[NSUB], pacc[NSUB];
#pragma unroll
    for (int u = 0; u < NSUB; ++u) { sacc[u] = f32x16(0.f); pacc[u] = f32x16(0.f); }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int u = 0; u < NSUB; ++u) {
        sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<D>(buf, 32 * u, s, lane), kf[s], sacc[u], 0, 0, 0);
        pacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<D>(buf + TILE, 32 * u, s, lane), vf[s], pacc[u], 0, 0, 0);
      }
    // P = exp(S*scale - lse), dS = P * (dP - delta)
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(slse + 32 * u + 8 * rr + 4 * hf);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(sdel + 32 * u + 8 * rr + 4 * hf);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = rr * 4 + j;
          const int qq = qt * QT + 32 * u + 8 * rr + 4 * hf + j;
          float pv = fast_exp2(fmaf(sacc[u][r], c, -l4[j] * kLog2e));
          if ((CAUSAL && key > qq) || key < kstart || key >= Lk || qq >= Lq) pv = 0.f;
          sacc[u][r] = pv;
          pacc[u][r] = pv * (pacc[u][r] - d4[j]);
        }
      }
    // dV += P^T dO ; dK += dS^T Q   (A operand = accumulator, B = transposed LDS fragment);
    // sub-tile order = the 32-row tile order, so every QT sums in the same order
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const frag8 pf = pack_frag(sacc[u], s);
        const frag8 df = pack_frag(pacc[u], s);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf, tr_frag<D>(buf + TILE, 32 * u + 16 * s, dt * 32, lane), dv[dt], 0, 0, 0);
          dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(df, tr_frag<D>(buf, 32 * u + 16 * s, dt * 32, lane), dk[dt], 0, 0, 0);
        }
      }
    if (more) {
      sq.store(nbuf);
      sdo.store(nbuf + TILE);
      store_aux(nbuf);
    }
    __syncthreads();
  }

  // dK/dV[key][d]: register r = key row, lane = d column
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kk = kb * 128 + wave * 32 + acc_row(r, hf);
      if (kk < Lk) {
        const int d = dt * 32 + (lane & 31);
        dK[((int64_t)b * Lk + kk) * lddk + (int64_t)h * D + d] = f2bf(dk[dt][r] * scale);
        dV[((int64_t)b * Lk + kk) * lddv + (int64_t)h * D + d] = f2bf(dv[dt][r]);
      }
    }
}

// Kernel B: dQ. A wave owns 32 query rows (Q, dO fragments in registers, lse/delta per
// lane); the workgroup sweeps 32-key K/V tiles. S^T = K Q^T, dP^T = V dO^T (query on the
// lane), dQ^T += K^T dS^T with K^T as a transposed LDS fragment.
template <int D, bool CAUSAL, int KT>
__global__ __launch_bounds__(256, 1) void attn_bwd_dq_k(
    const u16* __restrict__ Q, int64_t ldq, const u16* __restrict__ K, int64_t ldk,
    const u16* __restrict__ V, int64_t ldv, const u16* __restrict__ dO, int64_t lddo,
    const float* __restrict__ LSE, const float* __restrict__ DELTA, u16* __restrict__ dQ,
    int64_t lddq, int H, int Lq, int Lk, float scale, const int32_t* __restrict__ kv_start) {
  constexpr int TILE = KT * D * 2;
  constexpr int NSUB = KT / 32;  // 32-key sub-tiles per barrier
  constexpr int NS = D / 16;
  constexpr int ND = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nqb = (Lq + 127) / 128;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);  // as attn_fwd_k: one (b, h) per XCD range
  const int qi = lid % nqb, hb = lid / nqb;
  const int qb = CAUSAL ? (nqb - 1 - qi) : qi;
  const int h = hb % H, b = hb / H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hf = lane >> 5;
  const int q = qb * 128 + wave * 32 + (lane & 31);
  const int kstart = kv_start ? kv_start[b] : 0;

  const u16* Qb = Q + (int64_t)b * Lq * ldq + (int64_t)h * D;
  const u16* dOb = dO + (int64_t)b * Lq * lddo + (int64_t)h * D;
  const u16* Kb = K + (int64_t)b * Lk * ldk + (int64_t)h * D;
  const u16* Vb = V + (int64_t)b * Lk * ldv + (int64_t)h * D;

  frag8 qf[NS], of[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const bool ok = q < Lq;
    qf[s] = __builtin_bit_cast(frag8, ok ? *reinterpret_cast<const u16x8*>(Qb + (int64_t)q * ldq + 16 * s + 8 * hf) : u16x8(0));
    of[s] = __builtin_bit_cast(frag8, ok ? *reinterpret_cast<const u16x8*>(dOb + (int64_t)q * lddo + 16 * s + 8 * hf) : u16x8(0));
  }
  const float lse2 = (q < Lq) ? LSE[((int64_t)b * H + h) * Lq + q] * kLog2e : INFINITY;
  const float del = (q < Lq) ? DELTA[((int64_t)b * H + h) * Lq + q] : 0.f;
  const float c = scale * kLog2e;
  f32x16 dq[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) dq[i] = f32x16(0.f);

  int kend = Lk;
  if (CAUSAL) kend = min(Lk, qb * 128 + 128);
  const int ntiles = (kend + KT - 1) / KT;
  const int t0 = kstart / KT;

  Stage<KT, D> sk, sv;
  // buffer i: K at smem + 2*i*TILE, V right after it
#define bufK(i) (smem + 2 * (i) * TILE)
#define bufV(i) (smem + 2 * (i) * TILE + TILE)
  if (t0 < ntiles) {
    sk.load(Kb, ldk, t0 * KT, Lk);
    sv.load(Vb, ldv, t0 * KT, Lk);
    sk.store(bufK(0));
    sv.store(bufV(0));
  }
  __builtin_amdgcn_s_waitcnt(kVmcnt0);  // see attn_fwd_k: keeps hipcc from waiting on the prefetch
  __syncthreads();
  for (int t = t0; t < ntiles; ++t) {
    const int cur = (t - t0) & 1;
    const bool more = t + 1 < ntiles;
    if (more) {
      sk.load(Kb, ldk, (t + 1) * KT, Lk);
      sv.load(Vb, ldv, (t + 1) * KT, Lk);
    }
    f32x16 st[NSUB], dpt[NSUB];
#pragma unroll
    for (int u = 0; u < NSUB; ++u) { st[u] = f32x16(0.f); dpt[u] = f32x16(0.f); }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int u = 0; u < NSUB; ++u) {
        st[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<D>(bufK(cur), 32 * u, s, lane), qf[s], st[u], 0, 0, 0);
        dpt[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<D>(bufV(cur), 32 * u, s, lane), of[s], dpt[u], 0, 0, 0);
      }
    const int kbase = t * KT;
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kbase + 32 * u + acc_row(r, hf);
        float pv = fast_exp2(fmaf(st[u][r], c, -lse2));
        if (key >= Lk || key < kstart || (CAUSAL && key > q)) pv = 0.f;
        dpt[u][r] = pv * (dpt[u][r] - del);
      }
#pragma unroll
    for (int u = 0; u < NSUB; ++u)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const frag8 df = pack_frag(dpt[u], s);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
          dq[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag<D>(bufK(cur), 32 * u + 16 * s, dt * 32, lane), df, dq[dt], 0, 0, 0);
      }
    if (more) {
      sk.store(bufK(cur ^ 1));
      sv.store(bufV(cur ^ 1));
    }
    __syncthreads();
  }
  if (q < Lq) {
    u16* dQb = dQ + ((int64_t)b * Lq + q) * lddq + (int64_t)h * D;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        u16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = f2bf(dq[dt][rr * 4 + j] * scale);
        *reinterpret_cast<u16x4*>(dQb + dt * 32 + 8 * rr + 4 * hf) = w;
      }
  }
}

// ============================================================================================
// backward, 8-wave variants (the default): two waves per SIMD
// ============================================================================================
// The 4-wave kernels above keep one wave per SIMD (their K/V or Q/dO fragments plus two sets of
// 32x32 accumulators need > 256 registers), so every LDS read, exp and wait of a wave sits in
// front of its own MFMAs with nothing to overlap it. Here a workgroup has 8 waves over the same
// 128 keys (dK/dV) or 128 queries (dQ): waves w and w + 4 own the same 32-row slice and split
// the other dimension of every tile between them (query rows 0-31 / 32-63 of the 64-row query
// tile; keys 0-31 / 32-63 of the 64-key tile), so each SIMD runs two waves whose MFMAs cover
// each other's LDS / VALU phases. The pair's partial accumulators are added once at the end
// through LDS (fixed order: half 0 + half 1), so results stay bitwise reproducible.
//   dK/dV: K and V of the workgroup's 128 keys live in LDS for the whole sweep (row fragments
//   re-read per tile instead of 64 registers), Q / dO tiles double-buffered beside them.
//   dQ:    Q / dO fragments in registers, K / V tiles double-buffered in LDS.
template <int ROWS, int D, int NT>
struct StageN {
  static constexpr int kPer = ROWS * D / 8 / NT;  // 16-byte chunks per thread
  u16x8 r[kPer];
  DEV void load(const u16* base, int64_t ld, int row0, int nrows) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = threadIdx.x + NT * i;
      const int row = q / (D / 8), ch = q % (D / 8);
      r[i] = (row0 + row < nrows) ? *reinterpret_cast<const u16x8*>(base + (int64_t)(row0 + row) * ld + ch * 8)
                                  : u16x8(0);
    }
  }
  DEV void store(char* lds) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int q = threadIdx.x + NT * i;
      const int row = q / (D / 8), ch = q % (D / 8);
      *reinterpret_cast<u16x8*>(lds + kv_off<D>(row, ch)) = r[i];
    }
  }
};

template <int D, bool CAUSAL, bool DS_OUT = false, bool DMA = false>
__global__ __launch_bounds__(512, 1) void attn_bwd_dkdv8_k(
    const u16* __restrict__ Q, int64_t ldq, const u16* __restrict__ K, int64_t ldk,
    const u16* __restrict__ V, int64_t ldv, const u16* __restrict__ dO, int64_t lddo,
    const float* __restrict__ LSE, const float* __restrict__ DELTA, u16* __restrict__ dK,
    int64_t lddk, u16* __restrict__ dV, int64_t lddv, int H, int Lq, int Lk, float scale,
    const int32_t* __restrict__ kv_start, u16* __restrict__ dST, int64_t ldst, int64_t st_bh, int64_t st_blk) {
  constexpr int QT = 64, KB = 128;
  constexpr int TQ = QT * D * 2;          // bytes of a Q (or dO) tile
  constexpr int TK = KB * D * 2;          // bytes of the K (or V) image
  constexpr int NS = D / 16;
  constexpr int ND = D / 32;
  constexpr int BUF = 2 * TQ + 2 * QT * 4;  // [Q | dO | lse(64) | delta(64)]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sK = smem;
  char* sV = smem + TK;
  char* bufs = smem + 2 * TK;

  const int nkb = (Lk + KB - 1) / KB;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = lid % nkb, hb = lid / nkb;
  const int h = hb % H, b = hb / H;
  // wave index through readfirstlane: wave-uniform to the compiler (scalar slice / half branches
  // and row bases)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hf = lane >> 5;
  const int ksl = wave & 3, u = wave >> 2;          // 32-key slice, query half of each tile
  const int key = kb * KB + ksl * 32 + (lane & 31);  // this lane's key
  const int kstart = kv_start ? kv_start[b] : 0;
  // live queries of this key: [qlo, qlim) (empty for keys before kstart or past Lk)
  const int qlo = CAUSAL ? key : 0;
  const int qlim = (key < kstart || key >= Lk) ? qlo : Lq;
  const unsigned qspan = (unsigned)max(qlim - qlo, 0);

  const u16* Qb = Q + (int64_t)b * Lq * ldq + (int64_t)h * D;
  const u16* dOb = dO + (int64_t)b * Lq * lddo + (int64_t)h * D;
  const u16* Kb = K + (int64_t)b * Lk * ldk + (int64_t)h * D;
  const u16* Vb = V + (int64_t)b * Lk * ldv + (int64_t)h * D;
  const float* lseb = LSE + ((int64_t)b * H + h) * Lq;
  const float* delb = DELTA + ((int64_t)b * H + h) * Lq;

  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) { dk[i] = f32x16(0.f); dv[i] = f32x16(0.f); }
  const float c = scale * kLog2e;
  const int kmin = kb * KB;
  const int qt0 = CAUSAL ? (kmin / QT) : 0;
  const int nqt = (Lq + QT - 1) / QT;
  const bool block_live = kmin < Lk && (kmin + KB > kstart);

  StageT<QT, D, 512> sq, sdo;  // per-tile descriptors (see StageT)
  const unsigned voq = StageT<QT, D, 512>::lane_off(ldq), vodo = StageT<QT, D, 512>::lane_off(lddo);
  // DMA (cullavo_attn_set_bwd_stage(1)): Q / dO tiles by LDS-DMA into the swizzled image (as the
  // forward's StageDMA), no staging registers or ds_write
  StageDMA<QT, D, 8> dq_, ddo_;
  // DMA: per-lane LDS byte offsets of the asm fragment reads (rows relative to a 32-row slice /
  // a 16-key slice: the image swizzle depends on row & 15 only)
  unsigned roff_b[NS], toff_b[ND][2];
  if constexpr (DMA) {
    dq_.prep(ldq, wave, lane);
    ddo_.prep(lddo, wave, lane);
#pragma unroll
    for (int s = 0; s < NS; ++s) roff_b[s] = kv_off<D>(lane & 31, 2 * s + (lane >> 5));
    const int i = lane & 15, qq = i >> 2, pp = i & 3;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int ch = ((dt * 32 + 16 * ((lane >> 4) & 1)) >> 3) + (pp >> 1);
      toff_b[dt][0] = kv_off<D>(4 * hf + qq, ch) + 8 * (pp & 1);
      toff_b[dt][1] = kv_off<D>(4 * hf + qq + 8, ch) + 8 * (pp & 1);
    }
  }
  float aux = 0.f;
  // the next tile's lse / delta: loaded raw and first used when staged after the tile's compute
  // (the lse * log2 e at load time made the compiler wait for the load -- and for the in-flight
  // Q / dO prefetch -- at the top of every tile)
  bool aux_in = false;
  auto load_aux = [&](int qt) {
    if (threadIdx.x < 2 * QT) {
      const int qq = qt * QT + (int)threadIdx.x % QT;
      aux_in = qq < Lq;
      aux = (threadIdx.x < QT ? lseb : delb)[min(qq, Lq - 1)];
    }
  };
  auto store_aux = [&](char* buf) {
    if (threadIdx.x < 2 * QT)
      ((float*)(buf + 2 * TQ))[threadIdx.x] =
          threadIdx.x < QT ? (aux_in ? aux * kLog2e : INFINITY) : (aux_in ? aux : 0.f);
  };
  if (block_live) {
    StageN<KB, D, 512> skv;
    skv.load(Kb, ldk, kmin, Lk);
    skv.store(sK);
    skv.load(Vb, ldv, kmin, Lk);
    skv.store(sV);
    if (qt0 < nqt) {
      if constexpr (DMA) {
        dq_.issue(Qb, ldq, qt0 * QT, Lq, bufs, wave);
        ddo_.issue(dOb, lddo, qt0 * QT, Lq, bufs + TQ, wave);
      } else {
        sq.load(Qb, ldq, qt0 * QT, Lq, voq);
        sdo.load(dOb, lddo, qt0 * QT, Lq, vodo);
        sq.store(bufs);
        sdo.store(bufs + TQ);
      }
      load_aux(qt0);
      store_aux(bufs);
    }
  }
  __builtin_amdgcn_s_waitcnt(kVmcnt0);  // see attn_fwd_k: keeps hipcc from waiting on the prefetch
  __syncthreads();

  for (int qt = qt0; block_live && qt < nqt; ++qt) {
    const int cur = (qt - qt0) & 1;
    char* buf = bufs + cur * BUF;
    char* nbuf = bufs + (cur ^ 1) * BUF;
    const bool more = qt + 1 < nqt;
    if (more) {
      if constexpr (DMA) {
        dq_.issue(Qb, ldq, (qt + 1) * QT, Lq, nbuf, wave);  // nbuf was last read before the previous barrier
        ddo_.issue(dOb, lddo, (qt + 1) * QT, Lq, nbuf + TQ, wave);
      } else {
        sq.load(Qb, ldq, (qt + 1) * QT, Lq, voq);
        sdo.load(dOb, lddo, (qt + 1) * QT, Lq, vodo);
      }
      load_aux(qt + 1);
    }
    const float* slse = (const float*)(buf + 2 * TQ);
    const float* sdel = slse + QT;
    // S[q][key], dP[q][key] for this wave's 32 query rows of the tile
    f32x16 sacc = f32x16(0.f), pacc = f32x16(0.f);
    if constexpr (DMA) {
      // inline-asm fragment reads (a compiler-visible LDS read may alias the next tile's in-flight
      // LDS-DMA, so hipcc would wait vmcnt(0) in front of it), one k-step ahead of the MFMAs: the
      // four reads of step s + 1 are in flight while step s's two MFMAs issue
      const unsigned aq = lds_addr(buf) + 2u * D * 32u * u, ak = lds_addr(sK) + 2u * D * 32u * ksl;
      s16x8 q0, k0, d0, v0, q1, k1, d1, v1;
      __builtin_amdgcn_sched_barrier(0);
      rd4(q0, k0, d0, v0, aq + roff_b[0], ak + roff_b[0], aq + TQ + roff_b[0], ak + TK + roff_b[0]);
#pragma unroll
      for (int st = 0; st < NS; st += 2) {
        rd4(q1, k1, d1, v1, aq + roff_b[st + 1], ak + roff_b[st + 1], aq + TQ + roff_b[st + 1], ak + TK + roff_b[st + 1]);
        tie4<4>(q0, k0, d0, v0);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(frag8, q0), __builtin_bit_cast(frag8, k0), sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(frag8, d0), __builtin_bit_cast(frag8, v0), pacc, 0, 0, 0);
        if (st + 2 < NS) {
          rd4(q0, k0, d0, v0, aq + roff_b[st + 2], ak + roff_b[st + 2], aq + TQ + roff_b[st + 2], ak + TK + roff_b[st + 2]);
          tie4<4>(q1, k1, d1, v1);
        } else {
          tie4<0>(q1, k1, d1, v1);
        }
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(frag8, q1), __builtin_bit_cast(frag8, k1), sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(frag8, d1), __builtin_bit_cast(frag8, v1), pacc, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<D>(buf, 32 * u, s, lane), row_frag<D>(sK, 32 * ksl, s, lane), sacc, 0, 0, 0);
      pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<D>(buf + TQ, 32 * u, s, lane), row_frag<D>(sV, 32 * ksl, s, lane), pacc, 0, 0, 0);
    }
    }
    // query qq is live for this lane's key iff qlo <= qq < qlim: one unsigned compare per element
    const int qoff = qt * QT + 32 * u + 4 * hf - qlo;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const f32x4 l4 = *reinterpret_cast<const f32x4*>(slse + 32 * u + 8 * rr + 4 * hf);
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(sdel + 32 * u + 8 * rr + 4 * hf);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = rr * 4 + j;
        float pv = fast_exp2(fmaf(sacc[r], c, -l4[j]));  // lse staged as lse * log2(e)
        if ((unsigned)(qoff + 8 * rr + j) >= qspan) pv = 0.f;
        sacc[r] = pv;
        pacc[r] = pv * (pacc[r] - d4[j]);
      }
    }
    // dV += P^T dO ; dK += dS^T Q over this wave's 32 query rows
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const frag8 pf = pack_frag(sacc, s);
      const frag8 df = pack_frag(pacc, s);
      if (DS_OUT) {
        // dS^T[key][q] (the bf16 operand of dK) for the dQ kernel: registers 8s..8s+3 / 8s+4..8s+7
        // are query rows 16s + 4hf + 0..3 / 16s + 8 + 4hf + 0..3 of this wave's 32
        const u16x8 w = __builtin_bit_cast(u16x8, df);
        // (128-query block (qt QT) / 128 at st_blk: ds_layout)
        u16* row = dST + ((int64_t)b * H + h) * st_bh + (int64_t)((qt * QT) >> 7) * st_blk + (int64_t)key * ldst +
                   ((qt * QT) & 127) + 32 * u + 16 * s + 4 * hf;
        *reinterpret_cast<u16x4*>(row) = u16x4{w[0], w[1], w[2], w[3]};
        *reinterpret_cast<u16x4*>(row + 8) = u16x4{w[4], w[5], w[6], w[7]};
      }
      if constexpr (DMA) {
        // transposed dO / Q fragments by inline asm, one column block ahead of the MFMAs
        const unsigned kb = lds_addr(buf) + 2u * D * (32u * u + 16u * s);
        s16x4 dl0, dh0, ql0, qh0, dl1, dh1, ql1, qh1;
        __builtin_amdgcn_sched_barrier(0);
        rd4t(dl0, dh0, ql0, qh0, kb + TQ + toff_b[0][0], kb + TQ + toff_b[0][1], kb + toff_b[0][0], kb + toff_b[0][1]);
#pragma unroll
        for (int dt = 0; dt < ND; dt += 2) {
          rd4t(dl1, dh1, ql1, qh1, kb + TQ + toff_b[dt + 1][0], kb + TQ + toff_b[dt + 1][1], kb + toff_b[dt + 1][0],
               kb + toff_b[dt + 1][1]);
          tie4t<4>(dl0, dh0, ql0, qh0);
          dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf, tr_join(dl0, dh0), dv[dt], 0, 0, 0);
          dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(df, tr_join(ql0, qh0), dk[dt], 0, 0, 0);
          if (dt + 2 < ND) {
            rd4t(dl0, dh0, ql0, qh0, kb + TQ + toff_b[dt + 2][0], kb + TQ + toff_b[dt + 2][1], kb + toff_b[dt + 2][0],
                 kb + toff_b[dt + 2][1]);
            tie4t<4>(dl1, dh1, ql1, qh1);
          } else {
            tie4t<0>(dl1, dh1, ql1, qh1);
          }
          dv[dt + 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf, tr_join(dl1, dh1), dv[dt + 1], 0, 0, 0);
          dk[dt + 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(df, tr_join(ql1, qh1), dk[dt + 1], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      } else {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        dv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pf, tr_frag<D>(buf + TQ, 32 * u + 16 * s, dt * 32, lane), dv[dt], 0, 0, 0);
        dk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(df, tr_frag<D>(buf, 32 * u + 16 * s, dt * 32, lane), dk[dt], 0, 0, 0);
      }
      }
    }
    if (more) {
      if constexpr (!DMA) {
        sq.store(nbuf);
        sdo.store(nbuf + TQ);
      }
      store_aux(nbuf);
    }
    if constexpr (DMA) {  // the next tile's DMA landed (MFMAs kept in front of the wait)
      __builtin_amdgcn_sched_barrier(0);
      // DS_OUT: the tile's four dS^T stores (two 8-B stores per 16-query slice, after the DMA in
      // issue order) may stay in flight
      if constexpr (DS_OUT) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }

  // pair reduction: half 1 parks its partial sums in LDS, half 0 adds them and stores
  float* red = (float*)smem;  // [2 (dk, dv)][4 slices][ND][16][64] f32
  auto slot = [&](int which, int dt, int r) { return red + ((((which * 4 + ksl) * ND + dt) * 16 + r) * 64 + lane); };
  __syncthreads();
  if (u == 1) {
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) { *slot(0, dt, r) = dk[dt][r]; *slot(1, dt, r) = dv[dt][r]; }
  }
  __syncthreads();
  if (u == 0) {
    // wave-uniform row base (scalar), one 32-bit lane offset (4 hf rows + column lane & 31);
    // row r's offset acc_row(r, 0) * ld is scalar too, the column block dt * 32 an immediate:
    // one saddr store per element instead of 64-bit address arithmetic per element
    const int k0 = kb * KB + ksl * 32;
    u16* dKr = dK + ((int64_t)b * Lk + k0) * lddk + (int64_t)h * D;
    u16* dVr = dV + ((int64_t)b * Lk + k0) * lddv + (int64_t)h * D;
    const unsigned lk = (unsigned)(4 * hf * lddk + (lane & 31)) * 2u, lv = (unsigned)(4 * hf * lddv + (lane & 31)) * 2u;
    const int left = Lk - k0;  // rows of this slice that exist (>= 32 on all but the last block)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (acc_row(r, hf) < left) {
        u16* pk = dKr + (int64_t)acc_row(r, 0) * lddk;
        u16* pv = dVr + (int64_t)acc_row(r, 0) * lddv;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          *(u16*)((char*)pk + (lk + dt * 64u)) = f2bf((dk[dt][r] + *slot(0, dt, r)) * scale);
          *(u16*)((char*)pv + (lv + dt * 64u)) = f2bf(dv[dt][r] + *slot(1, dt, r));
        }
      }
    }
  }
}

// ============================================================================================
// backward dQ from the stored dS (mode 7)
// ============================================================================================
// The 8-wave dK/dV kernel writes dS^T[b, h][key][q] (bf16, the same rounded values its dK
// product consumes) for every (key, query) pair it visits; dQ^T = K^T dS^T then needs no S / dP
// recompute: one product instead of three. A wave owns 32 query columns, the workgroup sweeps
// 64-key tiles up to the causal diagonal with K and dS^T tiles staged in LDS, both operands
// read as transposed fragments (the same k order on both sides). dS^T has LkP =
// round_up(Lk, 128) rows (keys) of LqP = round_up(Lq, 128) queries (cullavo_attn_bwd_workspace).
template <int D, bool CAUSAL, bool DMA = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_ds_k(const u16* __restrict__ K, int64_t ldk,
                                                           const u16* __restrict__ dST, int64_t ldst, int64_t st_bh, int64_t st_blk,
                                                           int LkP, u16* __restrict__ dQ, int64_t lddq, int H,
                                                           int Lq, int Lk, float scale,
                                                           const int32_t* __restrict__ kv_start) {
  constexpr int KT = 64, QB = 128;
  constexpr int TK = KT * D * 2, TS = KT * QB * 2, BUF = TK + TS;
  constexpr int NS = KT / 16, ND = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nqb = (Lq + QB - 1) / QB;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qi = lid % nqb, hb = lid / nqb;
  const int qb = CAUSAL ? (nqb - 1 - qi) : qi;
  const int h = hb % H, b = hb / H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hf = lane >> 5;
  const int q = qb * QB + wave * 32 + (lane & 31);
  const int kstart = kv_start ? kv_start[b] : 0;
  const u16* Kb = K + (int64_t)b * Lk * ldk + (int64_t)h * D;
  const u16* Sb = dST + ((int64_t)b * H + h) * st_bh + qb * st_blk;

  f32x16 dq[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) dq[i] = f32x16(0.f);
  int kend = Lk;
  if (CAUSAL) kend = min(Lk, qb * QB + QB);
  const int ntiles = (kend + KT - 1) / KT;
  const int t0 = kstart / KT;

  StageT<KT, D> sk;
  StageT<KT, QB> ss;
  const unsigned vok = StageT<KT, D>::lane_off(ldk), vos = StageT<KT, QB>::lane_off(ldst);
  // DMA (cullavo_attn_set_bwd_stage bit 1): K and dS^T tiles by LDS-DMA into the swizzled
  // images. Every fragment of a tile is read into registers BEFORE the next tile's DMA is issued:
  // the transposed reads (builtin, no memory operand) would otherwise each wait for that DMA
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  StageDMA<KT, D, 4> dk_;
  StageDMA<KT, QB, 4> ds_;
  if constexpr (DMA) {
    dk_.prep(ldk, wu, lane);
    ds_.prep(ldst, wu, lane);
    if (t0 < ntiles) {
      dk_.issue(Kb, ldk, t0 * KT, Lk, smem, wu);
      ds_.issue(Sb, ldst, t0 * KT, LkP, smem + TK, wu);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = t0; t < ntiles; ++t) {
      char* bK = smem + ((t - t0) & 1) * BUF;
      char* bS = bK + TK;
      frag8 bsf[NS], kf[NS][ND];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        bsf[s] = tr_frag<QB>(bS, 16 * s, wave * 32, lane);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) kf[s][dt] = tr_frag<D>(bK, 16 * s, dt * 32, lane);
      }
      if (t + 1 < ntiles) {  // the other pair was last read before the previous barrier
        char* nK = smem + ((t - t0 + 1) & 1) * BUF;
        dk_.issue(Kb, ldk, (t + 1) * KT, Lk, nK, wu);
        ds_.issue(Sb, ldst, (t + 1) * KT, LkP, nK + TK, wu);
      }
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) dq[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[s][dt], bsf[s], dq[dt], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // the MFMAs issue before the wait for the DMA
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
  if (t0 < ntiles) {
    sk.load(Kb, ldk, t0 * KT, Lk, vok);
    ss.load(Sb, ldst, t0 * KT, LkP, vos);
    sk.store(smem);
    ss.store(smem + TK);
  }
  __builtin_amdgcn_s_waitcnt(kVmcnt0);
  __syncthreads();
  for (int t = t0; t < ntiles; ++t) {
    char* bK = smem + ((t - t0) & 1) * BUF;
    char* bS = bK + TK;
    const bool more = t + 1 < ntiles;
    if (more) {
      sk.load(Kb, ldk, (t + 1) * KT, Lk, vok);
      ss.load(Sb, ldst, (t + 1) * KT, LkP, vos);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const frag8 bs = tr_frag<QB>(bS, 16 * s, wave * 32, lane);
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
        dq[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag<D>(bK, 16 * s, dt * 32, lane), bs, dq[dt], 0, 0, 0);
    }
    if (more) {
      char* nK = smem + ((t - t0 + 1) & 1) * BUF;
      sk.store(nK);
      ss.store(nK + TK);
    }
    __syncthreads();
  }
  }
  if (q < Lq) {
    u16* dQb = dQ + ((int64_t)b * Lq + q) * lddq + (int64_t)h * D;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        u16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = f2bf(dq[dt][rr * 4 + j] * scale);
        *reinterpret_cast<u16x4*>(dQb + dt * 32 + 8 * rr + 4 * hf) = w;
      }
  }
}

// dQ = scale dS K from the stored dS^T, the LDS-DMA ring form (round 6; cullavo_attn_set_bwd_stage
// bit 2). attn_bwd_dq_ds_k keeps one 64-key tile in flight per workgroup (two per CU): 32 KiB of
// dS^T per CU against the ~50 KiB that HBM latency x the per-CU share of its bandwidth asks for,
// so it streams dS^T at ~3 TB/s (118 us per 7B layer, MFMA busy 0.14). Here one workgroup per CU
// holds NST = 4 stages of (K tile, dS^T tile) in LDS and keeps NST - 1 tiles in flight by
// LDS-DMA (counted vmcnt: the DMA pieces are the only vector-memory ops in the loop, 2 kPer per
// tile and wave), with the fragment reads by inline asm (a builtin LDS read would make the
// compiler wait for every DMA in flight first) tied by counted lgkmcnt. Same tiles, same MFMA
// order, same epilogue as attn_bwd_dq_ds_k: bitwise the same dQ.
// (NST, LAB: tools/lab/dq_lab.hip only -- LAB bit 0 skips the fragment reads and MFMAs, bit 1 the
// K tiles' DMA: timing floors, not results)
template <int D, bool CAUSAL, int NST = 4, int LAB = 0>
__global__ __launch_bounds__(256, 1) void attn_bwd_dq_ring_k(const u16* __restrict__ K, int64_t ldk,
                                                             const u16* __restrict__ dST, int64_t ldst, int64_t st_bh, int64_t st_blk,
                                                             int LkP, u16* __restrict__ dQ, int64_t lddq, int H,
                                                             int Lq, int Lk, float scale,
                                                             const int32_t* __restrict__ kv_start) {
  static_assert(NST >= 2 && NST <= 4, "2 to 4 stages");
  constexpr int KT = 64, QB = 128;
  constexpr int TK = KT * D * 2, TS = KT * QB * 2, BUF = TK + TS;
  constexpr int NS = KT / 16, ND = D / 32;
  constexpr unsigned KSTEP = 16 * D * 2, SSTEP = 16 * QB * 2;  // 16 rows: the image swizzle's period
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nqb = (Lq + QB - 1) / QB;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qi = lid % nqb, hb = lid / nqb;
  const int qb = CAUSAL ? (nqb - 1 - qi) : qi;
  const int h = hb % H, b = hb / H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hf = lane >> 5;
  const int q = qb * QB + wave * 32 + (lane & 31);
  const int kstart = kv_start ? kv_start[b] : 0;
  const u16* Kb = K + (int64_t)b * Lk * ldk + (int64_t)h * D;
  const u16* Sb = dST + ((int64_t)b * H + h) * st_bh + qb * st_blk;

  f32x16 dq[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) dq[i] = f32x16(0.f);
  int kend = Lk;
  if (CAUSAL) kend = min(Lk, qb * QB + QB);
  const int ntiles = (kend + KT - 1) / KT;
  const int t0 = kstart / KT;

  const int wu = __builtin_amdgcn_readfirstlane(wave);
  StageDMA<KT, D, 4> dk_;
  StageDMA<KT, QB, 4> ds_;
  dk_.prep(ldk, wu, lane);
  ds_.prep(ldst, wu, lane);
  constexpr int kOps = (LAB & 2 ? 0 : StageDMA<KT, D, 4>::kPer) + StageDMA<KT, QB, 4>::kPer;  // DMA pieces per tile and wave
  auto issue = [&](int t) {
    char* bK = smem + ((t - t0) % NST) * BUF;
    if constexpr (!(LAB & 2)) dk_.issue(Kb, ldk, t * KT, Lk, bK, wu);
    ds_.issue(Sb, ldst, t * KT, LkP, bK + TK, wu);
  };
  // per-lane LDS addresses of tr_frag's two halves (16-key step 0; step s adds s KSTEP / SSTEP)
  const unsigned sbase = lds_addr(smem);
  unsigned ko[ND][2], so[2];
  {
    const int i = lane & 15, qq = i >> 2, p = i & 3, r0 = 4 * hf + qq;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int ch = ((dt * 32 + 16 * ((lane >> 4) & 1)) >> 3) + (p >> 1);
      ko[dt][0] = sbase + kv_off<D>(r0, ch) + 8 * (p & 1);
      ko[dt][1] = sbase + kv_off<D>(r0 + 8, ch) + 8 * (p & 1);
    }
    const int ch = ((wave * 32 + 16 * ((lane >> 4) & 1)) >> 3) + (p >> 1);
    so[0] = sbase + TK + kv_off<QB>(r0, ch) + 8 * (p & 1);
    so[1] = sbase + TK + kv_off<QB>(r0 + 8, ch) + 8 * (p & 1);
  }
  // one 16-key step's fragments: dS^T (B operand) and the ND K^T fragments (A operands)
  struct Grp {
    s16x4 bl, bh, kl[ND], kh[ND];
  };
  // (ko / so as parameters: clang rejects a generic lambda's implicit capture used in asm operands)
  auto grp_issue = [](auto s_c, Grp& g, unsigned slot, const unsigned (&ko)[ND][2], const unsigned (&so)[2]) {
    constexpr unsigned S = decltype(s_c)::value;
    asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%4\n\tds_read_b64_tr_b16 %1, %3 offset:%4"
                 : "=&v"(g.bl), "=&v"(g.bh)
                 : "v"(so[0] + slot), "v"(so[1] + slot), "n"(S * SSTEP)
                 : "memory");
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
      asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%4\n\tds_read_b64_tr_b16 %1, %3 offset:%4"
                   : "=&v"(g.kl[dt]), "=&v"(g.kh[dt])
                   : "v"(ko[dt][0] + slot), "v"(ko[dt][1] + slot), "n"(S * KSTEP)
                   : "memory");
  };
  auto grp_tie = [](auto cnt_c, Grp& g) {
    constexpr int CNT = decltype(cnt_c)::value;
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(g.bl), "+v"(g.bh) : "n"(CNT) : "memory");
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) asm volatile("" : "+v"(g.kl[dt]), "+v"(g.kh[dt]));
    __builtin_amdgcn_sched_barrier(0);
  };
  auto grp_mfma = [&](const Grp& g) {
    const frag8 bs = tr_join(g.bl, g.bh);
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) dq[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_join(g.kl[dt], g.kh[dt]), bs, dq[dt], 0, 0, 0);
  };
  using C0 = std::integral_constant<int, 0>;
  using CG = std::integral_constant<int, 2 * (ND + 1)>;  // one group's reads
  static_assert(NS == 4 && 2 * (ND + 1) <= 15, "lgkmcnt counts one group in flight");

  for (int j = 0; j < NST - 1; ++j)
    if (t0 + j < ntiles) issue(t0 + j);
  for (int t = t0; t < ntiles; ++t) {
    // tile t landed: the tiles after it that are already issued may stay in flight
    const int after = min(NST - 2, ntiles - 1 - t);
    if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kOps) : "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kOps) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // every wave's pieces of tile t are in, and every wave is done reading the slot refilled next
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + NST - 1 < ntiles) issue(t + NST - 1);
    if constexpr (LAB & 1) continue;
    const unsigned slot = (unsigned)(((t - t0) % NST) * BUF);
    Grp ga, gb;
    grp_issue(std::integral_constant<unsigned, 0>{}, ga, slot, ko, so);
    grp_issue(std::integral_constant<unsigned, 1>{}, gb, slot, ko, so);
    grp_tie(CG{}, ga);
    grp_mfma(ga);
    grp_issue(std::integral_constant<unsigned, 2>{}, ga, slot, ko, so);
    grp_tie(CG{}, gb);
    grp_mfma(gb);
    grp_issue(std::integral_constant<unsigned, 3>{}, gb, slot, ko, so);
    grp_tie(CG{}, ga);
    grp_mfma(ga);
    grp_tie(C0{}, gb);
    grp_mfma(gb);
  }
  if (q < Lq) {
    u16* dQb = dQ + ((int64_t)b * Lq + q) * lddq + (int64_t)h * D;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        u16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = f2bf(dq[dt][rr * 4 + j] * scale);
        *reinterpret_cast<u16x4*>(dQb + dt * 32 + 8 * rr + 4 * hf) = w;
      }
  }
}

int64_t ds_rows(int Lk) { return cdiv(Lk, 128) * 128; }
int64_t ds_cols(int Lq) { return cdiv(Lq, 128) * 128; }

template <typename Kern>
void set_smem(Kern k, int bytes) {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

template <int D, bool CAUSAL>
int fwd_launch(const u16* q, int64_t ldq, const u16* k, int64_t ldk, const u16* v, int64_t ldv, u16* o,
               int64_t ldo, float* lse, int B, int H, int Lq, int Lk, float scale, const int32_t* ks,
               hipStream_t s) {
  const int smem = 4 * 64 * D * 2;
  static bool once = false;
  if (!once) {
    set_smem(attn_fwd_k<D, CAUSAL, 0>, smem);
    set_smem(attn_fwd_k<D, CAUSAL, 1>, smem);
    set_smem(attn_fwd_k<D, CAUSAL, 2>, smem);
    set_smem(attn_fwd_k<D, CAUSAL, 2, 1>, smem);
    set_smem(attn_fwd_k<D, CAUSAL, 4>, smem);
    set_smem(attn_fwd_k<D, CAUSAL, 5>, smem);
    set_smem(attn_fwd_k<D, CAUSAL, 6>, smem);
    set_smem(attn_fwd_pipe_k<D, CAUSAL>, smem);
    once = true;
  }
  const unsigned grid = (unsigned)(cdiv(Lq, 128) * H * B);
  const int stage = g_fwd_stage >= 0 ? g_fwd_stage : 7;
  if (stage == 7)
    attn_fwd_pipe_k<D, CAUSAL><<<grid, 256, smem, s>>>(q, ldq, k, ldk, v, ldv, o, ldo, lse, H, Lq, Lk, scale, ks);
  else if (stage == 6)
    attn_fwd_k<D, CAUSAL, 6><<<grid, 256, smem, s>>>(q, ldq, k, ldk, v, ldv, o, ldo, lse, H, Lq, Lk, scale, ks);
  else if (stage == 5)
    attn_fwd_k<D, CAUSAL, 5><<<grid, 256, smem, s>>>(q, ldq, k, ldk, v, ldv, o, ldo, lse, H, Lq, Lk, scale, ks);
  else if (stage == 4)
    attn_fwd_k<D, CAUSAL, 4><<<grid, 256, smem, s>>>(q, ldq, k, ldk, v, ldv, o, ldo, lse, H, Lq, Lk, scale, ks);
  else if (stage == 3)
    attn_fwd_k<D, CAUSAL, 2, 1><<<grid, 256, smem, s>>>(q, ldq, k, ldk, v, ldv, o, ldo, lse, H, Lq, Lk, scale, ks);
  else if (stage == 2)
    attn_fwd_k<D, CAUSAL, 2><<<grid, 256, smem, s>>>(q, ldq, k, ldk, v, ldv, o, ldo, lse, H, Lq, Lk, scale, ks);
  else if (stage == 1)
    attn_fwd_k<D, CAUSAL, 1><<<grid, 256, smem, s>>>(q, ldq, k, ldk, v, ldv, o, ldo, lse, H, Lq, Lk, scale, ks);
  else
    attn_fwd_k<D, CAUSAL, 0><<<grid, 256, smem, s>>>(q, ldq, k, ldk, v, ldv, o, ldo, lse, H, Lq, Lk, scale, ks);
  return cullavo_check_launch("attn_fwd");
}

template <int D, bool CAUSAL, int QT, int KT>
int bwd_launch(const u16* q, int64_t ldq, const u16* k, int64_t ldk, const u16* v, int64_t ldv, const u16* o,
               int64_t ldo, const u16* dout, int64_t lddo, const float* lse, float* delta, u16* dq, int64_t lddq,
               u16* dk, int64_t lddk, u16* dv, int64_t lddv, int B, int H, int Lq, int Lk, float scale,
               const int32_t* ks, hipStream_t s) {
  const int64_t rows = (int64_t)B * Lq * H;
  attn_delta_k<D><<<(unsigned)cdiv(rows * (D / 8), 256), 256, 0, s>>>(o, ldo, dout, lddo, delta, B, H, Lq);
  const int smem_a = 2 * (2 * QT * D * 2 + 2 * QT * 4);
  const int smem_b = 4 * KT * D * 2;
  static bool once = false;
  if (!once) {
    set_smem(attn_bwd_dkdv_k<D, CAUSAL, QT>, smem_a);
    set_smem(attn_bwd_dq_k<D, CAUSAL, KT>, smem_b);
    once = true;
  }
  const unsigned ga = (unsigned)(cdiv(Lk, 128) * H * B);
  attn_bwd_dkdv_k<D, CAUSAL, QT><<<ga, 256, smem_a, s>>>(q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, dk, lddk,
                                                      dv, lddv, H, Lq, Lk, scale, ks);
  const unsigned gb = (unsigned)(cdiv(Lq, 128) * H * B);
  attn_bwd_dq_k<D, CAUSAL, KT><<<gb, 256, smem_b, s>>>(q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, dq, lddq, H,
                                                    Lq, Lk, scale, ks);
  return cullavo_check_launch("attn_bwd");
}

// mode 4: the 8-wave dK/dV kernel + the 4-wave dQ kernel with 32-key tiles (the recompute path
// when no dS^T workspace is given; the 8-wave dQ kernel, mode 5, measured slower: 284 vs 251 us per
// 7B layer, and was removed in round 5)
template <int D, bool CAUSAL>
int bwd8_launch(const u16* q, int64_t ldq, const u16* k, int64_t ldk, const u16* v, int64_t ldv, const u16* o,
                int64_t ldo, const u16* dout, int64_t lddo, const float* lse, float* delta, u16* dq, int64_t lddq,
                u16* dk, int64_t lddk, u16* dv, int64_t lddv, int B, int H, int Lq, int Lk, float scale,
                const int32_t* ks, hipStream_t s) {
  const int64_t rows = (int64_t)B * Lq * H;
  attn_delta_k<D><<<(unsigned)cdiv(rows * (D / 8), 256), 256, 0, s>>>(o, ldo, dout, lddo, delta, B, H, Lq);
  // dK/dV: K, V images (2 x 128 x D) + 2 x [Q | dO | lse | delta] tiles of 64 rows; the pair
  // reduction reuses the front 2 x 4 x 32 x D f32 of it
  const int smem_a = std::max(2 * 128 * D * 2 + 2 * (2 * 64 * D * 2 + 2 * 64 * 4), 2 * 4 * 32 * D * 4);
  const int smem_b = 4 * 32 * D * 2;
  static bool once = false;
  if (!once) {
    set_smem(attn_bwd_dkdv8_k<D, CAUSAL>, smem_a);
    set_smem(attn_bwd_dkdv8_k<D, CAUSAL, false, true>, smem_a);
    set_smem(attn_bwd_dq_k<D, CAUSAL, 32>, smem_b);
    once = true;
  }
  if (g_bwd_stage & 1)
    attn_bwd_dkdv8_k<D, CAUSAL, false, true><<<(unsigned)(cdiv(Lk, 128) * H * B), 512, smem_a, s>>>(
        q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, dk, lddk, dv, lddv, H, Lq, Lk, scale, ks, nullptr, 0, 0, 0);
  else
    attn_bwd_dkdv8_k<D, CAUSAL><<<(unsigned)(cdiv(Lk, 128) * H * B), 512, smem_a, s>>>(
        q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, dk, lddk, dv, lddv, H, Lq, Lk, scale, ks, nullptr, 0, 0, 0);
  attn_bwd_dq_k<D, CAUSAL, 32><<<(unsigned)(cdiv(Lq, 128) * H * B), 256, smem_b, s>>>(
      q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, dq, lddq, H, Lq, Lk, scale, ks);
  return cullavo_check_launch("attn_bwd");
}

// mode 7: the 8-wave dK/dV kernel storing dS^T + dQ from it (workspace: B*H*LkP*LqP bf16)
template <int D, bool CAUSAL>
int bwd_ds_launch(const u16* q, int64_t ldq, const u16* k, int64_t ldk, const u16* v, int64_t ldv, const u16* o,
                  int64_t ldo, const u16* dout, int64_t lddo, const float* lse, float* delta, u16* dq, int64_t lddq,
                  u16* dk, int64_t lddk, u16* dv, int64_t lddv, int B, int H, int Lq, int Lk, float scale,
                  const int32_t* ks, u16* ds, hipStream_t s) {
  const int64_t rows = (int64_t)B * Lq * H;
  attn_delta_k<D><<<(unsigned)cdiv(rows * (D / 8), 256), 256, 0, s>>>(o, ldo, dout, lddo, delta, B, H, Lq);
  const int smem_a = std::max(2 * 128 * D * 2 + 2 * (2 * 64 * D * 2 + 2 * 64 * 4), 2 * 4 * 32 * D * 4);
  const int smem_b = 2 * (64 * D * 2 + 64 * 128 * 2);
  const int smem_r = 4 * (64 * D * 2 + 64 * 128 * 2);  // attn_bwd_dq_ring_k's 4 stages (128 KiB at D = 128)
  static bool once = false;
  if (!once) {
    set_smem(attn_bwd_dkdv8_k<D, CAUSAL, true>, smem_a);
    set_smem(attn_bwd_dkdv8_k<D, CAUSAL, true, true>, smem_a);
    set_smem(attn_bwd_dq_ds_k<D, CAUSAL>, smem_b);
    set_smem(attn_bwd_dq_ds_k<D, CAUSAL, true>, smem_b);
    if constexpr (D == 128) set_smem(attn_bwd_dq_ring_k<D, CAUSAL>, smem_r);
    once = true;
  }
  const int64_t LkP = ds_rows(Lk), LqP = ds_cols(Lq);
  // dS^T layout (ds_layout): row stride and 128-query block stride
  const bool blk = (g_bwd_stage & 8) != 0;
  const int64_t ldst = blk ? 128 : LqP, st_blk = blk ? LkP * 128 : 128;
  if (g_bwd_stage & 1)
    attn_bwd_dkdv8_k<D, CAUSAL, true, true><<<(unsigned)(cdiv(Lk, 128) * H * B), 512, smem_a, s>>>(
        q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, dk, lddk, dv, lddv, H, Lq, Lk, scale, ks, ds, ldst, LkP * LqP, st_blk);
  else
    attn_bwd_dkdv8_k<D, CAUSAL, true><<<(unsigned)(cdiv(Lk, 128) * H * B), 512, smem_a, s>>>(
        q, ldq, k, ldk, v, ldv, dout, lddo, lse, delta, dk, lddk, dv, lddv, H, Lq, Lk, scale, ks, ds, ldst, LkP * LqP, st_blk);
  if (D == 128 && (g_bwd_stage & 4))
    attn_bwd_dq_ring_k<D, CAUSAL><<<(unsigned)(cdiv(Lq, 128) * H * B), 256, smem_r, s>>>(
        k, ldk, ds, ldst, LkP * LqP, st_blk, (int)LkP, dq, lddq, H, Lq, Lk, scale, ks);
  else if (g_bwd_stage & 2)
    attn_bwd_dq_ds_k<D, CAUSAL, true><<<(unsigned)(cdiv(Lq, 128) * H * B), 256, smem_b, s>>>(
        k, ldk, ds, ldst, LkP * LqP, st_blk, (int)LkP, dq, lddq, H, Lq, Lk, scale, ks);
  else
    attn_bwd_dq_ds_k<D, CAUSAL><<<(unsigned)(cdiv(Lq, 128) * H * B), 256, smem_b, s>>>(
        k, ldk, ds, ldst, LkP * LqP, st_blk, (int)LkP, dq, lddq, H, Lq, Lk, scale, ks);
  return cullavo_check_launch("attn_bwd");
}


// backward tile shape (cullavo_attn_set_bwd_tiles): bit 0 -> 64 query rows per dK/dV
// barrier, bit 1 -> 64 keys per dQ barrier (else 32); -1 = per head dim, from the MI355X
// sweep in tools/attn_bench.py: D=128 causal 64/32 (730 vs 746 us), D=64 32/64 (636 vs 646 us)
int g_bwd_tiles = -1;

}  // namespace

extern "C" int cullavo_attn_set_stage(int buffer_loads) {
  const int prev = g_fwd_stage;
  if (buffer_loads >= -1 && buffer_loads <= 7) g_fwd_stage = buffer_loads;
  return prev;
}

extern "C" int cullavo_attn_set_bwd_stage(int mode) {
  const int prev = g_bwd_stage;
  if (mode >= 0 && mode <= 15) g_bwd_stage = mode;
  return prev;
}

extern "C" int cullavo_attn_set_rescale(float threshold, float* previous) {
  CV_REQUIRE(threshold >= 0.f && threshold <= 16.f, CULLAVO_EINVAL, "rescale threshold must be in [0, 16]");
  if (previous && hipMemcpyFromSymbol(previous, HIP_SYMBOL(g_rescale_thr), sizeof(float)) != hipSuccess)
    return CULLAVO_EHIP;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_rescale_thr), &threshold, sizeof(float)) != hipSuccess) return CULLAVO_EHIP;
  return CULLAVO_OK;
}

extern "C" int cullavo_attn_set_bwd_tiles(int mode) {
  const int prev = g_bwd_tiles;
  if ((mode >= -1 && mode <= 4) || mode == 7) g_bwd_tiles = mode;
  return prev;
}

extern "C" int cullavo_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                int64_t ldv, void* o, int64_t ldo, float* lse, int B, int H, int Lq, int Lk,
                                int D, float scale, int causal, const int32_t* kv_start, int dtype,
                                void* stream) {
  CV_REQUIRE(dtype == CULLAVO_DT_BF16 || dtype == CULLAVO_DT_F32, CULLAVO_EUNSUPPORTED, "attention: bf16 / f32");
  CV_REQUIRE(D == 16 || D == 32 || D == 64 || D == 128, CULLAVO_EUNSUPPORTED, "head_dim must be 16, 32, 64 or 128");
  CV_REQUIRE(!causal || Lq == Lk, CULLAVO_EINVAL, "causal attention needs Lq == Lk");
  CV_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 8 == 0, CULLAVO_EINVAL, "token strides must be multiples of 8");
  CV_REQUIRE(ldq >= (int64_t)H * D && ldk >= (int64_t)H * D && ldv >= (int64_t)H * D && ldo >= (int64_t)H * D,
             CULLAVO_EINVAL, "token stride smaller than H*D");
  if (B == 0 || H == 0 || Lq == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  if (dtype == CULLAVO_DT_F32 || D < 64)  // f32 parity mode / config-1 head dims: attn_generic.hip
    return cullavo_attn_generic_fwd(q, ldq, k, ldk, v, ldv, o, ldo, lse, B, H, Lq, Lk, D, scale, causal, kv_start,
                                    dtype, s);
  const u16 *Q = (const u16*)q, *K = (const u16*)k, *V = (const u16*)v;
  u16* O = (u16*)o;
  if (D == 128)
    return causal ? fwd_launch<128, true>(Q, ldq, K, ldk, V, ldv, O, ldo, lse, B, H, Lq, Lk, scale, kv_start, s)
                  : fwd_launch<128, false>(Q, ldq, K, ldk, V, ldv, O, ldo, lse, B, H, Lq, Lk, scale, kv_start, s);
  return causal ? fwd_launch<64, true>(Q, ldq, K, ldk, V, ldv, O, ldo, lse, B, H, Lq, Lk, scale, kv_start, s)
                : fwd_launch<64, false>(Q, ldq, K, ldk, V, ldv, O, ldo, lse, B, H, Lq, Lk, scale, kv_start, s);
}

// default: D=128 (the LM) mode 7 -- in the 7B shape 532 us per layer against 667 for mode 4
// (tools/attn_bench.py), the dQ kernel no longer recomputes S and dP; D=64 (the ViT) mode 2
static int bwd_mode(int D) { return g_bwd_tiles >= 0 ? g_bwd_tiles : (D == 128 ? 7 : 2); }

extern "C" size_t cullavo_attn_bwd_workspace(int B, int H, int Lq, int Lk, int D, int dtype) {
  if (dtype != CULLAVO_DT_BF16 || D < 64 || B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || (bwd_mode(D) != 7))
    return 0;
  return (size_t)B * H * ds_rows(Lk) * ds_cols(Lq) * 2;
}

extern "C" int cullavo_attn_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                int64_t ldv, const void* o, int64_t ldo, const void* dout, int64_t lddo,
                                const float* lse, float* delta, void* dq, int64_t lddq, void* dk,
                                int64_t lddk, void* dv, int64_t lddv, int B, int H, int Lq, int Lk, int D,
                                float scale, int causal, const int32_t* kv_start, int dtype, void* stream) {
  return cullavo_attn_bwd_ws(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, delta, dq, lddq, dk, lddk, dv, lddv,
                             B, H, Lq, Lk, D, scale, causal, kv_start, dtype, nullptr, 0, stream);
}

extern "C" int cullavo_attn_bwd_ws(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                   int64_t ldv, const void* o, int64_t ldo, const void* dout, int64_t lddo,
                                   const float* lse, float* delta, void* dq, int64_t lddq, void* dk,
                                   int64_t lddk, void* dv, int64_t lddv, int B, int H, int Lq, int Lk, int D,
                                   float scale, int causal, const int32_t* kv_start, int dtype, void* workspace,
                                   size_t workspace_bytes, void* stream) {

  CV_REQUIRE(dtype == CULLAVO_DT_BF16 || dtype == CULLAVO_DT_F32, CULLAVO_EUNSUPPORTED, "attention: bf16 / f32");
  CV_REQUIRE(D == 16 || D == 32 || D == 64 || D == 128, CULLAVO_EUNSUPPORTED, "head_dim must be 16, 32, 64 or 128");
  CV_REQUIRE(!causal || Lq == Lk, CULLAVO_EINVAL, "causal attention needs Lq == Lk");
  CV_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 8 == 0 && lddo % 8 == 0 && lddq % 8 == 0 &&
                 lddk % 8 == 0 && lddv % 8 == 0,
             CULLAVO_EINVAL, "token strides must be multiples of 8");
  if (B == 0 || H == 0 || Lq == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  if (dtype == CULLAVO_DT_F32 || D < 64)
    return cullavo_attn_generic_bwd(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, delta, dq, lddq, dk, lddk, dv,
                                    lddv, B, H, Lq, Lk, D, scale, causal, kv_start, dtype, s);
  const u16 *Q = (const u16*)q, *K = (const u16*)k, *V = (const u16*)v, *O = (const u16*)o, *dO = (const u16*)dout;
  u16 *dQ = (u16*)dq, *dK = (u16*)dk, *dV = (u16*)dv;
#define BWD4(DD, CC, QQ, KK) bwd_launch<DD, CC, QQ, KK>(Q, ldq, K, ldk, V, ldv, O, ldo, dO, lddo, lse, delta, dQ, lddq, dK, lddk, dV, lddv, B, H, Lq, Lk, scale, kv_start, s)
  // default: D=128 (the LM) the 8-wave dK/dV kernel + the 4-wave 32-key dQ kernel (mode 4;
  // in the 7B step 356 + 251 us per layer vs 467 + 251 for the 4-wave pair; the 8-wave dQ
  // kernel, mode 5, took 284 us);
  // D=64 (the ViT) the 4-wave kernels with 32-row dK/dV and 64-key dQ tiles (647 vs 797 us at
  // B=64, T=577, H=16): there the 4-wave kernels already hold K/V in registers at < 256
  // VGPRs and the 8-wave LDS re-reads cost more than the second wave hides (tools/attn_bench.py)
  int mode = bwd_mode(D);
  if (mode == 7) {
    if (workspace != nullptr && workspace_bytes >= cullavo_attn_bwd_workspace(B, H, Lq, Lk, D, dtype)) {
      u16* ds = (u16*)workspace;
#define BDS(DD, CC) bwd_ds_launch<DD, CC>(Q, ldq, K, ldk, V, ldv, O, ldo, dO, lddo, lse, delta, dQ, lddq, dK, lddk, dV, lddv, B, H, Lq, Lk, scale, kv_start, ds, s)
      if (D == 128) return causal ? BDS(128, true) : BDS(128, false);
      return causal ? BDS(64, true) : BDS(64, false);
#undef BDS
    }
    mode = 4;  // no dS workspace: the recompute path (same dK / dV kernel)
  }
  if (mode == 4) {
#define B8(DD, CC) bwd8_launch<DD, CC>(Q, ldq, K, ldk, V, ldv, O, ldo, dO, lddo, lse, delta, dQ, lddq, dK, lddk, dV, lddv, B, H, Lq, Lk, scale, kv_start, s)
    if (D == 128) return causal ? B8(128, true) : B8(128, false);
    return causal ? B8(64, true) : B8(64, false);
#undef B8
  }
  const int tiles = mode;
#define BWD(DD, CC) (tiles == 3 ? BWD4(DD, CC, 64, 64) : tiles == 2 ? BWD4(DD, CC, 32, 64) \
                     : tiles == 1 ? BWD4(DD, CC, 64, 32) : BWD4(DD, CC, 32, 32))
  if (D == 128) return causal ? BWD(128, true) : BWD(128, false);
  return causal ? BWD(64, true) : BWD(64, false);
#undef BWD
#undef BWD4
}
