// GEMM lab, round 3: the 256x256 tile with FOUR waves (one per SIMD), each owning a 128x128 output
// block (8 x 8 MFMA 16x16x32 tiles, 256 accumulator registers) -- the geometry of the hipBLASLt
// kernel that beats the production 8-wave kernel on the forward shapes
// (Cijk_..._MT256x256x32_MI16x16x1_..._MIWT8_8_..._WG32_8_1, profiles/r02). Forward layout only:
// C[M][N] = A[M][K] . B[N][K]^T, bf16 in, f32 accumulate, bf16 out; K % 32 == 0.
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/lab/gemm4w.hip -o tools/lab/libgemm4w.so
//   python tools/lab/gemm_lab.py --lib tools/lab/libgemm4w.so --variants 0,1 --shapes gate_up,lm_head,o
//
// BK = 32, three LDS stages of [256 rows][32 k] per operand (96 KiB), one barrier per K-tile.
// Step kt computes K-tile kt from fragments already in registers while it reads tile kt+1's
// fragments (registers of the other fragment set), writes or DMAs a later tile into the stage
// nobody reads, and issues the global loads of the tile after that.
//   variant 0: register staging (buffer_load_dwordx4 -> VGPR, ds_write_b128 one step later)
//   variants 1/2/3: LDS-DMA staging (buffer_load ... lds, counted vmcnt before the barrier) into
//   3/4/5 stages (tile kt+S issued at step kt: S-1 steps of latency budget)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

typedef unsigned short u16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 frag8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
#define DEV __device__ __forceinline__

namespace {

constexpr int BK = 32;
constexpr int OPB = 256 * BK * 2;  // 16 KiB per operand tile
constexpr int STAGE = 2 * OPB;
constexpr unsigned kOOB = 0x7FFFFFF0u;
// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8])
constexpr int kLgkm0 = 0xC07F;  // lgkmcnt(0)
constexpr int kVm8 = 0x0F78;    // vmcnt(8)
constexpr int kVm0 = 0x0F70;    // vmcnt(0)

// [256 rows][32 k] image, 64-B rows of four 16-B chunks; chunk c of row r sits in slot
// c ^ (3 * ((r >> 3) & 1)): conflict-free for ds_read_b128 fragment reads (lane l: row l & 15,
// chunk l >> 4) and for the staging writes (lanes 4r..4r+3: one row)
DEV int img(int row, int c) { return row * 64 + ((c ^ (((row >> 3) & 1) * 3)) << 4); }

DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

DEV __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

struct Frags {
  frag8 a[8], b[8];
};

// wait until at most n of this wave's LDS-DMA K-tiles (8 pieces each) are still in flight
DEV void wait_tiles(int n) {
  if (n <= 0) __builtin_amdgcn_s_waitcnt(0x0F70);       // vmcnt(0)
  else if (n == 1) __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8)
  else if (n == 2) __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
  else __builtin_amdgcn_s_waitcnt(0x4F78);              // vmcnt(24)
}

// sched_group_barrier masks
constexpr int kMFMA = 0x008, kDSR = 0x100, kDSW = 0x200, kVMR = 0x020;

// Round 3 (ASM variants): the MFMAs as inline asm with the accumulators constrained to AGPRs
// ("+a"), so hipcc keeps all 256 of them in the accumulator file and the two fragment sets in
// VGPRs instead of shuffling fragments through AGPRs (364 v_accvgpr moves per 128 MFMAs in the
// builtin version). Hazards (cdna_hip_programming.md "What hipcc does not do" item 2): the first
// K-step writes C from the literal 0 (no v_accvgpr_write -> MFMA pair); an accumulate chain on
// one register tuple needs no wait states; the last MFMAs' results get s_nop 11 (8-pass XDL: 12
// states) before the compiler's epilogue reads them.
DEV void mfma_acc(f32x4& c, const frag8& a, const frag8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
DEV void mfma_zero(f32x4& c, const frag8& a, const frag8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}

// AB: ablations (results wrong): 1 = no MFMAs (staging + fragment reads only), 2 = no staging
// (MFMAs + fragment reads of the prologue tiles only)
template <int V, int S, int IL, int AB = 0, int ASM = 0>
__global__ __launch_bounds__(256, 1) void g4w(const u16* __restrict__ A, const u16* __restrict__ B,
                                              u16* __restrict__ C, int M, int N, int K, int tiles_m, int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nwg = tiles_m * tiles_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  // groups of 4 N-tiles sweeping the M-tiles
  const int per_group = 4 * tiles_m;
  const int group = lid / per_group;
  const int first_n = group * 4;
  const int gsize = min(tiles_n - first_n, 4);
  const int n0 = (first_n + (lid % per_group) % gsize) * 256;
  const int m0 = ((lid % per_group) / gsize) * 256;

  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A, (int64_t)M * K * 2);
  const __amdgpu_buffer_rsrc_t rb = rsrc(B, (int64_t)N * K * 2);
  const int nk = K / BK;

  // staging geometry
  unsigned offA[4], offB[4];
  int lds_w[4];
  if constexpr (V != 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (t >> 2) + 64 * i, c = t & 3;
      offA[i] = m0 + row < M ? (unsigned)(((int64_t)(m0 + row) * K + c * 8) * 2) : kOOB;
      offB[i] = n0 + row < N ? (unsigned)(((int64_t)(n0 + row) * K + c * 8) * 2) : kOOB;
      lds_w[i] = img(row, c);
    }
  } else {
    // pieces wave + 4i (i = 0..3) of each operand: piece p = rows 16p..16p+15, lane l -> row
    // 16p + (l >> 2), slot l & 3 holding chunk (l & 3) ^ swz(row)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = wave + 4 * i;
      const int row = 16 * p + (lane >> 2);
      const int c = (lane & 3) ^ (((row >> 3) & 1) * 3);
      offA[i] = m0 + row < M ? (unsigned)(((int64_t)(m0 + row) * K + c * 8) * 2) : kOOB;
      offB[i] = n0 + row < N ? (unsigned)(((int64_t)(n0 + row) * K + c * 8) * 2) : kOOB;
      lds_w[i] = p * 1024;
    }
  }
  u32x4 st0[8], st1[8];
  // tiles >= nk read out of range (buffer loads return zeros): the staging ops stay unconditional,
  // in the MFMAs' basic block, where sched_group_barrier can interleave them
  auto gload = [&](int kt, u32x4 (&st)[8]) {
    const int so = kt * BK * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st[i] = __builtin_amdgcn_raw_buffer_load_b128(ra, offA[i], so, 0);
      st[4 + i] = __builtin_amdgcn_raw_buffer_load_b128(rb, offB[i], so, 0);
    }
  };
  auto swrite = [&](int kt, const u32x4 (&st)[8]) {
    char* s = smem + (kt % S) * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<u32x4*>(s + lds_w[i]) = st[i];
      *reinterpret_cast<u32x4*>(s + OPB + lds_w[i]) = st[4 + i];
    }
  };
  auto dma = [&](int kt) {
    char* s = smem + (kt % S) * STAGE;
    const int so = kt * BK * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(s + lds_w[i]), 16, offA[i], so, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(s + OPB + lds_w[i]), 16, offB[i], so, 0, 0);
    }
  };
  const int ra_row = wr * 128 + (lane & 15), rb_row = wc * 128 + (lane & 15), ch = lane >> 4;
  auto fread = [&](int kt, Frags& f) {
    const char* s = smem + (kt % S) * STAGE;
#pragma unroll
    for (int i = 0; i < 8; ++i) f.a[i] = *reinterpret_cast<const frag8*>(s + img(ra_row + i * 16, ch));
#pragma unroll
    for (int j = 0; j < 8; ++j) f.b[j] = *reinterpret_cast<const frag8*>(s + OPB + img(rb_row + j * 16, ch));
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: tiles 0 and 1 resident, the next ones on their way
  if constexpr (V == 0) {
    gload(0, st0);
    swrite(0, st0);
    gload(1, st0);
    swrite(1, st0);
    gload(2, st0);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
  } else if constexpr (V == 2) {
    gload(0, st0);
    swrite(0, st0);
    gload(1, st1);
    swrite(1, st1);
    gload(2, st0);
    gload(3, st1);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
  } else {
    // tiles 0 .. S-1 issued; tiles 0 and 1 must have landed
#pragma unroll
    for (int u = 0; u < S; ++u)
      if (u < nk) dma(u);
    wait_tiles(min(S, nk) - 2);
  }
  __builtin_amdgcn_s_barrier();
  Frags F0, F1;
  fread(0, F0);
  __builtin_amdgcn_s_waitcnt(kLgkm0);  // loop entry with no LDS op in flight (else the waitcnt
                                       // pass puts lgkmcnt(0) before every step's first MFMA)

  // step kt: MFMAs on tile kt (fragments in cur) with, under them, tile kt+1's fragment reads
  // into nxt and the staging of a later tile. P = kt & 1 (the 2-deep register staging's set).
  // ASM == 2: one wave per SIMD has no partner to hide its memory-instruction issue, so the step
  // spreads it over the MFMAs in program order (volatile asm MFMAs keep their place): before each
  // group of 8 MFMAs (one accumulator row) the two fragment reads of the next tile's row and one
  // LDS-DMA piece of tile kt+S
  auto step_il = [&](auto first_c, int kt, Frags& cur, Frags& nxt) {
    constexpr bool FIRST = decltype(first_c)::value;
    const char* rs = smem + ((kt + 1 < nk ? kt + 1 : kt) % S) * STAGE;
    char* ws = smem + ((kt + S) % S) * STAGE;
    const int so = (kt + S) * BK * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      nxt.a[i] = *reinterpret_cast<const frag8*>(rs + img(ra_row + i * 16, ch));
      nxt.b[i] = *reinterpret_cast<const frag8*>(rs + OPB + img(rb_row + i * 16, ch));
      if (i < 4) __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(ws + lds_w[i]), 16, offA[i], so, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(ws + OPB + lds_w[i - 4]), 16, offB[i - 4], so, 0, 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (FIRST) mfma_zero(acc[i][j], cur.b[j], cur.a[i]);
        else mfma_acc(acc[i][j], cur.b[j], cur.a[i]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    wait_tiles(S - 2);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();
  };
  // ASM == 2 with register staging (V == 2, 2 steps of latency): per group of 8 MFMAs the two
  // fragment reads, the LDS write of one piece of tile kt+2 (loaded two steps ago) and the global
  // load of that piece of tile kt+4 into the same registers
  auto step_il_reg = [&](auto first_c, int kt, Frags& cur, Frags& nxt, u32x4 (&stp)[8]) {
    constexpr bool FIRST = decltype(first_c)::value;
    const char* rs = smem + ((kt + 1 < nk ? kt + 1 : kt) % S) * STAGE;
    char* ws = smem + ((kt + 2) % S) * STAGE;
    const int so = (kt + 4) * BK * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      nxt.a[i] = *reinterpret_cast<const frag8*>(rs + img(ra_row + i * 16, ch));
      nxt.b[i] = *reinterpret_cast<const frag8*>(rs + OPB + img(rb_row + i * 16, ch));
      *reinterpret_cast<u32x4*>(ws + (i < 4 ? 0 : OPB) + lds_w[i & 3]) = stp[i];
      stp[i] = __builtin_amdgcn_raw_buffer_load_b128(i < 4 ? ra : rb, i < 4 ? offA[i] : offB[i - 4], so, 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (FIRST) mfma_zero(acc[i][j], cur.b[j], cur.a[i]);
        else mfma_acc(acc[i][j], cur.b[j], cur.a[i]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();
  };
  auto step = [&](auto first_c, int kt, Frags& cur, Frags& nxt, u32x4 (&stp)[8]) {
    constexpr bool FIRST = decltype(first_c)::value;
    if constexpr (ASM == 2 && V == 2) {
      step_il_reg(first_c, kt, cur, nxt, stp);
      return;
    } else if constexpr (ASM == 2) {
      step_il(first_c, kt, cur, nxt);
      return;
    }
    fread(AB == 2 ? (kt & 1) : kt + 1 < nk ? kt + 1 : kt, nxt);
    if constexpr (AB == 2) {
    } else if constexpr (V == 0) {
      swrite(kt + 2, st0);  // loaded last step (1 step of latency)
      gload(kt + 3, st0);
    } else if constexpr (V == 2) {
      swrite(kt + 2, stp);  // loaded two steps ago
      gload(kt + 4, stp);
    } else {
      dma(kt + S);  // into tile kt's stage: its fragments were read last step
    }
    if constexpr (AB == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(cur.a[i]), "v"(cur.b[i]));
    } else if constexpr (ASM) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if constexpr (FIRST) mfma_zero(acc[i][j], cur.b[j], cur.a[i]);
          else mfma_acc(acc[i][j], cur.b[j], cur.a[i]);
        }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur.b[j], cur.a[i], acc[i][j], 0, 0, 0);
    }
    if constexpr (IL) {
      // one memory op per MFMA gap: the wave (alone on its SIMD) issues them while the previous
      // MFMA occupies the matrix pipe, instead of in a burst with the pipe idle
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        __builtin_amdgcn_sched_group_barrier(kMFMA, 1, 0);
        __builtin_amdgcn_sched_group_barrier(kDSR, 1, 0);
        __builtin_amdgcn_sched_group_barrier(kMFMA, 1, 0);
        __builtin_amdgcn_sched_group_barrier(kDSR, 1, 0);
        __builtin_amdgcn_sched_group_barrier(kMFMA, 1, 0);
        if constexpr (V != 1) {
          __builtin_amdgcn_sched_group_barrier(kDSW, 1, 0);
          __builtin_amdgcn_sched_group_barrier(kMFMA, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(kVMR, 1, 0);
        __builtin_amdgcn_sched_group_barrier(kMFMA, V != 1 ? 4 : 5, 0);
      }
    }
    // keep the MFMAs on this side of the wait and the barrier (hipcc moves register-only MFMAs
    // across inline-asm waits, cdna_hip_programming.md rule 18): the LDS traffic issued above
    // runs under them
    __builtin_amdgcn_sched_barrier(0);
    // waits through the builtin, not inline asm: the compiler's waitcnt pass then knows the
    // fragments read above are retired and puts no lgkmcnt(0) in front of the next step's MFMAs
    if constexpr (V == 1 && AB != 2) {
      // tile kt + 2 (read next step) must have landed before this barrier; the newer ones fly
      wait_tiles(S - 2);
    }
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    __builtin_amdgcn_s_barrier();
  };
  using T0 = std::false_type;
  using T1 = std::true_type;
  int kt = 0;
  if constexpr (ASM) {
    // K-step 0 peeled (C from 0), then pairs from step 1: step kt reads fragment set kt & 1
    step(T1{}, 0, F0, F1, st0);
    kt = 1;
    for (; kt + 1 < nk; kt += 2) {
      step(T0{}, kt, F1, F0, st1);
      step(T0{}, kt + 1, F0, F1, st0);
    }
    if (kt < nk) step(T0{}, kt, F1, F0, st1);
    asm volatile("s_nop 11" : "+a"(acc[7][7]), "+a"(acc[7][6]), "+a"(acc[7][5]), "+a"(acc[7][4]),
                 "+a"(acc[7][3]), "+a"(acc[7][2]), "+a"(acc[7][1]), "+a"(acc[7][0]));
  } else {
    for (; kt + 1 < nk; kt += 2) {
      step(T0{}, kt, F0, F1, st0);
      step(T0{}, kt + 1, F1, F0, st1);
    }
    if (kt < nk) step(T0{}, kt, F0, F1, st0);
  }

#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + wc * 128 + j * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      const bf16x4 v = __builtin_convertvector(acc[i][j], bf16x4);
      *reinterpret_cast<bf16x4*>(C + (int64_t)m * N + n) = v;
    }
  }
}

template <int V, int S, int IL, int AB = 0, int ASM = 0>
int launch(int M, int N, int K, const void* A, const void* B, void* C, hipStream_t s) {
  const int smem = S * STAGE;
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)g4w<V, S, IL, AB, ASM>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    set = true;
  }
  const int tm = (M + 255) / 256, tn = (N + 255) / 256;
  g4w<V, S, IL, AB, ASM><<<tm * tn, 256, smem, s>>>((const u16*)A, (const u16*)B, (u16*)C, M, N, K, tm, tn);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace

extern "C" int lab_gemm(int v, int64_t M, int64_t N, int64_t K, const void* A, const void* B, void* C, void* stream) {
  if (K % BK) return 2;
  hipStream_t s = (hipStream_t)stream;
  switch (v) {
    case 0: return launch<0, 3, 0>((int)M, (int)N, (int)K, A, B, C, s);
    case 1: return launch<1, 3, 0>((int)M, (int)N, (int)K, A, B, C, s);
    case 2: return launch<1, 4, 0>((int)M, (int)N, (int)K, A, B, C, s);
    case 3: return launch<1, 5, 0>((int)M, (int)N, (int)K, A, B, C, s);
    case 4: return launch<1, 4, 1>((int)M, (int)N, (int)K, A, B, C, s);  // DMA, interleaved
    case 5: return launch<2, 3, 1>((int)M, (int)N, (int)K, A, B, C, s);  // registers 2-deep, interleaved
    case 6: return launch<2, 3, 0>((int)M, (int)N, (int)K, A, B, C, s);  // registers 2-deep
    case 7: return launch<0, 3, 1>((int)M, (int)N, (int)K, A, B, C, s);  // registers 1-deep, interleaved
    case 8: return launch<1, 4, 0, 1>((int)M, (int)N, (int)K, A, B, C, s);   // DMA staging alone (wrong)
    case 9: return launch<2, 3, 0, 1>((int)M, (int)N, (int)K, A, B, C, s);   // register staging alone (wrong)
    case 10: return launch<1, 4, 0, 2>((int)M, (int)N, (int)K, A, B, C, s);  // MFMA + fragment reads alone (wrong)
    // round 3: accumulators pinned to AGPRs (inline-asm MFMAs)
    case 11: return launch<1, 3, 0, 0, 1>((int)M, (int)N, (int)K, A, B, C, s);  // DMA, 3 stages
    case 12: return launch<1, 4, 0, 0, 1>((int)M, (int)N, (int)K, A, B, C, s);  // DMA, 4 stages
    case 13: return launch<1, 5, 0, 0, 1>((int)M, (int)N, (int)K, A, B, C, s);  // DMA, 5 stages
    case 14: return launch<2, 3, 0, 0, 1>((int)M, (int)N, (int)K, A, B, C, s);  // registers 2-deep
    case 15: return launch<1, 4, 0, 2, 1>((int)M, (int)N, (int)K, A, B, C, s);  // MFMA + fragment reads alone (wrong)
    case 16: return launch<1, 3, 0, 0, 2>((int)M, (int)N, (int)K, A, B, C, s);  // DMA 3 stages, interleaved by hand
    case 17: return launch<1, 4, 0, 0, 2>((int)M, (int)N, (int)K, A, B, C, s);  // DMA 4 stages, interleaved by hand
    case 18: return launch<1, 5, 0, 0, 2>((int)M, (int)N, (int)K, A, B, C, s);  // DMA 5 stages, interleaved by hand
    case 19: return launch<2, 3, 0, 0, 2>((int)M, (int)N, (int)K, A, B, C, s);  // registers 2-deep, interleaved by hand
  }
  return 3;
}
