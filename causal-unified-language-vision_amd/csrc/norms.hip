// RMSNorm (Llama) and LayerNorm (CLIP) forward/backward for gfx950.
// HBM-bound: one wave64 per row, 16 B per lane per access, the row held in registers between
// the statistics pass and the normalise pass (rows up to 8192 columns).
// Reference arithmetic: tf:llama/modeling_llama.py:53-70 (LlamaRMSNorm: f32 statistics,
// weight * x_hat.to(bf16)), torch.nn.LayerNorm as used by tf:clip/modeling_clip.py:353-384,642.
#include "common.h"

namespace {

constexpr int kRowsPerBlock = 4;   // 4 waves, one row each
constexpr int kBwdBlocks = 256;    // backward grid (weight-grad partials: 1024 wave slots)

// ------------------------------------------------------------------------------------------
// PREW (few rows: the KV-cache decode step's one row per sequence): the weight row is loaded
// together with x, before the reduction, so a launch waits out one memory round trip instead of
// two (7.4 us per decode-step norm at one row; the many-row training launches keep the registers)
template <typename T, int NCH, bool PREW = false>
__global__ __launch_bounds__(256) void rmsnorm_fwd_k(const T* __restrict__ x, const T* __restrict__ w,
                                                     T* __restrict__ y, float* __restrict__ rstd,
                                                     int64_t rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * cols;
  float v[NCH][8];
  float wp[PREW ? NCH : 1][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols) {
      load8(xr + col, v[c]);
      if constexpr (PREW) load8(w + col, wp[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)cols + eps);
  if (lane == 0) rstd[row] = r;
  T* yr = y + row * cols;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols) {
      float wv[8], o[8];
      if constexpr (PREW) {
#pragma unroll
        for (int j = 0; j < 8; ++j) wv[j] = wp[c][j];
      } else {
        load8(w + col, wv);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = wv[j] * Elt<T>::rnd(v[c][j] * r);
      store8(yr + col, o);
    }
  }
}

template <typename T, int NCH, bool WANT_DW, bool HAS_DRES>
__global__ __launch_bounds__(256) void rmsnorm_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const T* __restrict__ w, const float* __restrict__ rstd,
                                                     T* __restrict__ dx, const T* __restrict__ dres,
                                                     float* __restrict__ part, int64_t rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int wslot = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  const int nslots = gridDim.x * kRowsPerBlock;
  float acc[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  float wv[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols) load8(w + col, wv[c]);
  }
  for (int64_t row = wslot; row < rows; row += nslots) {
    const float r = rstd[row];
    float xv[NCH][8], g[NCH][8];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < cols) {
        float d[8];
        load8(x + row * cols + col, xv[c]);
        load8(dy + row * cols + col, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = xv[c][j] * r;
          g[c][j] = d[j] * wv[c][j];
          dot += g[c][j] * xh;
          if (WANT_DW) acc[c][j] += d[j] * Elt<T>::rnd(xh);
        }
      }
    }
    dot = wave_sum(dot) / (float)cols;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < cols) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = r * (g[c][j] - xv[c][j] * r * dot);
        if (HAS_DRES) {
          float rr[8];
          load8(dres + row * cols + col, rr);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rr[j];
        }
        store8(dx + row * cols + col, o);
      }
    }
  }
  if (WANT_DW) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < cols) store8(part + (int64_t)wslot * cols + col, acc[c]);
    }
  }
}

// RMSNorm backward, production form: 8-wave workgroups (two per CU) over contiguous row chunks,
// two waves per row, the row's x, dy and dres loads issued together, dw accumulated per wave in
// registers and folded per workgroup through LDS in slot order (deterministic) into ONE partial
// row per workgroup (<= 512 partial rows).
constexpr int kBwd8Blocks = 512;

// 8 raw elements kept in their storage type until used (register budget of 8-wave blocks)
template <typename T> struct Raw8;
template <> struct Raw8<u16> {
  u16x8 v;
  DEV void load(const u16* p) { v = *reinterpret_cast<const u16x8*>(p); }
  DEV float operator[](int j) const { return bf2f(v[j]); }
};
template <> struct Raw8<float> {
  f32x4 a, b;
  DEV void load(const float* p) {
    a = *reinterpret_cast<const f32x4*>(p);
    b = *reinterpret_cast<const f32x4*>(p + 4);
  }
  DEV float operator[](int j) const { return j < 4 ? a[j] : b[j - 4]; }
};

template <typename T, int NCH, bool WANT_DW, bool HAS_DRES>
__global__ __launch_bounds__(512, WANT_DW ? 2 : 4) void rmsnorm_bwd8_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                         const T* __restrict__ w, const float* __restrict__ rstd,
                                                         T* __restrict__ dx, const T* __restrict__ dres,
                                                         float* __restrict__ part, int64_t rows, int cols,
                                                         int64_t rows_per_block) {
  // two waves per row (wave = 2*slot + half; half h owns the 512-column chunks c = h, h+2, ...),
  // four rows in flight per workgroup, the row's dot product combined through LDS
  constexpr int NH = (NCH + 1) / 2;  // chunks per half
  extern __shared__ float sdw[];     // [cols] when WANT_DW
  __shared__ float pdot[2][4][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = wave >> 1, half = wave & 1;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float acc[NH][8];
#pragma unroll
  for (int c = 0; c < NH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  const int iters = (int)cdiv(r1 - r0, (int64_t)4);
  for (int it = 0; it < iters; ++it) {
    const int64_t row = r0 + 4 * it + slot;
    const bool live = row < r1;
    const float r = live ? rstd[row] : 0.f;
    Raw8<T> xr[NH], dr[NH], rr[NH];
#pragma unroll
    for (int c = 0; c < NH; ++c) {
      const int col = (2 * c + half) * 512 + lane * 8;
      if (live && 2 * c + half < NCH && col < cols) {
        xr[c].load(x + row * cols + col);
        dr[c].load(dy + row * cols + col);
        if (HAS_DRES) rr[c].load(dres + row * cols + col);
      }
    }
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NH; ++c) {
      const int col = (2 * c + half) * 512 + lane * 8;
      if (live && 2 * c + half < NCH && col < cols) {
        Raw8<T> wr;
        wr.load(w + col);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = xr[c][j] * r;
          dot += dr[c][j] * wr[j] * xh;
          if (WANT_DW) acc[c][j] += dr[c][j] * Elt<T>::rnd(xh);
        }
      }
    }
    dot = wave_sum(dot);
    if (lane == 0) pdot[it & 1][slot][half] = dot;
    __syncthreads();
    dot = (pdot[it & 1][slot][0] + pdot[it & 1][slot][1]) / (float)cols;
#pragma unroll
    for (int c = 0; c < NH; ++c) {
      const int col = (2 * c + half) * 512 + lane * 8;
      if (live && 2 * c + half < NCH && col < cols) {
        Raw8<T> wr;
        wr.load(w + col);
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o[j] = r * (dr[c][j] * wr[j] - xr[c][j] * r * dot);
          if (HAS_DRES) o[j] += rr[c][j];
        }
        store8(dx + row * cols + col, o);
      }
    }
  }
  if (WANT_DW) {  // fold the four row slots in order; the two halves own disjoint columns
    for (int sl = 0; sl < 4; ++sl) {
      if (slot == sl) {
#pragma unroll
        for (int c = 0; c < NH; ++c) {
          const int col = (2 * c + half) * 512 + lane * 8;
          if (2 * c + half < NCH && col < cols)
#pragma unroll
            for (int j = 0; j < 8; ++j) sdw[col + j] = (sl == 0 ? 0.f : sdw[col + j]) + acc[c][j];
        }
      }
      __syncthreads();
    }
    for (int col = threadIdx.x; col < cols; col += 512) part[(int64_t)blockIdx.x * cols + col] = sdw[col];
  }
}

// Pipelined form (the default with dw since round 2): one 8-wave workgroup per CU, two register sets,
// so the next rows' x / dy / dres loads are in flight while the current rows run their two
// passes, the dot-product barrier and their stores (rmsnorm_bwd8_k drains the loads at every
// iteration). Four waves per row (wave part p owns the 512-column chunks p, p+4, ...), two rows
// per iteration, so two register sets fit without spilling at 4096 columns. Per-element
// arithmetic is rmsnorm_bwd8_k's; the row's dot product adds its four wave partials in order
// (dx differs from rmsnorm_bwd8_k only in that sum's order); dw folds 256 partial rows in a fixed
// order (deterministic).
constexpr int kBwd8pBlocks = 256;
constexpr int kWpr = 4;             // waves per row
constexpr int kSlots = 8 / kWpr;    // rows per iteration

template <typename T, int NH, bool HAS_DRES>
struct BwdRows {
  Raw8<T> xr[NH], dr[NH], rr[NH];
  float r;
  DEV void load(const T* x, const T* dy, const T* dres, const float* rstd, int64_t row, bool live, int part,
                int lane, int nch, int cols) {
    r = live ? rstd[row] : 0.f;
#pragma unroll
    for (int c = 0; c < NH; ++c) {
      const int col = (kWpr * c + part) * 512 + lane * 8;
      if (live && kWpr * c + part < nch && col < cols) {
        xr[c].load(x + row * cols + col);
        dr[c].load(dy + row * cols + col);
        if (HAS_DRES) rr[c].load(dres + row * cols + col);
      }
    }
  }
};

template <typename T, int NCH, bool WANT_DW, bool HAS_DRES>
__global__ __launch_bounds__(512, 1) void rmsnorm_bwd8p_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const T* __restrict__ w, const float* __restrict__ rstd,
                                                          T* __restrict__ dx, const T* __restrict__ dres,
                                                          float* __restrict__ part, int64_t rows, int cols,
                                                          int64_t rows_per_block) {
  constexpr int NH = (NCH + kWpr - 1) / kWpr;
  extern __shared__ float sdw[];
  __shared__ float pdot[2][kSlots][kWpr];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int slot = wave / kWpr, wp = wave % kWpr;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(rows, r0 + rows_per_block);
  float acc[NH][8];
#pragma unroll
  for (int c = 0; c < NH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  const int iters = (int)cdiv(max(r1 - r0, (int64_t)0), (int64_t)kSlots);

  auto body = [&](const BwdRows<T, NH, HAS_DRES>& cur, int it) {
    const int64_t row = r0 + kSlots * it + slot;
    const bool live = row < r1;
    const float r = cur.r;
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NH; ++c) {
      const int col = (kWpr * c + wp) * 512 + lane * 8;
      if (live && kWpr * c + wp < NCH && col < cols) {
        Raw8<T> wr;
        wr.load(w + col);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = cur.xr[c][j] * r;
          dot += cur.dr[c][j] * wr[j] * xh;
          if (WANT_DW) acc[c][j] += cur.dr[c][j] * Elt<T>::rnd(xh);
        }
      }
    }
    dot = wave_sum(dot);
    if (lane == 0) pdot[it & 1][slot][wp] = dot;
    __syncthreads();
    dot = 0.f;
#pragma unroll
    for (int i = 0; i < kWpr; ++i) dot += pdot[it & 1][slot][i];
    dot /= (float)cols;
#pragma unroll
    for (int c = 0; c < NH; ++c) {
      const int col = (kWpr * c + wp) * 512 + lane * 8;
      if (live && kWpr * c + wp < NCH && col < cols) {
        Raw8<T> wr;
        wr.load(w + col);
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          o[j] = r * (cur.dr[c][j] * wr[j] - cur.xr[c][j] * r * dot);
          if (HAS_DRES) o[j] += cur.rr[c][j];
        }
        store8(dx + row * cols + col, o);
      }
    }
  };
  auto load = [&](BwdRows<T, NH, HAS_DRES>& dst, int it) {
    const int64_t row = r0 + kSlots * it + slot;
    dst.load(x, dy, dres, rstd, row, it < iters && row < r1, wp, lane, NCH, cols);
  };

  BwdRows<T, NH, HAS_DRES> ra, rb;
  load(ra, 0);
  for (int it = 0; it < iters; it += 2) {
    load(rb, it + 1);  // rows of the next iteration in flight under this one
    body(ra, it);
    if (it + 1 >= iters) break;
    load(ra, it + 2);
    body(rb, it + 1);
  }
  if (WANT_DW) {  // fold the row slots in order; the parts of a row own disjoint columns
    for (int sl = 0; sl < kSlots; ++sl) {
      if (slot == sl) {
#pragma unroll
        for (int c = 0; c < NH; ++c) {
          const int col = (kWpr * c + wp) * 512 + lane * 8;
          if (kWpr * c + wp < NCH && col < cols)
#pragma unroll
            for (int j = 0; j < 8; ++j) sdw[col + j] = (sl == 0 ? 0.f : sdw[col + j]) + acc[c][j];
        }
      }
      __syncthreads();
    }
    for (int col = threadIdx.x; col < cols; col += 512) part[(int64_t)blockIdx.x * cols + col] = sdw[col];
  }
}

// ------------------------------------------------------------------------------------------
template <typename T, int NCH>
__global__ __launch_bounds__(256) void layernorm_fwd_k(const T* __restrict__ x, const T* __restrict__ w,
                                                       const T* __restrict__ b, T* __restrict__ y,
                                                       float* __restrict__ mean_out,
                                                       float* __restrict__ rstd_out, int64_t rows,
                                                       int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * cols;
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols) {
      load8(xr + col, v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    }
  }
  const float mean = wave_sum(s) / (float)cols;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[c][j] - mean;
        ss += d * d;
      }
    }
  }
  const float r = rsqrtf(wave_sum(ss) / (float)cols + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = r;
  }
  T* yr = y + row * cols;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols) {
      float wv[8], bv[8], o[8];
      load8(w + col, wv);
      load8(b + col, bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * r * wv[j] + bv[j];
      store8(yr + col, o);
    }
  }
}

template <typename T, int NCH, bool WANT_DW, bool HAS_DRES>
__global__ __launch_bounds__(256) void layernorm_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const T* __restrict__ w,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       T* __restrict__ dx, const T* __restrict__ dres,
                                                       float* __restrict__ part, int64_t rows,
                                                       int cols) {
  const int lane = threadIdx.x & 63;
  const int wslot = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  const int nslots = gridDim.x * kRowsPerBlock;
  float accw[NCH][8], accb[NCH][8], wv[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
#pragma unroll
    for (int j = 0; j < 8; ++j) accw[c][j] = accb[c][j] = 0.f;
    const int col = c * 512 + lane * 8;
    if (col < cols) load8(w + col, wv[c]);
  }
  for (int64_t row = wslot; row < rows; row += nslots) {
    const float mu = mean[row], r = rstd[row];
    float xh[NCH][8], g[NCH][8];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < cols) {
        float d[8];
        load8(x + row * cols + col, xh[c]);
        load8(dy + row * cols + col, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] = (xh[c][j] - mu) * r;
          g[c][j] = d[j] * wv[c][j];
          sg += g[c][j];
          sgx += g[c][j] * xh[c][j];
          if (WANT_DW) {
            accw[c][j] += d[j] * xh[c][j];
            accb[c][j] += d[j];
          }
        }
      }
    }
    sg = wave_sum(sg) / (float)cols;
    sgx = wave_sum(sgx) / (float)cols;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < cols) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = r * (g[c][j] - sg - xh[c][j] * sgx);
        if (HAS_DRES) {
          float rr[8];
          load8(dres + row * cols + col, rr);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rr[j];
        }
        store8(dx + row * cols + col, o);
      }
    }
  }
  if (WANT_DW) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < cols) {
        store8(part + (int64_t)wslot * cols + col, accw[c]);
        store8(part + ((int64_t)nslots + wslot) * cols + col, accb[c]);
      }
    }
  }
}

// partial [nslots, cols] f32 -> out[c] = beta*out[c] + sum_p part[p][c]
// block = 64 columns x 16 slot groups (coalesced 256 B row segments), fixed summation order
template <typename TO>
__global__ __launch_bounds__(1024) void reduce_partials_k(const float* __restrict__ part, int nslots,
                                                          int cols, TO* __restrict__ out, float beta) {
  __shared__ float red[16][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c;
  float s = 0.f;
  if (col < cols)
    for (int p = g; p < nslots; p += 16) s += part[(int64_t)p * cols + col];
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && col < cols) {
    s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[i][c];
    if (beta != 0.f) s += beta * Elt<TO>::ld(out, col);
    Elt<TO>::st(out, col, s);
  }
}

int nch_for(int64_t cols) {
  if (cols <= 512) return 1;
  if (cols <= 1024) return 2;
  if (cols <= 2048) return 4;
  if (cols <= 4096) return 8;
  if (cols <= 6144) return 12;  // Llama-2-13B's 5120: three chunks per wave in the 4-waves-per-row kernel
  return 16;
}

#define NCH_DISPATCH(nch, ...)               \
  switch (nch) {                             \
    case 1: { constexpr int NC = 1; __VA_ARGS__; break; } \
    case 2: { constexpr int NC = 2; __VA_ARGS__; break; } \
    case 4: { constexpr int NC = 4; __VA_ARGS__; break; } \
    case 8: { constexpr int NC = 8; __VA_ARGS__; break; } \
    case 12: { constexpr int NC = 12; __VA_ARGS__; break; } \
    default: { constexpr int NC = 16; __VA_ARGS__; break; } \
  }

template <typename TO>
void launch_reduce(const float* part, int nslots, int cols, void* out, float beta, hipStream_t s) {
  reduce_partials_k<TO><<<cdiv(cols, 64), 1024, 0, s>>>(part, nslots, cols, (TO*)out, beta);
}

int bwd_blocks(int64_t rows) { return (int)std::min<int64_t>(kBwdBlocks, cdiv(rows, kRowsPerBlock)); }

}  // namespace

extern "C" size_t cullavo_norm_bwd_workspace(int64_t rows, int64_t cols) {
  return (size_t)2 * kBwdBlocks * kRowsPerBlock * cols * sizeof(float);
}

extern "C" int cullavo_rmsnorm_fwd(const void* x, const void* w, void* y, float* rstd, int64_t rows,
                                   int64_t cols, float eps, int dtype, void* stream) {
  CV_REQUIRE(cols % 8 == 0 && cols > 0 && cols <= 8192, CULLAVO_EINVAL, "cols must be a multiple of 8 in [8, 8192]");
  CV_REQUIRE(rows >= 0, CULLAVO_EINVAL, "rows < 0");
  if (rows == 0) return CULLAVO_OK;
  const int nb = (int)cdiv(rows, kRowsPerBlock);
  hipStream_t s = CV_STREAM(stream);
  const int nch = nch_for(cols);
  if (dtype == CULLAVO_DT_BF16 && rows <= 64 && nch <= 8) {
    NCH_DISPATCH(nch, rmsnorm_fwd_k<u16, NC, true><<<nb, 256, 0, s>>>((const u16*)x, (const u16*)w, (u16*)y, rstd, rows, (int)cols, eps));
  } else if (dtype == CULLAVO_DT_BF16) {
    NCH_DISPATCH(nch, rmsnorm_fwd_k<u16, NC><<<nb, 256, 0, s>>>((const u16*)x, (const u16*)w, (u16*)y, rstd, rows, (int)cols, eps));
  } else if (dtype == CULLAVO_DT_F32) {
    NCH_DISPATCH(nch, rmsnorm_fwd_k<float, NC><<<nb, 256, 0, s>>>((const float*)x, (const float*)w, (float*)y, rstd, rows, (int)cols, eps));
  } else {
    CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  }
  return cullavo_check_launch("rmsnorm_fwd");
}

static int g_rms_bwd_mode = 1;  // 1 = pipelined 8-wave kernel (default), 0 = rmsnorm_bwd8_k

extern "C" int cullavo_rmsnorm_set_bwd(int mode) {
  const int prev = g_rms_bwd_mode;
  if (mode == 0 || mode == 1) g_rms_bwd_mode = mode;
  return prev;
}

extern "C" int cullavo_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd,
                                   void* dx, const void* dres, void* dw, int w_dtype, float beta, float* ws,
                                   int64_t rows, int64_t cols, int dtype, void* stream) {
  CV_REQUIRE(cols % 8 == 0 && cols > 0 && cols <= 8192, CULLAVO_EINVAL, "cols must be a multiple of 8 in [8, 8192]");
  CV_REQUIRE(dw == nullptr || ws != nullptr, CULLAVO_EINVAL, "dw requires a workspace");
  if (rows == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const int nch = nch_for(cols);
  const bool want = dw != nullptr, hr = dres != nullptr;
  // more than 4096 columns (Llama-2-13B's 5120): the pipelined kernel with four waves per row
  // (at most 4 x 8 bf16 per lane per tensor and register set); the round-1 one-wave-per-row kernel
  // held 16 chunks of three tensors per lane and streamed 6400 x 5120 at 1.75 TB/s (config 5)
  const bool wide = nch > 8 && g_rms_bwd_mode == 0;
  // up to 4096 columns the pipelined kernel only pays when dw is wanted (measured,
  // tools/norm_bench.py: without dw the round-1 kernel's four waves per SIMD stream at ~5.8 TB/s)
  const bool pipe = !wide && g_rms_bwd_mode == 1 && (want || nch > 8);
  const int nb = wide ? bwd_blocks(rows) : (int)std::min<int64_t>(pipe ? kBwd8pBlocks : kBwd8Blocks, cdiv(rows, 4));
  const int64_t rpb = cdiv(rows, nb);
  const size_t lds = want ? (size_t)cols * sizeof(float) : 0;
#define RMB(T, WD, HR)                                                                                        \
  if (wide) rmsnorm_bwd_k<T, 16, WD, HR><<<nb, 256, 0, s>>>((const T*)dy, (const T*)x, (const T*)w, rstd, (T*)dx, (const T*)dres, ws, rows, (int)cols); \
  else if (pipe) NCH_DISPATCH(nch, rmsnorm_bwd8p_k<T, NC, WD, HR><<<nb, 512, lds, s>>>((const T*)dy, (const T*)x, (const T*)w, rstd, (T*)dx, (const T*)dres, ws, rows, (int)cols, rpb)) \
  else NCH_DISPATCH(nch, rmsnorm_bwd8_k<T, (NC > 8 ? 8 : NC), WD, HR><<<nb, 512, lds, s>>>((const T*)dy, (const T*)x, (const T*)w, rstd, (T*)dx, (const T*)dres, ws, rows, (int)cols, rpb))
  if (dtype == CULLAVO_DT_BF16) {
    if (want && hr) { RMB(u16, true, true); } else if (want) { RMB(u16, true, false); }
    else if (hr) { RMB(u16, false, true); } else { RMB(u16, false, false); }
  } else if (dtype == CULLAVO_DT_F32) {
    if (want && hr) { RMB(float, true, true); } else if (want) { RMB(float, true, false); }
    else if (hr) { RMB(float, false, true); } else { RMB(float, false, false); }
  } else {
    CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  }
#undef RMB
  if (want) {
    const int nslots = wide ? nb * kRowsPerBlock : nb;
    if (w_dtype == CULLAVO_DT_BF16) launch_reduce<u16>(ws, nslots, (int)cols, dw, beta, s);
    else launch_reduce<float>(ws, nslots, (int)cols, dw, beta, s);
  }
  return cullavo_check_launch("rmsnorm_bwd");
}

extern "C" int cullavo_layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean,
                                     float* rstd, int64_t rows, int64_t cols, float eps, int dtype,
                                     void* stream) {
  CV_REQUIRE(cols % 8 == 0 && cols > 0 && cols <= 8192, CULLAVO_EINVAL, "cols must be a multiple of 8 in [8, 8192]");
  if (rows == 0) return CULLAVO_OK;
  const int nb = (int)cdiv(rows, kRowsPerBlock);
  hipStream_t s = CV_STREAM(stream);
  const int nch = nch_for(cols);
  if (dtype == CULLAVO_DT_BF16) {
    NCH_DISPATCH(nch, layernorm_fwd_k<u16, NC><<<nb, 256, 0, s>>>((const u16*)x, (const u16*)w, (const u16*)b, (u16*)y, mean, rstd, rows, (int)cols, eps));
  } else if (dtype == CULLAVO_DT_F32) {
    NCH_DISPATCH(nch, layernorm_fwd_k<float, NC><<<nb, 256, 0, s>>>((const float*)x, (const float*)w, (const float*)b, (float*)y, mean, rstd, rows, (int)cols, eps));
  } else {
    CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  }
  return cullavo_check_launch("layernorm_fwd");
}

extern "C" int cullavo_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean,
                                     const float* rstd, void* dx, const void* dres, void* dw, void* db,
                                     int w_dtype, float beta, float* ws, int64_t rows, int64_t cols,
                                     int dtype, void* stream) {
  CV_REQUIRE(cols % 8 == 0 && cols > 0 && cols <= 8192, CULLAVO_EINVAL, "cols must be a multiple of 8 in [8, 8192]");
  CV_REQUIRE((dw == nullptr) == (db == nullptr), CULLAVO_EINVAL, "dw and db must both be given or both be null");
  CV_REQUIRE(dw == nullptr || ws != nullptr, CULLAVO_EINVAL, "dw requires a workspace");
  if (rows == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const int nb = bwd_blocks(rows);
  const int nch = nch_for(cols);
  const bool want = dw != nullptr, hr = dres != nullptr;
#define LNB(T, WD, HR) NCH_DISPATCH(nch, layernorm_bwd_k<T, NC, WD, HR><<<nb, 256, 0, s>>>((const T*)dy, (const T*)x, (const T*)w, mean, rstd, (T*)dx, (const T*)dres, ws, rows, (int)cols))
  if (dtype == CULLAVO_DT_BF16) {
    if (want && hr) { LNB(u16, true, true); } else if (want) { LNB(u16, true, false); }
    else if (hr) { LNB(u16, false, true); } else { LNB(u16, false, false); }
  } else if (dtype == CULLAVO_DT_F32) {
    if (want && hr) { LNB(float, true, true); } else if (want) { LNB(float, true, false); }
    else if (hr) { LNB(float, false, true); } else { LNB(float, false, false); }
  } else {
    CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  }
#undef LNB
  if (want) {
    const int nslots = nb * kRowsPerBlock;
    if (w_dtype == CULLAVO_DT_BF16) {
      launch_reduce<u16>(ws, nslots, (int)cols, dw, beta, s);
      launch_reduce<u16>(ws + (int64_t)nslots * cols, nslots, (int)cols, db, beta, s);
    } else {
      launch_reduce<float>(ws, nslots, (int)cols, dw, beta, s);
      launch_reduce<float>(ws + (int64_t)nslots * cols, nslots, (int)cols, db, beta, s);
    }
  }
  return cullavo_check_launch("layernorm_bwd");
}
