// Token embedding gather / deterministic scatter-add, the CLIP patch-embedding front end
// (im2col + CLS/pos + pre_layrnorm) and the llava image/text merge (index plan + row gather).
// All integer/byte work is HBM-bound row movement: one block per row, 16 B per lane.
#include "common.h"

namespace {

// ---- embedding (reference cullavo/arch_cullavo.py:582; tf nn.Embedding) ---------------------
__global__ __launch_bounds__(256) void embedding_fwd_k(const int64_t* __restrict__ ids, const u16* __restrict__ table,
                                                       int64_t vocab, int64_t dim, u16* __restrict__ out) {
  const int64_t i = blockIdx.x;
  const int64_t id = ids[i];
  const bool ok = id >= 0 && id < vocab;
  for (int64_t c = threadIdx.x; c < dim / 8; c += 256) {
    u16x8 v = ok ? *reinterpret_cast<const u16x8*>(table + id * dim + c * 8) : u16x8(0);
    *reinterpret_cast<u16x8*>(out + i * dim + c * 8) = v;
  }
}

// One block per token position i. The block that holds the FIRST occurrence of ids[i] sums
// every dout row with the same id in increasing position order (bitwise reproducible) and
// writes that table row once; later occurrences exit.
template <typename TT, typename TD>
__global__ __launch_bounds__(256) void embedding_bwd_k(const int64_t* __restrict__ ids, int64_t n,
                                                       const TD* __restrict__ dout, int64_t vocab,
                                                       int64_t dim, TT* __restrict__ dtable, float beta) {
  __shared__ int64_t first;
  __shared__ int match[256];
  __shared__ int nmatch;
  const int64_t i = blockIdx.x;
  const int64_t id = ids[i];
  if (id < 0 || id >= vocab) return;
  if (threadIdx.x == 0) first = n;
  __syncthreads();
  for (int64_t j = threadIdx.x; j <= i; j += 256)
    if (ids[j] == id) atomicMin((unsigned long long*)&first, (unsigned long long)j);
  __syncthreads();
  if (first != i) return;
  constexpr int kMaxC = 4;  // dim <= 8192
  float acc[kMaxC][8];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[c][e] = 0.f;
  const int nch = (int)(dim / 8);
  for (int64_t base = i; base < n; base += 256) {
    if (threadIdx.x == 0) nmatch = 0;
    __syncthreads();
    const int64_t j = base + threadIdx.x;
    const bool hit = j < n && ids[j] == id;
    // ordered compaction: ballot per wave, prefix over the 4 waves
    const unsigned long long bal = __ballot(hit);
    __shared__ int wcount[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) wcount[w] = __popcll(bal);
    __syncthreads();
    int off = 0;
    for (int k = 0; k < w; ++k) off += wcount[k];
    if (hit) match[off + __popcll(bal & ((1ull << lane) - 1ull))] = threadIdx.x;
    if (threadIdx.x == 0) nmatch = wcount[0] + wcount[1] + wcount[2] + wcount[3];
    __syncthreads();
    for (int m = 0; m < nmatch; ++m) {
      const int64_t row = base + match[m];
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) {
        const int ch = threadIdx.x + c * 256;
        if (ch < nch) {
          float v[8];
          load8(dout + row * dim + ch * 8, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[c][e] += v[e];
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) {
    const int ch = threadIdx.x + c * 256;
    if (ch < nch) {
      TT* dst = dtable + id * dim + ch * 8;
      if (beta != 0.f) {
        float o[8];
        load8(dst, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[c][e] += beta * o[e];
      }
      store8(dst, acc[c]);
    }
  }
}

// ---- CLIP patch embedding (tf:clip/modeling_clip.py:202-218) -------------------------------
template <typename TP, typename TO>
__global__ __launch_bounds__(256) void im2col_k(const TP* __restrict__ pix, int C, int H, int W, int patch,
                                                int gw, int P, TO* __restrict__ out, int64_t kpad) {
  const int64_t r = blockIdx.x;  // output row in [B*(1+P)]
  const int b = (int)(r / (1 + P));
  const int t = (int)(r % (1 + P));
  TO* o = out + r * kpad;
  const int kreal = C * patch * patch;
  for (int64_t c = threadIdx.x; c < kpad; c += 256) {
    float v = 0.f;
    if (t > 0 && c < kreal) {
      const int p = t - 1, py = p / gw, px = p % gw;
      const int ch = (int)(c / (patch * patch)), rem = (int)(c % (patch * patch));
      const int i = rem / patch, j = rem % patch;
      v = Elt<TP>::ld(pix, (((int64_t)b * C + ch) * H + (py * patch + i)) * W + px * patch + j);
    }
    Elt<TO>::st(o, c, v);  // the reference casts pixel_values to the conv weight dtype first
  }
}

template <typename TE, int NCH>
__global__ __launch_bounds__(256) void vision_embed_ln_k(const TE* __restrict__ x, const TE* __restrict__ cls,
                                                         const TE* __restrict__ pos, const TE* __restrict__ w,
                                                         const TE* __restrict__ b, TE* __restrict__ y,
                                                         int64_t rows, int T, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int t = (int)(row % T);
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols) {
      float pv[8];
      load8(x + row * cols + col, v[c]);
      load8(pos + (int64_t)t * cols + col, pv);
      if (t == 0) {
        float cv[8];
        load8(cls + col, cv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = Elt<TE>::rnd(cv[j] + pv[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = Elt<TE>::rnd(v[c][j] + pv[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    }
  }
  const float mean = wave_sum(s) / (float)cols;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols)
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += (v[c][j] - mean) * (v[c][j] - mean);
  }
  const float r = rsqrtf(wave_sum(ss) / (float)cols + eps);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < cols) {
      float wv[8], bv[8], o[8];
      load8(w + col, wv);
      load8(b + col, bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * r * wv[j] + bv[j];
      store8(y + row * cols + col, o);
    }
  }
}

// ---- llava merge plan (transformers ~4.37 _merge_input_ids_with_image_features) ------------
// One 1024-thread workgroup walks the batch rows in order (the image rows are numbered across
// the flattened (b, l) order, carried in `base`); inside a row every step is a workgroup-wide
// scan over 1024-element chunks, so the row costs a few scans instead of the L-long serial
// loops of one thread per row (806 -> tens of us at B=8, L=1088).
constexpr int kMergeThreads = 1024;

// inclusive scan over the workgroup; *total = sum over all threads
DEV int64_t wg_incl_scan(int64_t v, int64_t* lds, int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  if (lane == 63) lds[w] = v;
  __syncthreads();
  int64_t off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kMergeThreads / 64; ++k) {
    const int64_t x = lds[k];
    off += k < w ? x : 0;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return v + off;
}

__global__ __launch_bounds__(kMergeThreads) void merge_plan_k(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ mask, int B, int S, int L, int64_t image_token,
    int64_t P, int left_padding, int64_t* __restrict__ text_dst, int64_t* __restrict__ src,
    int64_t* __restrict__ mmask, int64_t* __restrict__ pos) {
  __shared__ int64_t lds[kMergeThreads / 64];
  const int t = threadIdx.x;
  const int64_t n_text = (int64_t)B * S;
  int64_t base = 0;  // image rows numbered so far (flattened (b, l) order)
  for (int b = 0; b < B; ++b) {
    const int64_t* idr = ids + (int64_t)b * S;
    const int64_t* mr = mask ? mask + (int64_t)b * S : nullptr;
    int64_t* srow = src + (int64_t)b * L;
    int64_t* mmrow = mmask + (int64_t)b * L;
    int64_t* prow = pos + (int64_t)b * L;
    // new_token_positions = cumsum(is_img * (P - 1) + 1) - 1; last = its final value
    int64_t total = 0, tot;
    for (int c0 = 0; c0 < S; c0 += kMergeThreads) {
      const int s = c0 + t;
      wg_incl_scan(s < S ? (idr[s] == image_token ? P : 1) : 0, lds, &tot);
      total += tot;
    }
    const int64_t nb_pad = (int64_t)L - 1 - (total - 1);
    for (int l = t; l < L; l += kMergeThreads) { srow[l] = -2; mmrow[l] = 0; }  // -2: not a text slot yet
    __syncthreads();
    int64_t carry = -1;
    for (int c0 = 0; c0 < S; c0 += kMergeThreads) {
      const int s = c0 + t;
      const bool img = s < S && idr[s] == image_token;
      const int64_t np = carry + wg_incl_scan(s < S ? (img ? P : 1) : 0, lds, &tot);
      carry += tot;
      if (s < S) {
        const int64_t dst = np + (left_padding ? nb_pad : 0);
        if (img) {
          text_dst[(int64_t)b * S + s] = -1;
        } else {
          // flattened merged row (b * L + dst) or -1 when the slot falls outside the row
          text_dst[(int64_t)b * S + s] = (dst >= 0 && dst < L) ? (int64_t)b * L + dst : -1;
          if (dst >= 0 && dst < L) {
            srow[dst] = (int64_t)b * S + s;
            mmrow[dst] = mr ? mr[s] : 1;
          }
        }
      }
    }
    __syncthreads();
    // image_to_overwrite = not-a-text-slot & (cumsum - 1 >= nb_pad); image slots get the next
    // image rows in order and mask |= 1; the other free slots stay -1
    int64_t cs_carry = 0, rank_carry = 0;
    for (int c0 = 0; c0 < L; c0 += kMergeThreads) {
      const int l = c0 + t;
      const bool fr = l < L && srow[l] == -2;
      const int64_t cs = cs_carry + wg_incl_scan(fr ? 1 : 0, lds, &tot);
      cs_carry += tot;
      const bool slot = fr && cs - 1 >= nb_pad;
      const int64_t rk = rank_carry + wg_incl_scan(slot ? 1 : 0, lds, &tot) - (slot ? 1 : 0);
      rank_carry += tot;
      if (fr) {
        if (slot) { srow[l] = n_text + base + rk; mmrow[l] = 1; }
        else srow[l] = -1;
      }
    }
    base += rank_carry;
    __syncthreads();
    // position_ids = (cumsum(mask) - 1).masked_fill(mask == 0, 1)
    int64_t mc = 0;
    for (int c0 = 0; c0 < L; c0 += kMergeThreads) {
      const int l = c0 + t;
      const int64_t m = l < L ? mmrow[l] : 0;
      const int64_t c = mc + wg_incl_scan(m, lds, &tot);
      mc += tot;
      if (l < L) prow[l] = m == 0 ? 1 : c - 1;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void row_gather2_k(const int64_t* __restrict__ src, const u16* __restrict__ a,
                                                     int64_t n_a, const u16* __restrict__ bsrc, int64_t dim,
                                                     u16* __restrict__ out) {
  const int64_t r = blockIdx.x;
  const int64_t s = src[r];
  const u16* p = s < 0 ? nullptr : (s < n_a ? a + s * dim : bsrc + (s - n_a) * dim);
  for (int64_t c = threadIdx.x; c < dim / 8; c += 256) {
    u16x8 v = p ? *reinterpret_cast<const u16x8*>(p + c * 8) : u16x8(0);
    *reinterpret_cast<u16x8*>(out + r * dim + c * 8) = v;
  }
}

}  // namespace

extern "C" int cullavo_embedding_fwd(const int64_t* ids, int64_t n, const void* table, int64_t vocab,
                                     int64_t dim, void* out, int dtype, void* stream) {
  CV_REQUIRE(dtype == CULLAVO_DT_BF16 || dtype == CULLAVO_DT_F32, CULLAVO_EUNSUPPORTED, "bf16 / f32");
  CV_REQUIRE(dim % 8 == 0, CULLAVO_EINVAL, "dim must be a multiple of 8");
  if (n == 0) return CULLAVO_OK;
  // a row copy: f32 rows move as twice as many 16-bit units
  const int64_t units = dtype == CULLAVO_DT_F32 ? dim * 2 : dim;
  embedding_fwd_k<<<(unsigned)n, 256, 0, CV_STREAM(stream)>>>(ids, (const u16*)table, vocab, units, (u16*)out);
  return cullavo_check_launch("embedding_fwd");
}

extern "C" int cullavo_embedding_bwd(const int64_t* ids, int64_t n, const void* dout, int64_t vocab,
                                     int64_t dim, void* dtable, int table_dtype, float beta, int dtype,
                                     void* stream) {
  CV_REQUIRE(dtype == CULLAVO_DT_BF16 || dtype == CULLAVO_DT_F32, CULLAVO_EUNSUPPORTED, "bf16 / f32");
  CV_REQUIRE(dim % 8 == 0 && dim <= 8192, CULLAVO_EINVAL, "dim must be a multiple of 8 and <= 8192");
  if (n == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
#define EBW(TT, TD) embedding_bwd_k<TT, TD><<<(unsigned)n, 256, 0, s>>>(ids, n, (const TD*)dout, vocab, dim, (TT*)dtable, beta)
  if (dtype == CULLAVO_DT_BF16) {
    if (table_dtype == CULLAVO_DT_BF16) EBW(u16, u16);
    else EBW(float, u16);
  } else {
    if (table_dtype == CULLAVO_DT_BF16) EBW(u16, float);
    else EBW(float, float);
  }
#undef EBW
  return cullavo_check_launch("embedding_bwd");
}

extern "C" int cullavo_im2col_patches(const void* pixels, int pix_dtype, int B, int C, int H, int W,
                                      int patch, void* out, int64_t kpad, int out_dtype, void* stream) {
  CV_REQUIRE(H % patch == 0 && W % patch == 0, CULLAVO_EINVAL, "image size must be a multiple of patch");
  CV_REQUIRE(kpad >= (int64_t)C * patch * patch, CULLAVO_EINVAL, "kpad too small");
  const int gw = W / patch, P = (H / patch) * gw;
  const int64_t rows = (int64_t)B * (1 + P);
  if (rows == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
#define I2C(TP, TO) im2col_k<TP, TO><<<(unsigned)rows, 256, 0, s>>>((const TP*)pixels, C, H, W, patch, gw, P, (TO*)out, kpad)
  if (out_dtype == CULLAVO_DT_BF16) {
    if (pix_dtype == CULLAVO_DT_F32) I2C(float, u16);
    else I2C(u16, u16);
  } else {
    if (pix_dtype == CULLAVO_DT_F32) I2C(float, float);
    else I2C(u16, float);
  }
#undef I2C
  return cullavo_check_launch("im2col_patches");
}

extern "C" int cullavo_vision_embed_ln(const void* x, const void* cls, const void* pos, const void* w,
                                       const void* b, void* y, int B, int T, int64_t dim, float eps,
                                       int dtype, void* stream) {
  CV_REQUIRE(dim % 8 == 0 && dim <= 8192, CULLAVO_EINVAL, "dim");
  CV_REQUIRE(dtype == CULLAVO_DT_BF16 || dtype == CULLAVO_DT_F32, CULLAVO_EUNSUPPORTED, "bf16 / f32");
  const int64_t rows = (int64_t)B * T;
  if (rows == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const int nb = (int)cdiv(rows, 4);
#define VEL1(T_, N) vision_embed_ln_k<T_, N><<<nb, 256, 0, s>>>((const T_*)x, (const T_*)cls, (const T_*)pos, (const T_*)w, (const T_*)b, (T_*)y, rows, T, (int)dim, eps)
#define VEL(N) do { if (dtype == CULLAVO_DT_F32) VEL1(float, N); else VEL1(u16, N); } while (0)
  if (dim <= 512) VEL(1);
  else if (dim <= 1024) VEL(2);
  else if (dim <= 2048) VEL(4);
  else if (dim <= 4096) VEL(8);
  else VEL(16);
#undef VEL
#undef VEL1
  return cullavo_check_launch("vision_embed_ln");
}

extern "C" int cullavo_merge_plan(const int64_t* ids, const int64_t* mask, int B, int S, int L,
                                  int64_t image_token, int64_t n_patches, int left_padding,
                                  int64_t* text_dst, int64_t* src, int64_t* merged_mask,
                                  int64_t* position_ids, void* stream) {
  CV_REQUIRE(B >= 0 && B <= 1024, CULLAVO_EINVAL, "B must be <= 1024");
  CV_REQUIRE(n_patches >= 1, CULLAVO_EINVAL, "n_patches");
  if (B == 0) return CULLAVO_OK;
  merge_plan_k<<<1, kMergeThreads, 0, CV_STREAM(stream)>>>(ids, mask, B, S, L, image_token, n_patches, left_padding,
                                                  text_dst, src, merged_mask, position_ids);
  return cullavo_check_launch("merge_plan");
}

extern "C" int cullavo_row_gather2(const int64_t* src, int64_t rows, const void* a, int64_t n_a,
                                   const void* b, int64_t dim, void* out, int dtype, void* stream) {
  CV_REQUIRE(dtype == CULLAVO_DT_BF16 || dtype == CULLAVO_DT_F32, CULLAVO_EUNSUPPORTED, "bf16 / f32");
  CV_REQUIRE(dim % 8 == 0, CULLAVO_EINVAL, "dim must be a multiple of 8");
  if (rows == 0) return CULLAVO_OK;
  const int64_t units = dtype == CULLAVO_DT_F32 ? dim * 2 : dim;  // row copy in 16-bit units
  row_gather2_k<<<(unsigned)rows, 256, 0, CV_STREAM(stream)>>>(src, (const u16*)a, n_a, (const u16*)b, units, (u16*)out);
  return cullavo_check_launch("row_gather2");
}
