// KV-cache decode for generate() (reference cullavo/arch_cullavo.py:
// 605-636 and the HF generate() loop it drives, :341-395).
//
// The cache is preallocated per layer as K, V [B, Lmax, H*D] bf16 (token stride ld_tok, batch
// stride ld_batch). Prefill writes the prompt's rotated keys and values with kv_append; each
// decode step appends one token and runs attn_decode: one query row per (batch, head) against
// keys [kv_start[b], kv_len[b]). Decode attention is HBM-bound (every cached key and value is
// read once per step), so it is split over the keys (flash-decoding): workgroup (chunk, h, b)
// scores kChunk keys with 8 lanes per key (each lane 16 dims, coalesced 256 B rows, all loads in
// flight before use), forms P.V with 16 dim-groups x 16 key-groups of 16 B loads, keeps the
// chunk's max / sum / unnormalised P.V in f32 partials, and a combine kernel rescales and sums
// the chunks in a fixed order (deterministic).
#include "common.h"

namespace {

// keys per workgroup: 64 gives the batch-1 step 32 heads x 18 chunks = 576 workgroups at the
// 1088-row prompt (128: 288, about one per CU, each waiting out a longer load ramp)
constexpr int kChunk = 64;
constexpr float kLog2e = 1.4426950408889634f;

__global__ __launch_bounds__(256) void kv_append_k(const u16* __restrict__ ks, int64_t ldks, const u16* __restrict__ vs,
                                                  int64_t ldvs, u16* __restrict__ kc, u16* __restrict__ vc,
                                                  int64_t ld_tok, int64_t ld_b, const int32_t* __restrict__ start,
                                                  int B, int Lnew, int64_t hd) {
  const int64_t per_row = hd / 8, total = (int64_t)B * Lnew * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t row = i / per_row, c = (i % per_row) * 8;
    const int b = (int)(row / Lnew), t = (int)(row % Lnew);
    const int64_t dst = (int64_t)b * ld_b + (int64_t)(start[b] + t) * ld_tok + c;
    *reinterpret_cast<u16x8*>(kc + dst) = *reinterpret_cast<const u16x8*>(ks + row * ldks + c);
    *reinterpret_cast<u16x8*>(vc + dst) = *reinterpret_cast<const u16x8*>(vs + row * ldvs + c);
  }
}

// ROPE (cullavo_attn_decode_rope): the step's RoPE + KV append fused in front (rope_append8_k's
// arithmetic, elementwise.hip): every workgroup rotates its head's query row itself (q is read, not
// rotated in place), the workgroup whose chunk holds the new row start[b] rotates that row's key,
// writes key and value to the cache and uses them from LDS (its own loads of that row may predate
// the write), and the keys attended are [kv_start[b], start[b] + 1).
struct DecodeRope {
  const u16* k;
  int64_t ldk;
  const u16* v;
  int64_t ldv;
  const int64_t* pos;
  float theta;
  const int32_t* start;
  u16* kc;
  u16* vc;
};

template <int D, bool ROPE = false>
__global__ __launch_bounds__(256) void attn_decode_k(const u16* __restrict__ Q, int64_t ldq, const u16* __restrict__ Kc,
                                                    const u16* __restrict__ Vc, int64_t ld_tok, int64_t ld_b,
                                                    const int32_t* __restrict__ kv_len,
                                                    const int32_t* __restrict__ kv_start, float scale_log2,
                                                    float* __restrict__ part_o, float* __restrict__ part_ml,
                                                    int H, int nchunk, DecodeRope rp = DecodeRope{}) {
  static_assert(D == 128, "decode attention is specialised for the LM head_dim");
  const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int t = threadIdx.x;
  const int pnew = ROPE ? rp.start[b] : -1;  // the appended row (ROPE)
  const int len = ROPE ? pnew + 1 : kv_len[b], k_lo = kv_start ? kv_start[b] : 0;
  const int kbeg = c * kChunk, kend = min(len, kbeg + kChunk);
  __shared__ float qs[D];
  __shared__ float ps[kChunk];
  __shared__ float red[8];
  __shared__ float oacc[16][D];
  __shared__ float cs[D / 2], sn[D / 2];
  __shared__ u16 kn[D], vn[D];
  const int64_t pidx = ((int64_t)b * H + h) * nchunk + c;
  if (kbeg >= kend) {  // chunk past this row's length: empty partial
    if (t < D) part_o[pidx * D + t] = 0.f;
    if (t == 0) { part_ml[2 * pidx] = -INFINITY; part_ml[2 * pidx + 1] = 0.f; }
  } else {
    const bool has_new = ROPE && pnew >= kbeg && pnew < kend;
    if constexpr (ROPE) {
      if (t < D / 2) {
        const float inv_freq = 1.0f / powf(rp.theta, (float)(2 * t) / (float)D);
        const float ang = (float)rp.pos[b] * inv_freq;
        cs[t] = Elt<u16>::rnd(cosf(ang));
        sn[t] = Elt<u16>::rnd(sinf(ang));
      }
      __syncthreads();
      // t < 64: the query pair (t, t + 64); 64 <= t < 128 (the new row's chunk): the key pair
      if (t < D / 2 || (has_new && t < D)) {
        const int i = t & (D / 2 - 1);
        const u16* src = t < D / 2 ? Q + (int64_t)b * ldq + (int64_t)h * D : rp.k + (int64_t)b * rp.ldk + (int64_t)h * D;
        const float x1 = bf2f(src[i]), x2 = bf2f(src[i + D / 2]);
        const float o1 = Elt<u16>::rnd(Elt<u16>::rnd(x1 * cs[i]) + Elt<u16>::rnd(-x2 * sn[i]));
        const float o2 = Elt<u16>::rnd(Elt<u16>::rnd(x2 * cs[i]) + Elt<u16>::rnd(x1 * sn[i]));
        if (t < D / 2) {
          qs[i] = o1 * scale_log2;
          qs[i + D / 2] = o2 * scale_log2;
        } else {
          const int64_t row = (int64_t)b * ld_b + (int64_t)pnew * ld_tok + (int64_t)h * D;
          kn[i] = f2bf(o1);
          kn[i + D / 2] = f2bf(o2);
          rp.kc[row + i] = f2bf(o1);
          rp.kc[row + i + D / 2] = f2bf(o2);
        }
      }
      if (has_new && t >= D && t < 2 * D) {
        const u16 vv = rp.v[(int64_t)b * rp.ldv + (int64_t)h * D + (t - D)];
        vn[t - D] = vv;
        rp.vc[(int64_t)b * ld_b + (int64_t)pnew * ld_tok + (int64_t)h * D + (t - D)] = vv;
      }
    } else {
      if (t < D) qs[t] = bf2f(Q[(int64_t)b * ldq + (int64_t)h * D + t]) * scale_log2;
    }
    const u16* Kb = Kc + (int64_t)b * ld_b + (int64_t)h * D;
    const u16* Vb = Vc + (int64_t)b * ld_b + (int64_t)h * D;
    // scores: 8 lanes per key (16 dims each, one 256 B row per key), 32 keys per pass; the K rows
    // and the V rows of P.V (which do not depend on the scores) are all in flight before the first
    // is consumed
    const int sub = t & 7, slot = t >> 3;
    constexpr int kPass = kChunk / 32;
    u16x8 kr[kPass][2];
#pragma unroll
    for (int pass = 0; pass < kPass; ++pass) {
      const int key = min(kbeg + pass * 32 + slot, kend - 1);
      const u16* kp = Kb + (int64_t)key * ld_tok + sub * 16;
      kr[pass][0] = *reinterpret_cast<const u16x8*>(kp);
      kr[pass][1] = *reinterpret_cast<const u16x8*>(kp + 8);
    }
    // P.V: thread (dim group dg of 8 dims, key group kg) sums keys kg, kg+16, ...
    const int dg = t & 15, kg = t >> 4;
    const int nk = kend - kbeg;
    u16x8 vr[kChunk / 16];
#pragma unroll
    for (int i = 0; i < kChunk / 16; ++i) {
      const int k = min(kg + 16 * i, nk - 1);
      vr[i] = *reinterpret_cast<const u16x8*>(Vb + (int64_t)(kbeg + k) * ld_tok + dg * 8);
    }
    __syncthreads();
    if (has_new) {  // the appended row from LDS (this workgroup's own cache write may not be visible)
#pragma unroll
      for (int pass = 0; pass < kPass; ++pass) {
        if (min(kbeg + pass * 32 + slot, kend - 1) == pnew) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            kr[pass][0][j] = kn[sub * 16 + j];
            kr[pass][1][j] = kn[sub * 16 + 8 + j];
          }
        }
      }
#pragma unroll
      for (int i = 0; i < kChunk / 16; ++i) {
        if (kbeg + min(kg + 16 * i, nk - 1) == pnew) {
#pragma unroll
          for (int j = 0; j < 8; ++j) vr[i][j] = vn[dg * 8 + j];
        }
      }
    }
    float qv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) qv[j] = qs[sub * 16 + j];
#pragma unroll
    for (int pass = 0; pass < kPass; ++pass) {
      const int key = kbeg + pass * 32 + slot;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += qv[j] * bf2f(kr[pass][0][j]) + qv[8 + j] * bf2f(kr[pass][1][j]);
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      acc += __shfl_xor(acc, 4);
      if (sub == 0) ps[pass * 32 + slot] = (key < kend && key >= k_lo) ? acc : -INFINITY;
    }
    __syncthreads();
    // chunk max and sum (kChunk scores, threads >= kChunk carry -inf / 0)
    const int lane = t & 63, wv = t >> 6;
    const float s = t < kChunk ? ps[t] : -INFINITY;
    float m = wave_max(s);
    if (lane == 0) red[wv] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float p = (s == -INFINITY) ? 0.f : exp2f(s - m);
    __syncthreads();
    if (t < kChunk) ps[t] = p;
    float l = wave_sum(p);
    if (lane == 0) red[4 + wv] = l;
    __syncthreads();
    l = red[4] + red[5] + red[6] + red[7];
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < kChunk / 16; ++i) {
      const int k = kg + 16 * i;
      const float pk = k < nk ? ps[k] : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += pk * bf2f(vr[i][j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) oacc[kg][dg * 8 + j] = o[j];
    __syncthreads();
    if (t < D) {
      float sum = 0.f;
#pragma unroll
      for (int g = 0; g < 16; ++g) sum += oacc[g][t];
      part_o[pidx * D + t] = sum;
    }
    if (t == 0) { part_ml[2 * pidx] = m; part_ml[2 * pidx + 1] = l; }
  }
}

// Combine: max over the chunks, then the rescaled sums in chunk order (deterministic). Up to
// kCombineRegs chunks (max_len <= 2048) every partial is loaded before the first is used.
constexpr int kCombineRegs = 2048 / kChunk;
template <int D>
__global__ __launch_bounds__(D) void attn_decode_combine_k(const float* __restrict__ part_o,
                                                          const float* __restrict__ part_ml, u16* __restrict__ O,
                                                          int64_t ldo, int H, int nchunk) {
  const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int64_t base = ((int64_t)b * H + h) * nchunk;
  float M = -INFINITY, L = 0.f, acc = 0.f;
  if (nchunk <= kCombineRegs) {
    float mc[kCombineRegs], lc[kCombineRegs], oc[kCombineRegs];
#pragma unroll
    for (int c = 0; c < kCombineRegs; ++c) {
      const bool in = c < nchunk;
      mc[c] = in ? part_ml[2 * (base + c)] : -INFINITY;
      lc[c] = in ? part_ml[2 * (base + c) + 1] : 0.f;
      oc[c] = in ? part_o[(base + c) * D + d] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < kCombineRegs; ++c) M = fmaxf(M, mc[c]);
    if (M != -INFINITY) {
#pragma unroll
      for (int c = 0; c < kCombineRegs; ++c) {
        if (mc[c] == -INFINITY) continue;
        const float w = exp2f(mc[c] - M);
        L += w * lc[c];
        acc += w * oc[c];
      }
    }
  } else {
    for (int c = 0; c < nchunk; ++c) M = fmaxf(M, part_ml[2 * (base + c)]);
    if (M != -INFINITY) {
      for (int c = 0; c < nchunk; ++c) {
        const float mc = part_ml[2 * (base + c)];
        if (mc == -INFINITY) continue;
        const float w = exp2f(mc - M);
        L += w * part_ml[2 * (base + c) + 1];
        acc += w * part_o[(base + c) * D + d];
      }
    }
  }
  O[(int64_t)b * ldo + (int64_t)h * D + d] = f2bf(L > 0.f ? acc / L : 0.f);  // no visible key -> 0
}

}  // namespace

extern "C" int cullavo_kv_append(const void* k, int64_t ldk, const void* v, int64_t ldv, void* k_cache,
                                 void* v_cache, int64_t ld_tok, int64_t ld_batch, const int32_t* start, int B,
                                 int Lnew, int64_t hd, void* stream) {
  CV_REQUIRE(hd % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ld_tok % 8 == 0 && ld_batch % 8 == 0, CULLAVO_EINVAL,
             "kv_append: sizes and strides must be multiples of 8");
  CV_REQUIRE(start != nullptr, CULLAVO_EINVAL, "kv_append: start positions");
  if (B == 0 || Lnew == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const int64_t work = (int64_t)B * Lnew * (hd / 8);
  const int g = (int)std::min<int64_t>(cdiv(work, 256), 8192);
  kv_append_k<<<g, 256, 0, s>>>((const u16*)k, ldk, (const u16*)v, ldv, (u16*)k_cache, (u16*)v_cache, ld_tok,
                                ld_batch, start, B, Lnew, hd);
  return cullavo_check_launch("kv_append");
}

extern "C" size_t cullavo_attn_decode_workspace(int B, int H, int max_len, int D) {
  const int64_t nchunk = cdiv((int64_t)std::max(max_len, 1), kChunk);
  return (size_t)B * H * nchunk * (D + 2) * sizeof(float);
}

extern "C" int cullavo_attn_decode_rope(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                        int64_t ldv, const int64_t* position_ids, float theta, void* k_cache,
                                        void* v_cache, int64_t ld_tok, int64_t ld_batch, const int32_t* start,
                                        const int32_t* kv_start, void* o, int64_t ldo, int B, int H, int max_len,
                                        int D, float scale, float* workspace, void* stream) {
  CV_REQUIRE(D == 128, CULLAVO_EUNSUPPORTED, "decode attention: head_dim 128");
  CV_REQUIRE(start != nullptr && position_ids != nullptr && workspace != nullptr && k != nullptr && v != nullptr,
             CULLAVO_EINVAL, "decode attention + rope: start / position_ids / workspace / k / v");
  CV_REQUIRE(ld_tok >= (int64_t)H * D && ldq >= (int64_t)H * D && ldk >= (int64_t)H * D && ldv >= (int64_t)H * D &&
                 ldo >= (int64_t)H * D && ld_tok % 8 == 0,
             CULLAVO_EINVAL, "decode attention + rope: strides");
  if (B == 0 || H == 0 || max_len <= 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const int nchunk = (int)cdiv((int64_t)max_len, kChunk);
  float* part_o = workspace;
  float* part_ml = workspace + (int64_t)B * H * nchunk * D;
  DecodeRope rp{(const u16*)k, ldk, (const u16*)v, ldv, position_ids, theta, start, (u16*)k_cache, (u16*)v_cache};
  attn_decode_k<128, true><<<dim3(nchunk, H, B), 256, 0, s>>>((const u16*)q, ldq, (const u16*)k_cache,
                                                              (const u16*)v_cache, ld_tok, ld_batch, nullptr,
                                                              kv_start, scale * kLog2e, part_o, part_ml, H, nchunk, rp);
  attn_decode_combine_k<128><<<dim3(H, B), 128, 0, s>>>(part_o, part_ml, (u16*)o, ldo, H, nchunk);
  return cullavo_check_launch("attn_decode_rope");
}

extern "C" int cullavo_attn_decode(const void* q, int64_t ldq, const void* k_cache, const void* v_cache,
                                   int64_t ld_tok, int64_t ld_batch, const int32_t* kv_len, const int32_t* kv_start,
                                   void* o, int64_t ldo, int B, int H, int max_len, int D, float scale,
                                   float* workspace, void* stream) {
  CV_REQUIRE(D == 128, CULLAVO_EUNSUPPORTED, "decode attention: head_dim 128");
  CV_REQUIRE(kv_len != nullptr && workspace != nullptr, CULLAVO_EINVAL, "decode attention: kv_len / workspace");
  CV_REQUIRE(ld_tok >= (int64_t)H * D && ldq >= (int64_t)H * D && ldo >= (int64_t)H * D && ld_tok % 8 == 0,
             CULLAVO_EINVAL, "decode attention: strides");
  if (B == 0 || H == 0 || max_len <= 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const int nchunk = (int)cdiv((int64_t)max_len, kChunk);
  float* part_o = workspace;
  float* part_ml = workspace + (int64_t)B * H * nchunk * D;
  attn_decode_k<128><<<dim3(nchunk, H, B), 256, 0, s>>>((const u16*)q, ldq, (const u16*)k_cache,
                                                        (const u16*)v_cache, ld_tok, ld_batch, kv_len, kv_start,
                                                        scale * kLog2e, part_o, part_ml, H, nchunk);
  attn_decode_combine_k<128><<<dim3(H, B), 128, 0, s>>>(part_o, part_ml, (u16*)o, ldo, H, nchunk);
  return cullavo_check_launch("attn_decode");
}
