// Lab: the dQ-from-dS^T ring kernel (attention.hip attn_bwd_dq_ring_k) at 2-4 stages, with the
// fragment reads + MFMAs (LAB bit 0) and / or the K tile DMA (bit 1) left out -- timing floors that
// say which part bounds the kernel, not results. Built by tools/lab/build_lab.sh dq_lab.hip dq;
// loaded after libcullavo_hip.so (RTLD_GLOBAL) by tools/lab/dq_lab.py.
#include "../../causal-unified-language-vision_amd/csrc/attention.hip"

namespace {
template <int NST, int LAB>
void run(const u16* K, int64_t ldk, const u16* ds, int64_t ldst, int64_t st_bh, int64_t st_blk, int LkP, u16* dq,
         int64_t lddq, int B, int H, int L, float scale, hipStream_t s) {
  const int smem = NST * (64 * 128 * 2 + 64 * 128 * 2);
  set_smem(attn_bwd_dq_ring_k<128, true, NST, LAB>, smem);
  attn_bwd_dq_ring_k<128, true, NST, LAB><<<(unsigned)(cdiv(L, 128) * H * B), 256, smem, s>>>(
      K, ldk, ds, ldst, st_bh, st_blk, LkP, dq, lddq, H, L, L, scale, nullptr);
}
}  // namespace

// variant = 10 * NST + LAB
extern "C" int dq_lab(int variant, const void* K, int64_t ldk, const void* ds, int64_t ldst, int64_t st_bh,
                      int64_t st_blk, int LkP, void* dq, int64_t lddq, int B, int H, int L, float scale, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const u16* k = (const u16*)K;
  const u16* d = (const u16*)ds;
  u16* o = (u16*)dq;
#define V(N, LB) \
  if (variant == 10 * N + LB) { run<N, LB>(k, ldk, d, ldst, st_bh, st_blk, LkP, o, lddq, B, H, L, scale, s); return 0; }
  V(2, 0) V(2, 1) V(2, 2) V(2, 3) V(3, 0) V(3, 1) V(3, 2) V(3, 3) V(4, 0) V(4, 1) V(4, 2) V(4, 3)
#undef V
  return -1;
}
