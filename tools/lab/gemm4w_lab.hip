// Ablation lab of the round-5 4-wave GEMM (tools/lab/gemm4w_r5.hip, lab tile mode 4): the same kernel with
// parts of its K-loop removed (results wrong), forward layout, bf16 out, for tools/lab/gemm_lab.py:
//   v = ABL bits: 0 full kernel, 1 no in-loop global loads, 2 no LDS writes, 4 no barrier,
//   8 no fragment reads (combinations allowed); v = 1000 + QABL: gemm4q_k (ks-region LDS-DMA pipeline); 2001: the tile-mode-4 launcher
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Iinclude tools/lab/gemm4w_lab.hip \
//     -o tools/lab/bin/libgemm4w_lab.so
#include "gemm4w_r5.hip"
#include "gemm4q.inc"

int cullavo_check_launch(const char*) { return hipGetLastError() == hipSuccess ? 0 : 1; }

template <int ABL>
int lab_launch(cvgemm::GemmArgs p, hipStream_t s) {
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)gemm4w_k<0, 0, CULLAVO_DT_BF16, ABL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, SMEM4);
    set = true;
  }
  p.tiles_m = (int)cdiv(p.M, T4);
  p.tiles_n = (int)cdiv(p.N, T4);
  p.sk_dp = p.tiles_m * p.tiles_n;
  gemm4w_k<0, 0, CULLAVO_DT_BF16, ABL><<<(unsigned)p.sk_dp, 256, SMEM4, s>>>(p);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

template <int Q>
int lab_launch_q(cvgemm::GemmArgs p, hipStream_t s) {
  static bool set = false;
  if (!set) {
    (void)hipFuncSetAttribute((const void*)gemm4q_k<0, 0, CULLAVO_DT_BF16, Q>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              SMEM4);
    set = true;
  }
  p.tiles_m = (int)cdiv(p.M, T4);
  p.tiles_n = (int)cdiv(p.N, T4);
  p.sk_dp = p.tiles_m * p.tiles_n;
  gemm4q_k<0, 0, CULLAVO_DT_BF16, Q><<<(unsigned)p.sk_dp, 256, SMEM4, s>>>(p);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int lab_gemm(int v, int64_t M, int64_t N, int64_t K, const void* A, const void* B, void* C, void* stream) {
  cvgemm::GemmArgs p{};
  p.A = (const u16*)A; p.B = (const u16*)B; p.C = C;
  p.M = M; p.N = N; p.K = K; p.lda = K; p.ldb = K; p.ldc = N;
  p.alpha = 1.f; p.act = CULLAVO_ACT_NONE; p.epi_lds = 1; p.group_m = -4;
  hipStream_t s = (hipStream_t)stream;
  if (v == 2001) return cvgemm_launch_4w(p, 0, 0, false, s);  // the tile-mode-4 launcher
  switch (v) {  // 1000 + QABL: gemm4q_k (ks-region LDS-DMA pipeline)
    case 1000: return lab_launch_q<0>(p, s);
    case 1001: return lab_launch_q<1>(p, s);
    case 1002: return lab_launch_q<2>(p, s);
    case 1006: return lab_launch_q<6>(p, s);
    case 1008: return lab_launch_q<8>(p, s);
    case 1009: return lab_launch_q<9>(p, s);
    case 1016: return lab_launch_q<16>(p, s);
    case 1032: return lab_launch_q<32>(p, s);
    case 1096: return lab_launch_q<96>(p, s);
    case 1104: return lab_launch_q<104>(p, s);
  }
  switch (v) {
#define C(V) case V: return lab_launch<V>(p, s);
    C(0) C(1) C(2) C(3) C(4) C(8) C(12) C(15) C(16) C(32) C(64) C(128) C(136) C(256) C(512)
#undef C
  }
  return 2;
}
