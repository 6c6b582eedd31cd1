// Issue-cost lab (round 5): what one memory instruction costs a wave that otherwise issues
// back-to-back v_mfma_f32_16x16x32_bf16, by instruction kind and waves per SIMD. The GEMM main
// loop question behind it: is an LDS-DMA piece (buffer_load_dwordx4 ... lds) dearer to issue
// beside MFMAs than the register-staging pair (buffer_load_dwordx4 -> VGPR, ds_write_b128)?
//
// Per iteration each wave issues 8 MFMAs on 8 independent accumulators (random bf16 operands in
// registers; round 5, second version: the first alternated two accumulators, whose dependent
// chains left bubbles the memory instructions hid in) and
//   V0: nothing else
//   V1: one LDS-DMA piece (1 KiB per wave-instruction, L2-resident source)
//   V2: one buffer_load_dwordx4 into VGPRs (its value consumed 4 loads later)
//   V3: one global_load_dwordx4 into VGPRs
//   V4: one ds_write_b128
//   V5: V2 + V4 (register staging: load, and write the value loaded 4 iterations earlier)
//   V6: two ds_read_b128
//   V7: four LDS-DMA pieces (the 8-wave kernel's one-loader-per-SIMD burst density)
// Time per iteration (ns, HIP events) is printed per variant and occupancy; the chip-wide rate of
// the MFMAs alone is the V0 line.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/lab/bin/issue_lab tools/lab/issue_lab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(8))) __bf16 frag8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int ITERS = 2048;
constexpr unsigned SRC_BYTES = 2u << 20;  // 2 MiB source: L2-resident on every XCD after the first pass

template <int V>
__global__ __launch_bounds__(512) void issue_k(const unsigned char* __restrict__ src, float* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // random-looking operand bits (DVFS: zero operands clock higher)
  unsigned h = (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  u32x4 ra, rb;
  for (int i = 0; i < 4; ++i) {
    h = h * 1664525u + 1013904223u;
    ra[i] = (h & 0x3FFF3FFFu) | 0x3C003C00u;
    h = h * 1664525u + 1013904223u;
    rb[i] = (h & 0x3FFF3FFFu) | 0x3C003C00u;
  }
  const frag8 fa = __builtin_bit_cast(frag8, ra), fb = __builtin_bit_cast(frag8, rb);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)SRC_BYTES, 0x00020000);
  const unsigned base = ((blockIdx.x * 8 + wave) * 1024u + lane * 16u) % SRC_BYTES;
  u32x4 r0 = {0, 0, 0, 0}, r1 = r0, r2 = r0, r3 = r0, sink = r0;
  char* lds_w = smem + wave * 8192;
  const unsigned lds_a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds_w + lane * 16;
  f32x4 c0 = acc[0], c1 = acc[1], c2 = acc[2], c3 = acc[3], c4 = acc[4], c5 = acc[5], c6 = acc[6], c7 = acc[7];
  // every instruction of the loop is inline asm (volatile: issued in program order, nothing hoisted
  // or merged); the register loads' values are consumed 4 iterations later behind a counted vmcnt(3)
#define MF(c) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(fa), "v"(fb) : "memory")
  for (int it = 0; it < ITERS; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned off = (base + (unsigned)(it + u) * 65536u) & (SRC_BYTES - 1);
      u32x4& slot = u == 0 ? r0 : u == 1 ? r1 : u == 2 ? r2 : r3;
      MF(c0);
      if constexpr (V == 1 || V == 7) {
#pragma unroll
        for (int p = 0; p < (V == 7 ? 4 : 1); ++p)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds_w + ((u * 4 + p) & 7) * 1024), 16,
                                                   (off + p * 1024u) & (SRC_BYTES - 1), 0, 0, 0);
        if (u == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      }
      if constexpr (V == 2 || V == 5) {
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        if constexpr (V == 5) asm volatile("ds_write_b128 %0, %1" :: "v"(lds_a + u * 1024), "v"(slot) : "memory");
        else sink ^= slot;
        asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(slot) : "v"(off), "s"(rsrc) : "memory");
      }
      if constexpr (V == 3) {
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        sink ^= slot;
        const unsigned char* ptr = src + off;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(slot) : "v"(ptr) : "memory");
      }
      if constexpr (V == 4)
        asm volatile("ds_write_b128 %0, %1" :: "v"(lds_a + u * 1024), "v"(ra) : "memory");
      if constexpr (V == 6) {
        u32x4 x, y;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:4096" : "=v"(x), "=v"(y) : "v"(lds_a + u * 1024)
                     : "memory");
        MF(c1); MF(c2); MF(c3);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(x), "+v"(y) :: "memory");
        sink ^= x ^ y;
        MF(c4); MF(c5); MF(c6); MF(c7);
        continue;
      }
      MF(c1); MF(c2); MF(c3); MF(c4); MF(c5); MF(c6); MF(c7);
    }
  }
#undef MF
  acc[0] = c0; acc[1] = c1; acc[2] = c2; acc[3] = c3; acc[4] = c4; acc[5] = c5; acc[6] = c6; acc[7] = c7;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  s += (float)(sink[0] ^ sink[1] ^ sink[2] ^ sink[3] ^ r0[0] ^ r1[1] ^ r2[2] ^ r3[3]);
  if (V == 1 || V == 7) s += (float)*reinterpret_cast<const unsigned*>(lds_w + lane * 4);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int V>
float run(int threads, const unsigned char* src, float* out) {
  const int blocks = 256 * 4;
  const int smem = 8 * 8192;
  hipFuncSetAttribute((const void*)issue_k<V>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  issue_k<V><<<blocks, threads, smem>>>(src, out);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(a);
    issue_k<V><<<blocks, threads, smem>>>(src, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  // one block per CU at a time (64 KiB LDS, 1-2 waves per SIMD): 4 rounds of ITERS iterations
  return best * 1e6f / (4.0f * ITERS);  // ns per iteration
}

int main() {
  unsigned char* src;
  float* out;
  hipMalloc(&src, SRC_BYTES);
  hipMemset(src, 0x3c, SRC_BYTES);
  hipMalloc(&out, 256 * 4 * 512 * 4);
  const char* names[8] = {"mfma only", "+1 LDS-DMA", "+1 buffer_load->vgpr", "+1 global_load->vgpr", "+1 ds_write_b128",
                          "+1 load->vgpr +1 ds_write", "+2 ds_read_b128", "+4 LDS-DMA"};
  for (int threads : {256, 512}) {
    float t[8];
    t[0] = run<0>(threads, src, out);
    t[1] = run<1>(threads, src, out);
    t[2] = run<2>(threads, src, out);
    t[3] = run<3>(threads, src, out);
    t[4] = run<4>(threads, src, out);
    t[5] = run<5>(threads, src, out);
    t[6] = run<6>(threads, src, out);
    t[7] = run<7>(threads, src, out);
    const double mfma_flops = 2.0 * 16 * 16 * 32 * 8 * (threads / 64) * 256.0;  // per iteration, chip-wide
    for (int v = 0; v < 8; ++v)
      printf("waves/SIMD %d  %-28s %8.2f ns/iter  %6.3fx  (MFMA %7.1f TF/s)\n", threads / 256, names[v], t[v],
             t[v] / t[0], mfma_flops / (t[v] * 1e-9) / 1e12);
  }
  hipFree(src);
  hipFree(out);
  return 0;
}
