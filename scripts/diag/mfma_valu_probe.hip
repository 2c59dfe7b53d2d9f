// Winograd feasibility probe (round 6, DESIGN.md §4 "Winograd F(2x2,3x3)"): how many vector instructions
// hide beside v_mfma_f32_16x16x32_f16 in the C = 128 trunk's regime (one wave per SIMD, operands in
// registers, random data), and at what clock the chip holds the denser stream.
//
// A Winograd trunk issues 384 MFMAs per board and layer instead of the edge tiles' 640 (1.67x fewer), but adds
// the input transform (V = B^T d B: ~576 v_pk_add_f16 per board-layer) and the output transform
// (Y = A^T M A: ~864 v_add_f32, or half as many v_pk_add_f32) -- about 2.6 vector instructions per MFMA, on
// top of the operand reads the direct trunk already places in the MFMA gaps.  This kernel measures cycles
// per MFMA and the in-kernel clock (s_memtime / s_memrealtime, 100 MHz) for NV independent vector adds per
// MFMA (f32, packed f16, packed f32), 8 independent accumulators, interleaved one MFMA : NV adds by
// sched_group_barrier.  Results go to a buffer of their own; nothing is computed from the stamps.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/diag/mfma_valu_probe.hip -o /tmp/mfma_valu_probe
//   /tmp/mfma_valu_probe > profiles/r06/winograd/mfma_valu_probe.json
#include <hip/hip_runtime.h>

#include <stdio.h>

#include <algorithm>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

enum { KIND_F32 = 0, KIND_PK16 = 1, KIND_PK32 = 2 };

__device__ __forceinline__ float hrand(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return (float)(x & 0xffff) / 65536.0f - 0.5f;
}

template <int NV, int KIND>
__global__ __launch_bounds__(256) void probe(float *out, unsigned long long *stamps, int iters, unsigned seed) {
  const unsigned tid = blockIdx.x * 256u + threadIdx.x;
  f16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (_Float16)hrand(seed + tid * 16u + i);
    b[i] = (_Float16)hrand(seed * 7u + tid * 16u + i);
  }
  f32x4 acc[8];
  for (int m = 0; m < 8; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float v[8];
  f16x2 h[8];
  f32x2 p[8];
  for (int j = 0; j < 8; ++j) {
    v[j] = hrand(seed + 99u * tid + j);
    h[j] = f16x2{(_Float16)v[j], (_Float16)(-v[j])};
    p[j] = f32x2{v[j], -v[j]};
  }
  const float dv = hrand(tid) * 1e-3f;
  const f16x2 dh = f16x2{(_Float16)dv, (_Float16)(-dv)};
  const f32x2 dp = f32x2{dv, -dv};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[m], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int k = (m * NV + j) & 7;
        if constexpr (KIND == KIND_F32) v[k] = v[k] + dv;
        else if constexpr (KIND == KIND_PK16) h[k] = h[k] + dh;
        else p[k] = p[k] + dp;
      }
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
      if constexpr (NV > 0) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);  // then NV vector ALU ops
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int m = 0; m < 8; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
  for (int j = 0; j < 8; ++j) s += v[j] + (float)h[j][0] + (float)h[j][1] + p[j][0] + p[j][1];
  out[tid] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t1 - t0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int NV, int KIND>
static void run(const char *kind, int iters, int blocks) {
  float *out;
  unsigned long long *st;
  (void)hipMalloc(&out, sizeof(float) * 256 * blocks);
  (void)hipMalloc(&st, sizeof(unsigned long long) * 2 * blocks);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // >= 2 s of back-to-back launches first (the clock the chip holds under this load), then the timed one
  for (int w = 0; w < 40; ++w) hipLaunchKernelGGL((probe<NV, KIND>), dim3(blocks), dim3(256), 0, 0, out, st, iters, 1234u + w);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((probe<NV, KIND>), dim3(blocks), dim3(256), 0, 0, out, st, iters, 777u);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(2 * blocks);
  (void)hipMemcpy(h.data(), st, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
  std::vector<double> cyc, clk;
  for (int b = 0; b < blocks; ++b) {
    cyc.push_back((double)h[2 * b]);
    clk.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 0.1);  // GHz: memtime ticks per 100 MHz tick / 10
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(clk.begin(), clk.end());
  const double mfmas = (double)iters * 8.0;
  const double flops = mfmas * 16.0 * 16.0 * 32.0 * 2.0 * 4.0 * blocks;  // 4 waves per block
  printf("{\"kind\": \"%s\", \"valu_per_mfma\": %d, \"cycles_per_mfma\": %.3f, \"clock_ghz\": %.4f, "
         "\"ms\": %.4f, \"tflops\": %.1f, \"blocks\": %d, \"iters\": %d}\n",
         kind, NV, cyc[blocks / 2] / mfmas, clk[blocks / 2], ms, flops / (ms * 1e-3) / 1e12, blocks, iters);
  fflush(stdout);
  (void)hipFree(out);
  (void)hipFree(st);
}

int main() {
  const int iters = 20000, blocks = 256;  // one 4-wave workgroup per CU: one wave per SIMD, as the trunk
  run<0, KIND_F32>("none", iters, blocks);
  run<1, KIND_F32>("v_add_f32", iters, blocks);
  run<2, KIND_F32>("v_add_f32", iters, blocks);
  run<3, KIND_F32>("v_add_f32", iters, blocks);
  run<4, KIND_F32>("v_add_f32", iters, blocks);
  run<6, KIND_F32>("v_add_f32", iters, blocks);
  run<2, KIND_PK16>("v_pk_add_f16", iters, blocks);
  run<3, KIND_PK16>("v_pk_add_f16", iters, blocks);
  run<4, KIND_PK16>("v_pk_add_f16", iters, blocks);
  run<2, KIND_PK32>("v_pk_add_f32", iters, blocks);
  run<0, KIND_F32>("none", iters, blocks);
  return 0;
}
