// trainconv.hip — the trainer's 3x3 residual-block convolutions on v_mfma_f32_16x16x32_f16 (round 5).
//
// The UpdateWorker's SGD step (updateworker.py:141-149 -> MCTreeSearch.update_from_memory, mcts.py:254-270)
// runs the ResidualTower (games/general/modules.py:13-40) forward and backward at batch 64 under fp16
// autocast.  MIOpen picks VALU dot2 Winograd kernels for those 3x3 convolutions (no MFMA; 26 us each,
// 46 % of a graphed step, profiles/r04/trainer/trainer_step_kernels.txt).  These kernels compute the same
// three products on the matrix cores, for the conv2d(x16, w16, b16, stride 1, padding 1) that autocast runs:
//
//   forward       y[b][co][p]  = b[co] + sum_{ci,tap} w[co][ci][tap] x[b][ci][p + tap]        (k_conv3x3)
//   input grad    dx[b][ci][p] = sum_{co,tap} w[co][ci][8 - tap] dy[b][co][p + tap]          (k_conv3x3 on
//                 the transposed, flipped weights: the same kernel)
//   weight grad   dw[co][ci][tap] = sum_{b,p} dy[b][co][p] x[b][ci][p + tap]                 (k_conv3x3_wgrad,
//                 split over boards, then k_conv3x3_reduce sums the splits in a fixed order; + db)
//
// Tensors are the module's own: NCHW fp16 activations [n][c][W][H] (cell p = x H + y), weights
// [co][ci][3][3]; fp32 accumulation, one rounding to fp16 at the end as MIOpen's fp16 kernels do.
// Deterministic (no atomics): the same bits every run, inside a captured HIP graph as well.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spmcts.h"

namespace tconv {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------------------------------------
// weight packing: w [co][ci][3][3] -> wf [co][tap][ci] (forward A operand rows) and wb [ci][tap][co] with the
// taps flipped (the input-gradient convolution's weights)
__global__ void k_pack(int cin, int cout, const _Float16 *__restrict__ w, _Float16 *__restrict__ wf,
                       _Float16 *__restrict__ wb) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cout * cin * 9) return;
  const int tap = i % 9, ci = (i / 9) % cin, co = i / (9 * cin);
  const _Float16 v = w[i];
  wf[((size_t)co * 9 + tap) * cin + ci] = v;
  wb[((size_t)ci * 9 + (8 - tap)) * cout + co] = v;
}

// ---------------------------------------------------------------------------------------------------------
// y[b][co][p] = bias[co] + sum_{ci, tap} wp[co][tap][ci] * x[b][ci][p + tap] (zero padding), NCHW fp16.
// One workgroup = one board x 32 output channels, 2 waves (16 channels each) x NT cell tiles of 16.  The
// board's input goes to LDS as padded rows [(W + 2)(H + 2)][CIN] (+ one zero row for the cells past W H of the
// last tile); lane 16 q + n reads 16 B of its cell's row at channels 32 k + 8 q (B operand) and its output
// channel's weights at the same channels (A operand, from global memory / L2).
template <int CIN, int NT>
__global__ __launch_bounds__(128) void k_conv3x3(int W, int H, int cout, const _Float16 *__restrict__ x,
                                                 const _Float16 *__restrict__ wp, const _Float16 *__restrict__ bias,
                                                 _Float16 *__restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int RSB = CIN * 2 + 16;  // row stride: a 16-B pad shifts consecutive rows by 4 banks
  const int b = blockIdx.x, cot = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, q = lane >> 4, n = lane & 15;
  const int HP = H + 2, NPR = (W + 2) * HP, ZR = NPR, cells = W * H;
  for (int i = tid; i < (NPR + 1) * RSB / 16; i += 128) ((uint4 *)lds)[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  const _Float16 *xb = x + (size_t)b * CIN * cells;
  for (int i = tid; i < CIN * cells; i += 128) {
    const int ci = i / cells, p = i - ci * cells, xx = p / H, yy = p - xx * H;
    *(_Float16 *)(lds + ((xx + 1) * HP + yy + 1) * RSB + ci * 2) = xb[i];
  }
  __syncthreads();
  int base[NT];
  bool ok[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int p = 16 * t + n;
    ok[t] = p < cells;
    base[t] = ok[t] ? ((p / H + 1) * HP + p % H + 1) : ZR;
  }
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int co = cot * 32 + wave * 16 + n;
  const _Float16 *wrow = wp + (size_t)co * 9 * CIN + 8 * q;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int toff = (tap / 3 - 1) * HP + (tap % 3 - 1);
    int roff[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) roff[t] = (ok[t] ? base[t] + toff : ZR) * RSB + 16 * q;
#pragma unroll
    for (int k = 0; k < CIN / 32; ++k) {
      const f16x8 a = *(const f16x8 *)(wrow + tap * CIN + 32 * k);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma(a, *(const f16x8 *)(lds + roff[t] + 64 * k), acc[t]);
    }
  }
  // D: lane 16 q + n holds output channels 4 q + r of the wave's 16, cell 16 t + n
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = cot * 32 + wave * 16 + 4 * q + r;
    const float bv = bias ? (float)bias[c] : 0.f;
    _Float16 *yc = y + ((size_t)b * cout + c) * cells;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int p = 16 * t + n;
      if (p < cells) yc[p] = (_Float16)(acc[t][r] + bv);
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// part[s][co][tap][ci] = sum over the boards of split s of sum_p dy[b][co][p] * x[b][ci][p + tap].
// GEMM over K = the cells of a padded grid (W + 2) x HP8 (HP8 = H + 2 rounded up to 8, so a row of the grid
// is 16 B and a dx shift is a whole number of 16-B slots): dy is placed on the grid (zero on the border),
// x three times, shifted by dy - 1 = -1, 0, +1 cells, so every B fragment (8 consecutive grid cells of one
// channel at shift (dx - 1) HP8) is one aligned 16-B LDS read.  Workgroup = 32 output x 32 input channels x
// one split of the batch; 4 waves = 2 x 2 sub-tiles of 16 x 16, all 9 taps (9 accumulators each).
template <int KK>  // k-steps of 32 grid cells per board
__global__ __launch_bounds__(256) void k_conv3x3_wgrad(int W, int H, int cin, int cout, int bps, int nb,
                                                       const _Float16 *__restrict__ x,
                                                       const _Float16 *__restrict__ dy, float *__restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int KP = 32 * KK;         // grid cells per board, padded to the k-steps
  constexpr int DS = KP + 8;          // sdy row (halfs): 16-B multiple
  constexpr int XS = KP + 24;         // sx row: 8 halfs of margin either side + the 16-B pad
  _Float16 *sdy = (_Float16 *)lds;                // [32 co][DS]
  _Float16 *sx = sdy + 32 * DS;                   // [3 dy][32 ci][XS], cell r at index 8 + r
  const int cot = blockIdx.x, cit = blockIdx.y, s = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, q = lane >> 4, n = lane & 15;
  const int HP = (H + 2 + 7) & ~7, cells = W * H;
  const int cs = wave & 1, is = wave >> 1;  // the wave's co / ci sub-tile of 16
  f32x4 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < bps; ++j) {
    const int b = s * bps + j;
    if (b >= nb) break;
    __syncthreads();  // the previous board's reads are done
    const _Float16 *dyb = dy + ((size_t)b * cout + cot * 32) * cells;
    const _Float16 *xb = x + ((size_t)b * cin + cit * 32) * cells;
    for (int i = tid; i < 32 * DS; i += 256) {
      const int c = i / DS, r = i - c * DS, gx = r / HP - 1, gy = r % HP - 1;
      const bool in = r < KP && gx >= 0 && gx < W && gy >= 0 && gy < H;
      sdy[i] = in ? dyb[(size_t)c * cells + gx * H + gy] : (_Float16)0.f;
    }
    for (int i = tid; i < 3 * 32 * XS; i += 256) {
      const int d = i / (32 * XS), rem = i - d * 32 * XS, c = rem / XS, r = rem - c * XS - 8 + d - 1;
      // grid cell r + (d - 1); r may run past either end of the grid (margins): zero there
      const int gx = r >= 0 ? r / HP - 1 : -1, gy = r >= 0 ? r % HP - 1 : -1;
      const bool in = r >= 0 && r < (W + 2) * HP && gx >= 0 && gx < W && gy >= 0 && gy < H;
      sx[i] = in ? xb[(size_t)c * cells + gx * H + gy] : (_Float16)0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const f16x8 a = *(const f16x8 *)(sdy + (cs * 16 + n) * DS + 32 * kk + 8 * q);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int d = tap % 3, dxo = (tap / 3 - 1) * HP;
        const f16x8 bb = *(const f16x8 *)(sx + (d * 32 + is * 16 + n) * XS + 8 + 32 * kk + 8 * q + dxo);
        acc[tap] = mfma(a, bb, acc[tap]);
      }
    }
  }
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = cot * 32 + cs * 16 + 4 * q + r, ci = cit * 32 + is * 16 + n;
      part[(((size_t)s * cout + co) * 9 + tap) * cin + ci] = acc[tap][r];
    }
}

// dw[co][ci][tap] = fp16(sum_s part[s][co][tap][ci]) (splits in order); blocks past the weights: db[co] =
// fp16(sum over boards and cells of dy[b][co][p]) in a fixed order (a 256-thread tree per channel)
__global__ __launch_bounds__(256) void k_conv3x3_reduce(int cin, int cout, int splits, int nb, int cells,
                                                        const float *__restrict__ part, const _Float16 *__restrict__ dy,
                                                        _Float16 *__restrict__ dw, _Float16 *__restrict__ db) {
  const int nw = cout * cin * 9;
  const int wblocks = (nw + 255) / 256;
  if ((int)blockIdx.x < wblocks) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nw) return;
    const int tap = i % 9, ci = (i / 9) % cin, co = i / (9 * cin);
    float acc = 0.f;
    for (int s = 0; s < splits; ++s) acc += part[(((size_t)s * cout + co) * 9 + tap) * cin + ci];
    dw[i] = (_Float16)acc;
    return;
  }
  const int co = blockIdx.x - wblocks;
  if (db == nullptr || co >= cout) return;
  __shared__ float red[256];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nb * cells; i += 256) {
    const int b = i / cells, p = i - b * cells;
    acc += (float)dy[((size_t)b * cout + co) * cells + p];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) db[co] = (_Float16)red[0];
}

// boards of up to 64 cells with H + 2 <= 8 (one 16-B grid row per x in the weight gradient) and an LDS tile of
// at most 100 padded rows; C in {128, 256} input channels, outputs a multiple of 32
static bool shape_ok(int W, int H, int cin, int cout) {
  return W >= 1 && H >= 1 && W * H <= 64 && H + 2 <= 8 && (W + 2) * (H + 2) <= 100 && (cin == 128 || cin == 256) &&
         cout % 32 == 0 && cout >= 32 && cout <= 1024;
}

template <int CIN, int NT>
static int launch_fwd(int n, int W, int H, int cout, const void *x, const void *wp, const void *bias, void *y,
                      hipStream_t s) {
  const size_t lds = (size_t)((W + 2) * (H + 2) + 1) * (CIN * 2 + 16);
  hipLaunchKernelGGL((k_conv3x3<CIN, NT>), dim3(n, cout / 32), dim3(128), lds, s, W, H, cout, (const _Float16 *)x,
                     (const _Float16 *)wp, (const _Float16 *)bias, (_Float16 *)y);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int CIN>
static int fwd_nt(int n, int W, int H, int cout, const void *x, const void *wp, const void *bias, void *y,
                  hipStream_t s) {
  switch ((W * H + 15) / 16) {
    case 1: return launch_fwd<CIN, 1>(n, W, H, cout, x, wp, bias, y, s);
    case 2: return launch_fwd<CIN, 2>(n, W, H, cout, x, wp, bias, y, s);
    case 3: return launch_fwd<CIN, 3>(n, W, H, cout, x, wp, bias, y, s);
    case 4: return launch_fwd<CIN, 4>(n, W, H, cout, x, wp, bias, y, s);
  }
  return -2;
}

}  // namespace tconv

extern "C" {

int spmcts_conv3x3_supported(int32_t width, int32_t height, int32_t cin, int32_t cout) {
  return tconv::shape_ok(width, height, cin, cout) && tconv::shape_ok(width, height, cout, cin) ? 1 : 0;
}

int spmcts_conv3x3_pack(int32_t cin, int32_t cout, const void *w, void *wf, void *wb, spmcts_stream stream) {
  if (cin <= 0 || cout <= 0 || !w || !wf || !wb) return -1;
  const int total = cin * cout * 9;
  hipLaunchKernelGGL(tconv::k_pack, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, cin, cout,
                     (const _Float16 *)w, (_Float16 *)wf, (_Float16 *)wb);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

int spmcts_conv3x3_fwd(int32_t n, int32_t width, int32_t height, int32_t cin, int32_t cout, const void *x,
                       const void *wpk, const void *bias, void *y, spmcts_stream stream) {
  if (!tconv::shape_ok(width, height, cin, cout)) return -2;
  if (n <= 0) return 0;
  if (!x || !wpk || !y) return -1;
  hipStream_t s = (hipStream_t)stream;
  if (cin == 128) return tconv::fwd_nt<128>(n, width, height, cout, x, wpk, bias, y, s);
  return tconv::fwd_nt<256>(n, width, height, cout, x, wpk, bias, y, s);
}

int spmcts_conv3x3_wgrad(int32_t n, int32_t width, int32_t height, int32_t cin, int32_t cout, const void *x,
                         const void *dy, float *part, int32_t splits, void *dw, void *db, spmcts_stream stream) {
  if (!tconv::shape_ok(width, height, cin, cout) || cin % 32) return -2;
  if (!x || !dy || !part || !dw || splits <= 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int HP = (height + 2 + 7) & ~7, kk = ((width + 2) * HP + 31) / 32;
  const int bps = (n + splits - 1) / splits;
  const size_t lds = (size_t)(32 * (32 * kk + 8) + 3 * 32 * (32 * kk + 24)) * 2;
  const dim3 grid(cout / 32, cin / 32, splits);
  if (n > 0) {
    switch (kk) {
      case 1: hipLaunchKernelGGL(tconv::k_conv3x3_wgrad<1>, grid, dim3(256), lds, s, width, height, cin, cout, bps, n,
                                 (const _Float16 *)x, (const _Float16 *)dy, part); break;
      case 2: hipLaunchKernelGGL(tconv::k_conv3x3_wgrad<2>, grid, dim3(256), lds, s, width, height, cin, cout, bps, n,
                                 (const _Float16 *)x, (const _Float16 *)dy, part); break;
      case 3: hipLaunchKernelGGL(tconv::k_conv3x3_wgrad<3>, grid, dim3(256), lds, s, width, height, cin, cout, bps, n,
                                 (const _Float16 *)x, (const _Float16 *)dy, part); break;
      case 4: hipLaunchKernelGGL(tconv::k_conv3x3_wgrad<4>, grid, dim3(256), lds, s, width, height, cin, cout, bps, n,
                                 (const _Float16 *)x, (const _Float16 *)dy, part); break;
      default: return -2;
    }
    if (hipGetLastError() != hipSuccess) return -3;
  } else {
    if (hipMemsetAsync(part, 0, (size_t)splits * cout * 9 * cin * sizeof(float), s) != hipSuccess) return -3;
  }
  const int wblocks = (cout * cin * 9 + 255) / 256;
  hipLaunchKernelGGL(tconv::k_conv3x3_reduce, dim3(wblocks + (db ? cout : 0)), dim3(256), 0, s, cin, cout, splits, n,
                     width * height, (const float *)part, (const _Float16 *)dy, (_Float16 *)dw, (_Float16 *)db);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // extern "C"
