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
//                 one slice of 8 boards per workgroup, then k_conv3x3_reduce sums the slices in a fixed
//                 order; + db)
//
// Tensors are the module's own: NCHW fp16 activations [n][c][W][H] (cell p = x H + y), the fp32 weight and
// bias parameters (rounded to fp16 on use, as autocast's casts round them, so no separate cast kernels run);
// fp32 accumulation, one rounding to fp16 at the end as MIOpen's fp16 kernels do; the weight and bias
// gradients are the fp16-rounded sums handed back as fp32 (what the cast's backward gives the parameter).
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
// weight packing: the fp32 parameter w [co][ci][3][3], rounded to fp16 as autocast's cast rounds it ->
// wf [co][tap][ci] (forward A operand rows) and wb [ci][tap][co] with the taps flipped (the input-gradient
// convolution's weights)
__global__ void k_pack(int cin, int cout, const float *__restrict__ w, _Float16 *__restrict__ wf,
                       _Float16 *__restrict__ wb) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cout * cin * 9) return;
  const int tap = i % 9, ci = (i / 9) % cin, co = i / (9 * cin);
  const _Float16 v = (_Float16)w[i];
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
                                                 const _Float16 *__restrict__ wp, const float *__restrict__ bias,
                                                 _Float16 *__restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int RSB = CIN * 2 + 16;  // row stride: a 16-B pad shifts consecutive rows by 4 banks
  constexpr int KS = CIN / 32;
  const int b = blockIdx.x, cot = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, q = lane >> 4, n = lane & 15;
  const int HP = H + 2, NPR = (W + 2) * HP, ZR = NPR, cells = W * H;
  // the wave's whole A operand (its 16 output channels' weights, 9 taps x CIN) is loaded first, so the
  // loads' latency runs under the input staging below instead of under every k-step
  const int co = cot * 32 + wave * 16 + n;
  const _Float16 *wrow = wp + (size_t)co * 9 * CIN + 8 * q;
  f16x8 a[9][KS];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int k = 0; k < KS; ++k) a[tap][k] = *(const f16x8 *)(wrow + tap * CIN + 32 * k);
  for (int i = tid; i < (NPR + 1) * RSB / 16; i += 128) ((uint4 *)lds)[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  // input staging: a thread takes 8 channels of one cell (8 coalesced 2-byte loads across the threads'
  // cells) and writes them as one 16-byte LDS row piece
  const _Float16 *xb = x + (size_t)b * CIN * cells;
  for (int i = tid; i < (CIN / 8) * cells; i += 128) {
    const int g = i / cells, p = i - g * cells, xx = p / H, yy = p - xx * H;
    f16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = xb[(size_t)(8 * g + j) * cells + p];
    *(f16x8 *)(lds + ((xx + 1) * HP + yy + 1) * RSB + g * 16) = v;
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
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int toff = (tap / 3 - 1) * HP + (tap % 3 - 1);
    int roff[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) roff[t] = (ok[t] ? base[t] + toff : ZR) * RSB + 16 * q;
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma(a[tap][k], *(const f16x8 *)(lds + roff[t] + 64 * k), acc[t]);
  }
  // D: lane 16 q + n holds output channels 4 q + r of the wave's 16, cell 16 t + n
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = cot * 32 + wave * 16 + 4 * q + r;
    const float bv = bias ? (float)(_Float16)bias[c] : 0.f;  // the fp32 bias as autocast's fp16 cast
    _Float16 *yc = y + ((size_t)b * cout + c) * cells;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int p = 16 * t + n;
      if (p < cells) yc[p] = (_Float16)(acc[t][r] + bv);
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// part[s][co][tap][ci] = sum over the 8 boards of slice s of sum_p dy[b][co][p] * x[b][ci][p + tap].
// The GEMM's K runs over (cell, board): a lane's 8 consecutive k are the slice's 8 boards at one cell, so
// both operands are stored board-innermost in LDS -- dy as [cell][co][8 boards], x on the zero-bordered
// padded grid as [(W + 2)(H + 2) rows][ci][8 boards] -- and a tap shift only moves the x row: every
// fragment is one aligned 16-B LDS read, and the zero border gives the convolution's padding.  A k-step of
// 32 covers 4 cells (lane quarter q: cell 4 ks + q).  Workgroup = 32 output x 32 input channels x one
// slice; 4 waves = 2 x 2 sub-tiles of 16 x 16, all 9 taps (9 accumulators each).
__global__ __launch_bounds__(256) void k_conv3x3_wgrad(int W, int H, int cin, int cout, int nb,
                                                       const _Float16 *__restrict__ x,
                                                       const _Float16 *__restrict__ dy, float *__restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int cot = blockIdx.x, cit = blockIdx.y, s = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, q = lane >> 4, n = lane & 15;
  const int HP = H + 2, NPR = (W + 2) * HP, cells = W * H, KSTEPS = (cells + 3) / 4;
  f16x8 *sdy = (f16x8 *)lds;               // [4 KSTEPS cells][32 co] (cells past W H: zero)
  f16x8 *sx = sdy + 4 * KSTEPS * 32;       // [NPR + 1 rows][32 ci] (the last row: zero, for those cells)
  const int ZR = NPR;
  // zero the padded-grid border, the zero row and the dy cells past W H
  for (int i = tid; i < (NPR + 1) * 32; i += 256) {
    const int r = i >> 5, gx = r / HP - 1, gy = r % HP - 1;
    if (r == ZR || gx < 0 || gx >= W || gy < 0 || gy >= H) sx[i] = f16x8{};
  }
  for (int i = cells * 32 + tid; i < 4 * KSTEPS * 32; i += 256) sdy[i] = f16x8{};
  // the slice's boards, board-innermost: 8 coalesced 2-byte loads (across the threads' cells) per piece
  const int b0 = s * 8;
  for (int i = tid; i < 32 * cells; i += 256) {
    const int c = i / cells, p = i - c * cells, xx = p / H, yy = p - xx * H;
    f16x8 vd, vx;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int b = b0 + j;
      const bool in = b < nb;
      vd[j] = in ? dy[((size_t)b * cout + cot * 32 + c) * cells + p] : (_Float16)0.f;
      vx[j] = in ? x[((size_t)b * cin + cit * 32 + c) * cells + p] : (_Float16)0.f;
    }
    sdy[p * 32 + c] = vd;
    sx[((xx + 1) * HP + yy + 1) * 32 + c] = vx;
  }
  __syncthreads();
  const int cs = wave & 1, is = wave >> 1;  // the wave's co / ci sub-tile of 16
  f32x4 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < KSTEPS; ++ks) {
    const int p = 4 * ks + q;
    const f16x8 av = sdy[p * 32 + cs * 16 + n];
    const bool ok = p < cells;
    const int r0 = ok ? (p / H + 1) * HP + p % H + 1 : ZR;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int r = ok ? r0 + (tap / 3 - 1) * HP + (tap % 3 - 1) : ZR;
      acc[tap] = mfma(av, sx[r * 32 + is * 16 + n], acc[tap]);
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

// dw[co][ci][tap] = fp16(sum_s part[s][co][tap][ci]) (slices in order); blocks past the weights: db[co] =
// fp16(sum over boards and cells of dy[b][co][p]) in a fixed order (a 256-thread tree per channel); both
// stored as fp32 values of the fp16 gradient, which is what autocast's weight cast hands its fp32 parameter
__global__ __launch_bounds__(256) void k_conv3x3_reduce(int cin, int cout, int splits, int nb, int cells,
                                                        const float *__restrict__ part, const _Float16 *__restrict__ dy,
                                                        float *__restrict__ dw, float *__restrict__ db) {
  const int nw = cout * cin * 9;
  const int wblocks = (nw + 255) / 256;
  if ((int)blockIdx.x < wblocks) {
    const int i = blockIdx.x * 256 + threadIdx.x;  // in part's [co][tap][ci] order: coalesced reads
    if (i >= nw) return;
    const int ci = i % cin, tap = (i / cin) % 9, co = i / (9 * cin);
    float acc = 0.f;
    for (int s = 0; s < splits; ++s) acc += part[(size_t)s * nw + i];
    dw[((size_t)co * cin + ci) * 9 + tap] = (float)(_Float16)acc;  // fp16 grad, as fp32 (the cast's backward)
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
  if (threadIdx.x == 0) db[co] = (float)(_Float16)red[0];
}

// boards of up to 64 cells with an LDS tile of at most 100 padded rows (and the weight gradient's dy and x
// slices within 64 KB of LDS); C in {128, 256} input channels, outputs a multiple of 32
static bool shape_ok(int W, int H, int cin, int cout) {
  const int cells = W * H, npr = (W + 2) * (H + 2);
  return W >= 1 && H >= 1 && cells <= 64 && npr <= 100 && 4 * ((cells + 3) / 4) + npr + 1 <= 128 &&
         (cin == 128 || cin == 256) && cout % 32 == 0 && cout >= 32 && cout <= 1024;
}

template <int CIN, int NT>
static int launch_fwd(int n, int W, int H, int cout, const void *x, const void *wp, const void *bias, void *y,
                      hipStream_t s) {
  const size_t lds = (size_t)((W + 2) * (H + 2) + 1) * (CIN * 2 + 16);
  hipLaunchKernelGGL((k_conv3x3<CIN, NT>), dim3(n, cout / 32), dim3(128), lds, s, W, H, cout, (const _Float16 *)x,
                     (const _Float16 *)wp, (const float *)bias, (_Float16 *)y);
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
                     (const float *)w, (_Float16 *)wf, (_Float16 *)wb);
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
  if (!x || !dy || !part || !dw || splits != (n + 7) / 8 || splits <= 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int cells = width * height, ksteps = (cells + 3) / 4, npr = (width + 2) * (height + 2);
  const size_t lds = (size_t)(4 * ksteps * 32 + (npr + 1) * 32) * 16;
  hipLaunchKernelGGL(tconv::k_conv3x3_wgrad, dim3(cout / 32, cin / 32, splits), dim3(256), lds, s, width, height, cin,
                     cout, n, (const _Float16 *)x, (const _Float16 *)dy, part);
  if (hipGetLastError() != hipSuccess) return -3;
  const int wblocks = (cout * cin * 9 + 255) / 256;
  hipLaunchKernelGGL(tconv::k_conv3x3_reduce, dim3(wblocks + (db ? cout : 0)), dim3(256), 0, s, cin, cout, splits, n,
                     cells, (const float *)part, (const _Float16 *)dy, (float *)dw, (float *)db);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // extern "C"
