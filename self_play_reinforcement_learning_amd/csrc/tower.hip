// tower.hip — fused residual-tower inference for the leaf evaluator (gfx950, bf16 MFMA).
//
// Evaluates the trunk of games/general/modules.py ResidualTower (stem conv3x3 +
// BN + ReLU, num_blocks x BasicBlock, and the two 1x1 head convs + BN + ReLU) for a
// batch of boards in ONE launch.  BatchNorm is folded into the conv weights/bias
// on the host (eval-mode statistics), so every layer is conv + bias (+ residual)
// + ReLU.
//
// One workgroup owns BOARDS whole boards (ROWS = 256 or 128 cell rows, NHWC) and
// keeps their activations resident in LDS for the whole tower: two ping-pong
// buffers X / Y of (ROWS + 1) rows x (C*2 + 16) bytes (the +16 pad makes the
// 16-byte MFMA operand reads bank-conflict free; row ROWS is all zeros and stands
// for the conv's zero padding).  A 3x3 conv is an implicit GEMM
//     out[c_out][cell] = sum_{tap, c_in} W[c_out][tap][c_in] * act[nbr(cell, tap)][c_in]
// on v_mfma_f32_32x32x16_bf16: A = weights (32 output channels x 16 k), streamed
// from global memory (L2/MALL resident, pre-swizzled so every wave reads one
// contiguous 1 KiB fragment per k-step), B = activations (16 k x 32 cells) read
// from LDS with a per-(tap, cell) neighbour table.  Each wave owns C/4 output
// channels for all ROWS cells; fp32 accumulators, bf16 activations between
// layers (as the bf16 PyTorch path).  HBM traffic per board: 42 x 3 input planes
// + 42 x 64 head features, i.e. the activations never leave the CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "spmcts.h"
#include "tower_edge.h"

namespace tower {

// The weight ring's loads for the next layer's first DEPTH k-steps are issued unconditionally (the
// last conv re-reads its own first steps, discarded): a conditional load made hipcc merge the ring
// registers with copies at every layer's last k-step, behind an s_waitcnt vmcnt(0) that drained
// the whole weight pipeline once per layer.
#ifndef SPMCTS_RING_ALWAYS
#define SPMCTS_RING_ALWAYS 1
#endif
constexpr bool kRingAlways = SPMCTS_RING_ALWAYS != 0;

// edge-tile layout tables (tower_edge.h): row -> (board, x, y) packed (the inverse map,
// EDGE_CELL_ROW_INIT, is used only by the host-side layout tests)
constexpr uint16_t kEdgeRow[256] = EDGE_ROW_INIT;
// [tap][row] source row (zero rows off the board, at bank positions no on-board lane of the
// 16-lane read group uses)
constexpr uint16_t kEdgeNbr[9 * 256] = EDGE_NBR_INIT;


typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// Element type of the weights, the LDS activations and the head features: bf16, or fp16 = the
// reference's own inference dtype (amp.autocast, inference_worker.py:117).  Operands travel in 16-byte
// containers typed bf16x8 whatever E is (a bit cast at the MFMA is free); both MFMA forms take the
// same cycles on gfx950 (MI355X_MICROARCH.md).  fp32 accumulation either way.
template <class E>
struct Ty;
template <>
struct Ty<__bf16> {
  static constexpr bool BF16 = true;
  static __device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  // relu of a pair, packed (v_cvt_pk_bf16_f32 + v_pk_max_i16: a negative bf16 is a negative int16)
  static __device__ __forceinline__ uint32_t relu_pk(f32x2 v) {
    const bf16x2 b = __builtin_convertvector(v, bf16x2);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2, b), i16x2{0, 0}));
  }
  static __device__ __forceinline__ f32x2 unpk(uint32_t x) {
    return f32x2{__uint_as_float(x << 16), __uint_as_float(x & 0xffff0000u)};
  }
  static __device__ __forceinline__ uint16_t from_bf16(__bf16 x) { return __builtin_bit_cast(uint16_t, x); }
};
template <>
struct Ty<_Float16> {
  static constexpr bool BF16 = false;
  static __device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  }
  // round to nearest even (as torch's fp16 casts), then relu as a signed 16-bit max with 0
  static __device__ __forceinline__ uint32_t relu_pk(f32x2 v) {
    const f16x2 b = __builtin_convertvector(v, f16x2);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2, b), i16x2{0, 0}));
  }
  static __device__ __forceinline__ f32x2 unpk(uint32_t x) {
    return __builtin_convertvector(__builtin_bit_cast(f16x2, x), f32x2);
  }
  static __device__ __forceinline__ uint16_t from_bf16(__bf16 x) {
    return __builtin_bit_cast(uint16_t, (_Float16)(float)x);
  }
};


template <int C_, int ROWS_, int W_, int H_, int CG_ = 2, int WAVES_ = 4, int ABL_ = 0, int DEPTH_ = 4, int OCC_ = 1,
          bool XMAJ_ = false, bool EDGE_ = false, class E_ = __bf16, bool ONEBUF_ = false, bool M16_ = false>
struct Cfg : Ty<E_> {
  // M16 (tower_m16.h): the block convs on v_mfma_f32_16x16x32 with the phys16 channel order
  static constexpr bool M16 = M16_;
  using E = E_;  // operand / activation element type (Ty)
  static constexpr int OCC = OCC_;  // resident workgroups per CU the register budget is sized for
  static constexpr int DEPTH = DEPTH_;  // weight-fragment prefetch distance (k-steps)
  static constexpr int C = C_, ROWS = ROWS_, W = W_, H = H_;
  // ABL: timing ablations for kernel analysis only (results are wrong): 1 = no accumulator init,
  // 2 = no epilogue store, 4 = no inter-layer barrier, 8 = no LDS operand reads in the k-loop,
  // 16 = no weight loads in the k-loop, 128 = half the weight loads (m = 0 only).
  // Schedule/epilogue alternatives (correct results): 64 = accumulator init with bias/residual
  // (instead of a zero first k-step and bias/residual in the epilogue), 256 = loads issued in a
  // burst between MFMA blocks (instead of one per MFMA gap), 2048 = packed-math epilogue,
  // 32768 = weight ring through 64-bit global addresses (instead of a buffer resource).
  static constexpr int ABL = ABL_;
  static constexpr int WAVES = WAVES_, THREADS = 64 * WAVES_;
  static constexpr int CG = CG_;            // waves split output channels into CG groups ...
  static constexpr int MG = WAVES_ / CG_;   // ... and cell rows into MG groups
  static constexpr int CELLS = W * H;
  static constexpr int BOARDS = ROWS / CELLS;
  static constexpr int VROWS = BOARDS * CELLS;
  static constexpr int RS = C * 2 + 16;  // bytes per LDS row
  static constexpr int ZROW = ROWS;
  // 16 zero rows: an off-board neighbour reads the zero row in its own bank position (rows r and
  // r + 16 share banks at a 4-dword row shift), so zero reads never conflict with on-board reads
  static constexpr int NZ = 16;
  static constexpr int NT = ROWS / 32 / MG;  // 32-cell tiles per wave
  static constexpr int MT = C / 32 / CG;     // 32-channel tiles per wave
  static constexpr int BUF = (ROWS + NZ) * RS;
  // Edge tiles (EDGE, a column-major-tile variant): rows ordered by tower_edge.h so that whole cell
  // tiles hold only x = 0, y = 0, x = W-1 or y = H-1 cells; 12 of the workgroup's 72 (tile, tap)
  // pairs read zero padding only and are skipped.  Neighbours are no longer affine row offsets:
  // a 9 x ROWS table of neighbour rows (zero rows for off-board) sits in LDS after the buffers.
  static constexpr bool EDGE = EDGE_ && XMAJ_;
  static constexpr int TAB = EDGE ? 9 * ROWS * 2 : 0;
  // ONEBUF (tower_wide.h): one activation buffer, convs in place between two barriers
  static constexpr bool ONEBUF = ONEBUF_;
  // ONEBUF also stages each conv's bias (C floats) in LDS
  static constexpr int LDS = (ONEBUF ? 1 : 2) * BUF + TAB + (ONEBUF ? C * 4 : 0);
  static constexpr int HEAD = C / 2;  // policy filter_factor | value filter_factor channels (filter_factor = C/4)
  static constexpr int HCT = HEAD / 32;  // head channel tiles
  static_assert(MT >= 1 && NT >= 1 && MT * NT <= (ONEBUF_ ? 16 : 8), "tile plan: at most 8 (one buffer: 16) accumulator tiles per wave");
  static_assert(CG * MG == WAVES, "wave plan");
  static_assert(BOARDS >= 1, "board larger than a tile");
  static_assert(LDS <= 163840, "LDS budget");
  static_assert(!EDGE_ || (W == 7 && H == 6 && ROWS == 256 && BOARDS == 6 && (MG == 2 || MG == 1)),
                "edge layout: 6 Connect4 boards, two row halves or one");
  // Row layout of the tile.  Board-major (default): row = board * CELLS + x * H + y.  Column-major
  // across boards (XMAJ): row = x * (BOARDS * H) + board * H + y, so each board column x of all the
  // tile's boards is BOARDS*H consecutive rows: with 6 boards (36 rows per column) cell tile 0 lies
  // in column 0 and tile 7 in column 6, whose dx = -1 / +1 taps read only zero padding and are
  // skipped (conv_layer_x): 6 of the 72 (tile, tap) pairs of the workgroup, 8.3 % of the MFMAs.
  // A neighbour stays an affine row offset in both layouts: dx * DX + dy.
  static constexpr bool XMAJ = XMAJ_;
  static constexpr int DX = XMAJ ? BOARDS * H : H;
  // (board, x, y) of a row < VROWS
  __host__ __device__ static constexpr int row_board(int row) {
    return EDGE ? kEdgeRow[row] >> 6 : XMAJ ? (row / H) % BOARDS : row / CELLS;
  }
  __host__ __device__ static constexpr int row_x(int row) {
    return EDGE ? (kEdgeRow[row] >> 3) & 7 : XMAJ ? row / (BOARDS * H) : (row % CELLS) / H;
  }
  __host__ __device__ static constexpr int row_y(int row) { return EDGE ? kEdgeRow[row] & 7 : row % H; }
  // does row `row` (< ROWS) hold a cell?  Board-major / column-major tiles: rows < VROWS; edge tiles: the
  // rows tower_edge.h does not mark as padding (255), which may sit anywhere in the tile
  __host__ __device__ static constexpr bool row_ok(int row) { return EDGE ? kEdgeRow[row] != 255 : row < VROWS; }
  // does any on-board row of cell tile T have an on-board neighbour for `tap`?
  __host__ __device__ static constexpr bool tile_tap_live(int T, int tap) {
    for (int r = T * 32; r < T * 32 + 32 && r < ROWS; ++r) {
      if (!row_ok(r)) continue;
      const int nx = row_x(r) + tap / 3 - 1, ny = row_y(r) + tap % 3 - 1;
      if (nx >= 0 && nx < W && ny >= 0 && ny < H) return true;
    }
    return false;
  }
  __host__ __device__ static constexpr int row_cell(int row) { return row_x(row) * H + row_y(row); }
  // does any on-board row of 32-row cell tile T have an on-board neighbour column x + dx?
  __host__ __device__ static constexpr bool tile_dx_live(int T, int dx) {
    for (int r = T * 32; r < T * 32 + 32 && r < ROWS; ++r) {
      if (!row_ok(r)) continue;
      const int nx = row_x(r) + dx;
      if (nx >= 0 && nx < W) return true;
    }
    return false;
  }
};

__device__ __forceinline__ bf16x8 lds_b128(const char *p) { return *(const bf16x8 *)p; }

// Weight fragments through a buffer resource: the per-lane part of the address is a constant
// 32-bit voffset (lane * 16) and the fragment's byte offset is a wave-uniform soffset, so a ring
// refill is one buffer_load_dwordx4 with no per-load 64-bit address arithmetic.
struct WBuf {
  __amdgpu_buffer_rsrc_t rsrc;
  int voff;
  template <int AUX = 0>
  __device__ __forceinline__ bf16x8 load(uint32_t byte_off) const {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, (int)byte_off, AUX);
    return __builtin_bit_cast(bf16x8, v);
  }
};

// One conv layer over the resident tile: src (LDS) -> dst (LDS), optional residual (LDS, == dst).
// KK = input channels / 16 (k-steps per tap), TAPS = 9 (3x3).
// Software pipeline: the 8 B (activation) fragments of step s+1 are read from LDS while
// the MFMAs of step s run, and the A (weight) fragment is fetched DEPTH steps ahead from
// L2/MALL (~4 x 256 MFMA cycles of cover for the memory latency).
// Per-lane neighbour geometry: for each of the wave's cell tiles t, the byte offset of the
// lane's cell row and a 9-bit mask of the taps whose neighbour lies on the board.
template <class K>
struct Nbr {
  int base[K::NT];
  int rowi[K::NT];
  uint32_t mask[K::NT];
  const uint16_t *tab;  // Cfg::EDGE: LDS neighbour-row table [9][ROWS]
  int off0[K::NT];      // tap 0's operand offsets (the same for every layer; set by finish())
  __device__ __forceinline__ void init(int r, int mg) {
#pragma unroll
    for (int t = 0; t < K::NT; ++t) {
      const int row = (mg * K::NT + t) * 32 + r;
      base[t] = row * K::RS;
      rowi[t] = row;
      uint32_t m = 0;
      if (K::row_ok(row)) {
        const int x = K::row_x(row), y = K::row_y(row);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int nx = x + tap / 3 - 1, ny = y + tap % 3 - 1;
          if (nx >= 0 && nx < K::W && ny >= 0 && ny < K::H) m |= 1u << tap;
        }
      }
      mask[t] = m;
    }
  }
  // once the table is in LDS: tap 0's offsets, kept for every layer's first operand reads (a table
  // read there would stall each layer start on an LDS round trip)
  __device__ __forceinline__ void finish() {
#pragma unroll
    for (int t = 0; t < K::NT; ++t) off0[t] = off(t, 0);
  }
  // Cfg::EDGE: the source row of tile t for `tap` (an LDS table read; times RS = off())
  __device__ __forceinline__ int row(int t, int tap) const { return (int)tab[tap * K::ROWS + rowi[t]]; }
  // byte offset of the source row of tile t for `tap` (the zero row when off the board); a
  // branch-free select (hipcc otherwise emits an exec-mask branch per tile and tap)
  __device__ __forceinline__ int off(int t, int tap) const {
    if constexpr (K::EDGE) return (int)tab[tap * K::ROWS + rowi[t]] * K::RS;
    const int dr = (tap / 3 - 1) * K::DX + (tap % 3 - 1);
    const int on = base[t] + dr * K::RS;
    const int zero = (K::ZROW + ((rowi[t] + dr) & (K::NZ - 1))) * K::RS;
    const int live = (int)((mask[t] >> tap) & 1u);
    return zero + live * (on - zero);
  }
};

// Channel order in LDS.  A lane's 16 accumulator values of a 32x32 MFMA tile are the output channels
// ct*32 + 8g + 4h + j (g, j = 0..3, h = lane half); they are stored at the PHYSICAL positions
// ct*32 + 16h + 4g + j, so that each lane's 16 values are one contiguous 32-byte run (two 16-byte
// LDS stores instead of four 8-byte ones; the epilogue's store burst is the layer boundary's cost).
// The next layer's weights are packed with their input channels in the same physical order
// (evaluator._pack_conv(in_perm=True)), so the MFMAs see consistent K chunks.
__device__ __forceinline__ int phys_off(int ct, int h, int g) { return (ct * 32 + 16 * h + 4 * g) * 2; }

// Accumulator initialisation: bias (and, for the second conv of a block, the residual input,
// which lives at the output location in dst) so the epilogue is only ReLU + bf16 + store.
template <class K, bool RESID>
__device__ __forceinline__ void acc_init(f32x16 (&acc)[K::MT][K::NT], const char *dst, const float *bias, int wave,
                                         int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int m = 0; m < K::MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = ((wave % K::CG) * K::MT + m) * 32 + 8 * g + 4 * h;
      const float4 bv = *(const float4 *)(bias + ch);
#pragma unroll
      for (int t = 0; t < K::NT; ++t) {
        float v0 = bv.x, v1 = bv.y, v2 = bv.z, v3 = bv.w;
        if (RESID) {
          const uint2 x = *(const uint2 *)(dst + (((wave / K::CG) * K::NT + t) * 32 + r) * K::RS +
                                           phys_off((wave % K::CG) * K::MT + m, h, g));
          const f32x2 lo = K::unpk(x.x), hi = K::unpk(x.y);
          v0 += lo[0];
          v1 += lo[1];
          v2 += hi[0];
          v3 += hi[1];
        }
        acc[m][t][4 * g + 0] = v0;
        acc[m][t][4 * g + 1] = v1;
        acc[m][t][4 * g + 2] = v2;
        acc[m][t][4 * g + 3] = v3;
      }
    }
}

// Epilogue with bias (and residual) added here instead of in the accumulator init (the first
// k-step's MFMAs then start from zero): out = relu(acc + bias (+ dst)), bf16, into dst.
template <class K, bool RESID>
__device__ __forceinline__ void acc_store_bias_relu(const f32x16 (&acc)[K::MT][K::NT], char *dst, const float *bias,
                                                    int wave, int lane) {
  static_assert(K::BF16, "timing-ablation epilogue: bf16 tiles only");
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int m = 0; m < K::MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = ((wave % K::CG) * K::MT + m) * 32 + 8 * g + 4 * h;
      const float4 bv = *(const float4 *)(bias + ch);
#pragma unroll
      for (int t = 0; t < K::NT; ++t) {
        char *p = dst + (((wave / K::CG) * K::NT + t) * 32 + r) * K::RS + phys_off((wave % K::CG) * K::MT + m, h, g);
        float v0 = acc[m][t][4 * g + 0] + bv.x, v1 = acc[m][t][4 * g + 1] + bv.y;
        float v2 = acc[m][t][4 * g + 2] + bv.z, v3 = acc[m][t][4 * g + 3] + bv.w;
        if (RESID) {
          const bf16x4 x = *(const bf16x4 *)p;
          v0 += (float)x[0];
          v1 += (float)x[1];
          v2 += (float)x[2];
          v3 += (float)x[3];
        }
        bf16x4 o;
        o[0] = (__bf16)fmaxf(v0, 0.f);
        o[1] = (__bf16)fmaxf(v1, 0.f);
        o[2] = (__bf16)fmaxf(v2, 0.f);
        o[3] = (__bf16)fmaxf(v3, 0.f);
        *(bf16x4 *)p = o;
      }
    }
}

// ReLU of a pair as bf16: convert, then a signed 16-bit max with 0 (a negative bf16 is a negative int16).
__device__ __forceinline__ uint32_t relu_pk_bf16(f32x2 v) { return Ty<__bf16>::relu_pk(v); }

// acc_store_bias_relu with the bias already in registers (bv[m][g] = bias[ch(m, g) .. + 4], loaded
// at the start of the layer so its global-load latency hides under the k-loop instead of stalling
// the epilogue).
template <class K, bool RESID>
__device__ __forceinline__ void acc_store_bias_relu_pre(const f32x16 (&acc)[K::MT][K::NT], char *dst,
                                                        const float4 (&bv)[K::MT][4], int wave, int lane) {
  const int r = lane & 31, h = lane >> 5;
  // per channel tile m: the residuals (block input) of its NT output runs are read in one batch
  // before any of them is written, so the LDS latency is paid once per batch instead of once per
  // read -> add -> write chain; each run is the lane's 16 channels, contiguous (phys_off)
#pragma unroll
  for (int m = 0; m < K::MT; ++m) {
    const int ct = (wave % K::CG) * K::MT + m;
    uint4 res[RESID ? K::NT : 1][2];
    if constexpr (RESID) {
#pragma unroll
      for (int t = 0; t < K::NT; ++t) {
        const char *p = dst + (((wave / K::CG) * K::NT + t) * 32 + r) * K::RS + phys_off(ct, h, 0);
        res[t][0] = *(const uint4 *)p;
        res[t][1] = *(const uint4 *)(p + 16);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < K::NT; ++t) {
      char *p = dst + (((wave / K::CG) * K::NT + t) * 32 + r) * K::RS + phys_off(ct, h, 0);
      uint32_t o[8];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v0 = acc[m][t][4 * g + 0] + bv[m][g].x, v1 = acc[m][t][4 * g + 1] + bv[m][g].y;
        float v2 = acc[m][t][4 * g + 2] + bv[m][g].z, v3 = acc[m][t][4 * g + 3] + bv[m][g].w;
        if constexpr (RESID) {
          const f32x2 x0 = K::unpk(((const uint32_t *)&res[t][g >> 1])[2 * (g & 1)]);
          const f32x2 x1 = K::unpk(((const uint32_t *)&res[t][g >> 1])[2 * (g & 1) + 1]);
          v0 += x0[0];
          v1 += x0[1];
          v2 += x1[0];
          v3 += x1[1];
        }
        // ReLU on the converted pairs (bf16: v_cvt_pk_bf16_f32 + v_pk_max_i16: identical bits to
        // converting max(v, 0), one instruction per pair instead of one per value)
        o[2 * g] = K::relu_pk(f32x2{v0, v1});
        o[2 * g + 1] = K::relu_pk(f32x2{v2, v3});
      }
      *(uint4 *)p = make_uint4(o[0], o[1], o[2], o[3]);
      *(uint4 *)(p + 16) = make_uint4(o[4], o[5], o[6], o[7]);
    }
  }
}

// Packed-math form of acc_store_bias_relu: v_pk_add_f32 for bias (and residual), one
// v_cvt_pk_bf16_f32 per pair, ReLU on the packed bf16 pair as a signed 16-bit max with 0
// (v_pk_max_i16: a bf16 with the sign bit set is a negative int16).

template <class K, bool RESID>
__device__ __forceinline__ void acc_store_bias_relu_pk(const f32x16 (&acc)[K::MT][K::NT], char *dst, const float *bias,
                                                       int wave, int lane) {
  static_assert(K::BF16, "timing-ablation epilogue: bf16 tiles only");
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int m = 0; m < K::MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = ((wave % K::CG) * K::MT + m) * 32 + 8 * g + 4 * h;
      const float4 bv = *(const float4 *)(bias + ch);
      const f32x2 b01 = {bv.x, bv.y}, b23 = {bv.z, bv.w};
#pragma unroll
      for (int t = 0; t < K::NT; ++t) {
        char *p = dst + (((wave / K::CG) * K::NT + t) * 32 + r) * K::RS + phys_off((wave % K::CG) * K::MT + m, h, g);
        f32x2 lo = f32x2{acc[m][t][4 * g + 0], acc[m][t][4 * g + 1]} + b01;
        f32x2 hi = f32x2{acc[m][t][4 * g + 2], acc[m][t][4 * g + 3]} + b23;
        if (RESID) {
          const uint2 x = *(const uint2 *)p;
          lo += f32x2{__uint_as_float(x.x << 16), __uint_as_float(x.x & 0xffff0000u)};
          hi += f32x2{__uint_as_float(x.y << 16), __uint_as_float(x.y & 0xffff0000u)};
        }
        *(uint2 *)p = make_uint2(relu_pk_bf16(lo), relu_pk_bf16(hi));
      }
    }
}

template <class K>
__device__ __forceinline__ void acc_store_relu(const f32x16 (&acc)[K::MT][K::NT], char *dst, int wave, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int m = 0; m < K::MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
#pragma unroll
      for (int t = 0; t < K::NT; ++t) {
        const uint2 o = make_uint2(K::relu_pk(f32x2{acc[m][t][4 * g + 0], acc[m][t][4 * g + 1]}),
                                   K::relu_pk(f32x2{acc[m][t][4 * g + 2], acc[m][t][4 * g + 3]}));
        *(uint2 *)(dst + (((wave / K::CG) * K::NT + t) * 32 + r) * K::RS + phys_off((wave % K::CG) * K::MT + m, h, g)) = o;
      }
    }
}

// One 3x3 conv layer over the resident tile: src (LDS) -> dst (LDS); RESID adds dst's old
// contents (the block input).  KK = input channels / 16 (k-steps per tap).
// Software pipeline: the NT B (activation) fragments of step s+1 are read from LDS while the
// MFMAs of step s run; the A (weight) fragment ring runs DEPTH steps ahead and continues into
// the next layer's weights (wn_off), so a layer starts with its first weights already in registers.
// (The A/B library's timing-ablation copy: tower_abl.h conv_layer_abl.)
template <class K, int KK, int DEPTH, bool RESID>
__device__ __forceinline__ void conv_layer(const char *src, char *dst, const Nbr<K> &nb, bf16x8 (&a)[DEPTH][K::MT],
                                           const float *bias, int wave, int lane, const WBuf &wb, uint32_t wl_off,
                                           uint32_t wn_off, int wn_steps) {
  // wl_off / wn_off: byte offset of (this layer / next layer, this wave's first channel tile, step 0);
  // channel tile m adds m * 9 * KK fragments of 1 KiB, step s adds s KiB
  constexpr uint32_t MSTRIDE = 9u * KK * 1024u;
  constexpr int STEPS = 9 * KK;
  static_assert(KK % DEPTH == 0, "ring slot must be a compile-time function of kk");
  const int h = lane >> 5;
  f32x16 acc[K::MT][K::NT];  // the first k-step starts from zero; bias and residual are added in the epilogue
  const int hoff = 16 * h;  // byte offset of this lane's 8 channels inside a 16-channel k-step
  // the epilogue's bias, fetched now, so the global-load latency hides under the k-loop
  float4 bv[K::MT][4];
#pragma unroll
  for (int m = 0; m < K::MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) bv[m][g] = *(const float4 *)(bias + ((wave % K::CG) * K::MT + m) * 32 + 8 * g + 4 * h);
  int off_cur[K::NT], off_nxt[K::NT];
#pragma unroll
  for (int t = 0; t < K::NT; ++t) off_cur[t] = nb.off(t, 0) + hoff;
  bf16x8 bc[K::NT], bn[K::NT];
#pragma unroll
  for (int t = 0; t < K::NT; ++t) bc[t] = lds_b128(src + off_cur[t]);

  // taps fully unrolled: a straight-line k-loop schedules 4-7 % faster than a rolled tap loop
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    if (tap + 1 < 9) {
#pragma unroll
      for (int t = 0; t < K::NT; ++t) off_nxt[t] = nb.off(t, tap + 1) + hoff;
    }
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int s = tap * KK + kk;
      if (kk + 1 < KK) {
#pragma unroll
        for (int t = 0; t < K::NT; ++t) bn[t] = lds_b128(src + off_cur[t] + (kk + 1) * 32);
      } else if (tap + 1 < 9) {
#pragma unroll
        for (int t = 0; t < K::NT; ++t) bn[t] = lds_b128(src + off_nxt[t]);
      }
      const int slot = kk % DEPTH;
      bf16x8 acur[K::MT];
#pragma unroll
      for (int m = 0; m < K::MT; ++m) acur[m] = a[slot][m];
      const int sn = s + DEPTH;
      if (sn < STEPS) {
#pragma unroll
        for (int m = 0; m < K::MT; ++m) a[slot][m] = wb.load(wl_off + m * MSTRIDE + (uint32_t)sn * 1024u);
      } else if (kRingAlways || sn - STEPS < wn_steps) {
#pragma unroll
        for (int m = 0; m < K::MT; ++m) a[slot][m] = wb.load(wn_off + m * MSTRIDE + (uint32_t)(sn - STEPS) * 1024u);
      }
      if (s == 0) {
#pragma unroll
        for (int t = 0; t < K::NT; ++t)
#pragma unroll
          for (int m = 0; m < K::MT; ++m)
            acc[m][t] = K::mfma(acur[m], bc[t], f32x16{});
      } else {
#pragma unroll
        for (int t = 0; t < K::NT; ++t)
#pragma unroll
          for (int m = 0; m < K::MT; ++m)
            acc[m][t] = K::mfma(acur[m], bc[t], acc[m][t]);
      }
      // interleave this step's loads (next B fragments, ring refill) between its MFMAs:
      // one LDS read or global load per MFMA gap instead of a burst between MFMA blocks
#pragma unroll
      for (int i = 0; i < K::NT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      }
#pragma unroll
      for (int i = 0; i < K::MT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
      }
      __builtin_amdgcn_sched_group_barrier(0x008, K::MT * K::NT - K::NT - K::MT, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < K::NT; ++t) bc[t] = bn[t];
    }
#pragma unroll
    for (int t = 0; t < K::NT; ++t) off_cur[t] = off_nxt[t];
  }
  acc_store_bias_relu_pre<K, RESID>(acc, dst, bv, wave, lane);
}

// Per-tap live cell tiles of a column-major / edge-tile layer (Cfg::XMAJ, Cfg::EDGE) for the waves of row
// group MG_: a tile all of whose rows lie in board column 0 (dx = -1) or W-1 (dx = +1), or whose taps read
// zero padding only (edge tiles), would multiply zeros; its MFMAs and operand reads are skipped (the
// skipped contributions are exact zeros).  Used by the 16x16x32 trunk (tower_m16.h) and the A/B library's
// 32x32x16 k-loops (tower_abl.h).
template <class K, int MG_>
struct XLive {
  static constexpr uint32_t mask(int g) {
    uint32_t m = 0;
    for (int t = 0; t < K::NT; ++t)
      if (K::tile_dx_live(MG_ * K::NT + t, g - 1)) m |= 1u << t;
    return m;
  }
  static constexpr uint32_t popc(uint32_t m) { return m ? (m & 1u) + popc(m >> 1) : 0u; }
  static constexpr uint32_t ALL = (1u << K::NT) - 1;
  static constexpr uint32_t LIVE[3] = {mask(0), mask(1), mask(2)};
  // tiles not live in group 0 miss the zero-start step 0: their accumulators start at zero
  static constexpr uint32_t ZPRE = ALL & ~LIVE[0];
  // per-tap live tiles (Cfg::EDGE: a tile can be dead for taps of one dy as well)
  static constexpr uint32_t lt(int tap) {
    uint32_t m = 0;
    for (int t = 0; t < K::NT; ++t)
      if (K::tile_tap_live(MG_ * K::NT + t, tap)) m |= 1u << t;
    return m;
  }
  static constexpr uint32_t ZPRE_T = ALL & ~lt(0);
};


// Stem: 3 input planes padded to one 16-channel k-step per tap (9 steps, weights loaded in place).
template <class K>
__device__ __forceinline__ void stem_layer(const char *src, char *dst, const Nbr<K> &nb, const bf16x8 *w,
                                           const float *bias, int wave, int lane) {
  const int h = lane >> 5;
  f32x16 acc[K::MT][K::NT];
  acc_init<K, false>(acc, dst, bias, wave, lane);
  bf16x8 a[9][K::MT];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int m = 0; m < K::MT; ++m) a[tap][m] = w[((size_t)((wave % K::CG) * K::MT + m) * 9 + tap) * 64 + lane];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int t = 0; t < K::NT; ++t) {
      const bf16x8 b = lds_b128(src + nb.off(t, tap) + 16 * h);
#pragma unroll
      for (int m = 0; m < K::MT; ++m)
        acc[m][t] = K::mfma(a[tap][m], b, acc[m][t]);
    }
  }
  acc_store_relu<K>(acc, dst, wave, lane);
}

// 1x1 head convs (C -> C/4 policy | C/4 value) + bias + ReLU, to global features
// [board][cell][C/2] (cell-major: the order the NHWC-reordered linear heads expect).
template <class K>
__device__ __forceinline__ void head_layer(const char *src, const bf16x8 *w, const float *bias, uint16_t *out,
                                           int board0, int batch, int wave, int lane) {
  constexpr int KK = K::C / 16;
  constexpr int GROUPS = K::WAVES / K::HCT;  // waves sharing one head channel tile
  constexpr int TILES = K::ROWS / 32;      // all cell tiles of the workgroup
  constexpr int TPW = TILES / GROUPS;      // cell tiles per wave
  static_assert(K::HCT * GROUPS == K::WAVES && TPW * GROUPS == TILES, "head tile plan");
  const int r = lane & 31, h = lane >> 5;
  const int ct = wave % K::HCT;
  const int t0 = (wave / K::HCT) * TPW;
  f32x16 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  // all KK weight fragments requested up front: one global-load latency instead of one per group
  bf16x8 wf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) wf[kk] = w[((size_t)ct * KK + kk) * 64 + lane];
  // the epilogue's bias too (fetched inside the store loop, each fetch waited behind the stores)
  float4 bvs[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) bvs[g] = *(const float4 *)(bias + ct * 32 + 8 * g + 4 * h);
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    const bf16x8 a = wf[kk];
    const int koff = (kk * 16 + 8 * h) * 2;
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int cell = (t0 + t) * 32 + r;
      const bf16x8 b = lds_b128(src + cell * K::RS + koff);
      acc[t] = K::mfma(a, b, acc[t]);
    }
  }
  // each lane's output rows, looked up once per cell tile (the row -> board/cell table is read from
  // global memory: looked up inside the store loop, every lookup waited for its own load)
  size_t obase[TPW];
  bool okr[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int row = (t0 + t) * 32 + r;
    const int rr = K::row_ok(row) ? row : 0;
    const int board = board0 + K::row_board(rr);
    okr[t] = K::row_ok(row) && board < batch;
    obase[t] = ((size_t)board * K::CELLS + K::row_cell(rr)) * K::HEAD;
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int ch = ct * 32 + 8 * g + 4 * h;
    const float4 bv = bvs[g];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if (!okr[t]) continue;
      *(uint2 *)(out + obase[t] + ch) = make_uint2(K::relu_pk(f32x2{acc[t][4 * g + 0] + bv.x, acc[t][4 * g + 1] + bv.y}),
                                                   K::relu_pk(f32x2{acc[t][4 * g + 2] + bv.z, acc[t][4 * g + 3] + bv.w}));
    }
  }
}

// Packed weight blob (bf16x8 units) and bias blob (floats), in layer order:
//   stem   [C/32][9][1][64 lanes]      k = 16 input channels (3 planes + 13 zero)
//   block  2 x [C/32][9][C/16][64]      per BasicBlock (conv1, conv2)
//   head   [C/64][1][C/16][64]          policy C/4 | value C/4 output channels
// lane l of fragment (ct, tap, kk) holds W[ct*32 + (l & 31)][tap][kk*16 + 8*(l >> 5) + j], j = 0..7.
// bias: stem C, blocks 2*C each, head C/2.
// One workgroup's tile: boards [board0, board0 + BOARDS) of the batch (board < batch), all layers.
#ifdef SPMCTS_AB
#include "tower_abl.h"  // timing ablations and the 32x32x16 column-group k-loops (A/B library only)
#endif
#include "tower_wide.h"
#include "tower_m16.h"
#include "tower_wide16.h"

template <class K>
__device__ __forceinline__ void tower_tile(char *smem, const __bf16 *planes, int batch, int board0, int n_blocks,
                                           const bf16x8 *wpk, const float *bias, uint16_t *out, uint4 *scr) {
  if constexpr (K::ONEBUF && K::M16) {
    wide16::tile<K>(smem, planes, batch, board0, n_blocks, wpk, bias, out, scr + blockIdx.x * (wide::Scr<K>::PER_WG / 16));
    return;
  } else if constexpr (K::ONEBUF) {
#ifdef SPMCTS_AB
    wide::tile<K>(smem, planes, batch, board0, n_blocks, wpk, bias, out, scr + blockIdx.x * (wide::Scr<K>::PER_WG / 16));
#else
    static_assert(K::M16, "the product's one-buffer trunk is the 16x16x32 form (tower_wide16.h)");
#endif
    return;
  }
  if constexpr (K::M16 && !K::ONEBUF) {
    m16::tile<K>(smem, planes, batch, board0, n_blocks, wpk, bias, out);
    return;
  }
  char *X = smem;
  char *Y = smem + K::BUF;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  Nbr<K> nb;
  nb.init(lane & 31, wave / K::CG);

  // zero rows + stem input: Y rows hold 16 channels (3 planes, 13 zeros)
  for (int i = tid; i < K::NZ * K::RS / 4; i += K::THREADS) {
    ((uint32_t *)(X + K::ZROW * K::RS))[i] = 0u;
    ((uint32_t *)(Y + K::ZROW * K::RS))[i] = 0u;
  }
  if constexpr (K::EDGE) {
    uint16_t *tab = (uint16_t *)(smem + 2 * K::BUF);
    static_assert(K::ROWS == 256 && K::ZROW == 256, "EDGE_NBR is laid out for 256-row tiles");
    // unrolled so all of a thread's table loads are in flight at once (a rolled loop waited for each)
#pragma unroll
    for (int j = 0; j < (9 * K::ROWS + K::THREADS - 1) / K::THREADS; ++j)
      if (9 * K::ROWS % K::THREADS == 0 || tid + j * K::THREADS < 9 * K::ROWS)
        tab[tid + j * K::THREADS] = kEdgeNbr[tid + j * K::THREADS];
    nb.tab = tab;
  }
  for (int row = tid; row < K::ROWS; row += K::THREADS) {
    const int board = board0 + K::row_board(row);
    uint16_t *dst = (uint16_t *)(Y + row * K::RS);
    const bool ok = K::row_ok(row) && board < batch;
    const size_t src = ((size_t)board * K::CELLS + K::row_cell(row)) * 3;
#pragma unroll
    for (int c = 0; c < 16; ++c) dst[c] = (ok && c < 3) ? K::from_bf16(planes[src + c]) : (uint16_t)0;
  }
  __syncthreads();
  nb.finish();

  constexpr int KK = K::C / 16;
  constexpr int DEPTH = K::DEPTH;
  constexpr size_t STEM = (size_t)K::C / 32 * 9 * 64;          // stem fragments
  constexpr size_t LAYER = (size_t)K::C / 32 * 9 * KK * 64;     // one block conv's fragments
  constexpr int LSTEPS = 9 * KK;
  stem_layer<K>(Y, X, nb, wpk, bias, wave, lane);
  __syncthreads();
  const bf16x8 *wblk = wpk + STEM;
  const float *b = bias + K::C;
  // per-wave weight streams: layer L, ctile (wave*MT + m) starts at wblk + L*LAYER + ct*LSTEPS*64 + lane
  bf16x8 ring[DEPTH][K::MT];
  const int n_convs = 2 * n_blocks;
  if (n_convs > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int m = 0; m < K::MT; ++m)
        ring[d][m] = wblk[(size_t)((wave % K::CG) * K::MT + m) * LSTEPS * 64 + (size_t)d * 64 + lane];
  }
  WBuf wb;
  wb.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)wpk, (short)0, 0x7fffffff, 0x00020000);
  wb.voff = lane * 16;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t ct0_off = (uint32_t)(STEM + (size_t)((wave_u % K::CG) * K::MT) * LSTEPS * 64) * 16u;
  for (int L = 0; L < n_convs; ++L) {
    const uint32_t wl_off = ct0_off + (uint32_t)((size_t)L * LAYER * 16u);
    const uint32_t wn_off = (kRingAlways && L + 1 == n_convs) ? wl_off : wl_off + (uint32_t)(LAYER * 16u);
    const int wn_steps = L + 1 < n_convs ? LSTEPS : 0;
#ifdef SPMCTS_AB
    if constexpr (K::XMAJ || K::ABL != 0) {  // the A/B library's 32x32x16 column-group trunks and ablations
      const bf16x8 *wl[K::MT], *wn[K::MT];
#pragma unroll
      for (int m = 0; m < K::MT; ++m) {
        const size_t ct = (size_t)((wave % K::CG) * K::MT + m) * LSTEPS * 64 + lane;
        wl[m] = wblk + (size_t)L * LAYER + ct;
        wn[m] = wblk + (size_t)(L + 1) * LAYER + ct;
      }
      conv_layer_ab<K, KK, DEPTH>(L, X, Y, nb, wl, wn, wn_steps, ring, b, wave, lane, wb, wl_off, wn_off);
      b += K::C;
      layer_barrier<K>();
      continue;
    }
#else
    static_assert(K::M16 || K::ONEBUF || (!K::XMAJ && K::ABL == 0),
                  "the product's board-major trunk (its column-group tiles: tower_m16.h, tower_wide16.h)");
#endif
    if ((L & 1) == 0) {
      conv_layer<K, KK, DEPTH, false>(X, Y, nb, ring, b, wave, lane, wb, wl_off, wn_off, wn_steps);
    } else {
      conv_layer<K, KK, DEPTH, true>(Y, X, nb, ring, b, wave, lane, wb, wl_off, wn_off, wn_steps);
    }
    b += K::C;
    __syncthreads();
  }
  const bf16x8 *w = wblk + (size_t)n_convs * LAYER;
  head_layer<K>(X, w, b, out, board0, batch, wave, lane);
}

#ifdef SPMCTS_AB
#include "tower_ring.h"  // the LDS weight-ring trunk (measured 3-6 % slower; A/B library only)
#endif

template <class K>
__global__ __launch_bounds__(K::THREADS) __attribute__((amdgpu_waves_per_eu(K::WAVES / 4 * K::OCC, K::WAVES / 4 * K::OCC))) void k_tower(
    const __bf16 *planes, int batch, int n_blocks, const bf16x8 *wpk, const float *bias, uint16_t *out, uint4 *scr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  tower_tile<K>(smem, planes, batch, blockIdx.x * K::BOARDS, n_blocks, wpk, bias, out, scr);
}

// Tail tile for a remainder of `rem` boards after whole rounds of full tiles: the smallest tile
// (fewest LDS rows, so the shortest workgroup) whose one round of `cus` workgroups covers it.
// 0 = half (KH), 1 = middle (KM), 2 = full (KF).
template <class KF, class KM, class KH>
__host__ __device__ __forceinline__ int tail_kind(int rem, int cus) {
  if (rem <= cus * KH::BOARDS) return 0;
  if (rem <= cus * KM::BOARDS) return 1;
  return 2;
}

// Device-count driven variant: the batch size is read from device memory (the arena's leaf-row
// counter), so the host never waits for it.  Workgroups are assigned as in launch_split: whole
// chip rounds of full-size tiles, then the remainder in one round of the smallest tile that covers
// it (tail_kind); surplus workgroups of the (maximum-size) grid exit at once.
template <class KF, class KM, class KH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_tower_dyn(
    const __bf16 *planes, const int32_t *count, int max_batch, int cus, int n_blocks, const bf16x8 *wpk,
    const float *bias, uint16_t *out, uint4 *scr) {
  static_assert(KF::THREADS == 256 && KM::THREADS == 256 && KH::THREADS == 256, "one block size");
  // residual scratch is sized per workgroup of the full tiles (scratch_bytes<KF>): a one-buffer tail tile
  // must be the full tile itself
  static_assert((!KM::ONEBUF || std::is_same<KM, KF>::value) && (!KH::ONEBUF || std::is_same<KH, KF>::value),
                "one-buffer tail tiles must be the full tiles");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = min(*count, max_batch);  // never past the caller's buffers
  const int full_wgs = (n / KF::BOARDS) / cus * cus;
  const int n_full = full_wgs * KF::BOARDS;
  const int rem = n - n_full;
  const int b = blockIdx.x;
  if constexpr (std::is_same<KM, KF>::value && std::is_same<KH, KF>::value) {
    // one tile kind: one inlined copy of the tile body (whole rounds and the tail alike)
    const int board0 = b < full_wgs ? b * KF::BOARDS : n_full + (b - full_wgs) * KF::BOARDS;
    if (board0 < n) tower_tile<KF>(smem, planes, n, board0, n_blocks, wpk, bias, out, scr);
    return;
  }
  if (b < full_wgs) {
    tower_tile<KF>(smem, planes, n, b * KF::BOARDS, n_blocks, wpk, bias, out, scr);
    return;
  }
  const int j = b - full_wgs;
  const int kind = tail_kind<KF, KM, KH>(rem, cus);
  if (kind == 0) {
    if (n_full + j * KH::BOARDS < n) tower_tile<KH>(smem, planes, n, n_full + j * KH::BOARDS, n_blocks, wpk, bias, out, scr);
  } else if (kind == 1) {
    if (n_full + j * KM::BOARDS < n) tower_tile<KM>(smem, planes, n, n_full + j * KM::BOARDS, n_blocks, wpk, bias, out, scr);
  } else {
    if (n_full + j * KF::BOARDS < n) tower_tile<KF>(smem, planes, n, n_full + j * KF::BOARDS, n_blocks, wpk, bias, out, scr);
  }
}

// ---------------------------------------------------------------------------------------
// Linear heads (modules.py:96-105 after the 1x1 convs), fused, for BOARDS boards per workgroup:
//   policy = softmax(pf @ Wp^T + bp)          pf = features[:, :, :ff]  (cell-major, K = cells*ff)
//   value  = tanh(relu(vf @ Wv^T + bv) @ wo + bo)                     vf = features[:, :, ff:]
// on v_mfma_f32_32x32x16_bf16 (M = 32 rows of which BOARDS are boards, N = 32 weight rows).
// The workgroup's features are staged once into LDS (coalesced; per-board stride padded by 16 B
// so the 16-B operand reads of 16 different boards are bank-conflict free); weight fragments are
// pre-swizzled on the host (one contiguous KiB per (32-row tile, 16-k step): lane (r, h) holds
// W[tile*32 + r][16 s + 8 h .. + 8]) and streamed through a 4-deep register ring.  Wave w owns
// value tiles [w*VTW, (w+1)*VTW) over all of K and the policy tile over a quarter of K; partial
// sums are combined in a fixed order (deterministic, batch-independent).
// Weight blob: tile 0 = Wp padded to 32 rows, tiles 1..VT = Wv; float blob: bp[32], bv[8ff], wo[8ff], bo.
template <int FF, int CELLS, int A>
struct HeadsCfg {
  static constexpr int K = CELLS * FF, KS = K / 16, HID = 8 * FF, VT = HID / 32, VTW = VT / 4;
  static constexpr int FROW = CELLS * 2 * FF * 2;  // feature bytes per board
  static constexpr int BOARDS = FROW * 16 + 16 * 16 <= 96 * 1024 ? 16 : 8;
  static constexpr int FS = FROW + 16;             // LDS stride per board
  static constexpr int KQ = (KS + 3) / 4;          // policy k-steps per wave
  static_assert(VT % 4 == 0 && FF % 16 == 0 && FROW % 16 == 0, "head tile plan");
};

template <int FF, int CELLS, int A, class E = __bf16>
__global__ __launch_bounds__(256) void k_heads(const uint16_t *feats, int n, const int32_t *count, const bf16x8 *wf,
                                               const float *hb, float *probs, float *values) {
  using H = HeadsCfg<FF, CELLS, A>;
  if (count) n = min(*count, n);  // n = the caller's buffer rows
  const int b0 = blockIdx.x * H::BOARDS;
  if (b0 >= n) return;
  __shared__ __attribute__((aligned(16))) char s_feat[H::BOARDS * H::FS];
  __shared__ float s_part[4][32];        // per-wave value partial sums
  __shared__ float s_pol[4][32][33];     // per-wave policy partial logits
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int nb = min(H::BOARDS, n - b0);
  // stage the features of this workgroup's boards (16 B per thread-iteration, coalesced)
  {
    constexpr int CH = H::FROW / 16;
    const uint4 *src = (const uint4 *)(feats + (size_t)b0 * CELLS * 2 * FF);
    for (int i = tid; i < H::BOARDS * CH; i += 256) {
      const int bd = i / CH, c = i % CH;
      const uint4 v = bd < nb ? src[(size_t)bd * CH + c] : make_uint4(0, 0, 0, 0);
      *(uint4 *)(s_feat + bd * H::FS + c * 16) = v;
    }
  }
  const float *bp = hb, *bv = hb + 32, *wo = hb + 32 + H::HID, *bo = hb + 32 + 2 * H::HID;
  const int row = r % H::BOARDS;  // rows >= BOARDS duplicate a board; their results are ignored
  const char *frow = s_feat + row * H::FS;
  f32x16 acc[H::VTW];
  f32x16 pacc = {};
#pragma unroll
  for (int v = 0; v < H::VTW; ++v) acc[v] = f32x16{};
  // weight ring: VTW value fragments (+ 1 policy fragment while s is in this wave's quarter)
  constexpr int D = 4;
  bf16x8 ring[D][H::VTW];
  const bf16x8 *wv = wf + (size_t)(1 + wave * H::VTW) * H::KS * 64 + lane;
  const bf16x8 *wp = wf + lane;
  const int q0 = wave * H::KQ, q1 = min(H::KS, q0 + H::KQ);
  __syncthreads();
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int v = 0; v < H::VTW; ++v) ring[d][v] = wv[((size_t)v * H::KS + d) * 64];
  bf16x8 pnext = wp[(size_t)q0 * 64];
  for (int s0 = 0; s0 < H::KS; s0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int s = s0 + d;
      if (s >= H::KS) break;
      const int k0 = 16 * s + 8 * h;
      const int cell = k0 / FF, c = k0 % FF;
      const bf16x8 av = *(const bf16x8 *)(frow + (cell * 2 * FF + FF + c) * 2);
      bf16x8 wcur[H::VTW];
#pragma unroll
      for (int v = 0; v < H::VTW; ++v) {
        wcur[v] = ring[d][v];
        if (s + D < H::KS) ring[d][v] = wv[((size_t)v * H::KS + s + D) * 64];
      }
#pragma unroll
      for (int v = 0; v < H::VTW; ++v) acc[v] = Ty<E>::mfma(av, wcur[v], acc[v]);
      if (s >= q0 && s < q1) {
        const bf16x8 ap = *(const bf16x8 *)(frow + (cell * 2 * FF + c) * 2);
        const bf16x8 pw = pnext;
        if (s + 1 < q1) pnext = wp[(size_t)(s + 1) * 64];
        pacc = Ty<E>::mfma(ap, pw, pacc);
      }
    }
  }
  // value: relu(acc + bv[col]) * wo[col], summed over the hidden units (cols)
  // D layout: lane (r, h): col = r, rows (boards) = (i & 3) + 8 * (i >> 2) + 4 * h
  float part[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) part[i] = 0.f;
#pragma unroll
  for (int v = 0; v < H::VTW; ++v) {
    const int col = (wave * H::VTW + v) * 32 + r;
    const float bb = bv[col], ww = wo[col];
#pragma unroll
    for (int i = 0; i < 16; ++i) part[i] += fmaxf(acc[v][i] + bb, 0.f) * ww;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float x = part[i];
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) x += __shfl_xor(x, off, 32);
    part[i] = x;
  }
  if (r == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s_part[wave][(i & 3) + 8 * (i >> 2) + 4 * h] = part[i];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) s_pol[wave][(i & 3) + 8 * (i >> 2) + 4 * h][r] = pacc[i];
  __syncthreads();
  if (tid < nb) {
    const int bd = b0 + tid;
    values[bd] = tanhf(((s_part[0][tid] + s_part[1][tid]) + (s_part[2][tid] + s_part[3][tid])) + bo[0]);
    float lg[A];
    float m = -INFINITY;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      lg[a] = ((s_pol[0][tid][a] + s_pol[1][tid][a]) + (s_pol[2][tid][a] + s_pol[3][tid][a])) + bp[a];
      m = fmaxf(m, lg[a]);
    }
    float e[A], sum = 0.f;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      e[a] = __expf(lg[a] - m);
      sum += e[a];
    }
    const float inv = 1.f / sum;
#pragma unroll
    for (int a = 0; a < A; ++a) probs[(size_t)bd * A + a] = e[a] * inv;
  }
}

// k_heads with room beside a trunk workgroup.  The trunk holds 152.5 KB of a CU's 160 KB LDS and
// 416 of each SIMD's 512 registers per lane, so k_heads (86 KB of staged features) could only run on
// a CU no trunk workgroup occupies: its 512 workgroups waited for the other lane's trunk workgroups
// to retire (0.8-1 ms per call in the bench against 11 us alone), and the lane's expand and next
// trunk launch waited behind it.  This form reads the features straight from global memory (L2:
// the trunk wrote them just before) as the MFMA A operand, fills all 32 MFMA rows with boards (32
// per workgroup, half the weight traffic of 16), keeps only the cross-wave sums in LDS (4.6 KB), and
// is held to 96 registers per lane, so one wave fits on each SIMD beside a trunk wave.  Same math
// in the same order as k_heads (per-wave k order, fixed-order cross-wave sums): bit-identical.
//
// C = 256 (FF = 64: 4 value tiles per wave, which spill at 96 registers in one pass) runs the value
// tiles in two passes of 2 over all of K (the features are read twice, from L2) within the same 96
// registers; the C = 256 trunk wave uses 400 of a SIMD's 512, so one heads wave fits beside it.
// part[] still sums the tiles in order 0..3: bit-identical.
template <int FF, int CELLS, int A, class E = __bf16, int WPE = 5, int VP = HeadsCfg<FF, CELLS, A>::VTW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_heads_co(
    const uint16_t *feats, int n, const int32_t *count, const bf16x8 *wf, const float *hb, float *probs, float *values) {
  using H = HeadsCfg<FF, CELLS, A>;
  static_assert(H::VTW % VP == 0, "value tiles per pass");
  constexpr int BOARDS = 32;
  if (count) n = min(*count, n);  // n = the caller's buffer rows
  const int b0 = blockIdx.x * BOARDS;
  if (b0 >= n) return;
  __shared__ float s_part[4][BOARDS];     // per-wave value partial sums
  constexpr int AP = (A + 7) / 8 * 8;
  __shared__ float s_pol[4][BOARDS][AP];  // per-wave policy partial logits
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int nb = min(BOARDS, n - b0);
  const float *bp = hb, *bv = hb + 32, *wo = hb + 32 + H::HID, *bo = hb + 32 + 2 * H::HID;
  // row r = board b0 + r (rows past the batch repeat its last board; their results are not stored)
  const char *frow = (const char *)feats + (size_t)(b0 + min(r, nb - 1)) * H::FROW;
  // value tiles first, then the policy quarter (each in k_heads' per-wave k order): only one set of
  // accumulators is live at a time, which keeps the wave inside 96 registers without spills
  const bf16x8 *wp = wf + lane;
  const int q0 = wave * H::KQ, q1 = min(H::KS, q0 + H::KQ);
  // the features of step s (value half at FF, policy half at 0), one step ahead
  auto feat = [&](int s, int half) {
    const int k0 = 16 * s + 8 * h;
    return *(const bf16x8 *)(frow + ((k0 / FF) * 2 * FF + half + k0 % FF) * 2);
  };
  float part[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) part[i] = 0.f;
#pragma unroll 1
  for (int v0 = 0; v0 < H::VTW; v0 += VP) {
    f32x16 acc[VP];
#pragma unroll
    for (int v = 0; v < VP; ++v) acc[v] = f32x16{};
    constexpr int D = 2;  // weight ring depth
    bf16x8 ring[D][VP];
    const bf16x8 *wv = wf + (size_t)(1 + wave * H::VTW + v0) * H::KS * 64 + lane;
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int v = 0; v < VP; ++v) ring[d][v] = wv[((size_t)v * H::KS + d) * 64];
    bf16x8 avn = feat(0, FF);
    for (int s0 = 0; s0 < H::KS; s0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int s = s0 + d;
        if (s >= H::KS) break;
        const bf16x8 av = avn;
        if (s + 1 < H::KS) avn = feat(s + 1, FF);
        bf16x8 wcur[VP];
#pragma unroll
        for (int v = 0; v < VP; ++v) {
          wcur[v] = ring[d][v];
          if (s + D < H::KS) ring[d][v] = wv[((size_t)v * H::KS + s + D) * 64];
        }
#pragma unroll
        for (int v = 0; v < VP; ++v) acc[v] = Ty<E>::mfma(av, wcur[v], acc[v]);
      }
    }
    // value: relu(acc + bv[col]) * wo[col], summed over the hidden units (cols); as k_heads
#pragma unroll
    for (int v = 0; v < VP; ++v) {
      const int col = (wave * H::VTW + v0 + v) * 32 + r;
      const float bb = bv[col], ww = wo[col];
#pragma unroll
      for (int i = 0; i < 16; ++i) part[i] += fmaxf(acc[v][i] + bb, 0.f) * ww;
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float x = part[i];
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) x += __shfl_xor(x, off, 32);
    part[i] = x;
  }
  if (r == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s_part[wave][(i & 3) + 8 * (i >> 2) + 4 * h] = part[i];
  }
  f32x16 pacc = {};
  if (q0 < q1) {
    bf16x8 pn = wp[(size_t)q0 * 64], apn = feat(q0, 0);
    for (int s = q0; s < q1; ++s) {
      const bf16x8 pw = pn, ap = apn;
      if (s + 1 < q1) {
        pn = wp[(size_t)(s + 1) * 64];
        apn = feat(s + 1, 0);
      }
      pacc = Ty<E>::mfma(ap, pw, pacc);
    }
  }
  if (r < A) {
#pragma unroll
    for (int i = 0; i < 16; ++i) s_pol[wave][(i & 3) + 8 * (i >> 2) + 4 * h][r] = pacc[i];
  }
  __syncthreads();
  if (tid < nb) {
    const int bd = b0 + tid;
    values[bd] = tanhf(((s_part[0][tid] + s_part[1][tid]) + (s_part[2][tid] + s_part[3][tid])) + bo[0]);
    float lg[A];
    float m = -INFINITY;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      lg[a] = ((s_pol[0][tid][a] + s_pol[1][tid][a]) + (s_pol[2][tid][a] + s_pol[3][tid][a])) + bp[a];
      m = fmaxf(m, lg[a]);
    }
    float e[A], sum = 0.f;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      e[a] = __expf(lg[a] - m);
      sum += e[a];
    }
    const float inv = 1.f / sum;
#pragma unroll
    for (int a = 0; a < A; ++a) probs[(size_t)bd * A + a] = e[a] * inv;
  }
}

// Head epilogue after one GEMM  Z = features[n][cells*2ff] @ Wc^T  (Wc = value rows [8ff]
// then policy rows [A], zero where a row meets the other head's channels):
//   value = tanh(sum_j relu(Z[j] + bv[j]) * wo[j] + bo), probs = softmax(Z[8ff + a] + bp[a]).
// One wave per board; the hidden-unit sum is a fixed-order lane reduction (deterministic).
template <int HID, int A>
__global__ __launch_bounds__(256) void k_head_epilogue(const __bf16 *Z, int ldz, int n, const float *hb,
                                                       float *probs, float *values) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (wave >= n) return;
  const __bf16 *z = Z + (size_t)wave * ldz;
  const float *bv = hb, *wo = hb + HID, *bo = hb + 2 * HID, *bp = hb + 2 * HID + 1;
  float acc = 0.f;
#pragma unroll
  for (int j = lane; j < HID; j += 64) acc += fmaxf((float)z[j] + bv[j], 0.f) * wo[j];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  float logit = lane < A ? (float)z[HID + lane] + bp[lane] : -INFINITY;
  float m = logit;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  const float e = lane < A ? __expf(logit - m) : 0.f;
  float sum = e;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
  if (lane < A) probs[(size_t)wave * A + lane] = e / sum;
  if (lane == 0) values[wave] = tanhf(acc + bo[0]);
}

// Residual scratch of the one-buffer trunk (tower_wide.h): one region per workgroup of a launch, one
// buffer per stream (launches on different streams run concurrently), grown on demand.
static uint4 *wide_scratch(hipStream_t s, size_t bytes) {
  struct Ent {
    hipStream_t s;
    void *p;
    size_t n;
  };
  static std::vector<Ent> tab;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  for (auto &e : tab)
    if (e.s == s) {
      if (e.n >= bytes) return (uint4 *)e.p;
      if (hipStreamSynchronize(s) != hipSuccess || hipFree(e.p) != hipSuccess) return nullptr;
      e.p = nullptr;
      e.n = 0;
      if (hipMalloc(&e.p, bytes) != hipSuccess) return nullptr;
      e.n = bytes;
      return (uint4 *)e.p;
    }
  void *p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  tab.push_back({s, p, bytes});
  return (uint4 *)p;
}

template <class K>
static size_t scratch_bytes(int grid) {
  if constexpr (K::ONEBUF) return (size_t)grid * wide::Scr<K>::PER_WG;
  return 0;
}

template <class K>
static int launch(const void *planes, int batch, int n_blocks, const void *w, const float *b, void *out,
                  hipStream_t s) {
  const int grid = (batch + K::BOARDS - 1) / K::BOARDS;
  if (grid <= 0) return 0;
  uint4 *scr = nullptr;
  if (const size_t sb = scratch_bytes<K>(grid)) {
    if (!(scr = wide_scratch(s, sb))) return -12;
  }
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void *)k_tower<K>, hipFuncAttributeMaxDynamicSharedMemorySize, K::LDS) !=
        hipSuccess)
      return -10;
    attr_set = true;
  }
  hipLaunchKernelGGL(k_tower<K>, dim3(grid), dim3(K::THREADS), K::LDS, s, (const __bf16 *)planes, batch, n_blocks,
                     (const bf16x8 *)w, b, (uint16_t *)out, scr);
  return hipGetLastError() == hipSuccess ? 0 : -11;
}

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}

// Full-size workgroups (one per CU, BOARDS boards each) for whole rounds of the chip, then the
// remainder in one round of the smallest tile that covers it (tail_kind: half-size tiles take about
// half the time, 4-board tiles three quarters): a batch of 3,700 boards costs 2.5 workgroup-rounds
// instead of 3, one of 4,096 boards 2.75.
template <class KF, class KM, class KH>
static int launch_split(const char *planes, int batch, int n_blocks, const void *w, const float *b, char *out,
                        hipStream_t s) {
  const int cus = num_cus();
  const int full_wgs = (batch / KF::BOARDS) / cus * cus;
  const int n_full = full_wgs * KF::BOARDS;
  const int rem = batch - n_full;
  int rc = 0;
  if (n_full > 0) rc = launch<KF>(planes, n_full, n_blocks, w, b, out, s);
  if (rc || rem <= 0) return rc;
  const char *p2 = planes + (size_t)n_full * KF::CELLS * 3 * 2;
  char *o2 = out + (size_t)n_full * KF::CELLS * KF::HEAD * 2;
  switch (tail_kind<KF, KM, KH>(rem, cus)) {
    case 0: return launch<KH>(p2, rem, n_blocks, w, b, o2, s);
    case 1: return launch<KM>(p2, rem, n_blocks, w, b, o2, s);
    default: return launch<KF>(p2, rem, n_blocks, w, b, o2, s);
  }
}

// pack: the launch runs beside launches on other streams (SPMCTS_TOWER_PACK): tiles are assigned
// as if the chip had one CU (all boards in full tiles, the last < BOARDS in one smaller tile); the
// other streams' workgroups fill the CUs a partial round would leave idle.
template <class KF, class KM, class KH>
static int launch_dyn(const void *planes, const int32_t *count, int max_batch, int n_blocks, const void *w,
                      const float *b, void *out, bool pack, hipStream_t s) {
  const int cus = pack ? 1 : num_cus();
  const int grid = (max_batch + KF::BOARDS - 1) / KF::BOARDS + (pack ? 1 : cus);
  uint4 *scr = nullptr;
  if (const size_t sb = scratch_bytes<KF>(grid)) {  // (the tail kinds KM / KH are two-buffer tiles)
    if (!(scr = wide_scratch(s, sb))) return -12;
  }
  constexpr int LDS = KF::LDS > KM::LDS ? (KF::LDS > KH::LDS ? KF::LDS : KH::LDS) : (KM::LDS > KH::LDS ? KM::LDS : KH::LDS);
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void *)k_tower_dyn<KF, KM, KH>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS) !=
        hipSuccess)
      return -10;
    attr_set = true;
  }
  hipLaunchKernelGGL((k_tower_dyn<KF, KM, KH>), dim3(grid), dim3(256), LDS, s, (const __bf16 *)planes, count,
                     max_batch, cus, n_blocks, (const bf16x8 *)w, b, (uint16_t *)out, scr);
  return hipGetLastError() == hipSuccess ? 0 : -11;
}

}  // namespace tower

namespace tower {
#ifdef SPMCTS_AB
// A/B library (make ab: libspmcts_ab.so, -DSPMCTS_AB) only: switches that select measured-slower
// alternates and timing ablations.  Read once.
static bool env_is(const char *name, const char *val) {
  const char *e = getenv(name);
  return e && strcmp(e, val) == 0;
}
static bool c256_board3() {  // SPMCTS_TOWER_C256=3: the C = 256 trunk on 3-board two-buffer tiles
  static const bool v = env_is("SPMCTS_TOWER_C256", "3");
  return v;
}
static bool wide_tails3() {  // SPMCTS_WIDE_TAILS=3: C = 256 launches with 3-board tail code
  static const bool v = env_is("SPMCTS_WIDE_TAILS", "3");
  return v;
}
// the C = 256 Connect4 trunk on the 16x16x32 one-buffer tiles (tower_wide16.h, its M16 weight layout) unless
// SPMCTS_TOWER_C256 (=32: round 4's 32x32x16 one-buffer tiles; =3: the 3-board tiles), SPMCTS_WIDE_TAILS or a
// SPMCTS_TOWER_CG probe code other than 25xx (all on the 32x32x16 layout) selects another set
static bool c256_m16() {  // (SPMCTS_TOWER_CG codes 25xx are variants of the 16x16x32 C = 256 trunk)
  static const bool cg25 = getenv("SPMCTS_TOWER_CG") && atoi(getenv("SPMCTS_TOWER_CG")) / 100 == 25;
  static const bool v = !getenv("SPMCTS_TOWER_C256") && !getenv("SPMCTS_WIDE_TAILS") && (!getenv("SPMCTS_TOWER_CG") || cg25);
  return v;
}
static bool heads_co256() {  // SPMCTS_HEADS_C256=lds: the LDS-staged C = 256 linear heads
  static const bool v = !env_is("SPMCTS_HEADS_C256", "lds");
  return v;
}
static bool heads_co() {  // SPMCTS_HEADS=lds: the LDS-staged linear heads
  static const bool v = !env_is("SPMCTS_HEADS", "lds");
  return v;
}
// SPMCTS_TOWER_M16=0: the 32x32x16 C = 128 Connect4 trunk (round 3's kernel set, its weight layout); the
// ring trunk and the SPMCTS_TOWER_CG variants take that layout too
static bool m16_trunk() {
  // SPMCTS_TOWER_CG codes 16xx are variants of the 16x16x32 trunk (its weight layout)
  static const bool cg16 = getenv("SPMCTS_TOWER_CG") && atoi(getenv("SPMCTS_TOWER_CG")) / 100 == 16;
  static const bool v =
      !env_is("SPMCTS_TOWER_M16", "0") && !getenv("SPMCTS_TOWER_RING") && (!getenv("SPMCTS_TOWER_CG") || cg16);
  return v;
}
#else
// The product library has exactly one kernel per (shape, dtype) and reads no switch; a switch of the
// A/B library set in the environment is refused (SPMCTS_ERR_AB_SWITCH) rather than silently ignored.
static constexpr bool m16_trunk() { return true; }
static constexpr bool c256_board3() { return false; }
static constexpr bool c256_m16() { return true; }
static constexpr bool wide_tails3() { return false; }
static constexpr bool heads_co256() { return true; }
static constexpr bool heads_co() { return true; }
#endif
// -5 when an A/B-library switch is set in a product build (read once)
static int ab_switch_guard() {
#ifdef SPMCTS_AB
  return 0;
#else
  static const int rc = [] {
    for (const char *n : {"SPMCTS_TOWER_CG", "SPMCTS_TOWER_RING", "SPMCTS_TOWER_C256", "SPMCTS_WIDE_TAILS", "SPMCTS_HEADS",
                          "SPMCTS_HEADS_C256", "SPMCTS_TREE_BLOCK", "SPMCTS_EXPAND_CO", "SPMCTS_TOWER_M16",
                          "SPMCTS_TREE_COPIES"})
      if (getenv(n)) return SPMCTS_ERR_AB_SWITCH;
    return 0;
  }();
  return rc;
#endif
}

// the instantiated tile sets of the device-count path, per board shape, channels and element type
template <class E>
static int forward_dev(int32_t width, int32_t height, int32_t channels, int32_t n_blocks, const void *planes_dev,
                       const int32_t *count_dev, int32_t max_batch, const void *weights_dev, const float *bias_dev,
                       void *features_dev, bool pack, hipStream_t s) {
  if (width == 7 && height == 6 && channels == 128) {
#ifdef SPMCTS_AB
    if (!m16_trunk())  // round 3's 32x32x16 set: 6-board edge tiles + 4- / 3-board board-major tails
      return launch_dyn<Cfg<128, 256, 7, 6, 2, 4, 0, 4, 1, true, true, E>, Cfg<128, 192, 7, 6, 2, 4, 0, 4, 1, false, false, E>,
                        Cfg<128, 128, 7, 6, 2, 4, 0, 4, 1, false, false, E>>(planes_dev, count_dev, max_batch, n_blocks,
                                                                            weights_dev, bias_dev, features_dev, pack, s);
#endif
    // 16x16x32 edge tiles for every board, tails included (tower_m16.h)
    using KM = Cfg<128, 256, 7, 6, 2, 4, 0, 2, 1, true, true, E, false, true>;
    return launch_dyn<KM, KM, KM>(planes_dev, count_dev, max_batch, n_blocks, weights_dev, bias_dev, features_dev, pack, s);
  }
  if (width == 7 && height == 6 && channels == 256) {
    // 6-board one-buffer edge tiles (tower_wide.h) with 3-board tails
    using K3 = Cfg<256, 128, 7, 6, 4, 4, 0, 4, 1, false, false, E>;
    using KW = Cfg<256, 256, 7, 6, 4, 4, 0, 2, 1, true, true, E, true>;
#ifdef SPMCTS_AB
    if (c256_board3())
      return launch_dyn<K3, K3, K3>(planes_dev, count_dev, max_batch, n_blocks, weights_dev, bias_dev, features_dev, pack, s);
    if (wide_tails3())  // SPMCTS_WIDE_TAILS=3: the round-3 set, 3-board tail tiles in one kernel with the 6-board body
      return launch_dyn<KW, K3, K3>(planes_dev, count_dev, max_batch, n_blocks, weights_dev, bias_dev, features_dev, pack,
                                    s);
    if (!c256_m16())  // SPMCTS_TOWER_C256=32: round 4's 32x32x16 one-buffer tiles for every board
      return launch_dyn<KW, KW, KW>(planes_dev, count_dev, max_batch, n_blocks, weights_dev, bias_dev, features_dev, pack, s);
#endif
    // every tile a 6-board one-buffer 16x16x32 tile (tower_wide16.h; a batch tail takes one partly empty tile),
    // so every board goes through the same arithmetic
    (void)sizeof(K3);
    (void)sizeof(KW);
    using KW16 = Cfg<256, 256, 7, 6, 4, 4, 0, 2, 1, true, true, E, true, true>;
    return launch_dyn<KW16, KW16, KW16>(planes_dev, count_dev, max_batch, n_blocks, weights_dev, bias_dev, features_dev,
                                        pack, s);
  }
  if (width == 3 && height == 3 && channels == 128)
    return launch_dyn<Cfg<128, 256, 3, 3, 2, 4, 0, 4, 1, false, false, E>, Cfg<128, 192, 3, 3, 2, 4, 0, 4, 1, false, false, E>,
                      Cfg<128, 128, 3, 3, 2, 4, 0, 4, 1, false, false, E>>(planes_dev, count_dev, max_batch, n_blocks,
                                                                          weights_dev, bias_dev, features_dev, pack, s);
  if (width == 3 && height == 3 && channels == 256)
    return launch_dyn<Cfg<256, 128, 3, 3, 4, 4, 0, 4, 1, false, false, E>, Cfg<256, 128, 3, 3, 4, 4, 0, 4, 1, false, false, E>,
                      Cfg<256, 128, 3, 3, 4, 4, 0, 4, 1, false, false, E>>(planes_dev, count_dev, max_batch, n_blocks,
                                                                          weights_dev, bias_dev, features_dev, pack, s);
  return -2;
}

// the host-count path (a batch size known on the host): the same tile sets, split on the host
template <class E>
static int forward_host(int32_t width, int32_t height, int32_t channels, int32_t n_blocks, const char *pl, int32_t batch,
                        const void *weights_dev, const float *bias_dev, char *ft, hipStream_t s) {
  if (width == 7 && height == 6 && channels == 128) {
#ifdef SPMCTS_AB
    if (!m16_trunk())
      return launch_split<Cfg<128, 256, 7, 6, 2, 4, 0, 4, 1, true, true, E>, Cfg<128, 192, 7, 6, 2, 4, 0, 4, 1, false, false, E>,
                          Cfg<128, 128, 7, 6, 2, 4, 0, 4, 1, false, false, E>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
#endif
    using KM = Cfg<128, 256, 7, 6, 2, 4, 0, 2, 1, true, true, E, false, true>;
    return launch<KM>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  }
  if (width == 7 && height == 6 && channels == 256) {
    using K3 = Cfg<256, 128, 7, 6, 4, 4, 0, 4, 1, false, false, E>;
#ifdef SPMCTS_AB
    if (c256_board3()) return launch<K3>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
    if (!c256_m16())  // the 32x32x16 one-buffer tiles with 3-board tails (round 4's host path)
      return launch_split<Cfg<256, 256, 7, 6, 4, 4, 0, 2, 1, true, true, E, true>, K3, K3>(pl, batch, n_blocks,
                                                                                         weights_dev, bias_dev, ft, s);
#endif
    (void)sizeof(K3);
    return launch<Cfg<256, 256, 7, 6, 4, 4, 0, 2, 1, true, true, E, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev,
                                                                                 ft, s);
  }
  if (width == 3 && height == 3 && channels == 128)
    return launch<Cfg<128, 256, 3, 3, 2, 4, 0, 4, 1, false, false, E>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  if (width == 3 && height == 3 && channels == 256)
    return launch<Cfg<256, 128, 3, 3, 4, 4, 0, 4, 1, false, false, E>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  return -2;
}
}  // namespace tower

#ifdef SPMCTS_AB
namespace tower {
// Ring trunk launch (tower_ring.h): full 6-board tiles only, for the C = 128 Connect4 net with at most
// ring::MAX_CONVS / 2 blocks.  count == nullptr: the batch is max_batch.
template <class E>
static int launch_ring(const void *planes, const int32_t *count, int max_batch, int n_blocks, const void *w,
                       const float *b, void *out, hipStream_t s) {
  using K = Cfg<128, 256, 7, 6, 2, 4, 0, 4, 1, true, true, E>;
  if (2 * n_blocks > ring::MAX_CONVS) return -2;
  const int grid = (max_batch + K::BOARDS - 1) / K::BOARDS;
  if (grid <= 0) return 0;
  const int lds = ring::Geo<K>::lds(2 * n_blocks);
  static int attr = 0;
  if (lds > attr) {
    if (hipFuncSetAttribute((const void *)ring::k_tower_ring<K>, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
      return -10;
    attr = lds;
  }
  hipLaunchKernelGGL(ring::k_tower_ring<K>, dim3(grid), dim3(256), lds, s, (const __bf16 *)planes, count, max_batch,
                     n_blocks, (const bf16x8 *)w, b, (uint16_t *)out);
  return hipGetLastError() == hipSuccess ? 0 : -11;
}

// SPMCTS_TOWER_RING=1 runs the ring trunk for the C = 128 Connect4 net instead of the two-buffer trunk
// (measured 3-6 % slower, DESIGN.md §4 "Round 3")
static bool ring_enabled(int n_blocks) {
  static const bool on = getenv("SPMCTS_TOWER_RING") && atoi(getenv("SPMCTS_TOWER_RING")) != 0;
  return on && 2 * n_blocks <= ring::MAX_CONVS;
}

// SPMCTS_TOWER_CG=<code>: timing alternatives and ablations of the C = 128 trunk (bf16; some give wrong
// results by design: DESIGN.md §4 has the measurements).  Returns 1 when no code is set.
static int forward_ab(int32_t width, int32_t height, int32_t channels, int32_t n_blocks, const char *pl, int32_t batch,
                      const void *weights_dev, const float *bias_dev, char *ft, hipStream_t s) {
  static const int cg = getenv("SPMCTS_TOWER_CG") ? atoi(getenv("SPMCTS_TOWER_CG")) : -1;
  if (cg < 0) return 1;
  if (width == 7 && height == 6 && channels == 128) {
    switch (cg) {
#define ABLATE(X) \
      case 100 + X: return launch<Cfg<128, 256, 7, 6, 2, 4, X>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      ABLATE(0) ABLATE(1) ABLATE(2) ABLATE(4) ABLATE(8) ABLATE(16) ABLATE(24) ABLATE(31) ABLATE(64) ABLATE(128)
      ABLATE(256) ABLATE(2048) ABLATE(32768)
#undef ABLATE
#define ABLATE_EDGE(X) \
      case 200 + X: return launch<Cfg<128, 256, 7, 6, 2, 4, X, 4, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      ABLATE_EDGE(0) ABLATE_EDGE(2) ABLATE_EDGE(4) ABLATE_EDGE(6) ABLATE_EDGE(8) ABLATE_EDGE(16) ABLATE_EDGE(24)
      ABLATE_EDGE(30) ABLATE_EDGE(128) ABLATE_EDGE(512)
      case 301: return launch<Cfg<128, 256, 7, 6, 2, 4, 4096, 4, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      // weight-major MFMA order within a k-step (bit-identical; clock / operand-toggling probe)
      case 304: return launch<Cfg<128, 256, 7, 6, 2, 4, 4194304, 4, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      // the 16x16x32 trunk (tower_m16.h, the default: DEPTH 2, grouped schedule) variants: weight ring 4 deep
      // (1604), the compiler's own schedule (1600)
      case 1604: return launch<Cfg<128, 256, 7, 6, 2, 4, 0, 4, 1, true, true, __bf16, false, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      case 1600: return launch<Cfg<128, 256, 7, 6, 2, 4, 256, 2, 1, true, true, __bf16, false, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      case 1602: return launch<Cfg<128, 256, 7, 6, 2, 4, 0, 2, 1, true, true, __bf16, false, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      // 4 channel quarters x all 8 cell tiles (one weight fragment per 16 MFMAs instead of per 8, twice the LDS
      // operand reads; the B fragments conflict-free since round 5): ring depth 2 (1640) and 4 (1644)
      case 1640: return launch<Cfg<128, 256, 7, 6, 4, 4, 0, 2, 1, true, true, __bf16, false, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      case 1644: return launch<Cfg<128, 256, 7, 6, 4, 4, 0, 4, 1, true, true, __bf16, false, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      // timing ablations of the shipped 16x16x32 trunk (wrong results): no weight loads in the k-loop (1616), no
      // LDS operand reads (1608) -- upper bounds on what fewer weight / operand fetches per MFMA could buy
      case 1616: return launch<Cfg<128, 256, 7, 6, 2, 4, 16, 2, 1, true, true, __bf16, false, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      case 1608: return launch<Cfg<128, 256, 7, 6, 2, 4, 8, 2, 1, true, true, __bf16, false, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      // timing ablation (wrong results): every layer streams layer 0's weights (an L2-resident set): what the
      // trunk's fabric re-stream of its 11.8 MB weight set costs
      case 1665: return launch<Cfg<128, 256, 7, 6, 2, 4, 65536, 2, 1, true, true, __bf16, false, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      // timing ablation (wrong results): two 16x16x32 MFMAs per 32x32x16 (the MFMA-shape clock probe)
      case 308: return launch<Cfg<128, 256, 7, 6, 2, 4, 8388608, 4, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      case 302: return launch<Cfg<128, 256, 7, 6, 2, 4, 8192, 4, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      case 316: return launch<Cfg<128, 256, 7, 6, 2, 4, 16384, 4, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
#undef ABLATE_EDGE
      // four channel quarters x one row group (each wave all 8 cell tiles, one weight fragment per k-step)
      case 400: return launch<Cfg<128, 256, 7, 6, 4, 4, 0, 4, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      case 408: return launch<Cfg<128, 256, 7, 6, 4, 4, 0, 8, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      // eight waves (two per SIMD): four channel quarters x two row halves, one weight fragment per k-step
      case 800: return launch<Cfg<128, 256, 7, 6, 4, 8, 0, 4, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      case 808: return launch<Cfg<128, 256, 7, 6, 4, 8, 0, 8, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
      case 250: return launch<Cfg<128, 256, 7, 6, 2, 4, 0, 8, 1, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);  // ring depth 8
      case 10: return launch_split<Cfg<128, 256, 7, 6, 2>, Cfg<128, 128, 7, 6, 2>, Cfg<128, 128, 7, 6, 2>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);  // two tile sizes only
      case 15: return launch_split<Cfg<128, 256, 7, 6, 2, 4, 0, 4, 1, true>, Cfg<128, 192, 7, 6, 2>, Cfg<128, 128, 7, 6, 2>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);  // column-major tiles without edge rows
      case 11: return launch_split<Cfg<128, 256, 7, 6, 2>, Cfg<128, 192, 7, 6, 2>, Cfg<128, 128, 7, 6, 2>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);  // board-major full tiles
      default: return 1;
    }
  }
  // the MFMA-shape clock probe on the C = 256 one-buffer trunk (timing only, wrong results: each 32x32x16 as two
  // 16x16x32 on the same operands, as code 308 for C = 128) and its reference (2300 = the shipped trunk)
  if (width == 7 && height == 6 && channels == 256 && cg == 2308)
    return launch_split<Cfg<256, 256, 7, 6, 4, 4, 8388608, 2, 1, true, true, __bf16, true>, Cfg<256, 128, 7, 6, 4>,
                        Cfg<256, 128, 7, 6, 4>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  if (width == 7 && height == 6 && channels == 256 && cg == 2300)
    return launch_split<Cfg<256, 256, 7, 6, 4, 4, 0, 2, 1, true, true, __bf16, true>, Cfg<256, 128, 7, 6, 4>,
                        Cfg<256, 128, 7, 6, 4>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  // the 16x16x32 one-buffer C = 256 trunk (tower_wide16.h, the product's) and two variants: a 4-deep weight ring
  // (2564), the compiler's own k-loop schedule (2556)
  if (width == 7 && height == 6 && channels == 256 && cg == 2560)
    return launch<Cfg<256, 256, 7, 6, 4, 4, 0, 2, 1, true, true, __bf16, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  if (width == 7 && height == 6 && channels == 256 && cg == 2564)
    return launch<Cfg<256, 256, 7, 6, 4, 4, 0, 4, 1, true, true, __bf16, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  if (width == 7 && height == 6 && channels == 256 && cg == 2556)
    return launch<Cfg<256, 256, 7, 6, 4, 4, 256, 2, 1, true, true, __bf16, true, true>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  if (width == 7 && height == 6 && channels == 256 && cg == 254)  // the one-buffer trunk with a 4-deep weight ring
    return launch_split<Cfg<256, 256, 7, 6, 4, 4, 0, 4, 1, true, true, __bf16, true>, Cfg<256, 128, 7, 6, 4>,
                        Cfg<256, 128, 7, 6, 4>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  // the round-3 residual-scratch pointer form (64-bit nontemporal accesses, 110 spills) against the shipped
  // buffer-resource form (tower_wide.h ScrBuf)
  if (width == 7 && height == 6 && channels == 256 && cg == 2566)
    return launch_split<Cfg<256, 256, 7, 6, 4, 4, 2097152, 2, 1, true, true, __bf16, true>, Cfg<256, 128, 7, 6, 4>,
                        Cfg<256, 128, 7, 6, 4>>(pl, batch, n_blocks, weights_dev, bias_dev, ft, s);
  return 1;
}
}  // namespace tower
#endif  // SPMCTS_AB

extern "C" int spmcts_tower_forward_dev(int32_t width, int32_t height, int32_t channels, int32_t n_blocks,
                                        const void *planes_dev, const int32_t *count_dev, int32_t max_batch,
                                        const void *weights_dev, const float *bias_dev, void *features_dev,
                                        int32_t flags, spmcts_stream stream) {
  using namespace tower;
  hipStream_t s = (hipStream_t)stream;
  if (n_blocks < 0 || max_batch < 0 || !count_dev || (flags & ~(SPMCTS_TOWER_PACK | SPMCTS_TOWER_F16))) return -3;
  if (const int g = ab_switch_guard()) return g;
  if (max_batch == 0) return 0;
  const bool pack = (flags & SPMCTS_TOWER_PACK) != 0;
#ifdef SPMCTS_AB
  if (width == 7 && height == 6 && channels == 128 && ring_enabled(n_blocks))
    return (flags & SPMCTS_TOWER_F16 ? launch_ring<_Float16> : launch_ring<__bf16>)(
        planes_dev, count_dev, max_batch, n_blocks, weights_dev, bias_dev, features_dev, s);
#endif
  if (flags & SPMCTS_TOWER_F16)
    return forward_dev<_Float16>(width, height, channels, n_blocks, planes_dev, count_dev, max_batch, weights_dev,
                                 bias_dev, features_dev, pack, s);
  return forward_dev<__bf16>(width, height, channels, n_blocks, planes_dev, count_dev, max_batch, weights_dev, bias_dev,
                             features_dev, pack, s);
}

extern "C" int spmcts_tower_forward(int32_t width, int32_t height, int32_t channels, int32_t n_blocks,
                                    const void *planes_dev, int32_t batch, const void *weights_dev,
                                    const float *bias_dev, void *features_dev, int32_t flags, spmcts_stream stream) {
  using namespace tower;
  hipStream_t s = (hipStream_t)stream;
  if (n_blocks < 0 || batch < 0 || (flags & ~SPMCTS_TOWER_F16)) return -3;
  if (const int g = ab_switch_guard()) return g;
  const char *pl = (const char *)planes_dev;
  char *ft = (char *)features_dev;
#ifdef SPMCTS_AB
  // the ring trunk serves both element types on both paths (as spmcts_tower_forward_dev)
  if (width == 7 && height == 6 && channels == 128 && ring_enabled(n_blocks) && !getenv("SPMCTS_TOWER_CG"))
    return (flags & SPMCTS_TOWER_F16 ? launch_ring<_Float16> : launch_ring<__bf16>)(
        planes_dev, nullptr, batch, n_blocks, weights_dev, bias_dev, features_dev, s);
  if (!(flags & SPMCTS_TOWER_F16)) {
    const int rc = forward_ab(width, height, channels, n_blocks, pl, batch, weights_dev, bias_dev, ft, s);
    if (rc != 1) return rc;
  }
#endif
  if (flags & SPMCTS_TOWER_F16)
    return forward_host<_Float16>(width, height, channels, n_blocks, pl, batch, weights_dev, bias_dev, ft, s);
  return forward_host<__bf16>(width, height, channels, n_blocks, pl, batch, weights_dev, bias_dev, ft, s);
}

template <class E>
static int tower_heads(int32_t width, int32_t height, int32_t channels, int32_t actions, const void *features_dev,
                       int32_t batch, const int32_t *count_dev, const void *head_w_dev, const float *head_b_dev,
                       float *probs_dev, float *values_dev, spmcts_stream stream) {
  using namespace tower;
  hipStream_t s = (hipStream_t)stream;
  if (batch <= 0) return batch < 0 ? -3 : 0;
  if (const int g = ab_switch_guard()) return g;
  // the co-resident k_heads_co (C = 256, FF = 64: two value passes of 2 tiles in 96 registers, beside the
  // C = 256 trunk); the A/B library's SPMCTS_HEADS=lds / SPMCTS_HEADS_C256=lds select the LDS-staged k_heads
#define HEADS_CO(FF, CELLS, A)                                                                              \
  hipLaunchKernelGGL((k_heads_co<FF, CELLS, A, E, 5, FF == 64 ? 2 : HeadsCfg<FF, CELLS, A>::VTW>),          \
                     dim3((batch + 31) / 32), dim3(256), 0, s, (const uint16_t *)features_dev, batch,       \
                     count_dev, (const bf16x8 *)head_w_dev, head_b_dev, probs_dev, values_dev)
#ifdef SPMCTS_AB
#define HEADS(FF, CELLS, A)                                                                                 \
  do {                                                                                                      \
    if (heads_co() && (FF == 32 || heads_co256()))                                                         \
      HEADS_CO(FF, CELLS, A);                                                                               \
    else                                                                                                    \
      hipLaunchKernelGGL((k_heads<FF, CELLS, A, E>), dim3((batch + HeadsCfg<FF, CELLS, A>::BOARDS - 1) /    \
                                                       HeadsCfg<FF, CELLS, A>::BOARDS), dim3(256), 0, s,     \
                         (const uint16_t *)features_dev, batch, count_dev, (const bf16x8 *)head_w_dev,      \
                         head_b_dev, probs_dev, values_dev);                                                \
  } while (0)
#else
#define HEADS(FF, CELLS, A) HEADS_CO(FF, CELLS, A)
#endif
  if (width == 7 && height == 6 && actions == 7 && channels == 128)
    HEADS(32, 42, 7);
  else if (width == 7 && height == 6 && actions == 7 && channels == 256)
    HEADS(64, 42, 7);
  else if (width == 3 && height == 3 && actions == 9 && channels == 128)
    HEADS(32, 9, 9);
  else if (width == 3 && height == 3 && actions == 9 && channels == 256)
    HEADS(64, 9, 9);
  else
    return -2;
#undef HEADS
#undef HEADS_CO
  return hipGetLastError() == hipSuccess ? 0 : -11;
}

extern "C" int spmcts_tower_heads(int32_t width, int32_t height, int32_t channels, int32_t actions,
                                  const void *features_dev, int32_t batch, const void *head_w_dev,
                                  const float *head_b_dev, float *probs_dev, float *values_dev, int32_t flags,
                                  spmcts_stream stream) {
  if (flags & ~SPMCTS_TOWER_F16) return -3;
  return (flags & SPMCTS_TOWER_F16 ? tower_heads<_Float16> : tower_heads<__bf16>)(
      width, height, channels, actions, features_dev, batch, nullptr, head_w_dev, head_b_dev, probs_dev, values_dev, stream);
}

extern "C" int spmcts_tower_heads_dev(int32_t width, int32_t height, int32_t channels, int32_t actions,
                                      const void *features_dev, const int32_t *count_dev, int32_t max_batch,
                                      const void *head_w_dev, const float *head_b_dev, float *probs_dev,
                                      float *values_dev, int32_t flags, spmcts_stream stream) {
  if (flags & ~SPMCTS_TOWER_F16) return -3;
  return (flags & SPMCTS_TOWER_F16 ? tower_heads<_Float16> : tower_heads<__bf16>)(
      width, height, channels, actions, features_dev, max_batch, count_dev, head_w_dev, head_b_dev, probs_dev,
      values_dev, stream);
}

extern "C" int spmcts_head_epilogue(int32_t hidden, int32_t actions, const void *z_dev, int32_t ldz, int32_t batch,
                                    const float *head_b_dev, float *probs_dev, float *values_dev,
                                    spmcts_stream stream) {
  using namespace tower;
  hipStream_t s = (hipStream_t)stream;
  if (batch <= 0) return batch < 0 ? -3 : 0;
  const int grid = (batch + 3) / 4;
#define EPI(HID, A)                                                                                       \
  hipLaunchKernelGGL((k_head_epilogue<HID, A>), dim3(grid), dim3(256), 0, s, (const __bf16 *)z_dev, ldz, batch, \
                     head_b_dev, probs_dev, values_dev)
  if (hidden == 256 && actions == 7)
    EPI(256, 7);
  else if (hidden == 512 && actions == 7)
    EPI(512, 7);
  else if (hidden == 256 && actions == 9)
    EPI(256, 9);
  else if (hidden == 512 && actions == 9)
    EPI(512, 9);
  else
    return -2;
#undef EPI
  return hipGetLastError() == hipSuccess ? 0 : -11;
}

extern "C" int spmcts_tower_supported(int32_t width, int32_t height, int32_t channels) {
  return ((width == 7 && height == 6) || (width == 3 && height == 3)) && (channels == 128 || channels == 256);
}

extern "C" int spmcts_tower_weight_layout(int32_t width, int32_t height, int32_t channels) {
  using namespace tower;
  if (!spmcts_tower_supported(width, height, channels)) return -2;
  if (width == 7 && height == 6 && channels == 128 && m16_trunk()) return SPMCTS_WLAYOUT_M16;
  if (width == 7 && height == 6 && channels == 256 && c256_m16()) return SPMCTS_WLAYOUT_M16;
  return SPMCTS_WLAYOUT_32X32;
}
