// tower_wide16.h — the C = 256 one-buffer trunk on v_mfma_f32_16x16x32_{bf16,f16} (round 5).
//
// Included by tower.hip (namespace tower) after tower_wide.h and tower_m16.h: the workgroup plan of
// tower_wide.h (6 boards in 256 edge-ordered rows, ONE activation buffer, the block input kept in a
// per-workgroup global scratch for the residual, 4 waves = 4 channel quarters x all 8 cell tiles, in-place
// epilogues between barriers) with the k-loop of tower_m16.h (each 32-row x 32-channel output tile as
// 2 x 2 tiles of 16 x 16 over K = 32 input channels, operand rows by lane_row, the phys16 channel order).
//   * per wave: 4 16-channel tiles (64 output channels: one whole phys16 group, so a lane's 16 outputs of
//     a cell are one contiguous 32-byte run) x 8 cell tiles x 2 row fragments = 64 f32x4 accumulators
//     (the full AGPR file, as the 32x32x16 form's 16 f32x16);
//   * the same FLOPs, LDS bytes and weight bytes per k-step as tower_wide.h; a timing probe on that kernel
//     (each 32x32x16 as two 16x16x32 on the same operands, A/B code 2308) ran the trunk 6.5 % faster at
//     a 1.90 vs 1.80 GHz clock (profiles/r05/c256/shape_probe.txt);
//   * residual scratch per workgroup: [wave][cell tile t][fragment h][64 lanes] x 32 bytes (the lane's run),
//     the same 128 KB as tower_wide.h's, through the same buffer resource (stores at soffset 0).
// Every tile of a launch is a 6-board tile (a batch tail takes one partly empty tile): every board goes
// through the same arithmetic, so outputs are batch-independent bit for bit.  The weight blob is the M16
// layout (evaluator._pack_conv_m16; spmcts_tower_weight_layout reports it for this shape).

namespace wide16 {

using m16::lane_row;
using m16::src_row;

template <class K>
__device__ __forceinline__ int soff(int wave, int t, int h) {
  return ((wave * K::NT + t) * 2 + h) * 64 * 32;
}

// In place: out = relu(acc + bias (+ the block input from scratch)); SAVE also stores the outputs to
// scratch (the next block's residual).  Every wave has finished reading the buffer (barrier before); a
// barrier publishes the outputs.
template <class K, bool RESID, bool SAVE>
__device__ __forceinline__ void epilogue(char *X, const f32x4 (&acc)[4][K::NT][2], const float4 (&bv)[4], uint4 *scr,
                                         int wave, int q, int rb, int lane) {
  const wide::ScrBuf<K> sb(scr);
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  const int ro = (64 * wave + 16 * q) * 2;  // the lane's run: channels 64 wave + 16 q .. + 16 (phys16)
  // residual reads two cell tiles at a time (32 registers in flight beside the 256 accumulator AGPRs)
  constexpr int TB = 2;
#pragma unroll
  for (int t0 = 0; t0 < K::NT; t0 += TB) {
    uint4 res[RESID ? TB : 1][2][2];
    if constexpr (RESID) {
#pragma unroll
      for (int i = 0; i < TB; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int so = soff<K>(wu, t0 + i, h);
          res[i][h][0] = sb.load(lane, 0, so);
          res[i][h][1] = sb.load(lane, 1, so);
        }
    }
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      const int t = t0 + i;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        char *p = X + (t * 32 + rb + h) * K::RS + ro;
        uint32_t o[8];
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
          // physical 4 mm + r within the run: output channel 64 wave + 16 mm + 4 q + r
          float v0 = acc[mm][t][h][0] + bv[mm].x, v1 = acc[mm][t][h][1] + bv[mm].y;
          float v2 = acc[mm][t][h][2] + bv[mm].z, v3 = acc[mm][t][h][3] + bv[mm].w;
          if constexpr (RESID) {
            const f32x2 x0 = K::unpk(((const uint32_t *)&res[i][h][mm >> 1])[2 * (mm & 1)]);
            const f32x2 x1 = K::unpk(((const uint32_t *)&res[i][h][mm >> 1])[2 * (mm & 1) + 1]);
            v0 += x0[0];
            v1 += x0[1];
            v2 += x1[0];
            v3 += x1[1];
          }
          o[2 * mm] = K::relu_pk(f32x2{v0, v1});
          o[2 * mm + 1] = K::relu_pk(f32x2{v2, v3});
        }
        const uint4 lo = make_uint4(o[0], o[1], o[2], o[3]), hi = make_uint4(o[4], o[5], o[6], o[7]);
        *(uint4 *)p = lo;
        *(uint4 *)(p + 16) = hi;
        if constexpr (SAVE) {
          const int so = soff<K>(wu, t, h);
          sb.store(lo, lane, 0, so);
          sb.store(hi, lane, 1, so);
        }
      }
    }
  }
  __syncthreads();
}

// One 3x3 conv over the resident tile, in place: tower_m16.h's k-loop (conv_tap, one channel quarter, all
// cell tiles), then the in-place epilogue.
template <class K, int DEPTH, bool RESID, bool SAVE>
__device__ __forceinline__ void conv(char *X, const Nbr<K> &nb, bf16x8 (&a)[DEPTH][4], const float *bias, int wave,
                                     int lane, const WBuf &wb, uint32_t wl_off, uint32_t wn_off, int wn_steps,
                                     uint4 *scr, float *sbias) {
  using Xl = XLive<K, 0>;
  constexpr int KK32 = K::C / 32;
  static_assert(K::C == K::THREADS, "one bias value per thread");
  static_assert(KK32 % DEPTH == 0, "ring slot must be a compile-time function of k");
  const int q = lane >> 4, rb = lane_row(lane & 15), qoff = 16 * q;
  // the epilogue's bias: one value per thread now, staged in LDS after the k-loop (as tower_wide.h)
  const float bmine = bias[threadIdx.x];
  f32x4 acc[4][K::NT][2];
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
#pragma unroll
    for (int mm = 0; mm < 4; ++mm)
      if ((Xl::ZPRE_T >> t) & 1u) acc[mm][t][0] = acc[mm][t][1] = f32x4{};
  int off_cur[K::NT][2], off_nxt[K::NT][2];
  bf16x8 bc[K::NT][2], bn[K::NT][2];
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
    if ((Xl::lt(0) >> t) & 1u) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        off_cur[t][h] = src_row(nb, 0, t, h, rb, 0) * K::RS + qoff;
        bc[t][h] = lds_b128(X + off_cur[t][h]);
      }
    }
#define TAPW16(T) \
  m16::conv_tap<K, KK32, DEPTH, 0, T>(X, nb, acc, bc, bn, off_cur, off_nxt, a, qoff, rb, wb, wl_off, wn_off, wn_steps)
  TAPW16(0); TAPW16(1); TAPW16(2); TAPW16(3); TAPW16(4); TAPW16(5); TAPW16(6); TAPW16(7); TAPW16(8);
#undef TAPW16
  sbias[threadIdx.x] = bmine;
  __syncthreads();  // every wave has read the layer input: outputs may overwrite it
  float4 bv[4];
#pragma unroll
  for (int mm = 0; mm < 4; ++mm) bv[mm] = *(const float4 *)(sbias + 16 * (4 * wave + mm) + 4 * q);
  epilogue<K, RESID, SAVE>(X, acc, bv, scr, wave, q, rb, lane);
}

// Stem (3 planes padded to one 16-channel k-step per tap, 32x32x16 as tower_wide.h's, bias in the
// accumulators), stored in the phys16 order in place; then each lane copies its runs (the first block's
// input) to scratch in the layout the epilogue reads.
template <class K>
__device__ __forceinline__ void stem(char *X, const Nbr<K> &nb, const bf16x8 *w, const float *bias, int wave, int lane,
                                     uint4 *scr) {
  const int h = lane >> 5;
  f32x16 acc[K::MT][K::NT];
  float4 bv[K::MT][4];
  wide::load_bias<K>(bv, bias, wave, lane);
#pragma unroll
  for (int m = 0; m < K::MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int t = 0; t < K::NT; ++t) {
        acc[m][t][4 * g + 0] = bv[m][g].x;
        acc[m][t][4 * g + 1] = bv[m][g].y;
        acc[m][t][4 * g + 2] = bv[m][g].z;
        acc[m][t][4 * g + 3] = bv[m][g].w;
      }
  bf16x8 a[9][K::MT];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int m = 0; m < K::MT; ++m) a[tap][m] = w[((size_t)(wave * K::MT + m) * 9 + tap) * 64 + lane];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int t = 0; t < K::NT; ++t) {
      const bf16x8 b = lds_b128(X + nb.off(t, tap) + 16 * h);
#pragma unroll
      for (int m = 0; m < K::MT; ++m) acc[m][t] = K::mfma(a[tap][m], b, acc[m][t]);
    }
  }
  __syncthreads();  // every wave has read the stem input
  m16::stem_store<K>(acc, X, wave, lane);
  __syncthreads();
  const wide::ScrBuf<K> sb(scr);
  const int wu = __builtin_amdgcn_readfirstlane(wave);
  const int q = lane >> 4, rb = lane_row(lane & 15), ro = (64 * wave + 16 * q) * 2;
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const char *p = X + (t * 32 + rb + hh) * K::RS + ro;
      const int so = soff<K>(wu, t, hh);
      sb.store(*(const uint4 *)p, lane, 0, so);
      sb.store(*(const uint4 *)(p + 16), lane, 1, so);
    }
}

// One workgroup's tile: boards [board0, board0 + BOARDS), all layers; scr = this workgroup's residual
// scratch (wide::Scr<K>::PER_WG bytes).
template <class K>
__device__ __forceinline__ void tile(char *smem, const __bf16 *planes, int batch, int board0, int n_blocks,
                                     const bf16x8 *wpk, const float *bias, uint16_t *out, uint4 *scr) {
  static_assert(K::EDGE && K::ONEBUF && K::M16 && K::MG == 1 && K::CG == 4 && K::WAVES == 4 && K::C == 256,
                "wide16 trunk: C = 256 6-board edge tiles, one buffer, 4 channel quarters x all cell tiles");
  static_assert(wide::Scr<K>::PER_WG == (size_t)K::WAVES * K::NT * 2 * 64 * 32, "scratch size");
  char *X = smem;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  Nbr<K> nb;
  nb.init(lane & 31, 0);
  for (int i = tid; i < K::NZ * K::RS / 4; i += K::THREADS) ((uint32_t *)(X + K::ZROW * K::RS))[i] = 0u;
  uint16_t *tab = (uint16_t *)(smem + K::BUF);
  float *sbias = (float *)(smem + K::BUF + K::TAB);
#pragma unroll
  for (int j = 0; j < (9 * K::ROWS + K::THREADS - 1) / K::THREADS; ++j)
    if (9 * K::ROWS % K::THREADS == 0 || tid + j * K::THREADS < 9 * K::ROWS)
      tab[tid + j * K::THREADS] = kEdgeNbr[tid + j * K::THREADS];
  nb.tab = tab;
  for (int row = tid; row < K::ROWS; row += K::THREADS) {
    const int board = board0 + K::row_board(row);
    uint16_t *dst = (uint16_t *)(X + row * K::RS);
    const bool ok = K::row_ok(row) && board < batch;
    const size_t src = ((size_t)board * K::CELLS + K::row_cell(row)) * 3;
#pragma unroll
    for (int c = 0; c < 16; ++c) dst[c] = (ok && c < 3) ? K::from_bf16(planes[src + c]) : (uint16_t)0;
  }
  __syncthreads();
  nb.finish();
  constexpr int KK32 = K::C / 32;
  constexpr int DEPTH = K::DEPTH;
  constexpr size_t STEM = (size_t)K::C / 32 * 9 * 64;         // stem fragments (32x32x16 layout)
  constexpr size_t LAYER = (size_t)K::C / 16 * 9 * KK32 * 64;  // one block conv's fragments (16x16x32 layout)
  constexpr int LSTEPS = 9 * KK32;
  stem<K>(X, nb, wpk, bias, wave, lane, scr);
  const bf16x8 *wblk = wpk + STEM;
  const float *b = bias + K::C;
  // per-wave weight streams: layer L, 16-channel tile (4 wave + mm) at wblk + L*LAYER + (4 wave + mm)*LSTEPS*64
  bf16x8 ring[DEPTH][4];
  const int n_convs = 2 * n_blocks;
  if (n_convs > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) ring[d][mm] = wblk[(size_t)(4 * wave + mm) * LSTEPS * 64 + (size_t)d * 64 + lane];
  }
  WBuf wb;
  wb.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)wpk, (short)0, 0x7fffffff, 0x00020000);
  wb.voff = lane * 16;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t ct0_off = (uint32_t)(STEM + (size_t)(4 * wave_u) * LSTEPS * 64) * 16u;
  // one iteration per residual block (a straight line; see tower_wide.h)
  for (int L = 0; L < n_convs; L += 2) {
    const uint32_t wl_off = ct0_off + (uint32_t)((size_t)L * LAYER * 16u);
    conv<K, DEPTH, false, false>(X, nb, ring, b, wave, lane, wb, wl_off, wl_off + (uint32_t)(LAYER * 16u), LSTEPS, scr,
                                 sbias);
    b += K::C;
    const uint32_t wl1 = wl_off + (uint32_t)(LAYER * 16u);
    const uint32_t wn1 = (kRingAlways && L + 2 == n_convs) ? wl1 : wl1 + (uint32_t)(LAYER * 16u);
    conv<K, DEPTH, true, true>(X, nb, ring, b, wave, lane, wb, wl1, wn1, L + 2 < n_convs ? LSTEPS : 0, scr, sbias);
    b += K::C;
  }
  head_layer<K>(X, wblk + (size_t)n_convs * LAYER, b, out, board0, batch, wave, lane);
}

}  // namespace wide16
