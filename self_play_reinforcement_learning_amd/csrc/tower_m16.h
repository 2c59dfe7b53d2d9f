// tower_m16.h — the C = 128 Connect4 trunk on v_mfma_f32_16x16x32_{bf16,f16} (round 4).
//
// Included by tower.hip (namespace tower): uses Cfg (M16), Nbr, XLive, WBuf, lds_b128, kRingAlways,
// stem_layer's k-loop shape and head_layer from there.
//
// The same workgroup plan as the 32x32x16 edge-tile trunk (6 boards in 256 edge-ordered rows, two LDS
// buffers, 4 waves = 2 channel halves x 2 row halves, 12 of the 72 (tile, tap) pairs skipped), with each
// 32-row x 32-channel output tile computed as 2 x 2 tiles of 16 x 16 over K = 32 input channels per MFMA:
//   * A (weights): fragment (16-channel tile, tap, 32-channel k-step), lane l = 16 q + n holds
//     W[16 ct + n][tap][physical input channels 32 k + 8 q .. + 8] (evaluator._pack_conv_m16);
//   * B (activations): lane l reads 16 bytes of row (tile t, row lane_row(l & 15) + h) at physical
//     channels 32 k + 8 q: the same rows and bytes per k-step as the 32x32x16 form, other lane addresses
//     (lane_row: the fragment's rows are the tile's rows of one residue parity, bank-conflict free);
//   * D: lane l holds output channels 16 mm + 4 q + r (r = 0..3) of that row; stored at the PHYSICAL
//     position 64 cg + 16 q + 4 mm + r (phys16), so each lane's 16 values of a cell are one contiguous
//     32-byte run (the next layer's weights take their input channels in this order; it is its own
//     inverse: evaluator.phys_channel_order_m16).
// Same FLOPs, the same LDS and weight bytes per k-step as the 32x32x16 form; the 16x16x32 MFMA holds a
// higher clock on this chip (MI355X_MICROARCH.md 'DVFS give-back' item 7): a timing probe in this kernel
// (two 16x16x32 per 32x32x16, same loads) ran 1.88 vs 1.72 GHz and 5 % faster (profiles/r04/mfma_shape/).
// Every tile of a launch is a 6-board tile (a batch tail takes one partly empty tile), so every board of
// a batch goes through the same arithmetic: outputs stay batch-independent bit for bit.

namespace m16 {

// 16-channel output tiles per wave: 4 with the 2 x 2 wave plan (channel halves x row halves, the product
// trunk), 2 with 4 x 1 (channel quarters x all rows, A/B code 1640)
template <class K>
constexpr int MM = K::C / 16 / K::CG;

// byte offset, within a row, of the physical run of lane quarter q for the wave's channel group cg: the
// wave's 16-channel tiles ct = MM cg + mm sit at 64 (ct / 4) + 16 q + 4 (ct % 4) + r (phys16), so its MM tiles
// are one run of 4 MM halfs (32 B for MM = 4, 16 B for MM = 2)
template <class K>
__device__ __forceinline__ int run_off(int cg, int q) {
  const int ct0 = MM<K> * cg;
  return (64 * (ct0 / 4) + 16 * q + 4 * (ct0 % 4)) * 2;
}

// Which of a 32-row tile's rows MFMA column n of fragment h (0, 1) stands for: row lane_row(n) + h.
// A B-fragment ds_read_b128 is serviced in 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32)
// (MI355X_MICROARCH.md §LDS); lane 16 q + n reads its row at 16-B slot (row + q + 4 k) mod 16 (272-B
// rows), so group 0 holds columns A = {0-3, 12-15} at quarter q and B = {4-11} at q + 1, group 1 the
// reverse.  With column n on row n (round 4) the two k offsets of a group collide (44 % of the trunk's LDS
// cycles were conflict cycles, profiles/r04/m16/stall_lds_pmc.txt): no permutation of one 16-row half
// avoids it (the A rows and the B rows + 1 would both have to fill the residues the other leaves).  Here
// fragment h takes the tile's 16 rows of residue parity h, each residue once in A and once in B: A's
// residues 2 i + h and B's 2 i + h + 1 are disjoint, so every group reads 16 distinct slots at the
// centre tap, and — the edge rows are residue-coloured (tower_edge.h: a tap shifts every row's residue
// by the same amount) — at every tap (tests/test_tower_edge_layout.py checks all 60 live (tile, tap)
// reads).  Each output element is the same MFMA sum as before, only in another column: bit-identical.
__device__ __forceinline__ int lane_row(int n) {
  const bool in_a = n < 4 || n >= 12;
  const int i = in_a ? (n < 4 ? n : n - 8) : n - 4;
  return (in_a ? 0 : 16) + 2 * i;
}

// the source row of (tile t, fragment h) for `tap`: the edge table, for this lane's row rb + h
template <class K>
__device__ __forceinline__ int src_row(const Nbr<K> &nb, int mg, int t, int h, int rb, int tap) {
  return (int)nb.tab[tap * K::ROWS + (mg * K::NT + t) * 32 + rb + h];
}

template <class K>
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (K::BF16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
}

// One tap of a layer: KK32 k-steps of 32 input channels; B fragments one k-step ahead (the next tap's
// first ones from its own rows), the weight ring DEPTH k-steps ahead and on into the next layer.
template <class K, int KK32, int DEPTH, int MG_, int TAP>
__device__ __forceinline__ void conv_tap(const char *src, const Nbr<K> &nb, f32x4 (&acc)[MM<K>][K::NT][2],
                                         bf16x8 (&bc)[K::NT][2], bf16x8 (&bn)[K::NT][2], int (&off_cur)[K::NT][2],
                                         int (&off_nxt)[K::NT][2], bf16x8 (&a)[DEPTH][MM<K>], int qoff, int rb,
                                         const WBuf &wb, uint32_t wl_off, uint32_t wn_off, int wn_steps) {
  using X = XLive<K, MG_>;
  constexpr int NM = MM<K>;
  constexpr uint32_t MSTRIDE = 9u * KK32 * 1024u;  // bytes between a wave's 16-channel tiles
  constexpr int STEPS = 9 * KK32;
  constexpr uint32_t LV = X::lt(TAP);
  constexpr uint32_t LVN = TAP < 8 ? X::lt(TAP < 8 ? TAP + 1 : 8) : 0u;
  constexpr int NTA = (int)X::popc(LV);
  if constexpr (TAP < 8) {
    // the next tap's source rows, read here and turned into byte offsets in this tap's last k-step
#pragma unroll
    for (int t = 0; t < K::NT; ++t)
      if ((LVN >> t) & 1u) {
        off_nxt[t][0] = src_row(nb, MG_, t, 0, rb, TAP + 1);
        off_nxt[t][1] = src_row(nb, MG_, t, 1, rb, TAP + 1);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int k = 0; k < KK32; ++k) {
    const int s = TAP * KK32 + k;
    if (k + 1 < KK32) {
#pragma unroll
      for (int t = 0; t < K::NT; ++t)
        if ((LV >> t) & 1u) {
          bn[t][0] = lds_b128(src + off_cur[t][0] + (k + 1) * 64);
          bn[t][1] = lds_b128(src + off_cur[t][1] + (k + 1) * 64);
        }
    } else if (TAP < 8) {
#pragma unroll
      for (int t = 0; t < K::NT; ++t)
        if ((LVN >> t) & 1u) {
          off_nxt[t][0] = off_nxt[t][0] * K::RS + qoff;
          off_nxt[t][1] = off_nxt[t][1] * K::RS + qoff;
          bn[t][0] = lds_b128(src + off_nxt[t][0]);
          bn[t][1] = lds_b128(src + off_nxt[t][1]);
        }
    }
    const int slot = k % DEPTH;
    bf16x8 acur[NM];
#pragma unroll
    for (int mm = 0; mm < NM; ++mm) acur[mm] = a[slot][mm];
    const int sn = s + DEPTH;
    if (sn < STEPS) {
#pragma unroll
      for (int mm = 0; mm < NM; ++mm) a[slot][mm] = wb.load(wl_off + mm * MSTRIDE + (uint32_t)sn * 1024u);
    } else if (kRingAlways || sn - STEPS < wn_steps) {
#pragma unroll
      for (int mm = 0; mm < NM; ++mm) a[slot][mm] = wb.load(wn_off + mm * MSTRIDE + (uint32_t)(sn - STEPS) * 1024u);
    }
#pragma unroll
    for (int t = 0; t < K::NT; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int mm = 0; mm < NM; ++mm)
          if ((LV >> t) & 1u)
            acc[mm][t][h] = mfma16<K>(acur[mm], bc[t][h], (TAP == 0 && k == 0) ? f32x4{} : acc[mm][t][h]);
    // one operand read or weight load per MFMA gap: 2 NTA LDS reads and NM weight loads among 2 NM NTA MFMAs
#pragma unroll
    for (int i = 0; i < 2 * NTA; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * NM * NTA - 2 * NTA - NM, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < K::NT; ++t) {
      bc[t][0] = bn[t][0];
      bc[t][1] = bn[t][1];
    }
  }
#pragma unroll
  for (int t = 0; t < K::NT; ++t) {
    off_cur[t][0] = off_nxt[t][0];
    off_cur[t][1] = off_nxt[t][1];
  }
}

#ifdef SPMCTS_AB
#include "tower_m16_abl.h"  // the k-loop's timing ablations (A/B library only)
#endif

// a tap of conv_layer: the product's conv_tap (or, in the A/B library, the ablation copy for a Cfg::ABL code)
template <class K, int KK32, int DEPTH, int MG_, int TAP>
__device__ __forceinline__ void tap(const char *src, const Nbr<K> &nb, f32x4 (&acc)[MM<K>][K::NT][2],
                                    bf16x8 (&bc)[K::NT][2], bf16x8 (&bn)[K::NT][2], int (&off_cur)[K::NT][2],
                                    int (&off_nxt)[K::NT][2], bf16x8 (&a)[DEPTH][MM<K>], int qoff, int rb,
                                    const WBuf &wb, uint32_t wl_off, uint32_t wn_off, int wn_steps) {
#ifdef SPMCTS_AB
  if constexpr (K::ABL != 0) {
    conv_tap_abl<K, KK32, DEPTH, MG_, TAP>(src, nb, acc, bc, bn, off_cur, off_nxt, a, qoff, rb, wb, wl_off, wn_off, wn_steps);
    return;
  }
#endif
  conv_tap<K, KK32, DEPTH, MG_, TAP>(src, nb, acc, bc, bn, off_cur, off_nxt, a, qoff, rb, wb, wl_off, wn_off, wn_steps);
}

// out = relu(acc + bias (+ the block input at the same physical positions, RESID)), into dst.
template <class K, bool RESID>
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[MM<K>][K::NT][2], char *dst, const float4 (&bv)[MM<K>],
                                         int cg, int mg, int q, int rb) {
  constexpr int NM = MM<K>, NU = NM / 2;  // the run: NU 16-byte pieces
#pragma unroll
  for (int t = 0; t < K::NT; ++t) {
    uint4 res[2][NU];
    if constexpr (RESID) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const char *p = dst + ((mg * K::NT + t) * 32 + rb + h) * K::RS + run_off<K>(cg, q);
#pragma unroll
        for (int u = 0; u < NU; ++u) res[h][u] = *(const uint4 *)(p + 16 * u);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      char *p = dst + ((mg * K::NT + t) * 32 + rb + h) * K::RS + run_off<K>(cg, q);
      uint32_t o[2 * NM];
#pragma unroll
      for (int mm = 0; mm < NM; ++mm) {
        // physical 4 mm + r within the run: output channel 16 mm + 4 q + r
        float v0 = acc[mm][t][h][0] + bv[mm].x, v1 = acc[mm][t][h][1] + bv[mm].y;
        float v2 = acc[mm][t][h][2] + bv[mm].z, v3 = acc[mm][t][h][3] + bv[mm].w;
        if constexpr (RESID) {
          const f32x2 x0 = K::unpk(((const uint32_t *)&res[h][mm >> 1])[2 * (mm & 1)]);
          const f32x2 x1 = K::unpk(((const uint32_t *)&res[h][mm >> 1])[2 * (mm & 1) + 1]);
          v0 += x0[0];
          v1 += x0[1];
          v2 += x1[0];
          v3 += x1[1];
        }
        o[2 * mm] = K::relu_pk(f32x2{v0, v1});
        o[2 * mm + 1] = K::relu_pk(f32x2{v2, v3});
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) *(uint4 *)(p + 16 * u) = make_uint4(o[4 * u], o[4 * u + 1], o[4 * u + 2], o[4 * u + 3]);
    }
  }
}

template <class K, int KK32, int DEPTH, bool RESID, int MG_>
__device__ __forceinline__ void conv_layer(const char *src, char *dst, const Nbr<K> &nb, bf16x8 (&a)[DEPTH][MM<K>],
                                           const float *bias, int cg, int lane, const WBuf &wb, uint32_t wl_off,
                                           uint32_t wn_off, int wn_steps) {
  using X = XLive<K, MG_>;
  constexpr int NM = MM<K>;
  static_assert(KK32 % DEPTH == 0, "ring slot must be a compile-time function of k");
  const int q = lane >> 4, rb = lane_row(lane & 15), qoff = 16 * q;
  float4 bv[NM];  // the epilogue's bias, fetched now (its latency hides under the k-loop)
#pragma unroll
  for (int mm = 0; mm < NM; ++mm) bv[mm] = *(const float4 *)(bias + 16 * (NM * cg + mm) + 4 * q);
  f32x4 acc[NM][K::NT][2];
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
#pragma unroll
    for (int mm = 0; mm < NM; ++mm)
      if ((X::ZPRE_T >> t) & 1u) acc[mm][t][0] = acc[mm][t][1] = f32x4{};
  int off_cur[K::NT][2], off_nxt[K::NT][2];
  bf16x8 bc[K::NT][2], bn[K::NT][2];
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
    if ((X::lt(0) >> t) & 1u) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        off_cur[t][h] = src_row(nb, MG_, t, h, rb, 0) * K::RS + qoff;
        bc[t][h] = lds_b128(src + off_cur[t][h]);
      }
    }
#define TAP16(T) tap<K, KK32, DEPTH, MG_, T>(src, nb, acc, bc, bn, off_cur, off_nxt, a, qoff, rb, wb, wl_off, wn_off, wn_steps)
  TAP16(0); TAP16(1); TAP16(2); TAP16(3); TAP16(4); TAP16(5); TAP16(6); TAP16(7); TAP16(8);
#undef TAP16
  epilogue<K, RESID>(acc, dst, bv, cg, MG_, q, rb);
}

// The stem's epilogue (32x32x16 accumulators, bias already in them): lane's output channels
// ct*32 + 8g + 4h + j go to their phys16 positions, four contiguous per (ct, g).
template <class K>
__device__ __forceinline__ void stem_store(const f32x16 (&acc)[K::MT][K::NT], char *dst, int wave, int lane) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int m = 0; m < K::MT; ++m) {
    const int ct = (wave % K::CG) * K::MT + m;  // 32-channel tile: half ct / 2, 16-tiles 2 (ct % 2) + g / 2
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int pos = 64 * (ct >> 1) + 16 * (2 * (g & 1) + h) + 4 * (2 * (ct & 1) + (g >> 1));
#pragma unroll
      for (int t = 0; t < K::NT; ++t) {
        const uint2 o = make_uint2(K::relu_pk(f32x2{acc[m][t][4 * g + 0], acc[m][t][4 * g + 1]}),
                                   K::relu_pk(f32x2{acc[m][t][4 * g + 2], acc[m][t][4 * g + 3]}));
        *(uint2 *)(dst + (((wave / K::CG) * K::NT + t) * 32 + r) * K::RS + pos * 2) = o;
      }
    }
  }
}

// The stem of the two-buffer kernel (3 planes padded to one 16-channel k-step per tap, 32x32x16) with
// the phys16 store.
template <class K>
__device__ __forceinline__ void stem(const char *src, char *dst, const Nbr<K> &nb, const bf16x8 *w, const float *bias,
                                     int wave, int lane) {
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
      for (int m = 0; m < K::MT; ++m) acc[m][t] = K::mfma(a[tap][m], b, acc[m][t]);
    }
  }
  stem_store<K>(acc, dst, wave, lane);
}

// One workgroup's tile (the two-buffer edge layout of tower_tile): stem (32x32x16) -> 2 n_blocks convs
// (16x16x32) -> head convs (head_layer, 32x32x16 over the phys16 channel order).
template <class K>
__device__ __forceinline__ void tile(char *smem, const __bf16 *planes, int batch, int board0, int n_blocks,
                                     const bf16x8 *wpk, const float *bias, uint16_t *out) {
  static_assert(K::EDGE && K::C == 128 && K::WAVES == 4 && !K::ONEBUF &&
                    ((K::CG == 2 && K::MG == 2) || (K::CG == 4 && K::MG == 1)),
                "m16 trunk: C = 128 edge tiles, 2 channel halves x 2 row halves (or 4 channel quarters x 1)");
  constexpr int NM = MM<K>;
  char *X = smem;
  char *Y = smem + K::BUF;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  Nbr<K> nb;
  nb.init(lane & 31, wave / K::CG);
  for (int i = tid; i < K::NZ * K::RS / 4; i += K::THREADS) {
    ((uint32_t *)(X + K::ZROW * K::RS))[i] = 0u;
    ((uint32_t *)(Y + K::ZROW * K::RS))[i] = 0u;
  }
  uint16_t *tab = (uint16_t *)(smem + 2 * K::BUF);
#pragma unroll
  for (int j = 0; j < (9 * K::ROWS + K::THREADS - 1) / K::THREADS; ++j)
    if (9 * K::ROWS % K::THREADS == 0 || tid + j * K::THREADS < 9 * K::ROWS)
      tab[tid + j * K::THREADS] = kEdgeNbr[tid + j * K::THREADS];
  nb.tab = tab;
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

  constexpr int KK32 = K::C / 32;
  constexpr int DEPTH = K::DEPTH;
  constexpr size_t STEM = (size_t)K::C / 32 * 9 * 64;         // stem fragments (32x32x16 layout)
  constexpr size_t LAYER = (size_t)K::C / 16 * 9 * KK32 * 64;  // one block conv's fragments (16x16x32 layout)
  constexpr int LSTEPS = 9 * KK32;
  stem<K>(Y, X, nb, wpk, bias, wave, lane);
  __syncthreads();
  const bf16x8 *wblk = wpk + STEM;
  const float *b = bias + K::C;
  const int cg = wave % K::CG;
  // per-wave weight streams: layer L, 16-channel tile (NM cg + mm) starts at wblk + L*LAYER + (NM cg + mm)*LSTEPS*64
  bf16x8 ring[DEPTH][NM];
  const int n_convs = 2 * n_blocks;
  if (n_convs > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int mm = 0; mm < NM; ++mm) ring[d][mm] = wblk[(size_t)(NM * cg + mm) * LSTEPS * 64 + (size_t)d * 64 + lane];
  }
  WBuf wb;
  wb.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)wpk, (short)0, 0x7fffffff, 0x00020000);
  wb.voff = lane * 16;
  const int cg_u = __builtin_amdgcn_readfirstlane(cg);
  const uint32_t ct0_off = (uint32_t)(STEM + (size_t)(NM * cg_u) * LSTEPS * 64) * 16u;
  for (int L = 0; L < n_convs; ++L) {
#ifdef SPMCTS_AB
    // timing ablation (A/B code 1665, wrong results): every layer streams layer 0's weights, an L2-resident
    // 295 KB set instead of 11.8 MB re-streamed from the fabric per round of workgroups
    const bool l2w = (K::ABL & 65536) != 0;
    const uint32_t wl_off = ct0_off + (l2w ? 0u : (uint32_t)((size_t)L * LAYER * 16u));
    const uint32_t wn_off = (l2w || (kRingAlways && L + 1 == n_convs)) ? wl_off : wl_off + (uint32_t)(LAYER * 16u);
#else
    const uint32_t wl_off = ct0_off + (uint32_t)((size_t)L * LAYER * 16u);
    const uint32_t wn_off = (kRingAlways && L + 1 == n_convs) ? wl_off : wl_off + (uint32_t)(LAYER * 16u);
#endif
    const int wn_steps = L + 1 < n_convs ? LSTEPS : 0;
    const bool even = (L & 1) == 0;
    if (K::MG == 1 || wave / K::CG == 0) {
      if (even) conv_layer<K, KK32, DEPTH, false, 0>(X, Y, nb, ring, b, cg, lane, wb, wl_off, wn_off, wn_steps);
      else conv_layer<K, KK32, DEPTH, true, 0>(Y, X, nb, ring, b, cg, lane, wb, wl_off, wn_off, wn_steps);
    } else if constexpr (K::MG == 2) {
      if (even) conv_layer<K, KK32, DEPTH, false, 1>(X, Y, nb, ring, b, cg, lane, wb, wl_off, wn_off, wn_steps);
      else conv_layer<K, KK32, DEPTH, true, 1>(Y, X, nb, ring, b, cg, lane, wb, wl_off, wn_off, wn_steps);
    }
    b += K::C;
    __syncthreads();
  }
  head_layer<K>(X, wblk + (size_t)n_convs * LAYER, b, out, board0, batch, wave, lane);
}

}  // namespace m16
