// tower_ring.h — the fused trunk with its weight stream shared through an LDS ring (round 3).
//
// Included by tower.hip (namespace tower): uses Cfg, Ty, Nbr-style neighbour tables, phys_off and
// head_layer from there.  Instantiated for the Connect4 ResNet-128 trunk (C = 128, 6-board
// edge-layout tiles of 256 rows, tower_edge.h).
//
// What changes against tower_tile (the two-buffer kernel):
//   * the weights of a k-step (4 channel tiles x 1 KiB fragments) are copied ONCE per CU into an LDS
//     ring by LDS-DMA (global_load_lds_dwordx4, one fragment per wave and k-step) and read from there
//     by the two waves of each channel half, instead of both waves loading the same fragment from
//     L2 into registers: half the weight requests per CU;
//   * the ring needs a workgroup barrier every phase of 2 k-steps (a DMA'd slot is readable by the
//     other waves only after its issuing wave's counted vmcnt and a barrier).  Barriers make the
//     waves run in lock step, so every phase must give the two row halves the same number of live
//     (tile, tap) MFMAs: each row half owns one dx-edge and one dy-edge tile (tiles {0, 6, 2, 3} and
//     {1, 7, 4, 5}), and the k-steps of taps 1 | 3 and 5 | 7 are interleaved kk by kk (their live
//     counts are 3 | 4 and 4 | 3 in one half, 4 | 3 and 3 | 4 in the other); every other tap has
//     equal counts in both halves;
//   * the LDS for the ring comes from holding ONE activation buffer: a conv reads the buffer for
//     all its k-steps, the waves meet at a barrier, then each wave writes its own outputs in place
//     (the first conv of a block first reads its output positions, the block input, into registers:
//     that is the residual the block's second conv adds), and a second barrier publishes them;
//   * the per-layer biases sit in LDS (copied once per workgroup), so the k-loop's only vector
//     memory instructions are the DMAs and the vmcnt counts are exact.
// Results are deterministic and batch-independent (every board goes through the same tile code);
// the k-step order differs from tower_tile's, so the bits differ from that kernel's.

namespace ring {

// timing ablations (wrong results; kernel analysis only): 1 = no DMAs in the k-loop, 2 = no phase
// barriers, 4 = no A-fragment reads from the ring
#ifndef SPMCTS_RING_ABL
#define SPMCTS_RING_ABL 0
#endif
constexpr int ABL = SPMCTS_RING_ABL;

constexpr int KK = 8;          // k-steps per tap (C = 128: 8 x 16 input channels)
constexpr int STEPS = 9 * KK;  // k-steps per conv layer
constexpr int R = 8;           // ring slots, one k-step (4 fragments) each
constexpr int D = 6;           // DMA lead in k-steps
constexpr int FRAG = 1024;     // one (32-channel tile, k-step) weight fragment
constexpr int SLOT = 4 * FRAG;
constexpr int MAX_CONVS = 48;  // bias table bound (n_blocks <= 24)

// row halves' tiles: each holds one dx-edge tile (0: x = 0, 6: x = 6) and one dy-edge tile (1: y = 0,
// 7: y = 5) of the edge layout
__host__ __device__ constexpr int tile_of(int mg, int t) {
  return mg == 0 ? (t == 0 ? 0 : t == 1 ? 6 : t + 0) : (t == 0 ? 1 : t == 1 ? 7 : t + 2);
}

// k-step order of a layer: segments {0}, {1|3}, {2}, {4}, {5|7}, {6}, {8}; a paired segment
// alternates its two taps kk by kk
struct Order {
  int tap[STEPS];
  int kk[STEPS];
};
__host__ __device__ constexpr Order make_order() {
  Order o{};
  int i = 0;
  const int seg[7][2] = {{0, -1}, {1, 3}, {2, -1}, {4, -1}, {5, 7}, {6, -1}, {8, -1}};
  for (int s = 0; s < 7; ++s)
    for (int k = 0; k < KK; ++k)
      for (int j = 0; j < 2; ++j) {
        if (seg[s][j] < 0) continue;
        o.tap[i] = seg[s][j];
        o.kk[i] = k;
        ++i;
      }
  return o;
}
constexpr Order kOrd = make_order();

template <class K>
struct Geo {
  static constexpr int RS = K::RS;
  static constexpr int X = 0;                       // the activation buffer: (ROWS + NZ) rows
  static constexpr int TAB = K::BUF;                // [9][ROWS] uint16 neighbour rows
  static constexpr int RING = TAB + 9 * K::ROWS * 2;
  static constexpr int BIAS = RING + R * SLOT;      // [n_convs][C] f32
  static constexpr int lds(int n_convs) { return BIAS + n_convs * K::C * 4; }
  static_assert(RING % 16 == 0 && BIAS % 16 == 0, "16-byte aligned regions");
  static_assert(BIAS + MAX_CONVS * K::C * 4 <= 163840, "LDS budget");
  // does tile t of row half mg have an on-board neighbour for `tap`?
  static constexpr bool live(int mg, int t, int tap) { return K::tile_tap_live(tile_of(mg, t), tap); }
  static constexpr uint32_t lmask(int mg, int tap) {
    uint32_t m = 0;
    for (int t = 0; t < K::NT; ++t)
      if (live(mg, t, tap)) m |= 1u << t;
    return m;
  }
  static constexpr int popc(uint32_t m) { return m ? (int)(m & 1u) + popc(m >> 1) : 0; }
  // the first step at which tile t is live (its accumulator starts from zero there)
  static constexpr int first(int mg, int t) {
    for (int i = 0; i < STEPS; ++i)
      if (live(mg, t, kOrd.tap[i])) return i;
    return STEPS;
  }
  // tiles whose accumulators start from zero at step i (a mask, so kernels test it at compile time)
  static constexpr uint32_t zmask(int mg, int i) {
    uint32_t m = 0;
    for (int t = 0; t < K::NT; ++t)
      if (first(mg, t) == i) m |= 1u << t;
    return m;
  }
  // phases (pairs of steps) are balanced: both row halves issue the same number of MFMAs
  static constexpr bool balanced() {
    for (int i = 0; i < STEPS; i += 2)
      if (popc(lmask(0, kOrd.tap[i])) + popc(lmask(0, kOrd.tap[i + 1])) !=
          popc(lmask(1, kOrd.tap[i])) + popc(lmask(1, kOrd.tap[i + 1])))
        return false;
    return true;
  }
};

__device__ __forceinline__ void lds_dma16(const void *gsrc, char *lds_dst) {
  __builtin_amdgcn_global_load_lds(gsrc, (__attribute__((address_space(3))) void *)lds_dst, 16, 0, 0);
}

// DMA of fragment `ct` (= the issuing wave) of step I (kOrd order) of conv layer Lx into ring `slot`.
// The source is the two-buffer kernel's weight blob as it is ([layer][ct][tap][kk][64 lanes][16 B]):
// a fragment is 1 KiB wherever it sits, so the ring needs no repacked copy.
template <int I>
__device__ __forceinline__ void issue_dma(char *ring, const char *wconv, int Lx, int slot, int ct, int lane) {
  constexpr int TAP = kOrd.tap[I], KKI = kOrd.kk[I];
  lds_dma16(wconv + (((size_t)Lx * 4 + ct) * STEPS + TAP * KK + KKI) * FRAG + lane * 16, ring + slot * SLOT + ct * FRAG);
}

// Per-wave state of the conv k-loop.
template <class K>
struct Wave {
  int lane, h, r, cg, mg;
  int rowi[K::NT];   // this lane's row of each tile
  int off[9][K::NT]; // byte offset (row * RS + 16h) of each tap's source row, per tile
};

// The conv k-loop of one layer for row half MG_: STEPS k-steps in kOrd order, A fragments from the
// ring slot of each step (one step ahead), B fragments from the activation buffer (one step ahead),
// one DMA per step for step + D, and the phase barrier after every second step.
template <class K, int MG_, int I>
__device__ __forceinline__ void ring_step(char *smem, const Wave<K> &w, f32x16 (&acc)[K::MT][K::NT],
                                          bf16x8 (&acur)[K::MT], bf16x8 (&anext)[K::MT], bf16x8 (&bcur)[K::NT],
                                          bf16x8 (&bnext)[K::NT], int L, int n_convs, const char *wconv, int ct) {
  using G = Geo<K>;
  constexpr int TAP = kOrd.tap[I];
  constexpr uint32_t LV = G::lmask(MG_, TAP);
  constexpr int NM = K::MT * G::popc(LV);  // MFMAs of this step
  constexpr bool HAS_NEXT = I + 1 < STEPS;
  constexpr int TAPN = HAS_NEXT ? kOrd.tap[I + 1] : 0;
  constexpr int KKN = HAS_NEXT ? kOrd.kk[I + 1] : 0;
  constexpr uint32_t LVN = HAS_NEXT ? G::lmask(MG_, TAPN) : 0u;
  constexpr int NDS = K::MT + G::popc(LVN);  // LDS reads issued this step (next step's A and B)
  constexpr uint32_t ZM = G::zmask(MG_, I);  // tiles starting from zero here
  const int J = L * STEPS + I;
  char *ring = smem + G::RING;
  // DMA of step J + D (this wave's fragment); past the last layer the last layer is re-read (keeps the
  // per-phase DMA count; the slot it lands in has been consumed)
  if constexpr (ABL & 1) {
  } else if constexpr (I + D < STEPS) {
    issue_dma<I + D>(ring, wconv, L, (J + D) % R, ct, w.lane);
  } else {
    issue_dma<I + D - STEPS>(ring, wconv, L + 1 < n_convs ? L + 1 : L, (J + D) % R, ct, w.lane);
  }
  // A fragments of the next step (the next layer's step 0 after the last step)
  if constexpr (ABL & 4) {
#pragma unroll
    for (int m = 0; m < K::MT; ++m) anext[m] = acur[m];
  } else {
    const char *slot = ring + ((J + 1) % R) * SLOT + w.lane * 16;
#pragma unroll
    for (int m = 0; m < K::MT; ++m) anext[m] = *(const bf16x8 *)(slot + (w.cg * K::MT + m) * FRAG);
  }
  // B fragments of the next step (within the layer: the buffer is rewritten after the last step)
  if constexpr (HAS_NEXT) {
#pragma unroll
    for (int t = 0; t < K::NT; ++t)
      if ((LVN >> t) & 1u) bnext[t] = *(const bf16x8 *)(smem + w.off[TAPN][t] + KKN * 32);
  }
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
#pragma unroll
    for (int m = 0; m < K::MT; ++m)
      if ((LV >> t) & 1u) {
        if ((ZM >> t) & 1u)
          acc[m][t] = K::mfma(acur[m], bcur[t], f32x16{});
        else
          acc[m][t] = K::mfma(acur[m], bcur[t], acc[m][t]);
      }
  // MFMA, the DMA, then one LDS read per MFMA gap
  __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
  __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (the DMA)
#pragma unroll
  for (int i = 0; i < NDS; ++i) {
    if (i + 1 < NM) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                   // DS read
  }
  if constexpr (NM - 1 > NDS) __builtin_amdgcn_sched_group_barrier(0x008, NM - 1 - NDS, 0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int m = 0; m < K::MT; ++m) acur[m] = anext[m];
#pragma unroll
  for (int t = 0; t < K::NT; ++t) bcur[t] = bnext[t];
  if constexpr (I & 1) {
    // phase end: this wave's DMAs up to the previous phase have landed (only this phase's two are
    // in flight) and its LDS reads are complete; after the barrier every wave may read those slots
    // and every wave's DMA may overwrite the slots read before it
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    if constexpr (!(ABL & 2)) __builtin_amdgcn_s_barrier();
  }
}

template <class K, int MG_, int... Is>
__device__ __forceinline__ void ring_steps(char *smem, const Wave<K> &w, f32x16 (&acc)[K::MT][K::NT],
                                           bf16x8 (&acur)[K::MT], bf16x8 (&anext)[K::MT], bf16x8 (&bcur)[K::NT],
                                           bf16x8 (&bnext)[K::NT], int L, int n_convs, const char *wconv, int ct,
                                           std::integer_sequence<int, Is...>) {
  (ring_step<K, MG_, Is>(smem, w, acc, acur, anext, bcur, bnext, L, n_convs, wconv, ct), ...);
}

// B fragments of a layer's first step (after the previous layer's outputs are published)
template <class K, int MG_>
__device__ __forceinline__ void first_b(const char *smem, const Wave<K> &w, bf16x8 (&bcur)[K::NT]) {
  constexpr uint32_t LV = Geo<K>::lmask(MG_, kOrd.tap[0]);
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
    if ((LV >> t) & 1u) bcur[t] = *(const bf16x8 *)(smem + w.off[kOrd.tap[0]][t] + kOrd.kk[0] * 32);
}

// In-place epilogue: every wave has finished reading the buffer (the last phase barrier).  RESID =
// false (a block's first conv): the lane's output positions hold the block input, read into `res`
// before they are overwritten.  RESID = true: out = relu(acc + bias + res).
template <class K, bool RESID, int MG_>
__device__ __forceinline__ void ring_epilogue(char *smem, const Wave<K> &w, const f32x16 (&acc)[K::MT][K::NT],
                                              uint4 (&res)[K::MT][K::NT][2], const float *bias_lds, bool save) {
  float4 bv[K::MT][4];
#pragma unroll
  for (int m = 0; m < K::MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) bv[m][g] = *(const float4 *)(bias_lds + (w.cg * K::MT + m) * 32 + 8 * g + 4 * w.h);
#pragma unroll
  for (int m = 0; m < K::MT; ++m) {
    const int ct = w.cg * K::MT + m;
    if (!RESID && save) {
#pragma unroll
      for (int t = 0; t < K::NT; ++t) {
        const char *p = smem + w.rowi[t] * K::RS + phys_off(ct, w.h, 0);
        res[m][t][0] = *(const uint4 *)p;
        res[m][t][1] = *(const uint4 *)(p + 16);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int t = 0; t < K::NT; ++t) {
      char *p = smem + w.rowi[t] * K::RS + phys_off(ct, w.h, 0);
      uint32_t o[8];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v0 = acc[m][t][4 * g + 0] + bv[m][g].x, v1 = acc[m][t][4 * g + 1] + bv[m][g].y;
        float v2 = acc[m][t][4 * g + 2] + bv[m][g].z, v3 = acc[m][t][4 * g + 3] + bv[m][g].w;
        if constexpr (RESID) {
          const f32x2 x0 = K::unpk(((const uint32_t *)&res[m][t][g >> 1])[2 * (g & 1)]);
          const f32x2 x1 = K::unpk(((const uint32_t *)&res[m][t][g >> 1])[2 * (g & 1) + 1]);
          v0 += x0[0];
          v1 += x0[1];
          v2 += x1[0];
          v3 += x1[1];
        }
        o[2 * g] = K::relu_pk(f32x2{v0, v1});
        o[2 * g + 1] = K::relu_pk(f32x2{v2, v3});
      }
      *(uint4 *)p = make_uint4(o[0], o[1], o[2], o[3]);
      *(uint4 *)(p + 16) = make_uint4(o[4], o[5], o[6], o[7]);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the outputs are written
  __builtin_amdgcn_s_barrier();        // ... and visible to every wave
}

// One conv layer for row half MG_ (k-loop, then the in-place epilogue)
template <class K, int MG_, bool RESID>
__device__ __forceinline__ void ring_conv(char *smem, const Wave<K> &w, bf16x8 (&acur)[K::MT],
                                          uint4 (&res)[K::MT][K::NT][2], int L, int n_convs, const char *wconv,
                                          int ct, bool save_res) {
  f32x16 acc[K::MT][K::NT];
  bf16x8 anext[K::MT], bcur[K::NT], bnext[K::NT];
  first_b<K, MG_>(smem, w, bcur);
  ring_steps<K, MG_>(smem, w, acc, acur, anext, bcur, bnext, L, n_convs, wconv, ct,
                     std::make_integer_sequence<int, STEPS>{});
  ring_epilogue<K, RESID, MG_>(smem, w, acc, res, (const float *)(smem + Geo<K>::BIAS) + L * K::C, save_res);
}

// Stem (conv3x3 over the 3 input planes, one 16-channel k-step per tap) in place: the input planes
// sit in the first 32 bytes of each row of the buffer.
template <class K>
__device__ __forceinline__ void ring_stem(char *smem, const Wave<K> &w, const bf16x8 *wst, const float *bias) {
  f32x16 acc[K::MT][K::NT];
  bf16x8 a[9][K::MT];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int m = 0; m < K::MT; ++m) a[tap][m] = wst[((size_t)(w.cg * K::MT + m) * 9 + tap) * 64 + w.lane];
  float4 bv[K::MT][4];
#pragma unroll
  for (int m = 0; m < K::MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) bv[m][g] = *(const float4 *)(bias + (w.cg * K::MT + m) * 32 + 8 * g + 4 * w.h);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
    for (int t = 0; t < K::NT; ++t) {
      const bf16x8 b = *(const bf16x8 *)(smem + w.off[tap][t]);
#pragma unroll
      for (int m = 0; m < K::MT; ++m) acc[m][t] = K::mfma(a[tap][m], b, tap == 0 ? f32x16{} : acc[m][t]);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_s_barrier();  // every wave has read its input rows
#pragma unroll
  for (int m = 0; m < K::MT; ++m) {
    const int ct = w.cg * K::MT + m;
#pragma unroll
    for (int t = 0; t < K::NT; ++t) {
      uint32_t o[8];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        o[2 * g] = K::relu_pk(f32x2{acc[m][t][4 * g + 0] + bv[m][g].x, acc[m][t][4 * g + 1] + bv[m][g].y});
        o[2 * g + 1] = K::relu_pk(f32x2{acc[m][t][4 * g + 2] + bv[m][g].z, acc[m][t][4 * g + 3] + bv[m][g].w});
      }
      char *p = smem + w.rowi[t] * K::RS + phys_off(ct, w.h, 0);
      *(uint4 *)p = make_uint4(o[0], o[1], o[2], o[3]);
      *(uint4 *)(p + 16) = make_uint4(o[4], o[5], o[6], o[7]);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_s_barrier();
}

template <class K, int MG_>
__device__ __forceinline__ void ring_convs(char *smem, const Wave<K> &w, int n_convs, const char *wconv, int ct) {
  bf16x8 acur[K::MT];
  {  // layer 0 step 0's A fragments (slot 0 was certified before the stem's barriers)
    const char *slot = smem + Geo<K>::RING + w.lane * 16;
#pragma unroll
    for (int m = 0; m < K::MT; ++m) acur[m] = *(const bf16x8 *)(slot + (w.cg * K::MT + m) * FRAG);
  }
  uint4 res[K::MT][K::NT][2];
  for (int L = 0; L + 1 < n_convs; L += 2) {
    ring_conv<K, MG_, false>(smem, w, acur, res, L, n_convs, wconv, ct, true);
    ring_conv<K, MG_, true>(smem, w, acur, res, L + 1, n_convs, wconv, ct, false);
  }
  if (n_convs & 1) ring_conv<K, MG_, false>(smem, w, acur, res, n_convs - 1, n_convs, wconv, ct, false);
}

// One workgroup's tile: boards [board0, board0 + BOARDS) of the batch, all layers.
template <class K>
__device__ __forceinline__ void ring_tile(char *smem, const __bf16 *planes, int batch, int board0, int n_blocks,
                                          const bf16x8 *wpk, const float *bias, uint16_t *out) {
  using G = Geo<K>;
  static_assert(K::EDGE && K::C == 128 && K::ROWS == 256 && K::MT == 2 && K::NT == 4 && K::CG == 2,
                "ring trunk: 6-board edge tiles of the C = 128 net, 2 x 2 waves");
  static_assert(G::balanced(), "ring trunk: phases must be balanced between the row halves");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n_convs = 2 * n_blocks;
  constexpr size_t STEM = (size_t)K::C / 32 * 9 * 64;
  constexpr size_t LAYER = (size_t)K::C / 32 * 9 * (K::C / 16) * 64;
  const char *wconv = (const char *)(wpk + STEM);
  const int ct = __builtin_amdgcn_readfirstlane(wave);  // the fragment this wave DMAs (wave-uniform)
  // 1. prime the ring: layer 0's steps 0 .. D-1 (one fragment per wave each)
  if (n_convs > 0) {
    char *ring = smem + G::RING;
    issue_dma<0>(ring, wconv, 0, 0, ct, lane);
    issue_dma<1>(ring, wconv, 0, 1, ct, lane);
    issue_dma<2>(ring, wconv, 0, 2, ct, lane);
    issue_dma<3>(ring, wconv, 0, 3, ct, lane);
    issue_dma<4>(ring, wconv, 0, 4, ct, lane);
    issue_dma<5>(ring, wconv, 0, 5, ct, lane);
    static_assert(D == 6, "priming: D steps");
  }
  // 2. zero rows, neighbour table, the conv biases, the stem input (3 planes + 13 zero channels)
  for (int i = tid; i < K::NZ * K::RS / 4; i += K::THREADS) ((uint32_t *)(smem + K::ZROW * K::RS))[i] = 0u;
  uint16_t *tab = (uint16_t *)(smem + G::TAB);
#pragma unroll
  for (int j = 0; j < 9 * K::ROWS / K::THREADS; ++j) tab[tid + j * K::THREADS] = kEdgeNbr[tid + j * K::THREADS];
  {
    float *bl = (float *)(smem + G::BIAS);
    const float *bg = bias + K::C;  // conv layers' biases (after the stem's)
    for (int i = tid; i < n_convs * K::C / 4; i += K::THREADS) ((float4 *)bl)[i] = ((const float4 *)bg)[i];
  }
  for (int row = tid; row < K::ROWS; row += K::THREADS) {
    const int board = board0 + K::row_board(row);
    uint16_t *dst = (uint16_t *)(smem + row * K::RS);
    const bool ok = K::row_ok(row) && board < batch;
    const size_t src = ((size_t)board * K::CELLS + K::row_cell(row)) * 3;
#pragma unroll
    for (int c = 0; c < 16; ++c) dst[c] = (ok && c < 3) ? K::from_bf16(planes[src + c]) : (uint16_t)0;
  }
  __syncthreads();  // (also waits for the priming DMAs: vmcnt(0))
  Wave<K> w;
  w.lane = lane;
  w.h = lane >> 5;
  w.r = lane & 31;
  w.cg = wave & 1;
  w.mg = wave >> 1;
#pragma unroll
  for (int t = 0; t < K::NT; ++t) {
    w.rowi[t] = tile_of(w.mg, t) * 32 + w.r;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) w.off[tap][t] = (int)tab[tap * K::ROWS + w.rowi[t]] * K::RS + 16 * w.h;
  }
  ring_stem<K>(smem, w, wpk, bias);
  if (n_convs > 0) {
    if (w.mg == 0)
      ring_convs<K, 0>(smem, w, n_convs, wconv, ct);
    else
      ring_convs<K, 1>(smem, w, n_convs, wconv, ct);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail DMAs (re-reads of the last layer)
  head_layer<K>(smem, wpk + STEM + (size_t)n_convs * LAYER, bias + K::C + (size_t)n_convs * K::C, out, board0, batch,
                wave, lane);
}

// Device-count launch: every board in full 6-board ring tiles (one tile code for every board keeps
// each board's result independent of its batch); surplus workgroups exit at once.
template <class K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_tower_ring(
    const __bf16 *planes, const int32_t *count, int max_batch, int n_blocks, const bf16x8 *wpk, const float *bias,
    uint16_t *out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = count ? min(*count, max_batch) : max_batch;
  const int b0 = blockIdx.x * K::BOARDS;
  if (b0 >= n) return;
  ring_tile<K>(smem, planes, n, b0, n_blocks, wpk, bias, out);
}

}  // namespace ring
