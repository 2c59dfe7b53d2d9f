// tower_wide.h — the C = 256 trunk on 6-board edge tiles with ONE activation buffer (round 3).
//
// Included by tower.hip (namespace tower): uses Cfg (ONEBUF), Nbr, XLive, conv_tap_x (tower_abl.h), phys_off
// and head_layer from there.  The product's C = 256 trunk is the 16x16x32 form of this plan (tower_wide16.h),
// which uses the residual scratch (Scr, ScrBuf) and load_bias below; the 32x32x16 k-loop, epilogue and tile
// of this file are built into the A/B library only (SPMCTS_AB).
//
// Two ping-pong buffers of a 6-board tile at C = 256 would need 2 x 143.6 KB of LDS, so the two-buffer
// kernel runs C = 256 on 3-board, board-major tiles (128 rows): no edge-tile skipping (every tap of
// every tile is issued) and each weight fragment serves 128 rows.  Here the 6-board edge layout of the
// C = 128 kernel (tower_edge.h) runs at C = 256 with one buffer:
//   * a conv reads the buffer for all its k-steps (conv_tap_x: 12 of the 72 (tile, tap) pairs of the
//     edge tiles read zero padding only and are skipped), the waves meet at a barrier, then each wave
//     writes its own output channels of all 256 rows in place, and a second barrier publishes them;
//   * the residual of a block's second conv (the block input, overwritten by the first conv's
//     outputs) goes through global memory: the stem and every second conv also store their outputs
//     (the next block input, the same bf16 / fp16 bits as in LDS) to a per-workgroup scratch region,
//     and the next second conv's epilogue reads them back, each lane its own 32-byte runs (the same
//     lane, tile and channel tile wrote them two layers earlier; coalesced 16-byte accesses);
//   * 4 waves = 4 channel quarters (64 output channels each) x all 8 cell tiles: 16 accumulator tiles
//     per wave (the full AGPR file), 2 weight fragments and 8 LDS operand reads per 16 MFMAs, so each
//     weight fragment serves 256 rows (half the weight requests per MFMA of the 3-board kernel).
// Every board's outputs are bit-identical to the 3-board kernel's (the skipped terms are exact zeros
// and the accumulation order per output is the same), so mixing the two tile kinds in one batch (the
// tails of k_tower_dyn) keeps results batch-independent.

namespace wide {


// residual scratch per workgroup: [wave][channel tile m][cell tile t][64 lanes] x 32 bytes
template <class K>
struct Scr {
  static constexpr size_t PER_WAVE = (size_t)K::MT * K::NT * 64 * 32;
  static constexpr size_t PER_WG = PER_WAVE * K::WAVES;
  __device__ static uint4 *at(uint4 *base, int wave, int m, int t, int lane) {
    return base + (((size_t)wave * K::MT + m) * K::NT + t) * 64 * 2 + lane * 2;
  }
};
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Residual-scratch access through a buffer resource over this workgroup's region: the per-lane part of a
// load's address is one 32-bit voffset (lane * 32 + half * 16) and the (wave, channel tile, cell tile) part a
// wave-uniform soffset, instead of 16 hoisted 64-bit addresses (the pointer form spilled 110 VGPRs on them).
// Stores take the whole offset in the voffset and soffset = 0: hipcc (ROCm 7.2) inserts no wait state between
// a buffer_store_dwordx4 whose soffset is an SGPR and a following VALU write of its data VGPRs (LLVM's
// store-data hazard check exempts a register soffset), and on gfx950 that form stored wrong data -- every
// C = 256 output differed (profiles/r04/c256_rsrc/probe_summary.txt: rsrc loads + pointer stores bit-equal,
// pointer loads + SGPR-soffset rsrc stores not).  With soffset = 0 the hazard check applies.
// A/B library: Cfg ABL bit 2097152 = the round-3 pointer form (nontemporal 64-bit accesses).
template <class K>
struct ScrBuf {
  static constexpr int AUX = 2;  // gfx950 CPol: nt, as the pointer form's nontemporal accesses
  __amdgpu_buffer_rsrc_t rsrc;
  __device__ __forceinline__ explicit ScrBuf(uint4 *base) {
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)Scr<K>::PER_WG, 0x00020000);
  }
  __device__ static __forceinline__ int soff(int wave, int m, int t) {
    return (int)(((size_t)wave * K::MT + m) * K::NT + t) * 64 * 32;
  }
  __device__ __forceinline__ uint4 load(int lane, int half, int so) const {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane * 32 + half * 16, so, AUX));
  }
  __device__ __forceinline__ void store(uint4 v, int lane, int half, int so) const {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rsrc, lane * 32 + half * 16 + so, 0, AUX);
  }
};
#ifdef SPMCTS_AB  // the 32x32x16 one-buffer trunk (A/B library only: SPMCTS_TOWER_C256=32, codes 23xx / 25xx)
template <class K>
constexpr bool kScrRsrc = (K::ABL & 2097152) == 0;

// In-place epilogue of a conv (or the stem): every wave has finished reading the buffer (barrier
// before), out = relu(acc + bias (+ residual from scratch)) into the lane's own rows; SAVE also stores
// the outputs to scratch (the next block's residual).  A barrier publishes the outputs.
template <class K, bool RESID, bool SAVE>
__device__ __forceinline__ void epilogue(char *X, const f32x16 (&acc)[K::MT][K::NT], const float4 (&bv)[K::MT][4],
                                         uint4 *scr, int wave, int lane) {
  const int r = lane & 31, h = lane >> 5;
  // residual reads in half batches of HT cell tiles (32 registers in flight instead of 64: the
  // epilogue sits beside 256 accumulator AGPRs, and the full batch spilled)
  constexpr int HT = K::NT / 2;
#pragma unroll
  for (int mh = 0; mh < 2 * K::MT; ++mh) {
    const int m = mh >> 1, t0 = (mh & 1) * HT;
    const int ct = wave * K::MT + m;  // CG = WAVES: wave w owns channel tiles [w*MT, (w+1)*MT)
    uint4 res[RESID ? HT : 1][2];
    if constexpr (RESID) {
#pragma unroll
      for (int i = 0; i < HT; ++i) {
        if constexpr (kScrRsrc<K>) {
          const ScrBuf<K> sb(scr);
          const int so = ScrBuf<K>::soff(__builtin_amdgcn_readfirstlane(wave), m, t0 + i);
          res[i][0] = sb.load(lane, 0, so);
          res[i][1] = sb.load(lane, 1, so);
        } else {
          // nontemporal (nt): served from L2, never from a vector-L1 line an earlier read left behind
          const u32x4 *p = (const u32x4 *)Scr<K>::at(scr, wave, m, t0 + i, lane);
          res[i][0] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(p));
          res[i][1] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(p + 1));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < HT; ++i) {
      const int t = t0 + i;
      char *p = X + (t * 32 + r) * K::RS + phys_off(ct, h, 0);
      uint32_t o[8];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v0 = acc[m][t][4 * g + 0] + bv[m][g].x, v1 = acc[m][t][4 * g + 1] + bv[m][g].y;
        float v2 = acc[m][t][4 * g + 2] + bv[m][g].z, v3 = acc[m][t][4 * g + 3] + bv[m][g].w;
        if constexpr (RESID) {
          const f32x2 x0 = K::unpk(((const uint32_t *)&res[i][g >> 1])[2 * (g & 1)]);
          const f32x2 x1 = K::unpk(((const uint32_t *)&res[i][g >> 1])[2 * (g & 1) + 1]);
          v0 += x0[0];
          v1 += x0[1];
          v2 += x1[0];
          v3 += x1[1];
        }
        o[2 * g] = K::relu_pk(f32x2{v0, v1});
        o[2 * g + 1] = K::relu_pk(f32x2{v2, v3});
      }
      const uint4 lo = make_uint4(o[0], o[1], o[2], o[3]), hi = make_uint4(o[4], o[5], o[6], o[7]);
      *(uint4 *)p = lo;
      *(uint4 *)(p + 16) = hi;
      if constexpr (SAVE && kScrRsrc<K>) {
        const ScrBuf<K> sb(scr);
        const int so = ScrBuf<K>::soff(__builtin_amdgcn_readfirstlane(wave), m, t);
        sb.store(lo, lane, 0, so);
        sb.store(hi, lane, 1, so);
      } else if constexpr (SAVE) {
        u32x4 *q = (u32x4 *)Scr<K>::at(scr, wave, m, t, lane);
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, lo), q);
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, hi), q + 1);
      }
    }
  }
  __syncthreads();
}
#endif  // SPMCTS_AB

template <class K>
__device__ __forceinline__ void load_bias(float4 (&bv)[K::MT][4], const float *bias, int wave, int lane) {
#pragma unroll
  for (int m = 0; m < K::MT; ++m)
#pragma unroll
    for (int g = 0; g < 4; ++g) bv[m][g] = *(const float4 *)(bias + (wave * K::MT + m) * 32 + 8 * g + 4 * (lane >> 5));
}

#ifdef SPMCTS_AB
// One 3x3 conv over the resident tile, in place (the k-loop is conv_layer_x's edge-tile path).
template <class K, int KK, int DEPTH, bool RESID, bool SAVE>
__device__ __forceinline__ void conv(char *X, const Nbr<K> &nb, bf16x8 (&a)[DEPTH][K::MT], const float *bias, int wave,
                                     int lane, const WBuf &wb, uint32_t wl_off, uint32_t wn_off, int wn_steps,
                                     uint4 *scr, float *sbias) {
  using Xl = XLive<K, 0>;
  static_assert(K::C == K::THREADS, "one bias value per thread");
  const int hoff = 16 * (lane >> 5);
  // the epilogue's bias: one value per thread fetched now (its latency hides under the k-loop), staged
  // in LDS at the end of the k-loop (1 register through the k-loop instead of the 32 of float4 bv[2][4];
  // the previous layer's epilogue finished reading the staging area at its closing barrier)
  const float bmine = bias[threadIdx.x];
  constexpr uint32_t ZP = Xl::ZPRE_T, LV0 = Xl::lt(0);
  f32x16 acc[K::MT][K::NT];
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
#pragma unroll
    for (int m = 0; m < K::MT; ++m)
      if ((ZP >> t) & 1u) acc[m][t] = f32x16{};
  int off_cur[K::NT], off_nxt[K::NT];
  bf16x8 bc[K::NT], bn[K::NT];
  // tap 0's operand rows from the LDS table at each layer start (one round trip per layer) rather than
  // 8 offsets held in registers through every layer: at 512 registers they were spilled and reloaded
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
    if ((LV0 >> t) & 1u) off_cur[t] = nb.off(t, 0) + hoff;
#pragma unroll
  for (int t = 0; t < K::NT; ++t)
    if ((LV0 >> t) & 1u) bc[t] = lds_b128(X + off_cur[t]);
#define TAPW(T) conv_tap_x<K, KK, DEPTH, 0, T>(X, nb, acc, bc, bn, off_cur, off_nxt, a, hoff, wb, wl_off, wn_off, wn_steps)
  TAPW(0); TAPW(1); TAPW(2); TAPW(3); TAPW(4); TAPW(5); TAPW(6); TAPW(7); TAPW(8);
#undef TAPW
  sbias[threadIdx.x] = bmine;
  __syncthreads();  // every wave has read the layer input: outputs may overwrite it
  float4 bv[K::MT][4];
  load_bias<K>(bv, sbias, wave, lane);
  epilogue<K, RESID, SAVE>(X, acc, bv, scr, wave, lane);
}

// Stem (3 input planes in the first 32 bytes of each row, one 16-channel k-step per tap), in place;
// its outputs are the first block's input, saved to scratch as well.
template <class K>
__device__ __forceinline__ void stem(char *X, const Nbr<K> &nb, const bf16x8 *w, const float *bias, int wave, int lane,
                                     uint4 *scr) {
  const int h = lane >> 5;
  // the accumulators start at the bias (as the two-buffer kernel's stem_layer: the same rounding order)
  f32x16 acc[K::MT][K::NT];
  float4 bv[K::MT][4];
  load_bias<K>(bv, bias, wave, lane);
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
  __syncthreads();
  const float4 zero[K::MT][4] = {};  // bias already in the accumulators (x + 0.0f == x, up to the sign of zero)
  epilogue<K, false, true>(X, acc, zero, scr, wave, lane);
}

// One workgroup's tile: boards [board0, board0 + BOARDS) of the batch, all layers; scr = this
// workgroup's residual scratch (Scr<K>::PER_WG bytes).
template <class K>
__device__ __forceinline__ void tile(char *smem, const __bf16 *planes, int batch, int board0, int n_blocks,
                                     const bf16x8 *wpk, const float *bias, uint16_t *out, uint4 *scr) {
  static_assert(K::EDGE && K::ONEBUF && K::MG == 1 && K::CG == K::WAVES && K::WAVES == 4,
                "wide trunk: 6-board edge tiles, one buffer, 4 channel quarters x all cell tiles");
  char *X = smem;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  Nbr<K> nb;
  nb.init(lane & 31, 0);
  for (int i = tid; i < K::NZ * K::RS / 4; i += K::THREADS) ((uint32_t *)(X + K::ZROW * K::RS))[i] = 0u;
  uint16_t *tab = (uint16_t *)(smem + K::BUF);
  float *sbias = (float *)(smem + K::BUF + K::TAB);  // the current conv's bias (K::C floats)
#pragma unroll
  for (int j = 0; j < (9 * K::ROWS + K::THREADS - 1) / K::THREADS; ++j)
    if (9 * K::ROWS % K::THREADS == 0 || tid + j * K::THREADS < 9 * K::ROWS)
      tab[tid + j * K::THREADS] = kEdgeNbr[tid + j * K::THREADS];
  nb.tab = tab;
  // stem input: each row's first 16 channels (3 planes, 13 zeros)
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
  constexpr int KK = K::C / 16;
  constexpr int DEPTH = K::DEPTH;
  constexpr size_t STEM = (size_t)K::C / 32 * 9 * 64;
  constexpr size_t LAYER = (size_t)K::C / 32 * 9 * KK * 64;
  constexpr int LSTEPS = 9 * KK;
  stem<K>(X, nb, wpk, bias, wave, lane, scr);
  const bf16x8 *wblk = wpk + STEM;
  const float *b = bias + K::C;
  bf16x8 ring[DEPTH][K::MT];
  const int n_convs = 2 * n_blocks;
  if (n_convs > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int m = 0; m < K::MT; ++m) ring[d][m] = wblk[(size_t)(wave * K::MT + m) * LSTEPS * 64 + (size_t)d * 64 + lane];
  }
  WBuf wb;
  wb.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)wpk, (short)0, 0x7fffffff, 0x00020000);
  wb.voff = lane * 16;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t ct0_off = (uint32_t)(STEM + (size_t)(wave_u * K::MT) * LSTEPS * 64) * 16u;
  // one loop iteration per residual block: its first conv, then its second (residual + save) -- a straight
  // line, where an odd/even branch per conv made the register allocator merge the two bodies' live ranges
  // at the branch (66 spilled VGPRs in round 4, reloaded there)
  for (int L = 0; L < n_convs; L += 2) {
    const uint32_t wl_off = ct0_off + (uint32_t)((size_t)L * LAYER * 16u);
    conv<K, KK, DEPTH, false, false>(X, nb, ring, b, wave, lane, wb, wl_off, wl_off + (uint32_t)(LAYER * 16u), LSTEPS,
                                     scr, sbias);
    b += K::C;
    const uint32_t wl1 = wl_off + (uint32_t)(LAYER * 16u);
    const uint32_t wn1 = (kRingAlways && L + 2 == n_convs) ? wl1 : wl1 + (uint32_t)(LAYER * 16u);
    conv<K, KK, DEPTH, true, true>(X, nb, ring, b, wave, lane, wb, wl1, wn1, L + 2 < n_convs ? LSTEPS : 0, scr, sbias);
    b += K::C;
  }
  head_layer<K>(X, wblk + (size_t)n_convs * LAYER, b, out, board0, batch, wave, lane);
}

#endif  // SPMCTS_AB

}  // namespace wide
