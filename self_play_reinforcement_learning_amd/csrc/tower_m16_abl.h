// tower_m16_abl.h -- A/B library only (make ab: libspmcts_ab.so, -DSPMCTS_AB): the 16x16x32 C = 128 trunk's
// k-loop with its timing ablations (SPMCTS_TOWER_CG 1600 / 1608 / 1616).  Included by tower_m16.h
// (namespace tower::m16) after the product's conv_tap, which it mirrors step for step.

// tower_m16.h's conv_tap with the Cfg::ABL timing ablations of the 16x16x32 trunk (results wrong by design):
// 8 = no LDS operand reads (code 1608), 16 = no weight loads in the k-loop (1616), 256 = the compiler's own
// schedule instead of one operand read or weight load per MFMA gap (1600; correct results).
template <class K, int KK32, int DEPTH, int MG_, int TAP>
__device__ __forceinline__ void conv_tap_abl(const char *src, const Nbr<K> &nb, f32x4 (&acc)[MM<K>][K::NT][2],
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
    if (K::ABL & 8) {  // timing ablation (A/B library only, wrong results): no LDS operand reads
    } else if (k + 1 < KK32) {
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
    if (K::ABL & 16) {  // timing ablation (A/B library only, wrong results): no weight loads in the k-loop
    } else if (sn < STEPS) {
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
    // (A/B: Cfg ABL 256 leaves the order to the compiler)
    if constexpr (!(K::ABL & 256)) {
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
    }
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

