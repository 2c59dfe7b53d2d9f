// spmcts.hip — MI355X (gfx950) batched self-play MCTS arena: kernels + C ABI.
//
// Replaces the per-game Python object tree of games/algos/mcts.py (MCNode /
// MCTreeSearch) and the episode loop of games/algos/selfplayworker.py
// (SelfPlayer) with one device-resident arena:
//
//   node store   one 32*APAD-byte record per "child block" (one per expansion):
//                n, vl, child (local block of the child's own children, -1 =
//                unexpanded), p, w, f64 flag per slot + the valid-children mask
//                (NodeRec).  A node = (block, slot); trees own disjoint block ranges.
//   trees        root node, root board (2 x u64 bitboards), root player, bump
//                allocator, Dirichlet noise, per-sim path scratch, RNG.
//   games        SelfPlayer state machine: board (policy frame), ply, swap_sides,
//                two trees, Move record buffers, export ring.
//
// Every simulation of every active tree runs in lock step:
//   k_select   one APAD-lane group per tree walks root -> leaf, scoring the A
//              children of each node lane-parallel in fp64 (bit-exact with the
//              reference's Python float arithmetic: fp-contract off), argmax via
//              in-group shuffles, jitter from Philox or the parity tape;
//              terminal leaves are backed up in place (no network call).
//   k_scan     orders pending leaves by tree id (deterministic rows).
//   k_encode   writes network input rows (planes or boards) for those leaves.
//   [network on the same stream — PyTorch ResNet or the table net]
//   k_expand   creates the leaf's child block from the priors, backs the value up.
//
// Compile: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see Makefile).
#include <hip/hip_runtime.h>
#include <rocrand/rocrand_normal.h>
#include <rocrand/rocrand_philox4x32_10.h>
#include <rocrand/rocrand_uniform.h>

#include "philox.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "board.h"
#include "spmcts.h"

#pragma clang fp contract(off)

using namespace spm;

// ----------------------------------------------------------------------------
// error reporting
// ----------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return fail(-(int)_e - 1000, std::string(#expr) + ": " + hipGetErrorString(_e));        \
  } while (0)

#define LAUNCH_CHECK()                                                                         \
  do {                                                                                         \
    hipError_t _e = hipGetLastError();                                                         \
    if (_e != hipSuccess) return fail(-(int)_e - 1000, std::string("launch: ") + hipGetErrorString(_e)); \
  } while (0)

// ----------------------------------------------------------------------------
// device view of an arena (passed by value to kernels)
// ----------------------------------------------------------------------------
typedef rocrand_state_philox4x32_10 Philox;

struct View {
  int T, cap, G, A;
  int iters;  // MCTreeSearch.iterations (bounds the last step of a K-in-flight search)
  int K, NS;  // simulations in flight per tree (virtual loss; 1 = sequential), pending slots = T * K
  double cpuct, x, alpha;
  int strong, evaluate, rng_mode, leaf_format, leaf_layout;
  // node store: one record of 32 * P bytes per child block (nd_* below)
  char *nodes;
  // trees
  int32_t *root;
  uint64_t *rpos, *rneg;
  int8_t *rplayer;
  int32_t *used;
  int32_t gc;         // 1: blocks_per_tree below the worst case -> compaction before a search (k_compact)
  int32_t *gc_list;   // [T][cap] scratch: live blocks (BFS order)
  int32_t *gc_map;    // [T][cap] scratch: old block -> new block (-1 dead)
  int32_t *tstarted;  // threaded search: search_node calls started in the current search (inactive: >= limit)
  double *noise;
  uint8_t *noise_on;
  int32_t *pnode;   // [T][MAXD] path node ids (root .. parent of leaf)
  int32_t *pn;      // [T][MAXD] their visit counts as read during select
  double *pw;       // [T][MAXD] their w as read during select
  int32_t *plen;
  int32_t *leaf;    // leaf node (local id)
  int32_t *leaf_n;
  double *leaf_w;
  uint64_t *lpos, *lneg;
  int8_t *lmover;
  uint8_t *need;
  Philox *rng;
  const double *tape;
  const int64_t *tape_end;  // [T] end offset
  int64_t *tape_cur;        // [T]
  int64_t *cnt;             // per-tree counters [T][8]
  int32_t *active;
  int32_t *row_tree;  // row -> pending slot (tree * K + j)
  int32_t *srow;      // pending slot -> row (K > 1)
  int32_t *row_count;
  // batch leaf dedup (K > 1, spmcts_set_leaf_dedup): pending leaves with the same network input share
  // one row.  dtab: open-addressing table of (generation << 32 | owner slot), dent: a slot's entry
  uint64_t *dtab;
  int32_t *dent;
  uint8_t *down;  // 1 = the slot owns its key's row, 2 = the leader lane's row serves it (set per step)
  int dedup, dmask;
  uint32_t dgen;
  // cross-lane dedup (round 6, spmcts_set_leaf_peer): a leader arena keeps each owner slot's key in okey
  // (2 x u64 per slot) for the step; a follower's owner slot whose key the leader evaluates this step
  // takes the leader's row (down 2, xpeer = the leader's owner slot), copied in by k_peer_push
  uint64_t *okey;
  int32_t *xpeer;
  int lead;     // 1: this arena has followers (k_dedup_owner writes okey)
  int peer_on;  // 1 in a follower's simulation-step launches (k_scan_need numbers down-2 slots after its own rows)
  // evaluation cache (round 6, spmcts_set_eval_cache): network outputs of the arena's own rows kept for `cwin`
  // generations (one per ply / search), keyed like the dedup table; an owner slot whose key is there takes
  // the cached outputs (down 3, xc = the entry) in a row after the network rows, filled by k_cache_io.
  // crec: one 64-byte record per entry (one line per probe): tag u64 ((generation << 32) | state, 0 = never used),
  // own u64, opp u64, then A probs + value as f32
  uint64_t *crec;
  int32_t *xc;
  int cwin, cmask;  // cwin 0 = off (also in launches where the cache is not live)
  uint32_t cgen;
  int cshared;  // 1: a follower lane using its leader's table (the leader inserts the rows it serves)
  int served;  // 1: k_scan_need numbers down-2 / down-3 slots after the network rows (peer_on or the cache)
  float *root_prior;
  uint32_t *err;
  // games
  uint64_t *gpos, *gneg;
  int32_t *gply;
  uint8_t *gswap, *gstate;
  int8_t *gresult;
  int64_t *gid;
  int8_t *mv_state;
  float *mv_probs;
  double *mv_q;
  uint8_t *mv_qf64;
  int32_t *mv_count;
  int8_t *ex_state;
  float *ex_probs;
  double *ex_q;
  uint8_t *ex_qf64;
  float *ex_z;
  int64_t *ex_game;
  int32_t *ex_count;
  int32_t ex_cap;
  int64_t *gcnt;  // games counters: [0] finished [1..6] results [7] next id [8] limit [9] exported
  int32_t *gscratch;
  // per-tree players (two-network arenas, compare_models / evaluation games)
  uint8_t *tnet;     // [T] network whose leaves this tree sends (0 / 1)
  uint8_t *tkind;    // [T] SPMCTS_PLAYER_*: MCTS, or a hard-coded player (hardcoded_players.py)
  int32_t *budget;   // [T] simulations per search of this tree (MCTreeSearch.iterations)
  // per-tree search settings (each side of an evaluation game is built from its own container's
  // kwargs, selfplayworker.py:71-81): Dirichlet alpha, strong_play, sims in flight (<= K)
  double *talpha;
  uint8_t *tstrong;
  int32_t *tK;
  int32_t seg1;      // first leaf row of network 1 (= number of network-0 trees)
  int32_t record;    // games mode: keep Move records (play_episode update=True)
  int32_t sim;       // index of the current simulation within the search (by value per launch)
};

// Node store.  A child block (the A children of one expanded node, P = APAD slots) is ONE contiguous
// record of 32 * P bytes: n i32[P] | vl i32[P] | child-block i32[P] | p f32[P] | w f64[P] | f64 flag
// u8[P] | valid-children mask u32 | pad.  The fields a select level scores (n, vl, child, p: the first
// 16 P bytes; w, the mask: the next) lie in two 128-byte lines for Connect4 (P = 8) instead of one line
// per field array.  Node id i = (tree * cap + block) * P + slot, as before; the flag is "w is a numpy
// float64" (strong_play dtype quirk, mcts.py:287/:308), vl is MCNode.virtual_loss (mcts.py:44).
template <int P>
struct NodeRec {
  static constexpr int N = 0, VL = 4 * P, C = 8 * P, PR = 12 * P, W = 16 * P, F = 24 * P, VM = 25 * P, BYTES = 32 * P;
  static_assert(VM + 4 <= BYTES && W % 8 == 0 && VM % 4 == 0, "record layout");
};
template <int P>
__host__ __device__ __forceinline__ char *nd_rec(const View &v, size_t i) {
  return v.nodes + (i / P) * (size_t)NodeRec<P>::BYTES;
}
template <int P>
__host__ __device__ __forceinline__ int32_t &nd_n(const View &v, size_t i) {
  return ((int32_t *)(nd_rec<P>(v, i) + NodeRec<P>::N))[i % P];
}
template <int P>
__host__ __device__ __forceinline__ int32_t &nd_vl(const View &v, size_t i) {
  return ((int32_t *)(nd_rec<P>(v, i) + NodeRec<P>::VL))[i % P];
}
template <int P>
__host__ __device__ __forceinline__ int32_t &nd_c(const View &v, size_t i) {
  return ((int32_t *)(nd_rec<P>(v, i) + NodeRec<P>::C))[i % P];
}
template <int P>
__host__ __device__ __forceinline__ float &nd_p(const View &v, size_t i) {
  return ((float *)(nd_rec<P>(v, i) + NodeRec<P>::PR))[i % P];
}
template <int P>
__host__ __device__ __forceinline__ double &nd_w(const View &v, size_t i) {
  return ((double *)(nd_rec<P>(v, i) + NodeRec<P>::W))[i % P];
}
template <int P>
__host__ __device__ __forceinline__ uint8_t &nd_f(const View &v, size_t i) {
  return ((uint8_t *)(nd_rec<P>(v, i) + NodeRec<P>::F))[i % P];
}
// valid-children mask of block `gb` = tree * cap + block
template <int P>
__host__ __device__ __forceinline__ uint32_t &nd_vm(const View &v, size_t gb) {
  return *(uint32_t *)(v.nodes + gb * (size_t)NodeRec<P>::BYTES + NodeRec<P>::VM);
}

enum { C_SIMS = 0, C_NN = 1, C_TERM = 2, C_DEPTH = 3, C_SETNODE = 4, C_MOVES = 5, C_LEAK = 6, C_GC = 7, C_HWM = 8, C_NCNT = 10 };
enum { GS_IDLE = 0, GS_ACTIVE = 1, GS_DONE = 2 };

__device__ __forceinline__ void set_err(const View &v, uint32_t f) { atomicOr(v.err, f); }

template <class G>
__device__ __forceinline__ size_t nbase(const View &v, int tree) {
  return (size_t)tree * (size_t)v.cap * G::APAD;
}

// ----------------------------------------------------------------------------
// RNG: Philox (rocRAND) or parity tape
// ----------------------------------------------------------------------------
struct TreeRng {
  PhiloxFields f;  // Philox mode: counter, key, substate (f.result is not carried; rng_store rebuilds it)
  int64_t cur, end;
};

__device__ __forceinline__ void rng_load(const View &v, int tree, TreeRng &r) {
  if (v.rng_mode == SPMCTS_RNG_TAPE) {
    r.cur = v.tape_cur[tree];
    r.end = v.tape_end[tree];
  } else {
    // memcpy: the rocRAND object read as its leading fields, without a type-punned access
    __builtin_memcpy(&r.f, (const void *)(v.rng + tree), sizeof(PhiloxFields));
  }
}

__device__ __forceinline__ void rng_store(const View &v, int tree, const TreeRng &r) {
  if (v.rng_mode == SPMCTS_RNG_TAPE) {
    v.tape_cur[tree] = r.cur;
  } else {
    // the state's leading fields, with rocRAND's output block rebuilt (philox.h); its Box-Muller
    // cache (the trailing fields, used only by the Dirichlet draws) is left as it was
    PhiloxFields f = r.f;
    philox_sync(f);
    __builtin_memcpy((void *)(v.rng + tree), &f, sizeof(PhiloxFields));
  }
}

// One double in [0, 1) for lane `j` of a k-wide vector draw (all lanes call it with the
// same state; the shared state then advances by k via rng_advance).
__device__ __forceinline__ double rng_lane(const View &v, const TreeRng &r, int j, bool *tape_err) {
  if (v.rng_mode == SPMCTS_RNG_TAPE) {
    const int64_t i = r.cur + j;
    if (i >= r.end) {
      *tape_err = true;
      return 0.0;
    }
    return v.tape[i];
  }
  // = skipahead(2j) + rocrand_uniform_double, without the run-time index into the output block
  return 1.0 - philox_uniform_at(r.f, 2ull * (unsigned long long)j);  // rocRAND gives (0, 1]
}

__device__ __forceinline__ void rng_advance(const View &v, TreeRng &r, int k) {
  if (v.rng_mode == SPMCTS_RNG_TAPE)
    r.cur += k;
  else
    philox_skip(r.f, 2ull * (unsigned long long)k);  // skipahead(2k) minus its output-block refresh
}

// Child jitter of a P-lane tree group, lane j < A using its draw (= rng_lane(j)); every lane of the
// group must call it.  Tape mode reads lane j's tape entry; Philox mode computes each output block
// once per group and shares it through shuffles (philox.h philox_uniform_group).
template <class G>
__device__ __forceinline__ double rng_group(const View &v, const TreeRng &r, int lane, int gbase, bool *tape_err) {
  if (v.rng_mode == SPMCTS_RNG_TAPE) return lane < G::A ? rng_lane(v, r, lane, tape_err) : 0.0;
  return 1.0 - philox_uniform_group<G::APAD>(r.f, lane, gbase);
}

// sequential scalar draw (single thread)
__device__ __forceinline__ double rng_next(const View &v, TreeRng &r, bool *tape_err) {
  double u = rng_lane(v, r, 0, tape_err);
  rng_advance(v, r, 1);
  return u;
}

// Gamma(alpha, 1): alpha == 1 -> Exp(1) = -log U; otherwise Marsaglia-Tsang.
__device__ double gamma_draw(Philox *s, double alpha) {
  if (alpha == 1.0) return -log(rocrand_uniform_double(s));
  double boost = 1.0;
  if (alpha < 1.0) {
    boost = pow(rocrand_uniform_double(s), 1.0 / alpha);
    alpha += 1.0;
  }
  const double d = alpha - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  for (int it = 0; it < 256; ++it) {
    const double xn = rocrand_normal_double(s);
    double t = 1.0 + c * xn;
    if (t <= 0.0) continue;
    t = t * t * t;
    const double u = rocrand_uniform_double(s);
    if (log(u) < 0.5 * xn * xn + d - d * t + d * log(t)) return d * t * boost;
  }
  return d * boost;
}

// ----------------------------------------------------------------------------
// small helpers
// ----------------------------------------------------------------------------
template <class G>
__device__ __forceinline__ void reset_tree(const View &v, int tree, int player, const float *prior) {
  constexpr int P = G::APAD;
  const size_t nb = nbase<G>(v, tree);
  const size_t bb = (size_t)tree * v.cap;
  // block 0 = pseudo block holding the root in slot 0; block 1 = root's children
  nd_n<P>(v, nb + 0) = 0;
  nd_w<P>(v, nb + 0) = 0.0;
  nd_p<P>(v, nb + 0) = 0.f;
  nd_c<P>(v, nb + 0) = 1;
  nd_f<P>(v, nb + 0) = 0;
  if (v.K > 1) {
    nd_vl<P>(v, nb + 0) = 0;
    for (int j = 0; j < P; ++j) nd_vl<P>(v, nb + P + j) = 0;
  }
  for (int j = 0; j < P; ++j) {
    nd_n<P>(v, nb + P + j) = 0;
    nd_w<P>(v, nb + P + j) = 0.0;
    nd_p<P>(v, nb + P + j) = j < G::A ? prior[j] : 0.f;
    nd_c<P>(v, nb + P + j) = -1;
    nd_f<P>(v, nb + P + j) = 0;
  }
  nd_vm<P>(v, bb + 0) = 1u;
  nd_vm<P>(v, bb + 1) = legal_mask<G>(Board{0, 0});
  v.used[tree] = 2;
  v.root[tree] = 0;
  v.rpos[tree] = 0;
  v.rneg[tree] = 0;
  v.rplayer[tree] = (int8_t)player;
  v.noise_on[tree] = 0;
  v.tstarted[tree] = 0x3fffffff;  // no search in progress
  for (int j = 0; j < v.K; ++j) v.need[(size_t)tree * v.K + j] = 0;
}

// terminal value of _expand_node (mcts.py:305-313) for `tree`'s own strong_play; r = reward * mover
__device__ __forceinline__ double terminal_value(bool strong, Board parent, int r) {
  if (strong) {
    const int num_steps = popc(parent.pos | parent.neg) + 1;  // np.sum(np.abs(state)) + 1
    return (1.18 - ((double)(9 * num_steps) / 350.0)) * (double)r;
  }
  return (double)r;
}
__device__ __forceinline__ double terminal_value(const View &v, int tree, Board parent, int r) {
  if (v.tstrong[tree]) {
    const int num_steps = popc(parent.pos | parent.neg) + 1;  // np.sum(np.abs(state)) + 1
    return (1.18 - ((double)(9 * num_steps) / 350.0)) * (double)r;
  }
  return (double)r;
}

// Dirichlet root noise (add_noise, mcts.py:49-53): A components, invalid children included.
template <class G>
__device__ void draw_noise(const View &v, int tree) {
  double g[G::A];
  if (v.rng_mode == SPMCTS_RNG_TAPE) {
    TreeRng r;
    rng_load(v, tree, r);
    bool terr = false;
    for (int j = 0; j < G::A; ++j) g[j] = rng_lane(v, r, j, &terr);
    rng_advance(v, r, G::A);
    if (terr) set_err(v, SPMCTS_ERR_TAPE);
    rng_store(v, tree, r);
  } else {
    // rocRAND's own Gamma path on the whole state (Box-Muller cache included); stores keep its
    // invariant result == philox10(counter), so the state is rocRAND-consistent here
    Philox st = v.rng[tree];
    double acc = 0.0;
    for (int j = 0; j < G::A; ++j) {
      g[j] = gamma_draw(&st, v.talpha[tree]);
      acc += g[j];
    }
    const double inv = acc > 0.0 ? 1.0 / acc : 0.0;
    for (int j = 0; j < G::A; ++j) g[j] *= inv;
    v.rng[tree] = st;
  }
  for (int j = 0; j < G::A; ++j) v.noise[(size_t)tree * G::APAD + j] = g[j];
  v.noise_on[tree] = 1;
  v.tstarted[tree] = 0;  // a search begins: `iterations` search_node calls to start
}

// ----------------------------------------------------------------------------
// kernels: resets / noise
// ----------------------------------------------------------------------------
template <class G>
__global__ void k_tree_reset(View v, const int32_t *trees, const int8_t *players, const float *priors, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = trees[i];
  if (t < 0 || t >= v.T) {
    set_err(v, SPMCTS_ERR_STATE);
    return;
  }
  reset_tree<G>(v, t, players[i], priors ? priors + (size_t)i * G::A : v.root_prior + 16 * v.tnet[t]);
}

template <class G>
__global__ void k_search_begin(View v, const int32_t *trees, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = trees[i];
  v.active[i] = t;
  if (t < 0) return;
  draw_noise<G>(v, t);
}

// ----------------------------------------------------------------------------
// kernel: subtree recycling (node-store compaction of one tree before a search)
// ----------------------------------------------------------------------------
// The reference keeps every node of a game alive (backup runs to the original root, mcts.py:94-98;
// its _prune, mcts.py:197-199, is never called), but nothing above the active root is ever read
// again.  When a tree's remaining blocks cannot hold one more search (iterations + K + 2 blocks:
// one per network expansion, the _set_node expansion, slack), the blocks still reachable from the
// active root are slid down to the front of the tree's region, in their old order, and every child
// index is remapped:
//   * block 0 slot 0 becomes the root (its record copied there: n, w, p, children, dtype flag, vl);
//   * the live blocks (BFS from the root's child block, level-synchronous over the workgroup) keep
//     their relative order, so new index <= old index and the move can run in place, chunk by chunk
//     (a chunk is read completely before any of it is written);
//   * the root's child block is the oldest live block (everything below it was allocated after it),
//     so it lands at block 1 and the relation "child block > parent block" is preserved.
// Results are unchanged bit for bit (tests run the parity fixtures with a tiny blocks_per_tree).
// Without an explicit blocks_per_tree the store is sized for the worst case and this never runs.
template <class G>
__global__ __launch_bounds__(256) void k_compact(View v, int n_active) {
  constexpr int P = G::APAD;
  constexpr int NT = 256;
  __shared__ int s_head, s_tail, s_carry, s_scan[NT];
  const int slot = blockIdx.x;
  if (slot >= n_active) return;
  const int tree = v.active[slot];
  if (tree < 0 || !v.gc) return;
  const int need = min(v.budget[tree], v.iters) + v.K + 2;
  const int used = v.used[tree];
  if (v.cap - used >= need) return;
  const int tid = threadIdx.x;
  const size_t nb = nbase<G>(v, tree);
  const size_t bb = (size_t)tree * v.cap;
  int32_t *list = v.gc_list + bb;
  int32_t *map = v.gc_map + bb;
  const int root = v.root[tree];
  const int croot = nd_c<P>(v, nb + root);
  // 1. live blocks: BFS from the root's child block
  if (tid == 0) {
    s_head = 0;
    s_tail = 0;
    if (croot >= 0) {
      list[0] = croot;
      s_tail = 1;
    }
  }
  for (int b = tid; b < used; b += NT) map[b] = -1;
  __syncthreads();
  for (;;) {
    const int head = s_head, tail = s_tail;
    if (head == tail) break;
    __syncthreads();
    for (int k = head * P + tid; k < tail * P; k += NT) {
      const int blk = list[k / P], j = k % P;
      const int c = j < G::A ? nd_c<P>(v, nb + (size_t)blk * P + j) : -1;
      if (c >= 0) list[atomicAdd(&s_tail, 1)] = c;
    }
    __threadfence_block();
    __syncthreads();
    if (tid == 0) s_head = tail;
    __syncthreads();
  }
  const int L = s_tail;
  for (int k = tid; k < L; k += NT) map[list[k]] = 0;
  __threadfence_block();
  __syncthreads();
  // 2. new indices: 1 + rank among the live blocks in old order (block-wide scan in chunks)
  if (tid == 0) s_carry = 1;
  __syncthreads();
  for (int c0 = 0; c0 < used; c0 += NT) {
    const int b = c0 + tid;
    const int live = (b < used && map[b] == 0) ? 1 : 0;
    s_scan[tid] = live;
    __syncthreads();
    for (int off = 1; off < NT; off <<= 1) {
      const int add = tid >= off ? s_scan[tid - off] : 0;
      __syncthreads();
      s_scan[tid] += add;
      __syncthreads();
    }
    if (live) map[b] = s_carry + s_scan[tid] - 1;
    __syncthreads();
    if (tid == NT - 1) s_carry += s_scan[NT - 1];
    __syncthreads();
  }
  __threadfence_block();
  __syncthreads();
  // 3. the root record into block 0 slot 0 (block 0 is never a destination: live blocks map to >= 1)
  if (tid == 0) {
    const int32_t rn = nd_n<P>(v, nb + root);
    const double rw = nd_w<P>(v, nb + root);
    const float rp = nd_p<P>(v, nb + root);
    const uint8_t rf = nd_f<P>(v, nb + root);
    const int32_t rvl = v.K > 1 ? nd_vl<P>(v, nb + root) : 0;
    nd_n<P>(v, nb) = rn;
    nd_w<P>(v, nb) = rw;
    nd_p<P>(v, nb) = rp;
    nd_f<P>(v, nb) = rf;
    nd_c<P>(v, nb) = croot >= 0 ? map[croot] : croot;
    if (v.K > 1) nd_vl<P>(v, nb) = rvl;
    nd_vm<P>(v, bb) = 1u;
    v.root[tree] = 0;
  }
  __threadfence_block();
  __syncthreads();
  // 4. slide the live blocks down, chunk by chunk; child indices remapped
  for (int c0 = 1; c0 < used; c0 += NT / P) {
    const int b = c0 + tid / P, j = tid % P;
    const int dst = b < used ? map[b] : -1;
    int32_t n = 0, c = -1, vl = 0;
    double w = 0.0;
    float pr = 0.f;
    uint8_t f = 0;
    uint32_t vm = 0;
    if (dst >= 0) {
      const size_t i = nb + (size_t)b * P + j;
      n = nd_n<P>(v, i);
      w = nd_w<P>(v, i);
      pr = nd_p<P>(v, i);
      c = nd_c<P>(v, i);
      f = nd_f<P>(v, i);
      if (v.K > 1) vl = nd_vl<P>(v, i);
      if (j == 0) vm = nd_vm<P>(v, bb + b);
      if (c >= 0) c = map[c];
    }
    __syncthreads();
    if (dst >= 0) {
      const size_t o = nb + (size_t)dst * P + j;
      nd_n<P>(v, o) = n;
      nd_w<P>(v, o) = w;
      nd_p<P>(v, o) = pr;
      nd_c<P>(v, o) = c;
      nd_f<P>(v, o) = f;
      if (v.K > 1) nd_vl<P>(v, o) = vl;
      if (j == 0) nd_vm<P>(v, bb + dst) = vm;
    }
    __threadfence_block();
    __syncthreads();
  }
  if (tid == 0) {
    v.used[tree] = 1 + L;
    v.cnt[(size_t)tree * C_NCNT + C_GC] += 1;
    if (v.cap - (1 + L) < need) set_err(v, SPMCTS_ERR_POOL);  // the live subtree alone fills the store
  }
}

// ----------------------------------------------------------------------------
// kernel: select (search_node, mcts.py:340-367)
// ----------------------------------------------------------------------------
// P-lane group reductions on DPP lane permutations (a few cycles each) instead of ds_bpermute (an LDS
// round trip each, ~100 cycles on the tree kernels' dependent chain): partners lane ^ 1 and lane ^ 2
// (quad_perm), then lane ^ 7 (row_half_mirror: the other quad of the 8-lane group) and lane ^ 15
// (row_mirror: the other half of a 16-lane group).  After the two quad steps every lane holds its quad's
// result, so the mirror steps combine whole quads / halves: every lane ends with the group's result.
// Only lanes of the same group are read (the permutations stay within 4, 8 or 16 lanes).
enum { DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140 };
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const int2 v = __builtin_bit_cast(int2, x);
  return __builtin_bit_cast(double, make_int2(dpp_i<CTRL>(v.x), dpp_i<CTRL>(v.y)));
}

// argmax with the lowest index on ties (associative and commutative, so the butterfly order does not
// change the result)
template <int P, int CTRL>
__device__ __forceinline__ void argmax_step(double &s, int &idx) {
  const double so = dpp_d<CTRL>(s);
  const int io = dpp_i<CTRL>(idx);
  if (so > s || (so == s && io < idx)) {
    s = so;
    idx = io;
  }
}
template <int P>
__device__ __forceinline__ void group_argmax(double &s, int &idx) {
  static_assert(P == 8 || P == 16, "tree groups of 8 or 16 lanes");
  argmax_step<P, DPP_XOR1>(s, idx);
  argmax_step<P, DPP_XOR2>(s, idx);
  argmax_step<P, DPP_HALF_MIRROR>(s, idx);
  if constexpr (P == 16) argmax_step<P, DPP_MIRROR>(s, idx);
}

// group_argmax that also hands every lane the winning lane's child fields (the payload moves with the
// index through the butterfly, so no ds_bpermute from lane `a` afterwards)
template <int CTRL>
__device__ __forceinline__ void argmax_carry_step(double &s, int &idx, int &c0, int &c1, int &c2, double &d0) {
  const double so = dpp_d<CTRL>(s), d0o = dpp_d<CTRL>(d0);
  const int io = dpp_i<CTRL>(idx), c0o = dpp_i<CTRL>(c0), c1o = dpp_i<CTRL>(c1), c2o = dpp_i<CTRL>(c2);
  if (so > s || (so == s && io < idx)) {
    s = so;
    idx = io;
    c0 = c0o;
    c1 = c1o;
    c2 = c2o;
    d0 = d0o;
  }
}
template <int P>
__device__ __forceinline__ void group_argmax_carry(double &s, int &idx, int &c0, int &c1, int &c2, double &d0) {
  static_assert(P == 8 || P == 16, "tree groups of 8 or 16 lanes");
  argmax_carry_step<DPP_XOR1>(s, idx, c0, c1, c2, d0);
  argmax_carry_step<DPP_XOR2>(s, idx, c0, c1, c2, d0);
  argmax_carry_step<DPP_HALF_MIRROR>(s, idx, c0, c1, c2, d0);
  if constexpr (P == 16) argmax_carry_step<DPP_MIRROR>(s, idx, c0, c1, c2, d0);
}

template <int P>
__device__ __forceinline__ int group_or(int x) {
  static_assert(P == 8 || P == 16, "tree groups of 8 or 16 lanes");
  x |= dpp_i<DPP_XOR1>(x);
  x |= dpp_i<DPP_XOR2>(x);
  x |= dpp_i<DPP_HALF_MIRROR>(x);
  if constexpr (P == 16) x |= dpp_i<DPP_MIRROR>(x);
  return x;
}

template <class G>
__global__ __launch_bounds__(64) void k_select(View v, int n_active) {
  constexpr int P = G::APAD;
  constexpr int GPB = 64 / P;  // groups (trees) per block
  __shared__ int32_t s_node[GPB][G::MAXD];
  __shared__ int32_t s_n[GPB][G::MAXD];
  __shared__ double s_w[GPB][G::MAXD];

  const int lane = threadIdx.x & (P - 1);
  const int grp = threadIdx.x / P;
  const int slot = blockIdx.x * GPB + grp;
  if (slot >= n_active) return;
  const int tree = v.active[slot];
  if (tree < 0) return;
  if (v.sim >= v.budget[tree]) return;  // this tree's search is complete (per-player iterations)

  const size_t nb = nbase<G>(v, tree);
  const size_t bb = (size_t)tree * v.cap;
  int node = v.root[tree];
  Board b{v.rpos[tree], v.rneg[tree]};
  int player = v.rplayer[tree];
  const bool noise = v.noise_on[tree] != 0;
  const double nz = (noise && lane < G::A) ? v.noise[(size_t)tree * P + lane] : 0.0;
  TreeRng rng;
  rng_load(v, tree, rng);
  bool terr = false;

  int node_n = nd_n<P>(v, nb + node);
  double node_w = nd_w<P>(v, nb + node);
  // the node's child block: read for the root; below it, the child entry read with the parent's
  // block already holds it (one dependent global load per level instead of two)
  int cb = nd_c<P>(v, nb + node);
  int depth = 0;
  for (;;) {
    if (lane == 0) {
      s_node[grp][depth] = node;
      s_n[grp][depth] = node_n;
      s_w[grp][depth] = node_w;
    }
    if (cb < 0) {  // an expanded node is required here
      if (lane == 0) set_err(v, SPMCTS_ERR_STATE);
      return;
    }
    const uint32_t vm = nd_vm<P>(v, bb + cb);
    const size_t ci = nb + (size_t)cb * P + lane;
    int cn = 0, cc = -1;
    double cw = 0.0;
    float cp = 0.f;
    if (lane < G::A) {
      cn = nd_n<P>(v, ci);
      cw = nd_w<P>(v, ci);
      cp = nd_p<P>(v, ci);
      cc = nd_c<P>(v, ci);
    }
    const int gbase = (threadIdx.x & 63) & ~(P - 1);
    // the jitter does not depend on the child block: drawn here, it overlaps the loads above
    bool terr_j = false;
    const double jit = rng_group<G>(v, rng, lane, gbase, &terr_j);
    const bool valid = (lane < G::A) && ((vm >> lane) & 1u);
    double score = -10000000000.0;  // mcts.py:347
    if (valid) {
      // q (mcts.py:59-62): children carry no virtual loss in sequential mode
      const double q = cn ? cw / (double)cn : 0.0;
      // p_eff (mcts.py:64-69): noise only on the active root's children
      const double pe = (depth == 0 && noise) ? nz * v.x + (double)cp * (1.0 - v.x) : (double)cp;
      // u (mcts.py:71-78): parent.n + parent.virtual_loss, and the parent holds vl = 1 here
      const double u = ((v.cpuct * pe) * sqrt((double)(node_n + 1))) / (double)(1 + cn);
      // select_prob (mcts.py:80-84): -child.player * q + u = parent.player * q + u
      score = (player > 0 ? q : -q) + u;
    }
    if (!group_or<P>(valid ? 1 : 0)) {  // mcts.py:349-354
      if (lane == 0) set_err(v, SPMCTS_ERR_NOCHILD);
      return;
    }
    // argmax(select_probs + 1e-6 * rand(A)) (mcts.py:355): first index on ties
    terr = terr || terr_j;
    double s = -INFINITY;
    if (lane < G::A) s = score + 0.000001 * jit;
    rng_advance(v, rng, G::A);
    int a = lane;
    group_argmax<P>(s, a);
    const int cc_a = __shfl(cc, gbase + a, 64);
    const int cn_a = __shfl(cn, gbase + a, 64);
    const double cw_a = __shfl(cw, gbase + a, 64);
    const int child = cb * P + a;
    if (cc_a < 0) {
      // leaf reached: _expand_node (mcts.py:301-321)
      Board nb2 = b;
      int rew = 0, done = 0;
      const int st = step<G>(nb2, a, player, &rew, &done);
      if (lane == 0) {
        if (st != STEP_OK) set_err(v, SPMCTS_ERR_STATE);
        int64_t *cnt = v.cnt + (size_t)tree * C_NCNT;
        cnt[C_SIMS] += 1;
        cnt[C_DEPTH] += depth + 1;
        if (done) {
          // terminal: value r (or strong_play shaping), no children, backup in place
          const double val = terminal_value(v, tree, b, rew * player);
          const bool strong = v.tstrong[tree] != 0;
          for (int k = 0; k <= depth; ++k) {
            const size_t idx = nb + s_node[grp][k];
            nd_n<P>(v, idx) = s_n[grp][k] + 1;
            nd_w<P>(v, idx) = s_w[grp][k] + val;
            if (strong) nd_f<P>(v, idx) = 1;
          }
          nd_n<P>(v, nb + child) = cn_a + 1;
          nd_w<P>(v, nb + child) = cw_a + val;
          if (strong) nd_f<P>(v, nb + child) = 1;
          cnt[C_TERM] += 1;
        } else {
          // pending network evaluation: stash the path for k_expand
          const size_t pb = (size_t)tree * G::MAXD;
          for (int k = 0; k <= depth; ++k) {
            v.pnode[pb + k] = s_node[grp][k];
            v.pn[pb + k] = s_n[grp][k];
            v.pw[pb + k] = s_w[grp][k];
          }
          v.plen[tree] = depth + 1;
          v.leaf[tree] = child;
          v.leaf_n[tree] = cn_a;
          v.leaf_w[tree] = cw_a;
          v.lpos[tree] = nb2.pos;
          v.lneg[tree] = nb2.neg;
          v.lmover[tree] = (int8_t)player;
          v.need[tree] = 1;
        }
        if (terr) set_err(v, SPMCTS_ERR_TAPE);
        rng_store(v, tree, rng);
      }
      return;
    }
    // descend
    play<G>(b, a, player);
    node = child;
    node_n = cn_a;
    node_w = cw_a;
    cb = cc_a;
    player = -player;
    ++depth;
    if (depth >= G::MAXD) {
      if (lane == 0) set_err(v, SPMCTS_ERR_STATE);
      return;
    }
  }
}

// ----------------------------------------------------------------------------
// threaded search: K simulations in flight per tree with virtual loss (the reference's
// thread_count search_node calls under an InferenceProxy, mcts.py:154, :328-331, :340-367).
//
// The reference's K threads each run select -> wait for the network -> backup, then take the next
// search_node task, so at any time ~K sims are in flight and a thread's next select sees the other
// K-1 sims still pending (a ROLLING window).  The arena fixes the order of that rolling schedule:
// pending slots j = 0..K-1 of a tree are completed in slot order, and each freed slot is refilled
// right after its backup (FIFO: the oldest pending sim returns first), so every select after the
// first K sees K-1 pending sims, as with the reference's threads.  One network batch still holds
// the K pending leaves of every tree.  Sims that end without a network call (a terminal leaf: backed
// up at once; a leak: every child invalid or locked, mcts.py:349-354, vl left in place) do not
// occupy a slot: the slot takes the next sim at once, as the reference's thread takes its next task.
// oracle/mcts.py (OracleTree.search, threads=K) restates exactly this schedule; the G6 fixture
// (threaded_stats.json) pins its statistics to the reference's own threaded search.
// ----------------------------------------------------------------------------
enum { SIM_DONE = 0, SIM_PENDING = 1, SIM_LEAK = 2, SIM_ERROR = -1 };

// The searching tree's root, loaded once per kernel and kept in registers across the K fills /
// backups / refills (it is on every path): node id, its child block (fixed during a search: the
// root is expanded), board, player, and its visit count and virtual loss — and its child block
// (lane j < A: child j's n, w, p, child index, vl; the valid mask), the first level every sim
// scores.  Every store a sim or backup makes to these nodes is made to the registers as well (the
// same arithmetic), so depth 0 reads no memory.
struct TreeRoot {
  bool strong;  // the tree's strong_play (read once: a global load in a sim would wait on its stores)
  int node, cb, player, n, vl;
  double w;  // the root's w (terminal backups write it from here, no read-modify-write)
  Board b;
  int cn, cc, cvl;
  double cw;
  float cp;
  uint32_t vm;
};

template <class G>
__device__ __forceinline__ TreeRoot load_root(const View &v, int tree) {
  constexpr int P = G::APAD;
  const size_t nb = nbase<G>(v, tree);
  TreeRoot R;
  R.strong = v.tstrong[tree] != 0;
  R.node = v.root[tree];
  R.b = Board{v.rpos[tree], v.rneg[tree]};
  R.player = v.rplayer[tree];
  R.n = nd_n<P>(v, nb + R.node);
  R.vl = nd_vl<P>(v, nb + R.node);
  R.w = nd_w<P>(v, nb + R.node);
  R.cb = nd_c<P>(v, nb + R.node);
  const int lane = threadIdx.x & (P - 1);
  R.cn = 0;
  R.cc = -1;
  R.cvl = 0;
  R.cw = 0.0;
  R.cp = 0.f;
  R.vm = 0u;
  if (R.cb >= 0) {
    R.vm = nd_vm<P>(v, (size_t)tree * v.cap + R.cb);
    if (lane < G::A) {
      const size_t ci = nb + (size_t)R.cb * P + lane;
      R.cn = nd_n<P>(v, ci);
      R.cw = nd_w<P>(v, ci);
      R.cp = nd_p<P>(v, ci);
      R.cc = nd_c<P>(v, ci);
      R.cvl = nd_vl<P>(v, ci);
    }
  }
  return R;
}

// The path of the sim in flight, in LDS (one group per tree): node ids and, per level, the node's n, vl
// (this sim's virtual loss included) and w as this sim read them, and where the node's record sits (cs: a
// BlockCache slot, kRootRegs for the root and the root's children, kUncached).  One wave owns the tree, so
// nothing changes them between the read and this sim's backup: a terminal backup writes n + 1, w + value,
// vl - 1 from here instead of reading the nodes again (one memory round trip less per terminal sim).
struct PathLds {
  int32_t *node, *n, *vl, *cs;
  double *w;
};
enum { kUncached = -1, kRootRegs = -2 };

// Per-launch LDS copies of the child blocks a tree's sims read (round 5).  One wave owns a tree for the
// whole launch, so a block's record, copied in from global memory the first time a level reads it, stays
// exact as long as every store the launch makes to the block is made to the copy as well (write-through:
// the global record stays current for later launches).  A level that hits reads LDS instead of issuing a
// dependent global load, and a sim whose stores all went to copied blocks or to the root and its children
// (kept in registers for the launch, TreeRoot) needs no fence before the next sim: nothing it wrote is read
// back from global memory in this launch.  With the copies full, stores to uncopied blocks set `dirty`,
// and the next global read of node records waits on a workgroup fence first (round 4's per-sim fence).
// The copies hold everything a level reads (n, vl, child block, p, w, the valid mask); the strong-play
// flag is written to global memory only (nothing in a launch reads it).
template <int P, int S>
struct BlockCache {
  static constexpr int BYTES = NodeRec<P>::BYTES;
  int32_t *tag;  // [S] tree-local block index of each copy (16-byte aligned)
  char *rec;     // [S][BYTES] the copies
  int cnt = 0;   // copies in use (group-uniform)
  bool dirty = false;  // stores to uncopied blocks since the last fence (group-uniform)
  __device__ __forceinline__ void fence_if_dirty() {
    if (dirty) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      dirty = false;
    }
  }
  // the slot holding block `blk` or kUncached; every lane may ask for its own block
  __device__ __forceinline__ int find(int blk) const {
    int hit = kUncached;
    if constexpr (S > 0) {
#pragma unroll
      for (int i = 0; i < S / 4; ++i) {
        if (4 * i >= cnt) break;
        const int4 t = ((const int4 *)tag)[i];
        if (t.x == blk && 4 * i + 0 < cnt) hit = 4 * i + 0;
        if (t.y == blk && 4 * i + 1 < cnt) hit = 4 * i + 1;
        if (t.z == blk && 4 * i + 2 < cnt) hit = 4 * i + 2;
        if (t.w == blk && 4 * i + 3 < cnt) hit = 4 * i + 3;
      }
    }
    return hit;
  }
  // copy block `blk` (global record `g`) into a free slot (group-uniform call); kUncached when full
  __device__ __forceinline__ int insert(int blk, const char *g, int lane) {
    if constexpr (S == 0) {
      return kUncached;
    } else {
      if (cnt >= S) return kUncached;
      fence_if_dirty();
      const int s = cnt++;
      const uint4 *src = (const uint4 *)(g + 32 * lane);  // P lanes x 32 bytes = the record
      const uint4 a = src[0], b = src[1];
      uint4 *dst = (uint4 *)(rec + s * BYTES + 32 * lane);
      dst[0] = a;
      dst[1] = b;
      if (lane == 0) tag[s] = blk;
      return s;
    }
  }
  // a new block's copy from the values the caller stores to global memory (k_expand_vl); kUncached when full
  __device__ __forceinline__ int insert_new(int blk, int lane, float p, uint32_t vm) {
    if constexpr (S == 0) {
      return kUncached;
    } else {
      if (cnt >= S) return kUncached;
      const int s = cnt++;
      char *r = rec + s * BYTES;
      ((int32_t *)(r + NodeRec<P>::N))[lane] = 0;
      ((int32_t *)(r + NodeRec<P>::VL))[lane] = 0;
      ((int32_t *)(r + NodeRec<P>::C))[lane] = -1;
      ((float *)(r + NodeRec<P>::PR))[lane] = p;
      ((double *)(r + NodeRec<P>::W))[lane] = 0.0;
      if (lane == 0) {
        *(uint32_t *)(r + NodeRec<P>::VM) = vm;
        tag[s] = blk;
      }
      return s;
    }
  }
  template <class T>
  __device__ __forceinline__ T &at(int s, int off, int a) const {
    return ((T *)(rec + s * BYTES + off))[a];
  }
  __device__ __forceinline__ uint32_t vm(int s) const { return *(const uint32_t *)(rec + s * BYTES + NodeRec<P>::VM); }
};

#ifdef SPMCTS_TREE_PROF
// Profiling build only (make prof: libspmcts_prof.so): shader-clock cycles per sim phase, summed over the
// trees, per kernel (select: [0, 8), expand: [8, 16)) -- [0..5] the phases of TP_* below, [6] the largest
// per-tree launch time, [7] the most sims one tree ran in one launch
__device__ unsigned long long g_tprof[16];
enum { TP_LOAD = 0, TP_SCORE = 1, TP_ARGMAX = 2, TP_LEAF = 3, TP_DESCEND = 4, TP_RNG = 5, TP_OTHER = 5 };
#define TP_MARK(sc, i)                                 \
  do {                                                 \
    const unsigned long long t_ = clock64();           \
    (sc).tp[i] += t_ - (sc).tlast;                     \
    (sc).tlast = t_;                                   \
  } while (0)
#else
#define TP_MARK(sc, i) \
  do {                 \
  } while (0)
#endif

// The tree's counters of one kernel launch (the same value in every lane of the group), added to the
// arena's counters once at the end of the launch instead of a read-modify-write per sim.
struct SimCnt {
  int64_t sims = 0, depth = 0, term = 0, leak = 0, nn = 0, hwm = 0;
#ifdef SPMCTS_TREE_PROF
  unsigned long long tp[6] = {0, 0, 0, 0, 0, 0}, tlast = 0, t0 = 0;
  int64_t sims0 = 0;
  __device__ void prof_begin() {
    t0 = tlast = clock64();
    sims0 = sims;
  }
  __device__ void prof_flush(int base) const {
    const unsigned long long t1 = clock64();
    for (int i = 0; i < 6; ++i) atomicAdd(&g_tprof[base + i], tp[i]);
    atomicMax(&g_tprof[base + 6], t1 - t0);
    atomicMax(&g_tprof[base + 7], (unsigned long long)(sims - sims0));
  }
#endif
  __device__ void flush(int64_t *cnt) const {
    cnt[C_SIMS] += sims;
    cnt[C_DEPTH] += depth;
    cnt[C_TERM] += term;
    cnt[C_LEAK] += leak;
    cnt[C_NN] += nn;
    cnt[C_HWM] = max(cnt[C_HWM], hwm);
  }
};

// One search_node with virtual loss (mcts.py:340-367) for pending slot j of `tree`, run by the
// tree's P-lane group.  vl += 1 on every node passed (mcts.py:345), children scored with
// q = (w - vl)/(n + vl) and u = c p sqrt(N + vl_parent)/(1 + n + vl) (mcts.py:59-78), pending leaves
// locked (child-block index -2, score -1e10, mcts.py:86-88).  Returns SIM_PENDING with the leaf
// locked and its path stashed in slot j, SIM_DONE for a terminal leaf (backed up, path vl removed),
// SIM_LEAK for a leak, SIM_ERROR on a corrupt tree; R (the root in registers) and the block copies bc are
// updated to match.  The return value is uniform across the group.
template <class G, int S>
__device__ int sim_vl(const View &v, int tree, int j, TreeRoot &R, TreeRng &rng, bool &terr, const PathLds &pl,
                      bool noise, double nz, SimCnt &sc, BlockCache<G::APAD, S> &bc) {
  constexpr int P = G::APAD;
  const int lane = threadIdx.x & (P - 1);
  const int gbase = (threadIdx.x & 63) & ~(P - 1);
  const size_t nb = nbase<G>(v, tree);
  const size_t bb = (size_t)tree * v.cap;
  const int ps = tree * v.K + j;
  int node = R.node;
  Board b = R.b;
  int player = R.player;
  int node_n = R.n;
  int node_vl = R.vl + 1;  // this sim's virtual loss on the node (mcts.py:345)
  double node_w = R.w;
  int cb = R.cb;
  int ncs = kRootRegs;  // where path node `depth`'s record sits
  R.vl += 1;
  int depth = 0;
  int a0 = 0;  // the root child this sim took (path node 1)
  for (;;) {
    if (lane == 0) {
      pl.node[depth] = node;
      pl.n[depth] = node_n;
      pl.vl[depth] = node_vl;
      pl.w[depth] = node_w;
      pl.cs[depth] = ncs;
      if (ncs >= 0) bc.template at<int32_t>(ncs, NodeRec<P>::VL, node % P) = node_vl;
    }
    // the global store of the path's virtual loss waits for the sim's end (one store per path node, all
    // at once): gfx950's vmcnt counts stores too, so a store here would hold up the next level's loads.
    // `dirty` is set where those stores are issued (leak, pending, terminal below), not here: nothing of
    // this sim is in flight yet, so the levels of one sim read without a fence.
    if (depth == 1 && lane == a0) R.cvl = node_vl;  // the root child's vl, in registers too
    if (cb < 0) {
      if (lane == 0) set_err(v, SPMCTS_ERR_STATE);
      return SIM_ERROR;
    }
    uint32_t vm;
    int cn = 0, cc = -1, cvl = 0;
    double cw = 0.0;
    float cp = 0.f;
    int lcs = kRootRegs;  // where this level's child block (cb) sits
    if (depth == 0) {  // the root's child block, from registers
      vm = R.vm;
      cn = R.cn;
      cw = R.cw;
      cp = R.cp;
      cc = R.cc;
      cvl = R.cvl;
    } else {
      lcs = bc.find(cb);
      if (lcs == kUncached) lcs = bc.insert(cb, nd_rec<P>(v, nb + (size_t)cb * P), lane);
      if (lcs >= 0) {
        vm = bc.vm(lcs);
        if (lane < G::A) {
          cn = bc.template at<int32_t>(lcs, NodeRec<P>::N, lane);
          cw = bc.template at<double>(lcs, NodeRec<P>::W, lane);
          cp = bc.template at<float>(lcs, NodeRec<P>::PR, lane);
          cc = bc.template at<int32_t>(lcs, NodeRec<P>::C, lane);
          cvl = bc.template at<int32_t>(lcs, NodeRec<P>::VL, lane);
        }
      } else {
        bc.fence_if_dirty();
        vm = nd_vm<P>(v, bb + cb);
        const size_t ci = nb + (size_t)cb * P + lane;
        if (lane < G::A) {
          cn = nd_n<P>(v, ci);
          cw = nd_w<P>(v, ci);
          cp = nd_p<P>(v, ci);
          cc = nd_c<P>(v, ci);
          cvl = nd_vl<P>(v, ci);
        }
      }
    }
#ifdef SPMCTS_TREE_PROF
    // (profiling: the loads completed before the jitter, to time the two apart)
    if (cn == -12345 || cw == -1.5 || cp == -1.5f || cvl == -12345 || vm == 0xdeadbeefu) sc.tp[TP_OTHER] += 1;
    TP_MARK(sc, TP_LOAD);
#endif
    // the jitter does not depend on the child block: drawn here, it overlaps the loads above
    bool terr_j = false;
    const double jit = rng_group<G>(v, rng, lane, gbase, &terr_j);
    // valid (mcts.py:86-88): valid move and not locked by a pending sim
    const bool valid = (lane < G::A) && ((vm >> lane) & 1u) && cc != -2;
#ifdef SPMCTS_TREE_PROF
    if (jit == -1.5) sc.tp[TP_OTHER] += 1;
    TP_MARK(sc, TP_RNG);
#endif
    double score = -10000000000.0;
    if (valid) {
      // q (mcts.py:59-62): (w - vl) / (n + vl)
      const int ne = cn + cvl;
      const double q = ne ? (cw - (double)cvl) / (double)ne : 0.0;
      const double pe = (depth == 0 && noise) ? nz * v.x + (double)cp * (1.0 - v.x) : (double)cp;
      // u (mcts.py:71-78): sqrt(parent.n + parent.virtual_loss) / (1 + n + virtual_loss)
      const double u = ((v.cpuct * pe) * sqrt((double)(node_n + node_vl))) / (double)(1 + cn + cvl);
      score = (player > 0 ? q : -q) + u;
    }
    if (!group_or<P>(valid ? 1 : 0)) {  // mcts.py:349-354: return, virtual loss left in place
      int unc = 0;
      for (int k = lane; k <= depth; k += P) {
        nd_vl<P>(v, nb + pl.node[k]) = pl.vl[k];
        unc |= pl.cs[k] == kUncached;
      }
      if (group_or<P>(unc)) bc.dirty = true;
      sc.leak += 1;
      return SIM_LEAK;
    }
    terr = terr || terr_j;  // (a leak consumes no draw, so its tape check does not count)
    double s = -INFINITY;
    if (lane < G::A) s = score + 0.000001 * jit;
    rng_advance(v, rng, G::A);
    TP_MARK(sc, TP_SCORE);
    int a = lane;
    int cc_a = cc, cn_a = cn, cvl_a = cvl;
    double cw_a = cw;
    group_argmax_carry<P>(s, a, cc_a, cn_a, cvl_a, cw_a);  // lane a's child fields in every lane
    const int child = cb * P + a;
    TP_MARK(sc, TP_ARGMAX);
    if (cc_a < 0) {
      // leaf: _expand_node (mcts.py:301-321)
      Board nb2 = b;
      int rew = 0, done = 0;
      const int st = step<G>(nb2, a, player, &rew, &done);
      if (done) {
        // terminal: backup (mcts.py:94-98) then remove the path's virtual loss (:365); one lane per
        // path node, the values this sim read (pl: written by lane 0 of this wave, LDS stays in order)
        const double val = terminal_value(R.strong, b, rew * player);
        const bool strong = R.strong;
        int unc = 0;
        for (int k = lane; k <= depth; k += P) {
          const int nk = pl.node[k], ck = pl.cs[k];
          const size_t idx = nb + nk;
          const int32_t n1 = pl.n[k] + 1, vl1 = pl.vl[k] - 1;
          const double w1 = pl.w[k] + val;
          nd_n<P>(v, idx) = n1;
          nd_w<P>(v, idx) = w1;
          if (strong) nd_f<P>(v, idx) = 1;
          nd_vl<P>(v, idx) = vl1;
          if (ck >= 0) {
            bc.template at<int32_t>(ck, NodeRec<P>::N, nk % P) = n1;
            bc.template at<double>(ck, NodeRec<P>::W, nk % P) = w1;
            bc.template at<int32_t>(ck, NodeRec<P>::VL, nk % P) = vl1;
          }
          unc |= ck == kUncached;
        }
        if (lane == 0) {
          nd_n<P>(v, nb + child) = cn_a + 1;
          nd_w<P>(v, nb + child) = cw_a + val;
          if (strong) nd_f<P>(v, nb + child) = 1;
          if (lcs >= 0) {
            bc.template at<int32_t>(lcs, NodeRec<P>::N, a) = cn_a + 1;
            bc.template at<double>(lcs, NodeRec<P>::W, a) = cw_a + val;
          }
        }
        if (group_or<P>(unc) || lcs == kUncached) bc.dirty = true;
        R.n += 1;  // the root is path node 0
        R.vl -= 1;
        R.w += val;
        if (depth >= 1 && lane == a0) {  // path node 1, the root child a0
          R.cn += 1;
          R.cw += val;
          R.cvl -= 1;
        }
        if (depth == 0 && lane == a) {  // the terminal leaf is a root child
          R.cn += 1;
          R.cw += val;
        }
        sc.term += 1;
      } else {
        const size_t pb = (size_t)ps * G::MAXD;
        int unc = 0;
        for (int k = lane; k <= depth; k += P) {
          const int nk = pl.node[k];
          v.pnode[pb + k] = nk;
          nd_vl<P>(v, nb + nk) = pl.vl[k];
          unc |= pl.cs[k] == kUncached;
        }
        if (group_or<P>(unc)) bc.dirty = true;
      }
      sc.sims += 1;
      sc.depth += depth + 1;
      if (lane == 0) {
        if (st != STEP_OK) set_err(v, SPMCTS_ERR_STATE);
        if (!done) {
          // lock the leaf (mcts.py:359); the path was stashed above for the backup
          nd_c<P>(v, nb + child) = -2;
          if (lcs >= 0) bc.template at<int32_t>(lcs, NodeRec<P>::C, a) = -2;
          v.plen[ps] = depth + 1;
          v.leaf[ps] = child;
          v.lpos[ps] = nb2.pos;
          v.lneg[ps] = nb2.neg;
          v.lmover[ps] = (int8_t)player;
          v.need[ps] = 1;
        }
      }
      if (!done && lcs == kUncached) bc.dirty = true;
      if (!done && depth == 0 && lane == a) R.cc = -2;
      TP_MARK(sc, TP_LEAF);
      return done ? SIM_DONE : SIM_PENDING;
    }
    if (depth == 0) a0 = a;
    play<G>(b, a, player);
    node = child;
    node_n = cn_a;
    node_vl = cvl_a + 1;
    node_w = cw_a;
    cb = cc_a;
    ncs = lcs;  // the child's record is in this level's block
    player = -player;
    ++depth;
    TP_MARK(sc, TP_DESCEND);
    if (depth >= G::MAXD) {
      if (lane == 0) set_err(v, SPMCTS_ERR_STATE);
      return SIM_ERROR;
    }
  }
}

// Refill pending slot j: start sims until one waits for the network or the tree's budget of
// search_node calls is spent (`started` counts them, mcts.py:328-331 submits `iterations`).  No fence
// between sims: a sim reads what the previous one wrote from the block copies or the registers, and
// the copies' `dirty` rule fences before any global read of node records after an uncopied store.
template <class G, int S>
__device__ int fill_slot_vl(const View &v, int tree, int j, int limit, int &started, TreeRoot &R, TreeRng &rng,
                            bool &terr, const PathLds &pl, bool noise, double nz, SimCnt &sc,
                            BlockCache<G::APAD, S> &bc) {
  while (started < limit) {
    ++started;
    const int r = sim_vl<G, S>(v, tree, j, R, rng, terr, pl, noise, nz, sc, bc);
    if (r == SIM_PENDING || r == SIM_ERROR) return r;
  }
  return SIM_DONE;
}

// LDS block copies per tree: none in the shipped kernels.  Measured (profiles/r05/tree2/): with 16
// copies per tree the isolated expand ran 250 -> 295-300 us and select unchanged (a launch starts with no
// copies, so most blocks are copied once and read once; and the levels of a sim are a chain of short
// dependent LDS / permute / FP64 latencies, not memory round trips: scripts/bench_tree.py --prof).
// The A/B library keeps them behind SPMCTS_TREE_COPIES=1.
template <int TB>
constexpr int kCopies = 0;

// First step of a search: fill the K slots of every searching tree.
template <class G, int TB = 64, int S = kCopies<TB>>
__global__ __launch_bounds__(TB) void k_select_vl(View v, int n_active) {
  constexpr int P = G::APAD;
  constexpr int GPB = TB / P;
  constexpr int S1 = S > 0 ? S : 4;
  __shared__ int32_t s_node[GPB][G::MAXD], s_n[GPB][G::MAXD], s_vl[GPB][G::MAXD], s_cs[GPB][G::MAXD];
  __shared__ double s_w[GPB][G::MAXD];
  __shared__ __attribute__((aligned(16))) int32_t s_tag[GPB][S1];
  __shared__ __attribute__((aligned(16))) char s_rec[S > 0 ? GPB : 1][S > 0 ? S : 1][NodeRec<P>::BYTES];
  const int lane = threadIdx.x & (P - 1);
  const int grp = threadIdx.x / P;
  const PathLds pl{s_node[grp], s_n[grp], s_vl[grp], s_cs[grp], s_w[grp]};
  BlockCache<P, S> bc;
  bc.tag = s_tag[grp];
  bc.rec = S > 0 ? &s_rec[grp][0][0] : nullptr;
  const int slot = blockIdx.x * (int)(blockDim.x / P) + grp;  // blockDim = 64 (GPB trees) or P (one tree)
  if (slot >= n_active) return;
  const int tree = v.active[slot];
  if (tree < 0) return;
  const int limit = min(v.budget[tree], v.iters);
  int started = v.tstarted[tree];
  if (started >= limit) return;
  const bool noise = v.noise_on[tree] != 0;
  const double nz = (noise && lane < G::A) ? v.noise[(size_t)tree * P + lane] : 0.0;
  TreeRng rng;
  rng_load(v, tree, rng);
  TreeRoot R = load_root<G>(v, tree);
  bool terr = false;
  SimCnt sc;
#ifdef SPMCTS_TREE_PROF
  sc.prof_begin();
#endif
  const int kt = v.tK[tree];  // this tree's sims in flight (its own thread_count, <= K)
  for (int j = 0; j < kt; ++j) {
    if (v.need[tree * v.K + j]) continue;
    // SIM_ERROR (a corrupt tree: the sticky SPMCTS_ERR_STATE flag is set) ends the tree's launch; the counters
    // of the sims completed before it are still flushed below (the failing sim's path vl is not written)
    if (fill_slot_vl<G, S>(v, tree, j, limit, started, R, rng, terr, pl, noise, nz, sc, bc) == SIM_ERROR) break;
  }
  if (lane == 0) {
#ifdef SPMCTS_TREE_PROF
    sc.prof_flush(0);
#endif
    sc.flush(v.cnt + (size_t)tree * C_NCNT);
    v.tstarted[tree] = started;
    if (terr) set_err(v, SPMCTS_ERR_TAPE);
    rng_store(v, tree, rng);
  }
}
// ----------------------------------------------------------------------------
// kernel: compaction of pending leaves into rows (tree order => deterministic)
// ----------------------------------------------------------------------------
// Two segments: leaves of network-0 trees in rows [0, n0), of network-1 trees in rows
// [seg1, seg1 + n1) (single-network arenas: seg1 = T, n1 = 0).
// count_out (optional): [0] = n0 + n1, [1] = n0, [2] = n1.
// ----------------------------------------------------------------------------
// batch leaf dedup (K > 1): the network input of a pending leaf is its (own, opp) stone planes from
// the mover's view (k_encode), so leaves with equal (own, opp) of the same network get one row and
// one evaluation; the trunk and heads are deterministic and batch-independent, so every leaf still
// receives exactly the outputs its own row would have produced.  Owner of a key = its lowest slot
// (deterministic); the table is cleared by generation stamps instead of a memset per step.
// ----------------------------------------------------------------------------
template <class G>
__device__ __forceinline__ void leaf_key(const View &v, int t, uint64_t &own, uint64_t &opp) {
  const int mover = v.lmover[t];
  own = mover > 0 ? v.lpos[t] : v.lneg[t];
  opp = mover > 0 ? v.lneg[t] : v.lpos[t];
  if (v.tnet[t / v.K]) own |= 1ull << 63;  // rows of the two networks never merge (cell bits < 63)
}

__device__ __forceinline__ uint32_t leaf_hash(uint64_t a, uint64_t b) {
  uint64_t x = a ^ (b * 0x9E3779B97F4A7C15ull);
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}

template <class G>
__global__ __launch_bounds__(256) void k_dedup_insert(View v) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= v.NS || !v.need[t]) return;
  uint64_t own, opp;
  leaf_key<G>(v, t, own, opp);
  const unsigned long long mine = ((unsigned long long)v.dgen << 32) | (uint32_t)t;
  unsigned long long *tab = (unsigned long long *)v.dtab;
  uint32_t h = leaf_hash(own, opp) & (uint32_t)v.dmask;
  for (int probe = 0; probe <= v.dmask; ++probe) {
    // claim the entry if it holds an older generation; a failed CAS returns the current value, which
    // during this kernel can only have become this generation's (at most two rounds)
    unsigned long long w = tab[h];
    while ((uint32_t)(w >> 32) != v.dgen) {
      const unsigned long long old = atomicCAS(tab + h, w, mine);
      if (old == w) {
        v.dent[t] = (int)h;
        return;
      }
      w = old;
    }
    uint64_t so, sp;
    leaf_key<G>(v, (int)(uint32_t)w, so, sp);
    if (so == own && sp == opp) {
      atomicMin(tab + h, mine);  // the lowest slot of the key owns the row
      v.dent[t] = (int)h;
      return;
    }
    h = (h + 1) & (uint32_t)v.dmask;
  }
  set_err(v, SPMCTS_ERR_STATE);  // unreachable: the table has >= 2 NS entries
}

// owner flags, one independent load pair per slot (the scan below then reads one byte per slot
// instead of a dependent dent -> dtab chain per slot in its serial chunk loop); a leader lane also
// keeps each owner's key for its followers' lookups this step (okey: nothing else writes it until its
// next step's k_dedup_owner, which runs after every follower's lookup of this step)
// Evaluation cache (spmcts_set_eval_cache): linear probing over at most CACHE_PROBES entries from the key's
// hash.  An entry's tag is (generation << 32 | state): 0 = never used, CACHE_READY = key and outputs published,
// CACHE_BUSY = being written.  A lookup sees READY entries whose generation is within the window of its own
// (0 <= cgen - gen < cwin); an insert may take an entry that was never used or whose READY generation is more
// than cwin behind its own (one generation of slack: the two lanes of a shared table are at most one ply apart,
// so no entry a lane can still see, or renew, is taken by the other).  Tags never return to 0, so every entry
// before a live key's entry in its probe chain has been in use since the key went in, and a lookup may stop at
// the first never-used entry.  Publication: CAS to BUSY, key and outputs stored, then the READY tag stored with
// release semantics (agent scope); a lookup confirms a candidate by acquire re-reads (cache_find), so a READY key
// is never read torn (a lane sharing its leader's table reads it while the leader's expand inserts on another
// stream).
constexpr int CACHE_PROBES = 32;
constexpr unsigned long long CACHE_READY = 1ull, CACHE_BUSY = 2ull;

constexpr int CACHE_REC = 8;  // u64 words per record (64 bytes): tag, own, opp, (A + 1) f32 (A <= 9)
static_assert(24 + 4 * (C4::A + 1) <= 8 * CACHE_REC && 24 + 4 * (TTT::A + 1) <= 8 * CACHE_REC, "cache record");

__device__ __forceinline__ unsigned long long *cache_rec(const View &v, uint32_t h) {
  return (unsigned long long *)v.crec + (size_t)h * CACHE_REC;
}
__device__ __forceinline__ float *cache_out(const View &v, uint32_t h) {
  return (float *)(cache_rec(v, h) + 3);
}

__device__ __forceinline__ bool cache_live_tag(const View &v, unsigned long long tag) {
  const int d = (int)(v.cgen - (uint32_t)(tag >> 32));
  return (tag & 0xffffffffull) == CACHE_READY && d >= 0 && d < v.cwin;
}

__device__ __forceinline__ bool cache_free_tag(const View &v, unsigned long long tag) {
  const int d = (int)(v.cgen - (uint32_t)(tag >> 32));
  return tag == 0 || ((tag & 0xffffffffull) == CACHE_READY && d > v.cwin);
}

// The probe loop reads records with plain loads (a stale line only makes a miss or an early stop: the position
// is then evaluated); a candidate is confirmed after an acquire fence by atomic re-reads of its tag and key, so a
// hit is a READY record whose key and outputs were published before the tag.
__device__ __forceinline__ int cache_find(const View &v, uint64_t own, uint64_t opp) {
  uint32_t h = leaf_hash(own, opp) & (uint32_t)v.cmask;
  for (int p = 0; p < CACHE_PROBES; ++p) {
    const unsigned long long *r = cache_rec(v, h);
    const unsigned long long tag = r[0];
    if (tag == 0) return -1;
    if (cache_live_tag(v, tag) && r[1] == own && r[2] == opp) {
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      unsigned long long *rw = cache_rec(v, h);
      const unsigned long long t2 = __hip_atomic_load(rw, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long o2 = __hip_atomic_load(rw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long q2 = __hip_atomic_load(rw + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return cache_live_tag(v, t2) && o2 == own && q2 == opp ? (int)h : -1;
    }
    h = (h + 1) & (uint32_t)v.cmask;
  }
  return -1;
}

// an owner slot's key in the cache: down 3, the entry in xc, its generation renewed (kept while in use)
template <class G>
__device__ __forceinline__ bool cache_hit(const View &v, int t) {
  uint64_t own, opp;
  leaf_key<G>(v, t, own, opp);
  const int e = cache_find(v, own, opp);
  if (e < 0) return false;
  __hip_atomic_store(cache_rec(v, e), ((unsigned long long)v.cgen << 32) | CACHE_READY, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  v.xc[t] = e;
  return true;
}

template <class G>
__global__ __launch_bounds__(256) void k_dedup_owner(View v) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= v.NS) return;
  const bool own = v.need[t] && (int)(uint32_t)v.dtab[v.dent[t]] == t;
  v.down[t] = own ? (v.cwin && cache_hit<G>(v, t) ? 3 : 1) : 0;
  if (own && v.lead) {
    uint64_t a, b;
    leaf_key<G>(v, t, a, b);
    v.okey[2 * (size_t)t] = a;
    v.okey[2 * (size_t)t + 1] = b;
  }
}

// Follower lane (spmcts_set_leaf_peer), a simulation step: owner flags as k_dedup_owner, and each owner
// slot's key looked up in the leader lane's table of the same step (generation pgen, probed as the
// leader's k_dedup_insert placed it: a key present this generation sits before the first entry of an
// older one).  A hit takes the leader's row: down 2, xpeer = the leader's owner slot.  Outputs are pure
// functions of the leaf planes (the fused trunk is batch-independent), so the leaf still gets exactly
// the outputs its own row would have produced.
template <class G>
__global__ __launch_bounds__(256) void k_dedup_owner_peer(View v, const uint64_t *ptab, const uint64_t *pkey,
                                                          const uint8_t *pdown, int pmask, uint32_t pgen) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= v.NS) return;
  int d = 0, xp = -1;
  if (v.need[t] && (int)(uint32_t)v.dtab[v.dent[t]] == t) {
    d = 1;
    if (v.cwin && cache_hit<G>(v, t)) {  // the follower's own cache first: no wait on the leader's outputs
      v.down[t] = 3;
      v.xpeer[t] = -1;
      return;
    }
    uint64_t own, opp;
    leaf_key<G>(v, t, own, opp);
    uint32_t h = leaf_hash(own, opp) & (uint32_t)pmask;
    for (int probe = 0; probe <= pmask; ++probe) {
      const unsigned long long w = ptab[h];
      if ((uint32_t)(w >> 32) != pgen) break;  // not in the leader's batch
      const int s = (int)(uint32_t)w;
      if (pkey[2 * (size_t)s] == own && pkey[2 * (size_t)s + 1] == opp) {
        if (pdown[s] == 1) {  // a row the leader's network evaluates (not one its cache fills at its expand)
          d = 2;
          xp = s;
        }
        break;
      }
      h = (h + 1) & (uint32_t)pmask;
    }
  }
  v.down[t] = (uint8_t)d;
  v.xpeer[t] = xp;
}

// the leader's outputs of this step into the follower's rows of the slots it serves (down 2), on the
// leader's stream after its heads (spmcts_peer_push): probs [row][A] f32, values [row] f32
__global__ __launch_bounds__(256) void k_peer_push(View v, const int32_t *psrow, const float *pprobs,
                                                   const float *pvalues, float *probs, float *values) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= v.NS || v.down[t] != 2) return;
  const int r1 = v.srow[t], r0 = psrow[v.xpeer[t]];
  for (int a = 0; a < v.A; ++a) probs[(size_t)r1 * v.A + a] = pprobs[(size_t)r0 * v.A + a];
  values[r1] = pvalues[r0];
}

// Evaluation cache at the expand of a step whose rows consulted it (single-network arenas): a cache-served
// owner slot (down 3) gets its entry's outputs in its row; a slot whose row holds network outputs (down 1:
// its own network's, down 2: the leader's, pushed before this -- unless the table is the leader's own, which
// the leader fills) puts them in the cache under the current generation (nothing is cached when no entry
// within CACHE_PROBES is free).  Duplicates (down 0) read their owner's row.
template <class G>
__global__ __launch_bounds__(256) void k_cache_io(View v, float *probs0, float *values0, float *probs1,
                                                  float *values1) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= v.NS || !v.need[t]) return;
  const int d = v.down[t];
  if (d == 0) return;
  const int A = v.A;
  // network-1 rows (two-network arenas) live in their own output buffers, indexed by row - seg1
  const int row = v.srow[t];
  const bool n1 = row >= v.seg1;
  const int r = n1 ? row - v.seg1 : row;
  float *values = n1 ? values1 : values0;
  float *pr = (n1 ? probs1 : probs0) + (size_t)r * A;
  if (d == 3) {
    const float *c = cache_out(v, v.xc[t]);
    for (int a = 0; a < A; ++a) pr[a] = c[a];
    values[r] = c[A];
    return;
  }
  if (d == 2 && v.cshared) return;
  uint64_t own, opp;
  leaf_key<G>(v, t, own, opp);
  uint32_t h = leaf_hash(own, opp) & (uint32_t)v.cmask;
  const unsigned long long gen = (unsigned long long)v.cgen << 32;
  for (int p = 0; p < CACHE_PROBES; ++p) {
    unsigned long long *rec = cache_rec(v, h);
    unsigned long long w = __hip_atomic_load(rec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (cache_free_tag(v, w)) {  // never used, or behind the window (+1): free to take
      const unsigned long long old = atomicCAS(rec, w, gen | CACHE_BUSY);
      if (old == w) {
        rec[1] = own;
        rec[2] = opp;
        float *c = cache_out(v, h);
        for (int a = 0; a < A; ++a) c[a] = pr[a];
        c[A] = values[r];
        __hip_atomic_store(rec, gen | CACHE_READY, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      w = old;  // another insert took it first: probe on
    }
    h = (h + 1) & (uint32_t)v.cmask;
  }
}

__device__ __forceinline__ bool row_owner(const View &v, int t) { return v.dedup ? v.down[t] == 1 : v.need[t] != 0; }

// duplicates read their owner's row
__global__ __launch_bounds__(256) void k_dedup_alias(View v) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= v.NS || !v.need[t]) return;
  const int s = (int)(uint32_t)v.dtab[v.dent[t]];
  if (s != t) v.srow[t] = v.srow[s];
}

// 512 threads = two waves per SIMD: the kernel runs while the other lane's trunk holds every CU, in the
// registers a trunk wave leaves free on its SIMD (512 - 424 = 88 per lane beside the C = 128 trunk; a
// 1,024-thread block needs 4 x 24 there and waited for a trunk workgroup to retire: 37 -> 90 us average
// in the bench trace, profiles/r04_bench_prof/; 256 threads: 64 us, two rounds of flag loads per pass)
constexpr int SCAN_THREADS = 512;
constexpr int SCAN_WAVES = SCAN_THREADS / 64;

__global__ __launch_bounds__(SCAN_THREADS) void k_scan_need(View v, int32_t *count_out) {
  // wave totals of the two segments' owner counts (a two-level scan: 6 shuffle steps within each wave,
  // 3 over the 8 wave totals, 2 barriers; the round-3 1,024-entry Hillis-Steele scan took 20 barriers
  // and 8 KB of LDS)
  __shared__ int32_t s_w0[SCAN_WAVES], s_w1[SCAN_WAVES], s_w2[SCAN_WAVES], s_w4[SCAN_WAVES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int T = v.NS;  // pending slots (tree * K + j), tree order then in-flight order
  const int chunk = (T + SCAN_THREADS - 1) / SCAN_THREADS;
  const int lo = min(T, tid * chunk), hi = min(T, lo + chunk);
  // c0 / c1: network-0 / network-1 rows the networks evaluate; c2 / c4: served rows (leader- or cache-served) of
  // network 0 / 1, numbered after the evaluated rows of their segment; c3: cache-served rows (a counter)
  int c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0;
  const bool two = v.seg1 < v.NS;  // two-network arena (single-network: no tnet loads)
  // unrolled so each thread's chunk of flags is fetched in one round of independent loads
  if (v.served) {
#pragma unroll 16
    for (int t = lo; t < hi; ++t) {
      const int d = v.down[t];
      const bool n1 = two && v.tnet[t / v.K] != 0;
      c0 += d == 1 && !n1;
      c1 += d == 1 && n1;
      c2 += d >= 2 && !n1;
      c4 += d >= 2 && n1;
      c3 += d == 3;
    }
  } else {
#pragma unroll 16
    for (int t = lo; t < hi; ++t)
      if (row_owner(v, t)) {
        if (v.tnet[t / v.K]) ++c1; else ++c0;
      }
  }
  // inclusive scans of (c0, c1, c2, c4) in thread order: within the wave, then over the wave totals
  int i0 = c0, i1 = c1, i2 = c2, i4 = c4;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int a0 = __shfl_up(i0, off, 64), a1 = __shfl_up(i1, off, 64), a2 = __shfl_up(i2, off, 64);
    const int a4 = __shfl_up(i4, off, 64);
    if (lane >= off) {
      i0 += a0;
      i1 += a1;
      i2 += a2;
      i4 += a4;
    }
  }
  if (lane == 63) {
    s_w0[wave] = i0;
    s_w1[wave] = i1;
    s_w2[wave] = i2;
    s_w4[wave] = i4;
  }
  __syncthreads();
  if (wave == 0) {
    int w0 = lane < SCAN_WAVES ? s_w0[lane] : 0, w1 = lane < SCAN_WAVES ? s_w1[lane] : 0;
    int w2 = lane < SCAN_WAVES ? s_w2[lane] : 0, w4 = lane < SCAN_WAVES ? s_w4[lane] : 0;
#pragma unroll
    for (int off = 1; off < SCAN_WAVES; off <<= 1) {
      const int a0 = __shfl_up(w0, off, 64), a1 = __shfl_up(w1, off, 64), a2 = __shfl_up(w2, off, 64);
      const int a4 = __shfl_up(w4, off, 64);
      if (lane >= off) {
        w0 += a0;
        w1 += a1;
        w2 += a2;
        w4 += a4;
      }
    }
    if (lane < SCAN_WAVES) {
      s_w0[lane] = w0;
      s_w1[lane] = w1;
      s_w2[lane] = w2;
      s_w4[lane] = w4;
    }
  }
  __syncthreads();
  i0 += wave ? s_w0[wave - 1] : 0;
  i1 += wave ? s_w1[wave - 1] : 0;
  i2 += wave ? s_w2[wave - 1] : 0;
  i4 += wave ? s_w4[wave - 1] : 0;
  int r0 = i0 - c0, r1 = v.seg1 + i1 - c1;
  if (v.served) {
    // served rows follow all evaluated rows of their network's segment
    int r2 = s_w0[SCAN_WAVES - 1] + i2 - c2, r4 = v.seg1 + s_w1[SCAN_WAVES - 1] + i4 - c4;
#pragma unroll 16
    for (int t = lo; t < hi; ++t) {
      const int d = v.down[t];
      if (d == 0) continue;
      const bool n1 = two && v.tnet[t / v.K] != 0;
      if (d == 1) {
        const int r = n1 ? r1++ : r0++;
        v.row_tree[r] = t;
        v.srow[t] = r;
      } else {
        v.srow[t] = n1 ? r4++ : r2++;
      }
    }
    if (v.cwin) {  // cache-served rows (counters.cache_rows)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) c3 += __shfl_xor(c3, off, 64);
      if (lane == 0 && c3) atomicAdd((unsigned long long *)&v.gcnt[11], (unsigned long long)c3);
    }
  } else {
#pragma unroll 16
    for (int t = lo; t < hi; ++t)
      if (row_owner(v, t)) {
        const int r = v.tnet[t / v.K] ? r1++ : r0++;
        v.row_tree[r] = t;
        if (v.K > 1) v.srow[t] = r;
      }
  }
  if (tid == SCAN_THREADS - 1) {  // the last thread's inclusive prefix is each segment's total
    v.row_count[0] = i0;
    v.row_count[1] = i1;
    v.gcnt[10] += i0 + i1;  // network rows emitted (counters.nn_rows)
    if (count_out) {
      count_out[0] = i0 + i1;
      count_out[1] = i0;
      count_out[2] = i1;
    }
  }
}

__device__ __forceinline__ bool row_live(const View &v, int row) {
  return row < v.seg1 ? row < v.row_count[0] : row - v.seg1 < v.row_count[1];
}

// ----------------------------------------------------------------------------
// kernel: leaf encoding (preprocess, games/general/modules.py:115-125; input = state*mover)
// ----------------------------------------------------------------------------
template <class G>
__global__ void k_encode(View v, void *out) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int row = (int)(gid / G::CELLS);
  const int cell = (int)(gid % G::CELLS);
  if (row >= v.NS || !row_live(v, row)) return;
  const int t = v.row_tree[row];
  const int x = cell / G::H, y = cell % G::H;
  const uint64_t bit = 1ull << cell_bit<G>(x, y);
  const int mover = v.lmover[t];
  const uint64_t own = mover > 0 ? v.lpos[t] : v.lneg[t];
  const uint64_t opp = mover > 0 ? v.lneg[t] : v.lpos[t];
  const int c_own = (own & bit) ? 1 : 0, c_opp = (opp & bit) ? 1 : 0;
  const int c_emp = 1 - c_own - c_opp;
  if (v.leaf_format == SPMCTS_LEAF_BOARD_I64) {
    ((int64_t *)out)[(size_t)row * G::CELLS + cell] = (int64_t)(c_own - c_opp);
    return;
  }
  size_t i0, i1, i2;
  if (v.leaf_layout == SPMCTS_NHWC) {
    const size_t base = ((size_t)row * G::CELLS + cell) * 3;
    i0 = base;
    i1 = base + 1;
    i2 = base + 2;
  } else {
    const size_t base = (size_t)row * 3 * G::CELLS + cell;
    i0 = base;
    i1 = base + G::CELLS;
    i2 = base + 2 * G::CELLS;
  }
  if (v.leaf_format == SPMCTS_LEAF_F32) {
    float *o = (float *)out;
    o[i0] = (float)c_emp;
    o[i1] = (float)c_own;
    o[i2] = (float)c_opp;
  } else {
    const uint16_t one = v.leaf_format == SPMCTS_LEAF_F16 ? 0x3C00 : 0x3F80;
    uint16_t *o = (uint16_t *)out;
    o[i0] = c_emp ? one : 0;
    o[i1] = c_own ? one : 0;
    o[i2] = c_opp ? one : 0;
  }
}

// ----------------------------------------------------------------------------
// kernel: expand + backup of network-evaluated leaves (mcts.py:316-321, :94-98)
// ----------------------------------------------------------------------------
template <class G>
__global__ __launch_bounds__(64) void k_expand(View v, const float *probs0, const float *values0,
                                               const float *probs1, const float *values1) {
  constexpr int P = G::APAD;
  const int lane = threadIdx.x & (P - 1);
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) / P;
  if (row >= v.T || !row_live(v, row)) return;
  // network-1 rows read their outputs from the second network's buffers (row - seg1)
  const bool s1 = row >= v.seg1;
  const float *prow = s1 ? probs1 + (size_t)(row - v.seg1) * G::A : probs0 + (size_t)row * G::A;
  const float vrow = s1 ? values1[row - v.seg1] : values0[row];
  const int tree = v.row_tree[row];
  const size_t nb = nbase<G>(v, tree);
  const size_t bb = (size_t)tree * v.cap;
  const int blk = v.used[tree];
  if (blk >= v.cap) {
    if (lane == 0) set_err(v, SPMCTS_ERR_POOL);
    return;
  }
  const int leaf = v.leaf[tree];
  // create_children (mcts.py:103-107): A children in action order, validity = valid_moves
  {
    const size_t ci = nb + (size_t)blk * P + lane;
    nd_n<P>(v, ci) = 0;
    nd_w<P>(v, ci) = 0.0;
    nd_p<P>(v, ci) = lane < G::A ? prow[lane] : 0.f;
    nd_c<P>(v, ci) = -1;
    nd_f<P>(v, ci) = 0;
  }
  const int mover = v.lmover[tree];
  // network(s, parent.player) returns value * player (modules.py:109-112)
  const double val = (double)vrow * (double)mover;
  const int plen = v.plen[tree];
  const size_t pb = (size_t)tree * G::MAXD;
  for (int k = lane; k < plen; k += P) {
    const size_t idx = nb + v.pnode[pb + k];
    nd_n<P>(v, idx) = v.pn[pb + k] + 1;
    nd_w<P>(v, idx) = v.pw[pb + k] + val;
  }
  if (lane == 0) {
    nd_vm<P>(v, bb + blk) = legal_mask<G>(Board{v.lpos[tree], v.lneg[tree]});
    nd_c<P>(v, nb + leaf) = blk;
    nd_n<P>(v, nb + leaf) = v.leaf_n[tree] + 1;
    nd_w<P>(v, nb + leaf) = v.leaf_w[tree] + val;
    v.used[tree] = blk + 1;
    v.need[tree] = 0;
    v.cnt[(size_t)tree * C_NCNT + C_NN] += 1;
    v.cnt[(size_t)tree * C_NCNT + C_HWM] = max(v.cnt[(size_t)tree * C_NCNT + C_HWM], (int64_t)(blk + 1));
  }
}

// ----------------------------------------------------------------------------
// kernel: the network replies of the threaded search, slot by slot (mcts.py:360-365): create_children,
// backup (n += 1, w += v on the leaf and its path), unlock, vl -= 1 on the path — and, while the
// search has sims left, refill the slot at once (the rolling schedule above).  Read-modify-write:
// earlier slots of the same tree have changed the shared ancestors.  Pending leaves of trees that
// are not searching (a _set_node expansion, slot 0, path length 0) are completed without a refill.
// ----------------------------------------------------------------------------
template <class G, int TB, int S>
__device__ __forceinline__ void expand_vl_body(View v, const float *probs0, const float *values0,
                                               const float *probs1, const float *values1);

template <class G, int TB = 64, int S = kCopies<TB>>
__global__ __launch_bounds__(TB) void k_expand_vl(View v, const float *probs0, const float *values0,
                                                  const float *probs1, const float *values1) {
  expand_vl_body<G, TB, S>(v, probs0, values0, probs1, values1);
}

// The same held to 96 registers (SPMCTS_EXPAND_CO=1, a timing variant): its waves then fit on a SIMD
// beside a trunk wave (416 registers) instead of waiting for the trunk workgroup to retire, at the
// price of register spills on the dependent chain.
template <class G>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void k_expand_vl_co(
    View v, const float *probs0, const float *values0, const float *probs1, const float *values1) {
  expand_vl_body<G, 64, 0>(v, probs0, values0, probs1, values1);
}

template <class G, int TB, int S>
__device__ __forceinline__ void expand_vl_body(View v, const float *probs0, const float *values0,
                                               const float *probs1, const float *values1) {
  constexpr int P = G::APAD;
  constexpr int GPB = TB / P;
  constexpr int KMAX = P;  // slots whose records one lane each prefetches (spmcts_arena_create: K <= P)
  constexpr int S1 = S > 0 ? S : 4;
  __shared__ int32_t s_node[GPB][G::MAXD], s_n[GPB][G::MAXD], s_vl[GPB][G::MAXD], s_cs[GPB][G::MAXD];
  __shared__ double s_w[GPB][G::MAXD];
  __shared__ __attribute__((aligned(16))) int32_t s_tag[GPB][S1];
  __shared__ __attribute__((aligned(16))) char s_rec[S > 0 ? GPB : 1][S > 0 ? S : 1][NodeRec<P>::BYTES];
  // the prefetched path nodes (k < P) and network outputs of each slot, per tree group; each LDS word
  // is written and later read by the same wave (LDS operations of a wave stay in order)
  __shared__ int32_t s_pnode[GPB][KMAX][P];
  __shared__ float s_pr[GPB][KMAX][P];
  __shared__ float s_vr[GPB][KMAX];
  const int lane = threadIdx.x & (P - 1);
  const int grp = threadIdx.x / P;
  const int gbase = (threadIdx.x & 63) & ~(P - 1);
  const int tree = (blockIdx.x * blockDim.x + threadIdx.x) / P;
  if (tree >= v.T) return;
  const PathLds pl{s_node[grp], s_n[grp], s_vl[grp], s_cs[grp], s_w[grp]};
  BlockCache<P, S> bc;
  bc.tag = s_tag[grp];
  bc.rec = S > 0 ? &s_rec[grp][0][0] : nullptr;
  const int K = v.K;
  const size_t nb = nbase<G>(v, tree);
  const size_t bb = (size_t)tree * v.cap;
  // prefetch (independent loads, one round trip): lane j < K holds pending slot j's record, every lane
  // the j-th path node of each slot; the tree's counters
  const int psl = tree * K + (lane < K ? lane : 0);
  const int my_need = lane < K ? (int)v.need[psl] : 0;
  const int my_srow = v.srow[psl], my_leaf = v.leaf[psl], my_plen = v.plen[psl];
  const int my_mover = v.lmover[psl];
  const uint64_t my_pos = v.lpos[psl], my_neg = v.lneg[psl];
  {
    int pn[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j)
      pn[j] = (j < K && lane < G::MAXD) ? v.pnode[(size_t)(tree * K + j) * G::MAXD + lane] : 0;
#pragma unroll
    for (int j = 0; j < KMAX; ++j) s_pnode[grp][j][lane] = pn[j];
  }
  if (!group_or<P>(my_need)) return;
  const int limit = min(v.budget[tree], v.iters);
  int started = v.tstarted[tree];
  const bool refill = started < limit;
  int used = v.used[tree];
  const bool noise = v.noise_on[tree] != 0;
  const double nz = (noise && lane < G::A) ? v.noise[(size_t)tree * P + lane] : 0.0;
  TreeRng rng;
  TreeRoot R;
  if (refill) {
    rng_load(v, tree, rng);
    R = load_root<G>(v, tree);
  }
  // the network outputs of the pending slots (second round trip: they depend on the rows)
  {
    float pr[KMAX], vr[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      const int nj = __shfl(my_need, gbase + j, 64), row = __shfl(my_srow, gbase + j, 64);
      pr[j] = 0.f;
      vr[j] = 0.f;
      if (j < K && nj) {
        const bool s1 = row >= v.seg1;
        const float *prow = s1 ? probs1 + (size_t)(row - v.seg1) * G::A : probs0 + (size_t)row * G::A;
        if (lane < G::A) pr[j] = prow[lane];
        vr[j] = s1 ? values1[row - v.seg1] : values0[row];
      }
    }
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      s_pr[grp][j][lane] = pr[j];
      if (lane == 0) s_vr[grp][j] = vr[j];
    }
  }
  bool terr = false;
  SimCnt sc;
#ifdef SPMCTS_TREE_PROF
  sc.prof_begin();
#endif
  // one copy of the slot body (a rolled loop: the unrolled form was 70 KB of code, more than the
  // instruction cache two CUs share, for a kernel that runs one wave per CU on a latency chain)
#pragma unroll 1
  for (int j = 0; j < K; ++j) {
    const int ps = tree * K + j;
    if (__shfl(my_need, gbase + j, 64)) {
      const int leaf = __shfl(my_leaf, gbase + j, 64), plen = __shfl(my_plen, gbase + j, 64);
      const int mover = __shfl(my_mover, gbase + j, 64);
      const uint64_t lpos = __shfl(my_pos, gbase + j, 64), lneg = __shfl(my_neg, gbase + j, 64);
      const int blk = used;
      if (blk >= v.cap) {  // sticky SPMCTS_ERR_POOL; the counters of the slots done so far are still flushed
        if (lane == 0) set_err(v, SPMCTS_ERR_POOL);
        break;
      }
      ++used;
      const float pnew = lane < G::A ? s_pr[grp][j][lane] : 0.f;
      const uint32_t vmnew = legal_mask<G>(Board{lpos, lneg});
      {
        const size_t ci = nb + (size_t)blk * P + lane;
        nd_n<P>(v, ci) = 0;
        nd_w<P>(v, ci) = 0.0;
        nd_p<P>(v, ci) = pnew;
        nd_c<P>(v, ci) = -1;
        nd_f<P>(v, ci) = 0;
        nd_vl<P>(v, ci) = 0;
      }
      const double val = (double)s_vr[grp][j] * (double)mover;
      if (!refill) {
        // no sims in this launch (nothing copied, the root not in registers): read-modify-write backup of the
        // path (distinct nodes): one lane per path node, the node ids prefetched; a node's depth fixes its
        // lane, so the slots' updates of a shared ancestor are one lane's program order
        for (int k = lane; k < plen; k += P) {
          const size_t idx = nb + (k < P ? s_pnode[grp][j][k] : v.pnode[(size_t)ps * G::MAXD + k]);
          nd_n<P>(v, idx) += 1;
          nd_w<P>(v, idx) += val;
          nd_vl<P>(v, idx) -= 1;
        }
        if (lane == 0) {
          nd_vm<P>(v, bb + blk) = vmnew;
          nd_c<P>(v, nb + leaf) = blk;
          nd_n<P>(v, nb + leaf) += 1;
          nd_w<P>(v, nb + leaf) += val;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      } else {
        // with sims in this launch: the root and its children from the registers (TreeRoot), deeper path
        // nodes and the leaf from their block copies when copied (write-through), else read-modify-write in
        // global memory after a fence if an uncopied store is outstanding (BlockCache)
        if (lane == 0) nd_vm<P>(v, bb + blk) = vmnew;
        if (bc.insert_new(blk, lane, pnew, vmnew) == kUncached) bc.dirty = true;
        const int a1 = plen > 1 ? s_pnode[grp][j][1] - R.cb * P : 0;  // path node 1: root child a1
        const int r1n = __shfl(R.cn, gbase + a1, 64), r1vl = __shfl(R.cvl, gbase + a1, 64);
        const double r1w = __shfl(R.cw, gbase + a1, 64);
        bc.fence_if_dirty();
        int unc = 0;
        for (int k = lane; k < plen; k += P) {
          const int nk = k < P ? s_pnode[grp][j][k] : v.pnode[(size_t)ps * G::MAXD + k];
          const size_t idx = nb + nk;
          if (k == 0) {  // the root
            nd_n<P>(v, idx) = R.n + 1;
            nd_w<P>(v, idx) = R.w + val;
            nd_vl<P>(v, idx) = R.vl - 1;
          } else if (k == 1) {  // root child a1
            nd_n<P>(v, idx) = r1n + 1;
            nd_w<P>(v, idx) = r1w + val;
            nd_vl<P>(v, idx) = r1vl - 1;
          } else {
            const int ck = bc.find(nk / P);
            if (ck >= 0) {
              int32_t &n = bc.template at<int32_t>(ck, NodeRec<P>::N, nk % P);
              double &w = bc.template at<double>(ck, NodeRec<P>::W, nk % P);
              int32_t &vl = bc.template at<int32_t>(ck, NodeRec<P>::VL, nk % P);
              const int32_t n1 = n + 1, vl1 = vl - 1;
              const double w1 = w + val;
              n = n1;
              w = w1;
              vl = vl1;
              nd_n<P>(v, idx) = n1;
              nd_w<P>(v, idx) = w1;
              nd_vl<P>(v, idx) = vl1;
            } else {
              nd_n<P>(v, idx) += 1;
              nd_w<P>(v, idx) += val;
              nd_vl<P>(v, idx) -= 1;
              unc = 1;
            }
          }
        }
        // the leaf: a root child (plen 1, registers: lane la), or a deeper node
        const int la = leaf - R.cb * P;
        if (plen == 1) {
          if (lane == la) {
            nd_c<P>(v, nb + leaf) = blk;
            nd_n<P>(v, nb + leaf) = R.cn + 1;
            nd_w<P>(v, nb + leaf) = R.cw + val;
          }
        } else {
          const int cl = bc.find(leaf / P);  // group-uniform
          if (lane == 0) {
            if (cl >= 0) {
              bc.template at<int32_t>(cl, NodeRec<P>::C, leaf % P) = blk;
              int32_t &n = bc.template at<int32_t>(cl, NodeRec<P>::N, leaf % P);
              double &w = bc.template at<double>(cl, NodeRec<P>::W, leaf % P);
              const int32_t n1 = n + 1;
              const double w1 = w + val;
              n = n1;
              w = w1;
              nd_c<P>(v, nb + leaf) = blk;
              nd_n<P>(v, nb + leaf) = n1;
              nd_w<P>(v, nb + leaf) = w1;
            } else {
              nd_c<P>(v, nb + leaf) = blk;
              nd_n<P>(v, nb + leaf) += 1;
              nd_w<P>(v, nb + leaf) += val;
            }
          }
          unc |= cl == kUncached;
        }
        if (group_or<P>(unc)) bc.dirty = true;
      }
      if (lane == 0) {
        v.used[tree] = blk + 1;
        v.need[ps] = 0;
      }
      sc.nn += 1;
      sc.hwm = max(sc.hwm, (int64_t)(blk + 1));
      if (refill && plen > 0) {  // the root is the path's first node
        R.n += 1;
        R.vl -= 1;
        R.w += val;
      }
      if (refill && plen > 1) {  // path node 1 is a root child: its copy in registers
        if (lane == s_pnode[grp][j][1] - R.cb * P) {
          R.cn += 1;
          R.cw += val;
          R.cvl -= 1;
        }
      } else if (refill && plen == 1) {  // the leaf itself is a root child
        if (lane == leaf - R.cb * P) {
          R.cc = blk;
          R.cn += 1;
          R.cw += val;
        }
      }
      if (refill && fill_slot_vl<G, S>(v, tree, j, limit, started, R, rng, terr, pl, noise, nz, sc, bc) == SIM_ERROR)
        break;  // sticky SPMCTS_ERR_STATE; counters flushed below
    }
  }
  if (lane == 0) {
#ifdef SPMCTS_TREE_PROF
    sc.prof_flush(8);
#endif
    sc.flush(v.cnt + (size_t)tree * C_NCNT);
  }
  if (refill && lane == 0) {
    v.tstarted[tree] = started;
    if (terr) set_err(v, SPMCTS_ERR_TAPE);
    rng_store(v, tree, rng);
  }
}

// ----------------------------------------------------------------------------
// _play (mcts.py:272-299): choose the move from root visit counts
// ----------------------------------------------------------------------------
struct PlayOut {
  int action;
  bool recorded;
  double q;
  uint8_t qf64;
};

// numpy kahan_sum used by RandomState.choice's validation
__device__ __forceinline__ double kahan_sum(const double *p, int n) {
  double s = p[0], c = 0.0;
  for (int i = 1; i < n; ++i) {
    const double y = p[i] - c;
    const double t = s + y;
    c = (t - s) - y;
    s = t;
  }
  return s;
}

template <class G>
__device__ PlayOut play_move_choice(const View &v, int tree, double temp, float *probs_out) {
  constexpr int P = G::APAD;
  const size_t nb = nbase<G>(v, tree);
  const int root = v.root[tree];
  const int cb = nd_c<P>(v, nb + root);
  PlayOut o{0, false, 0.0, 0};
  int n[G::A];
  for (int j = 0; j < G::A; ++j) n[j] = cb >= 0 ? nd_n<P>(v, nb + (size_t)cb * P + j) : 0;
  double t = temp;
  if (v.evaluate) t = t / 20.0;
  const double inv = 1.0 / t;
  double pp[G::A];
  for (int j = 0; j < G::A; ++j) pp[j] = inv == 1.0 ? (double)n[j] : pow((double)n[j], inv);
  double s = 0.0;
  for (int j = 0; j < G::A; ++j) s = s + pp[j];
  double pr[G::A];
  for (int j = 0; j < G::A; ++j) pr[j] = pp[j] / s;
  // np.random.choice(A, p) validation (ValueError -> argmax fallback, mcts.py:290-295)
  bool ok = true;
  for (int j = 0; j < G::A; ++j)
    if (pr[j] < 0.0 || pr[j] != pr[j]) ok = false;
  if (ok && fabs(kahan_sum(pr, G::A) - 1.0) > 1.4901161193847656e-08) ok = false;
  if (ok) {
    TreeRng r;
    rng_load(v, tree, r);
    bool terr = false;
    const double u = rng_next(v, r, &terr);
    rng_store(v, tree, r);
    if (terr) set_err(v, SPMCTS_ERR_TAPE);
    double cdf[G::A];
    double c = 0.0;
    for (int j = 0; j < G::A; ++j) {
      c = c + pr[j];
      cdf[j] = c;
    }
    const double last = cdf[G::A - 1];
    int a = 0;
    for (int j = 0; j < G::A; ++j) {
      cdf[j] = cdf[j] / last;
      if (cdf[j] <= u) a = j + 1;  // searchsorted(u, side='right') on a non-decreasing cdf
    }
    if (a >= G::A) a = G::A - 1;
    o.action = a;
    o.recorded = true;
    for (int j = 0; j < G::A; ++j) probs_out[j] = (float)pr[j];
    const int rn = nd_n<P>(v, nb + root);
    if (v.K > 1) {
      // q (mcts.py:59-62) with the root's virtual loss, nonzero after a leaked sim (:349-354)
      const int rvl = nd_vl<P>(v, nb + root);
      o.q = (rn + rvl) ? (nd_w<P>(v, nb + root) - (double)rvl) / (double)(rn + rvl) : 0.0;
    } else {
      o.q = rn ? nd_w<P>(v, nb + root) / (double)rn : 0.0;
    }
    o.qf64 = nd_f<P>(v, nb + root);
  } else {
    int best = 0;
    for (int j = 1; j < G::A; ++j)
      if (n[j] > n[best]) best = j;
    o.action = best;
  }
  v.noise_on[tree] = 0;  // remove_noise (mcts.py:55-57)
  v.cnt[(size_t)tree * C_NCNT + C_MOVES] += 1;
  return o;
}

template <class G>
__device__ __forceinline__ void write_state(Board b, int8_t *dst) {
  for (int x = 0; x < G::W; ++x)
    for (int y = 0; y < G::H; ++y) dst[x * G::H + y] = cell_value<G>(b, x, y);
}

template <class G>
__global__ void k_search_end(View v, int n_active, double temp, int32_t *actions, int8_t *states, float *tprobs,
                             double *qs, uint8_t *qf64, uint8_t *recorded) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_active) return;
  const int tree = v.active[i];
  if (tree < 0) return;
  float pr[G::A];
  const PlayOut o = play_move_choice<G>(v, tree, temp, pr);
  actions[i] = o.action;
  recorded[i] = o.recorded ? 1 : 0;
  qs[i] = o.q;
  qf64[i] = o.qf64;
  for (int j = 0; j < G::A; ++j) tprobs[(size_t)i * G::A + j] = o.recorded ? pr[j] : 0.f;
  write_state<G>(Board{v.rpos[tree], v.rneg[tree]}, states + (size_t)i * G::CELLS);
}

// _set_node (mcts.py:201-209) for one tree; returns false on an illegal action.
template <class G>
__device__ bool set_node(const View &v, int tree, int a) {
  constexpr int P = G::APAD;
  const size_t nb = nbase<G>(v, tree);
  const size_t bb = (size_t)tree * v.cap;
  const int root = v.root[tree];
  const int cb = nd_c<P>(v, nb + root);
  if (cb < 0 || a < 0 || a >= G::A || !((nd_vm<P>(v, bb + cb) >> a) & 1u)) {
    set_err(v, SPMCTS_ERR_ACTION);
    return false;
  }
  const int child = cb * P + a;
  const int rp = v.rplayer[tree];
  Board b{v.rpos[tree], v.rneg[tree]};
  int rew = 0, done = 0;
  step<G>(b, a, rp, &rew, &done);
  if (nd_n<P>(v, nb + child) == 0) {
    int64_t *cnt = v.cnt + (size_t)tree * C_NCNT;
    cnt[C_SETNODE] += 1;
    if (done) {
      const double val = terminal_value(v, tree, Board{v.rpos[tree], v.rneg[tree]}, rew * rp);
      nd_n<P>(v, nb + child) = 1;
      nd_w<P>(v, nb + child) = nd_w<P>(v, nb + child) + val;
      if (v.tstrong[tree]) nd_f<P>(v, nb + child) = 1;
    } else {
      const int ps = tree * v.K;  // pending slot 0 of the tree
      v.plen[ps] = 0;
      v.leaf[ps] = child;
      v.leaf_n[ps] = 0;
      v.leaf_w[ps] = nd_w<P>(v, nb + child);
      v.lpos[ps] = b.pos;
      v.lneg[ps] = b.neg;
      v.lmover[ps] = (int8_t)rp;
      v.need[ps] = 1;
    }
  }
  v.root[tree] = child;
  v.rpos[tree] = b.pos;
  v.rneg[tree] = b.neg;
  v.rplayer[tree] = (int8_t)(-rp);
  return true;
}

template <class G>
__global__ void k_play_action(View v, const int32_t *trees, const int32_t *actions, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = trees[i];
  if (t < 0 || t >= v.T) return;
  set_node<G>(v, t, actions[i]);
}

// ----------------------------------------------------------------------------
// games: SelfPlayer.play_episode state machine (selfplayworker.py:164-224)
// ----------------------------------------------------------------------------
template <class G>
__device__ void start_game(const View &v, int g, int64_t id, const float *priors) {
  const bool swap = (id & 1) != 0;  // swap_sides = not i % 2 == 0 (self_play_parallel.py:237)
  v.gpos[g] = 0;
  v.gneg[g] = 0;
  v.gply[g] = 0;
  v.gswap[g] = swap ? 1 : 0;
  v.gstate[g] = GS_ACTIVE;
  v.gresult[g] = 0;
  v.gid[g] = id;
  v.mv_count[2 * g] = 0;
  v.mv_count[2 * g + 1] = 0;
  // policy.reset(-1 if swap else 1), opposing.reset(1 if swap else -1)  (:175-176)
  reset_tree<G>(v, 2 * g, swap ? -1 : 1, priors ? priors : v.root_prior + 16 * v.tnet[2 * g]);
  reset_tree<G>(v, 2 * g + 1, swap ? 1 : -1, priors ? priors + G::A : v.root_prior + 16 * v.tnet[2 * g + 1]);
}

template <class G>
__global__ void k_games_start(View v, const int32_t *slots, const float *priors, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int g = slots[i];
  if (g < 0 || g >= v.G) {
    set_err(v, SPMCTS_ERR_STATE);
    return;
  }
  start_game<G>(v, g, v.gcnt[7] + i, priors ? priors + (size_t)i * 2 * G::A : nullptr);
}

__global__ void k_games_bump_id(View v, int n) { v.gcnt[7] += n; }

template <class G>
__global__ void k_games_begin_ply(View v) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= v.G) return;
  if (v.gstate[g] != GS_ACTIVE) {
    v.active[g] = -1;
    return;
  }
  // policy moves on even plies unless swap_sides (:178-183)
  const int mover = (v.gply[g] + v.gswap[g]) & 1;
  const int tree = 2 * g + mover;
  if (v.tkind[tree] != SPMCTS_PLAYER_MCTS) {  // hard-coded players do not search
    v.active[g] = -1;
    return;
  }
  v.active[g] = tree;
  draw_noise<G>(v, tree);
}

// Hard-coded opponents (games/general/hardcoded_players.py).  `own` = the player's stones,
// `enemy` = the other side's, in the player's own env frame (its stones are +1: play_move passes
// player * -1 to the opposing policy, selfplayworker.py:221-224); `look` = the player sign given to
// reset(player) (selfplayworker.py:175-176), which OneStepLookahead uses as "self.player".
// OneStepLookahead (:18-33): first any move after which step(a, look) ends the game, then any move
// after which step(a, -look) does, else uniform over the legal moves.  Random (:45-49): uniform.
// The uniform draw uses the tree's Philox stream (the reference's `random` module stream is not
// reproduced).
template <class G>
__device__ int hardcoded_move(const View &v, int tree, int kind, Board envb, int look) {
  const uint32_t legal = legal_mask<G>(envb);
  if (kind == SPMCTS_PLAYER_LOOKAHEAD) {
    for (int pass = 0; pass < 2; ++pass) {
      const int who = pass == 0 ? look : -look;
      for (int a = 0; a < G::A; ++a) {
        if (!((legal >> a) & 1u)) continue;
        Board b = envb;
        int rew = 0, done = 0;
        step<G>(b, a, who, &rew, &done);
        if (done) return a;
      }
    }
  }
  const int n = popc((uint64_t)legal);
  if (n == 0) return 0;
  TreeRng r;
  rng_load(v, tree, r);
  bool terr = false;
  const double u = rng_next(v, r, &terr);
  rng_store(v, tree, r);
  if (terr) set_err(v, SPMCTS_ERR_TAPE);
  int k = (int)(u * (double)n);
  if (k >= n) k = n - 1;
  for (int a = 0; a < G::A; ++a)
    if ((legal >> a) & 1u) {
      if (k == 0) return a;
      --k;
    }
  return 0;
}

template <class G>
__global__ void k_games_end_ply(View v) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= v.G) return;
  if (v.gstate[g] != GS_ACTIVE) return;
  const int mover = (v.gply[g] + v.gswap[g]) & 1;
  const int tree = 2 * g + mover;
  const int m = v.mv_count[tree];
  float pr[G::A];
  PlayOut o{0, false, 0.0, 0};
  const int kind = v.tkind[tree];
  if (kind == SPMCTS_PLAYER_MCTS) {
    o = play_move_choice<G>(v, tree, 1.0, pr);
  } else {
    const Board envb = mover == 0 ? Board{v.gpos[g], v.gneg[g]} : Board{v.gneg[g], v.gpos[g]};
    o.action = hardcoded_move<G>(v, tree, kind, envb, v.rplayer[tree]);
  }
  if (o.recorded && v.record) {
    if (m < G::MAXM) {
      const size_t rec = (size_t)tree * G::MAXM + m;
      write_state<G>(Board{v.rpos[tree], v.rneg[tree]}, v.mv_state + rec * G::CELLS);
      for (int j = 0; j < G::A; ++j) v.mv_probs[rec * G::A + j] = pr[j];
      v.mv_q[rec] = o.q;
      v.mv_qf64[rec] = o.qf64;
      v.mv_count[tree] = m + 1;
    } else {
      set_err(v, SPMCTS_ERR_STATE);
    }
  }
  // env.step in the policy's frame (play_move :221-224): policy plays +1, opponent -1
  const int p_env = mover == 0 ? 1 : -1;
  Board gb{v.gpos[g], v.gneg[g]};
  int rew = 0, done = 0;
  const int st = step<G>(gb, o.action, p_env, &rew, &done);
  if (st != STEP_OK) set_err(v, SPMCTS_ERR_ACTION);
  v.gpos[g] = gb.pos;
  v.gneg[g] = gb.neg;
  v.gply[g] += 1;
  if (done) {
    v.gstate[g] = GS_DONE;
    v.gresult[g] = (int8_t)(rew * p_env);  // r = r * player (:218)
    return;  // both trees are discarded with the game
  }
  if (v.tkind[2 * g] == SPMCTS_PLAYER_MCTS) set_node<G>(v, 2 * g, o.action);
  if (v.tkind[2 * g + 1] == SPMCTS_PLAYER_MCTS) set_node<G>(v, 2 * g + 1, o.action);
}

// finished games: offsets into the export ring + refill ids (single block, slot order)
template <class G>
__global__ __launch_bounds__(1024) void k_games_finish_scan(View v, int refill, int32_t *out) {
  __shared__ int32_t s_rec[1024];
  __shared__ int32_t s_fin[1024];
  const int tid = threadIdx.x;
  const int Gn = v.G;
  const int chunk = (Gn + 1023) / 1024;
  const int lo = min(Gn, tid * chunk), hi = min(Gn, lo + chunk);
  int rec = 0, fin = 0;
  for (int g = lo; g < hi; ++g)
    if (v.gstate[g] == GS_DONE) {
      rec += v.mv_count[2 * g] + v.mv_count[2 * g + 1];
      fin += 1;
    }
  s_rec[tid] = rec;
  s_fin[tid] = fin;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int a1 = tid >= off ? s_rec[tid - off] : 0;
    const int a2 = tid >= off ? s_fin[tid - off] : 0;
    __syncthreads();
    s_rec[tid] += a1;
    s_fin[tid] += a2;
    __syncthreads();
  }
  const int base_rec = v.ex_count[0];
  int r0 = base_rec + s_rec[tid] - rec;
  int f0 = s_fin[tid] - fin;
  // per-game: record offset and finish index (for refill ids) in gscratch[2*g], [2*g+1]
  for (int g = lo; g < hi; ++g)
    if (v.gstate[g] == GS_DONE) {
      v.gscratch[2 * g] = r0;
      v.gscratch[2 * g + 1] = f0;
      r0 += v.mv_count[2 * g] + v.mv_count[2 * g + 1];
      f0 += 1;
    }
  __syncthreads();
  if (tid == 0) {
    const int total_rec = s_rec[1023], total_fin = s_fin[1023];
    int64_t started = v.gcnt[7];
    int64_t limit = v.gcnt[8];
    int64_t can = 0;
    if (refill) {
      if (limit < 0) {
        can = total_fin;
      } else {
        const int64_t room = limit - started;
        can = room < 0 ? 0 : (room < (int64_t)total_fin ? room : (int64_t)total_fin);
      }
    }
    v.gscratch[2 * Gn] = (int32_t)can;     // refills this ply
    v.gscratch[2 * Gn + 1] = (int32_t)(started & 0x7fffffff);
    ((int64_t *)(v.gscratch + 2 * Gn + 2))[0] = started;
    v.gcnt[7] = started + can;
    v.gcnt[0] += total_fin;
    if (base_rec + total_rec > v.ex_cap) atomicOr(v.err, SPMCTS_ERR_EXPORT);
    v.ex_count[0] = min(v.ex_cap, base_rec + total_rec);
    v.gcnt[9] += min(total_rec, v.ex_cap - base_rec);
    if (out) {
      out[0] = total_fin;
      out[1] = v.ex_count[0];
    }
  }
}

template <class G>
__global__ void k_games_finish_apply(View v) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= v.G) return;
  if (v.gstate[g] != GS_DONE) return;
  const int r = v.gresult[g];
  const int swap = v.gswap[g];
  // results breakdown (self_play_parallel.py:302-327): reward in the policy's view
  atomicAdd((unsigned long long *)&v.gcnt[1 + swap * 3 + (r == 1 ? 0 : (r == 0 ? 1 : 2))], 1ull);
  // push_to_queue: policy's moves with r, then opposing's with -r (selfplayworker.py:186-190)
  int off = v.gscratch[2 * g];
  for (int side = 0; side < 2; ++side) {
    const int tree = 2 * g + side;
    const float z = side == 0 ? (float)r : (float)(-r);
    const int m = v.mv_count[tree];
    for (int k = 0; k < m; ++k, ++off) {
      if (off >= v.ex_cap) continue;
      const size_t src = (size_t)tree * G::MAXM + k;
      for (int c = 0; c < G::CELLS; ++c) v.ex_state[(size_t)off * G::CELLS + c] = v.mv_state[src * G::CELLS + c];
      for (int j = 0; j < G::A; ++j) v.ex_probs[(size_t)off * G::A + j] = v.mv_probs[src * G::A + j];
      v.ex_q[off] = v.mv_q[src];
      v.ex_qf64[off] = v.mv_qf64[src];
      v.ex_z[off] = z;
      v.ex_game[off] = v.gid[g];
    }
  }
  const int fin_idx = v.gscratch[2 * g + 1];
  const int can = v.gscratch[2 * v.G];
  const int64_t started = ((const int64_t *)(v.gscratch + 2 * v.G + 2))[0];
  if (fin_idx < can) {
    start_game<G>(v, g, started + fin_idx, nullptr);
  } else {
    v.gstate[g] = GS_IDLE;
  }
}

__global__ void k_export(View v, int A, int cells, int8_t *st, float *pr, double *q, uint8_t *qf, float *z, int64_t *gid,
                         int max_records, int32_t *count_out) {
  const int n = min(v.ex_count[0], max_records);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && count_out) count_out[0] = n;
  if (i >= n) return;
  for (int c = 0; c < cells; ++c) st[(size_t)i * cells + c] = v.ex_state[(size_t)i * cells + c];
  for (int j = 0; j < A; ++j) pr[(size_t)i * A + j] = v.ex_probs[(size_t)i * A + j];
  q[i] = v.ex_q[i];
  qf[i] = v.ex_qf64[i];
  z[i] = v.ex_z[i];
  gid[i] = v.ex_game[i];
}

__global__ void k_export_clear(View v) { v.ex_count[0] = 0; }

// ----------------------------------------------------------------------------
// stand-alone kernels
// ----------------------------------------------------------------------------
template <class G>
__global__ void k_env_step(const int8_t *boards, const int32_t *actions, const int8_t *players, const uint8_t *over,
                           int n, int8_t *out, int8_t *reward, uint8_t *done, int8_t *status, uint8_t *valid) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Board b = from_cells<G>(boards + (size_t)i * G::CELLS);
  int rew = 0, dn = 0, st;
  if (over && over[i]) {
    st = STEP_GAME_OVER;
    dn = 1;
  } else {
    st = step<G>(b, actions[i], players[i], &rew, &dn);
  }
  for (int x = 0; x < G::W; ++x)
    for (int y = 0; y < G::H; ++y) out[(size_t)i * G::CELLS + x * G::H + y] = cell_value<G>(b, x, y);
  reward[i] = (int8_t)rew;
  done[i] = (uint8_t)dn;
  status[i] = (int8_t)st;
  const uint32_t lm = legal_mask<G>(b);
  for (int a = 0; a < G::A; ++a) valid[(size_t)i * G::A + a] = (lm >> a) & 1u;
}

// table network (oracle/table_net.py) from leaf rows
template <class G>
__global__ void k_table_net(const void *leaves, int fmt, int layout, int n, uint64_t salt, const uint64_t *salts,
                            float *probs, float *values) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t h = 0xCBF29CE484222325ull;
  for (int cell = 0; cell < G::CELLS; ++cell) {
    int c = 0;
    if (fmt == SPMCTS_LEAF_BOARD_I64) {
      const int64_t val = ((const int64_t *)leaves)[(size_t)i * G::CELLS + cell];
      c = val == 1 ? 1 : (val == -1 ? 2 : 0);
    } else {
      size_t i1, i2;
      if (layout == SPMCTS_NHWC) {
        i1 = ((size_t)i * G::CELLS + cell) * 3 + 1;
        i2 = i1 + 1;
      } else {
        i1 = (size_t)i * 3 * G::CELLS + G::CELLS + cell;
        i2 = i1 + G::CELLS;
      }
      float own, opp;
      if (fmt == SPMCTS_LEAF_F32) {
        own = ((const float *)leaves)[i1];
        opp = ((const float *)leaves)[i2];
      } else {
        own = ((const uint16_t *)leaves)[i1] ? 1.f : 0.f;
        opp = ((const uint16_t *)leaves)[i2] ? 1.f : 0.f;
      }
      c = own != 0.f ? 1 : (opp != 0.f ? 2 : 0);
    }
    h = (h ^ (uint64_t)(c + 3 * cell + 1)) * 0x100000001B3ull;
  }
  h ^= salts ? salts[i] : salt;
  uint32_t k[G::A];
  uint32_t tot = 0;
  for (int j = 0; j < G::A; ++j) {
    k[j] = 1u + (uint32_t)((splitmix64(h + (uint64_t)j) >> 40) & 0xFFFFull);
    tot += k[j];
  }
  const float ft = (float)tot;
  for (int j = 0; j < G::A; ++j) probs[(size_t)i * G::A + j] = __fdiv_rn((float)k[j], ft);
  const int raw = (int)((splitmix64(h ^ 0x5DEECE66Dull) >> 40) & 0xFFFFull) - 32768;
  values[i] = __fdiv_rn((float)raw, 32768.0f);
}

__global__ void k_copy_probe(const float4 *src, float4 *dst, size_t n4) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n4; i += stride) dst[i] = src[i];
}

// ----------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------
struct spmcts_arena {
  spmcts_config cfg;
  int device;
  int A, W, H, P, cells, maxd, maxm;
  View v;
  std::vector<void *> allocs;
  int n_active;  // active-set size for select / search_end
  int tree_block;  // threads per workgroup of the threaded tree kernels: 64 (64/P trees per wave) or P (one)
  // cross-lane dedup (spmcts_set_leaf_peer): a follower's leader, a leader's followers, and the events that
  // order the two streams (leader: ev_ins after its table of a step; follower: ev_rows after its rows,
  // ev_push after the leader's outputs reached its rows)
  spmcts_arena *peer = nullptr;
  std::vector<spmcts_arena *> followers;
  hipEvent_t ev_ins = nullptr, ev_rows = nullptr, ev_push = nullptr, ev_lead = nullptr;
  hipStream_t push_stream = nullptr;  // a follower's stream for k_peer_push (spmcts_peer_push)
  bool peer_step = false;  // the last launch_rows of this follower used the leader's table
  bool push_pending = false;  // the leader's stream has not yet waited for this follower's last push
  // evaluation cache (spmcts_set_eval_cache): its allocations, and whether the last launch_rows consulted it
  // (the next expand then runs k_cache_io)
  std::vector<void *> cache_allocs;
  bool cache_step = false;
  bool cache_shared_step = false;  // that launch used the leader's table (cache_view)
  const uint64_t *cache_tab = nullptr;  // the table that launch looked its keys up in
};

// The evaluation-cache table of a launch: a follower lane (spmcts_set_leaf_peer) whose leader runs a cache of
// the same window, one generation apart at most, uses the leader's table -- one table for the GPU's lanes, so a
// position either lane evaluated serves both -- and inserts only the rows its own network evaluated; otherwise
// the arena's own table.
#ifdef SPMCTS_AB
// SPMCTS_CACHE_SHARE=0 (A/B library): follower lanes keep a table of their own (the first form)
static bool cache_share_off() {
  static const bool v = getenv("SPMCTS_CACHE_SHARE") && strcmp(getenv("SPMCTS_CACHE_SHARE"), "0") == 0;
  return v;
}
#else
static constexpr bool cache_share_off() { return false; }
#endif

static bool cache_view(const spmcts_arena *h, View &v) {
  v.cshared = 0;
  const spmcts_arena *p = h->peer;
  if (cache_share_off()) return false;
  if (!v.cwin || !p || p->v.cwin != v.cwin || !p->v.crec) return false;
  const int d = (int)(v.cgen - p->v.cgen);
  if (d < -1 || d > 1) return false;
  v.crec = p->v.crec;
  v.cmask = p->v.cmask;
  v.cshared = 1;
  return true;
}

static int geometry(const spmcts_config *c, int *A, int *P, int *cells, int *maxd, int *maxm) {
  if (c->game == SPMCTS_CONNECT4 && c->width == 7 && c->height == 6) {
    *A = C4::A; *P = C4::APAD; *cells = C4::CELLS; *maxd = C4::MAXD; *maxm = C4::MAXM;
    return 0;
  }
  if (c->game == SPMCTS_TICTACTOE && c->width == 3 && c->height == 3) {
    *A = TTT::A; *P = TTT::APAD; *cells = TTT::CELLS; *maxd = TTT::MAXD; *maxm = TTT::MAXM;
    return 0;
  }
  return fail(-2, "unsupported game/board size (instantiated: connect4 7x6, tictactoe 3x3)");
}

// worst-case node blocks per tree per game: root pseudo block + root children + one
// block per expansion; a tree searches at most ceil(cells/2) times and play_action
// expands at most once per ply.
static int default_cap(const spmcts_config *c, int cells) {
  const long long it = std::max(1, c->iterations);
  const long long cap = 2 + ((cells + 1) / 2) * it + cells + 2;
  return (int)std::min<long long>(cap, 1 << 26);
}

struct Plan {
  size_t off = 0;
  std::vector<std::pair<void **, size_t>> items;
  template <class T>
  void add(T **p, size_t count) {
    items.push_back({(void **)p, sizeof(T) * std::max<size_t>(count, 1)});
  }
  size_t total() const {
    size_t t = 0;
    for (auto &it : items) t += (it.second + 255) & ~size_t(255);
    return t;
  }
};

// device address of a field of node i (host side; off = the field's NodeRec offset in units of P bytes)
static const char *node_field(const spmcts_arena *h, int off, int elt, size_t i) {
  const size_t P = h->P;
  return h->v.nodes + (i / P) * 32 * P + off * P + (i % P) * elt;
}

static void plan_arena(spmcts_arena *h, Plan &pl) {
  View &v = h->v;
  const size_t T = v.T, P = h->P, cap = v.cap, G = v.G;
  pl.add(&v.nodes, T * cap * 32 * P);  // 32 * P bytes per child block (NodeRec)
  pl.add(&v.root, T);
  pl.add(&v.rpos, T);
  pl.add(&v.rneg, T);
  pl.add(&v.rplayer, T);
  pl.add(&v.used, T);
  pl.add(&v.gc_list, v.gc ? T * cap : 1);
  pl.add(&v.gc_map, v.gc ? T * cap : 1);
  pl.add(&v.tstarted, T);
  pl.add(&v.noise, T * P);
  pl.add(&v.noise_on, T);
  const size_t NS = v.NS;  // pending slots
  pl.add(&v.pnode, NS * h->maxd);
  pl.add(&v.pn, NS * h->maxd);
  pl.add(&v.pw, NS * h->maxd);
  pl.add(&v.plen, NS);
  pl.add(&v.leaf, NS);
  pl.add(&v.leaf_n, NS);
  pl.add(&v.leaf_w, NS);
  pl.add(&v.lpos, NS);
  pl.add(&v.lneg, NS);
  pl.add(&v.lmover, NS);
  pl.add(&v.need, NS);
  pl.add(&v.rng, T);
  pl.add((int64_t **)&v.tape_end, T);
  pl.add(&v.tape_cur, T);
  pl.add(&v.cnt, T * C_NCNT);
  pl.add(&v.active, std::max(T, G));
  pl.add(&v.row_tree, NS);
  pl.add(&v.srow, NS);
  pl.add(&v.row_count, 4);
  {
    size_t tab = 1;
    while (tab < 2 * NS) tab <<= 1;
    v.dmask = (int)(tab - 1);
    pl.add(&v.dtab, v.K > 1 ? tab : 1);
    pl.add(&v.dent, v.K > 1 ? NS : 1);
    pl.add(&v.down, v.K > 1 ? NS : 1);
    pl.add(&v.okey, v.K > 1 ? 2 * NS : 1);
    pl.add(&v.xpeer, v.K > 1 ? NS : 1);
  }
  pl.add(&v.root_prior, 32);  // [net][16]
  pl.add(&v.err, 4);
  pl.add(&v.gpos, G);
  pl.add(&v.gneg, G);
  pl.add(&v.gply, G);
  pl.add(&v.gswap, G);
  pl.add(&v.gstate, G);
  pl.add(&v.gresult, G);
  pl.add(&v.gid, G);
  pl.add(&v.mv_state, 2 * G * h->maxm * h->cells);
  pl.add(&v.mv_probs, 2 * G * h->maxm * h->A);
  pl.add(&v.mv_q, 2 * G * h->maxm);
  pl.add(&v.mv_qf64, 2 * G * h->maxm);
  pl.add(&v.mv_count, 2 * G);
  const size_t X = std::max<size_t>(64, 4 * G * h->maxm);
  v.ex_cap = (int32_t)X;
  pl.add(&v.ex_state, X * h->cells);
  pl.add(&v.ex_probs, X * h->A);
  pl.add(&v.ex_q, X);
  pl.add(&v.ex_qf64, X);
  pl.add(&v.ex_z, X);
  pl.add(&v.ex_game, X);
  pl.add(&v.ex_count, 4);
  pl.add(&v.gcnt, 16);
  pl.add(&v.gscratch, 2 * G + 8);
  pl.add(&v.tnet, T);
  pl.add(&v.tkind, T);
  pl.add(&v.budget, T);
  pl.add(&v.talpha, T);
  pl.add(&v.tstrong, T);
  pl.add(&v.tK, T);
}

static int setup_view(spmcts_arena *h, const spmcts_config *cfg) {
  int A, P, cells, maxd, maxm;
  if (geometry(cfg, &A, &P, &cells, &maxd, &maxm)) return -2;
  h->cfg = *cfg;
  h->A = A;
  h->P = P;
  h->cells = cells;
  h->maxd = maxd;
  h->maxm = maxm;
  h->W = cfg->width;
  h->H = cfg->height;
  View &v = h->v;
  memset(&v, 0, sizeof(v));
  v.T = cfg->n_trees;
  v.G = cfg->n_games;
  v.A = A;
  v.cap = cfg->blocks_per_tree > 0 ? cfg->blocks_per_tree : default_cap(cfg, cells);
  v.gc = v.cap < default_cap(cfg, cells) ? 1 : 0;  // below the worst case: recycle subtrees (k_compact)
  v.cpuct = cfg->cpuct;
  v.x = cfg->x_noise;
  v.alpha = cfg->alpha;
  v.strong = cfg->strong_play;
  v.evaluate = cfg->evaluate;
  v.rng_mode = cfg->rng_mode;
  v.leaf_format = cfg->leaf_format;
  v.leaf_layout = cfg->leaf_layout;
  v.K = std::max(1, cfg->search_threads);
  if (v.K > P) return fail(-3, "search_threads must not exceed the lane group (8 for connect4, 16 for tictactoe)");
  v.iters = std::max(1, cfg->iterations);
  v.NS = v.T * v.K;
  v.seg1 = v.NS;
  v.record = 1;
  v.sim = 0;
  if (v.T <= 0) return fail(-3, "n_trees must be > 0");
  if (v.G < 0 || 2 * (long long)v.G > v.T) return fail(-3, "games mode needs n_trees >= 2 * n_games");
  if (v.T > (1 << 24)) return fail(-3, "too many trees");
  if (v.K > 64 || (long long)v.T * v.K > (1 << 24)) return fail(-3, "search_threads too large");
  if (v.cap < 4) return fail(-3, "blocks_per_tree too small");
  if ((long long)v.cap * P >= (1ll << 31)) return fail(-3, "blocks_per_tree too large");
  return 0;
}

__global__ void k_rng_init(View v, uint64_t seed, uint64_t sub0) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= v.T) return;
  Philox s;
  rocrand_init(seed, sub0 + (uint64_t)t, 0ull, &s);
  v.rng[t] = s;
  v.tape_cur[t] = 0;
  ((int64_t *)v.tape_end)[t] = 0;
  for (int j = 0; j < v.K; ++j) v.need[(size_t)t * v.K + j] = 0;
  v.tstarted[t] = 0x3fffffff;
  v.noise_on[t] = 0;
  v.tnet[t] = 0;
  v.tkind[t] = SPMCTS_PLAYER_MCTS;
  v.budget[t] = 0x7fffffff;
  v.talpha[t] = v.alpha;
  v.tstrong[t] = (uint8_t)(v.strong ? 1 : 0);
  v.tK[t] = v.K;
  for (int k = 0; k < C_NCNT; ++k) v.cnt[(size_t)t * C_NCNT + k] = 0;
}

__global__ void k_games_init(View v) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g == 0) {
    for (int k = 0; k < 16; ++k) v.gcnt[k] = 0;
    v.gcnt[8] = -1;  // unlimited refill
    v.ex_count[0] = 0;
    v.err[0] = 0;
    v.row_count[0] = 0;
    v.row_count[1] = 0;
  }
  if (g >= v.G) return;
  v.gstate[g] = GS_IDLE;
  v.mv_count[2 * g] = 0;
  v.mv_count[2 * g + 1] = 0;
}

#define DISPATCH(h, KCALL)                                             \
  do {                                                                 \
    if ((h)->cfg.game == SPMCTS_CONNECT4) {                            \
      using GG = C4;                                                   \
      KCALL;                                                           \
    } else {                                                           \
      using GG = TTT;                                                  \
      KCALL;                                                           \
    }                                                                  \
  } while (0)

static inline int nblk(long long n, int b) { return (int)std::max<long long>(1, (n + b - 1) / b); }

__global__ void k_set_tape(View v, const int64_t *offsets) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= v.T) return;
  v.tape_cur[t] = offsets[t];
  ((int64_t *)v.tape_end)[t] = offsets[t + 1];
}

template <class G>
static int env_step_host_t(int8_t *board, int32_t action, int32_t player, int32_t *reward, int32_t *done) {
  Board b = from_cells<G>(board);
  int r = 0, d = 0;
  const int st = step<G>(b, action, player, &r, &d);
  for (int x = 0; x < G::W; ++x)
    for (int y = 0; y < G::H; ++y) board[x * G::H + y] = cell_value<G>(b, x, y);
  *reward = r;
  *done = d;
  return st;
}

extern "C" {

int spmcts_version(void) { return 1; }

const char *spmcts_last_error(void) { return g_last_error.c_str(); }

int spmcts_arena_bytes(const spmcts_config *cfg, uint64_t *bytes_out) {
  spmcts_arena tmp;
  if (setup_view(&tmp, cfg)) return -2;
  Plan pl;
  plan_arena(&tmp, pl);
  *bytes_out = pl.total();
  return 0;
}

int spmcts_arena_create(const spmcts_config *cfg, int device, spmcts_arena **out) {
  if (!cfg || !out) return fail(-1, "null argument");
  spmcts_arena *h = new spmcts_arena();
  h->device = device;
  h->n_active = 0;
  int rc = setup_view(h, cfg);
  if (rc) {
    delete h;
    return rc;
  }
#ifndef SPMCTS_AB
  for (const char *n : {"SPMCTS_TREE_BLOCK", "SPMCTS_EXPAND_CO", "SPMCTS_TREE_COPIES", "SPMCTS_PEER_PUSH",
                        "SPMCTS_CACHE_SHARE"})
    if (getenv(n)) {
      delete h;
      return fail(SPMCTS_ERR_AB_SWITCH, std::string(n) + " is a switch of the A/B library (make ab: libspmcts_ab.so)");
    }
#endif
  {
    // Threads per workgroup of the threaded tree kernels (SPMCTS_TREE_BLOCK): P = one tree per wave,
    // 64 = one wave of 64/P trees, 128..512 = 2..8 such waves.  A tree-kernel wave (~170 VGPRs) leaves no
    // room on its SIMD for a trunk wave (416 registers), so each tree workgroup keeps a whole CU away from
    // the other lane's trunk launch while it runs: fewer, fuller workgroups block fewer CUs.
#ifdef SPMCTS_AB
    const char *e = getenv("SPMCTS_TREE_BLOCK");  // A/B library only (64 measured best)
    const int tb = e ? atoi(e) : 64;
#else
    const int tb = 64;
#endif
    h->tree_block = (tb == h->P || (tb >= 64 && tb <= 512 && tb % 64 == 0)) ? tb : 64;
  }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete h;
    return fail(-1000 - (int)e, std::string("hipSetDevice: ") + hipGetErrorString(e));
  }
  Plan pl;
  plan_arena(h, pl);
  for (auto &it : pl.items) {
    void *p = nullptr;
    e = hipMalloc(&p, it.second);
    if (e != hipSuccess) {
      for (void *q : h->allocs) (void)hipFree(q);
      delete h;
      return fail(-1000 - (int)e, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    h->allocs.push_back(p);
    *it.first = p;
  }
  if (h->v.K > 1) (void)hipMemset(h->v.dtab, 0, sizeof(uint64_t) * ((size_t)h->v.dmask + 1));  // generation 0
  hipLaunchKernelGGL(k_rng_init, dim3(nblk(h->v.T, 256)), dim3(256), 0, 0, h->v, cfg->seed, cfg->subsequence0);
  hipLaunchKernelGGL(k_games_init, dim3(nblk(std::max(1, h->v.G), 256)), dim3(256), 0, 0, h->v);
  // default root prior: uniform (replaced by spmcts_set_root_prior)
  std::vector<float> pri(32, 0.f);
  for (int j = 0; j < h->A; ++j) pri[j] = pri[16 + j] = 1.0f / h->A;
  e = hipMemcpy(h->v.root_prior, pri.data(), 32 * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    for (void *q : h->allocs) (void)hipFree(q);
    delete h;
    return fail(-1000 - (int)e, std::string("arena init: ") + hipGetErrorString(e));
  }
  *out = h;
  return 0;
}

int spmcts_arena_destroy(spmcts_arena *h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  (void)spmcts_set_leaf_peer(h, nullptr);
  for (spmcts_arena *f : h->followers) {  // a destroyed leader leaves its followers lane-local
    f->peer = nullptr;
    f->peer_step = false;
  }
  for (hipEvent_t e : {h->ev_ins, h->ev_rows, h->ev_push, h->ev_lead})
    if (e) (void)hipEventDestroy(e);
  if (h->push_stream) (void)hipStreamDestroy(h->push_stream);
  for (void *p : h->allocs) (void)hipFree(p);
  for (void *p : h->cache_allocs) (void)hipFree(p);
  delete h;
  return 0;
}

int spmcts_set_leaf_peer(spmcts_arena *h, spmcts_arena *leader) {
  if (!h) return fail(-1, "null arena");
  if (h->peer) {
    auto &f = h->peer->followers;
    f.erase(std::remove(f.begin(), f.end(), h), f.end());
    h->peer = nullptr;
  }
  h->peer_step = false;
  h->push_pending = false;
  if (!leader) return 0;
  if (leader == h) return fail(-3, "an arena cannot be its own leader");
  if (leader->peer || !h->followers.empty()) return fail(-3, "one level of lanes: a leader cannot follow");
  if (leader->cfg.game != h->cfg.game || leader->device != h->device)
    return fail(-3, "leader and follower must play the same game on the same device");
  if (h->v.K < 2 || leader->v.K != h->v.K) return fail(-3, "cross-lane dedup needs equal search_threads > 1");
  if (h->v.seg1 < h->v.NS || leader->v.seg1 < leader->v.NS) return fail(-3, "cross-lane dedup: single-network arenas");
  for (hipEvent_t *e : {&leader->ev_ins, &h->ev_rows, &h->ev_push, &h->ev_lead})
    if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
  leader->followers.push_back(h);
  h->peer = leader;
  return 0;
}

#ifdef SPMCTS_AB
// SPMCTS_PEER_PUSH=leader (A/B library): the push on the leader's own stream ahead of its expand (round 6's
// first form), instead of on the follower's push stream
static bool push_on_leader() {
  static const bool v = getenv("SPMCTS_PEER_PUSH") && strcmp(getenv("SPMCTS_PEER_PUSH"), "leader") == 0;
  return v;
}
#else
static constexpr bool push_on_leader() { return false; }
#endif

int spmcts_peer_push(spmcts_arena *h, float *probs_dev, float *values_dev, const float *leader_probs_dev,
                     const float *leader_values_dev, spmcts_stream stream, spmcts_stream leader_stream) {
  if (!h) return fail(-1, "null arena");
  if (!h->peer_step) return 0;
  if (!probs_dev || !values_dev || !leader_probs_dev || !leader_values_dev) return fail(-1, "null argument");
  const hipStream_t s = (hipStream_t)stream, ls = (hipStream_t)leader_stream;
  if (push_on_leader()) {
    // on the leader's stream, after its heads of this step (ahead of its expand)
    HIP_TRY(hipStreamWaitEvent(ls, h->ev_rows, 0));
    hipLaunchKernelGGL(k_peer_push, dim3(nblk(h->v.NS, 256)), dim3(256), 0, ls, h->v, h->peer->v.srow,
                       leader_probs_dev, leader_values_dev, probs_dev, values_dev);
    HIP_TRY(hipEventRecord(h->ev_push, ls));
  } else {
    // on the follower's own push stream, once the leader's outputs of this step (everything the caller has
    // issued on leader_stream: its heads) and our rows are there; the leader's stream goes on at once (its
    // expand does not wait) and waits for the push only before it next rewrites its table, keys or outputs
    // (launch_rows: its next step's rows)
    if (!h->push_stream) HIP_TRY(hipStreamCreateWithFlags(&h->push_stream, hipStreamNonBlocking));
    HIP_TRY(hipEventRecord(h->ev_lead, ls));
    HIP_TRY(hipStreamWaitEvent(h->push_stream, h->ev_lead, 0));
    HIP_TRY(hipStreamWaitEvent(h->push_stream, h->ev_rows, 0));
    hipLaunchKernelGGL(k_peer_push, dim3(nblk(h->v.NS, 256)), dim3(256), 0, h->push_stream, h->v, h->peer->v.srow,
                       leader_probs_dev, leader_values_dev, probs_dev, values_dev);
    HIP_TRY(hipEventRecord(h->ev_push, h->push_stream));
    h->push_pending = true;
  }
  HIP_TRY(hipStreamWaitEvent(s, h->ev_push, 0));
  h->peer_step = false;
  LAUNCH_CHECK();
  return 0;
}

int spmcts_arena_geometry(const spmcts_arena *h, int32_t *A, int32_t *W, int32_t *H, int32_t *bpt, int32_t *nt,
                          int32_t *ng) {
  if (!h) return fail(-1, "null arena");
  if (A) *A = h->A;
  if (W) *W = h->W;
  if (H) *H = h->H;
  if (bpt) *bpt = h->v.cap;
  if (nt) *nt = h->v.T;
  if (ng) *ng = h->v.G;
  return 0;
}

int spmcts_set_root_prior(spmcts_arena *h, const float *probs_dev, spmcts_stream stream) {
  if (!h || !probs_dev) return fail(-1, "null argument");
  HIP_TRY(hipMemcpyAsync(h->v.root_prior, probs_dev, sizeof(float) * h->A, hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return 0;
}

int spmcts_set_tape(spmcts_arena *h, const double *tape_dev, const int64_t *offsets_dev, spmcts_stream stream) {
  if (!h || !offsets_dev) return fail(-1, "null argument");
  if (h->cfg.rng_mode != SPMCTS_RNG_TAPE) return fail(-4, "arena is not in tape RNG mode");
  h->v.tape = tape_dev;
  hipLaunchKernelGGL(k_set_tape, dim3(nblk(h->v.T, 256)), dim3(256), 0, (hipStream_t)stream, h->v, offsets_dev);
  LAUNCH_CHECK();
  return 0;
}

int spmcts_tree_reset(spmcts_arena *h, const int32_t *trees_dev, const int8_t *root_player_dev,
                      const float *priors_dev, int32_t n, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  if (n <= 0) return 0;
  DISPATCH(h, hipLaunchKernelGGL(k_tree_reset<GG>, dim3(nblk(n, 128)), dim3(128), 0, (hipStream_t)stream, h->v,
                                 trees_dev, root_player_dev, priors_dev, n));
  LAUNCH_CHECK();
  return 0;
}

int spmcts_search_begin(spmcts_arena *h, const int32_t *trees_dev, int32_t n, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  if (n > std::max(h->v.T, h->v.G)) return fail(-3, "too many active trees");
  h->n_active = n;
  h->v.sim = 0;
  if (h->v.cwin) ++h->v.cgen;  // a new evaluation-cache generation per search
  if (n <= 0) return 0;
  DISPATCH(h, hipLaunchKernelGGL(k_search_begin<GG>, dim3(nblk(n, 128)), dim3(128), 0, (hipStream_t)stream, h->v,
                                 trees_dev, n));
  if (h->v.gc) DISPATCH(h, hipLaunchKernelGGL(k_compact<GG>, dim3(n), dim3(256), 0, (hipStream_t)stream, h->v, n));
  LAUNCH_CHECK();
  return 0;
}

// cross-lane dedup is live for this step: a follower whose leader and itself dedup (spmcts_set_leaf_peer)
static bool peer_live(const spmcts_arena *h) { return h->peer && h->v.dedup && h->peer->v.dedup; }

// `sim_step`: a simulation step's rows (spmcts_select / spmcts_leaf_rows), where a follower lane looks its
// owner keys up in its leader's table; the end-of-ply expansions (spmcts_play_action, games_end_ply) stay
// lane-local
static int launch_rows(spmcts_arena *h, void *leaves_dev, int32_t *leaf_count_dev, hipStream_t s, bool sim_step) {
  h->peer_step = false;
  for (spmcts_arena *f : h->followers)  // a leader rewrites its table, keys and (later) outputs only after the pushes
    if (f->push_pending) {
      HIP_TRY(hipStreamWaitEvent(s, f->ev_push, 0));
      f->push_pending = false;
    }
  View v = h->v;
  v.peer_on = 0;
  // the evaluation cache is live in leaf-dedup launches (spmcts_set_eval_cache)
  h->cache_step = v.cwin > 0 && v.dedup;
  if (!h->cache_step) v.cwin = 0;
  h->cache_shared_step = h->cache_step && cache_view(h, v);
  h->cache_tab = h->cache_step ? v.crec : nullptr;
  v.served = h->cache_step ? 1 : 0;
  if (v.dedup) {
    if (++h->v.dgen == 0) ++h->v.dgen;  // generation 0 = the zeroed table
    v.dgen = h->v.dgen;
    v.lead = h->followers.empty() ? 0 : 1;
    DISPATCH(h, hipLaunchKernelGGL(k_dedup_insert<GG>, dim3(nblk(v.NS, 256)), dim3(256), 0, s, v));
    if (sim_step && peer_live(h)) {
      // the leader's table and keys of this step are complete (its ev_ins), and stay so until this step's
      // rows are numbered (the leader's stream waits for our ev_rows before it moves on: spmcts_peer_push)
      const spmcts_arena *p = h->peer;
      HIP_TRY(hipStreamWaitEvent(s, p->ev_ins, 0));
      v.peer_on = 1;
      v.served = 1;
      DISPATCH(h, hipLaunchKernelGGL(k_dedup_owner_peer<GG>, dim3(nblk(v.NS, 256)), dim3(256), 0, s, v,
                                     p->v.dtab, p->v.okey, p->v.down, p->v.dmask, p->v.dgen));
    } else {
      DISPATCH(h, hipLaunchKernelGGL(k_dedup_owner<GG>, dim3(nblk(v.NS, 256)), dim3(256), 0, s, v));
    }
    if (v.lead) HIP_TRY(hipEventRecord(h->ev_ins, s));
  }
  hipLaunchKernelGGL(k_scan_need, dim3(1), dim3(SCAN_THREADS), 0, s, v, leaf_count_dev);
  if (v.dedup) hipLaunchKernelGGL(k_dedup_alias, dim3(nblk(v.NS, 256)), dim3(256), 0, s, v);
  if (v.peer_on) {
    HIP_TRY(hipEventRecord(h->ev_rows, s));
    h->peer_step = true;  // spmcts_peer_push brings the leader's outputs before the expand
  }
  if (leaves_dev) {
    const long long total = (long long)v.NS * h->cells;
    DISPATCH(h, hipLaunchKernelGGL(k_encode<GG>, dim3(nblk(total, 256)), dim3(256), 0, s, v, leaves_dev));
  }
  LAUNCH_CHECK();
  return 0;
}

#ifdef SPMCTS_AB
// SPMCTS_TREE_COPIES=1 (A/B library): the threaded tree kernels with 16 LDS block copies per tree
static bool tree_copies() {
  static const bool v = getenv("SPMCTS_TREE_COPIES") && strcmp(getenv("SPMCTS_TREE_COPIES"), "1") == 0;
  return v;
}
#endif

#ifdef SPMCTS_TREE_PROF
// the per-phase cycle sums of the tree kernels since the last reset (g_tprof), into out[16]
extern "C" int spmcts_ab_tree_prof(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tprof), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long zero[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_tprof), zero, sizeof(zero)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

int spmcts_select_tree(spmcts_arena *h, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  hipStream_t s = (hipStream_t)stream;
  const int n = h->n_active;
  if (n > 0) {
    const int gpb = 64 / h->P;
    if (h->v.K > 1) {
      const int tb = h->tree_block, tpb = tb / h->P;
#ifdef SPMCTS_AB
      if (tb > 64)
        DISPATCH(h, hipLaunchKernelGGL((k_select_vl<GG, 512>), dim3(nblk(n, tpb)), dim3(tb), 0, s, h->v, n));
      else if (tree_copies())
        DISPATCH(h, hipLaunchKernelGGL((k_select_vl<GG, 64, 16>), dim3(nblk(n, tpb)), dim3(tb), 0, s, h->v, n));
      else
#endif
        DISPATCH(h, hipLaunchKernelGGL(k_select_vl<GG>, dim3(nblk(n, tpb)), dim3(tb), 0, s, h->v, n));
    } else {
      DISPATCH(h, hipLaunchKernelGGL(k_select<GG>, dim3(nblk(n, gpb)), dim3(64), 0, s, h->v, n));
    }
  }
  h->v.sim += h->v.K;
  LAUNCH_CHECK();
  return 0;
}

int spmcts_leaf_rows(spmcts_arena *h, void *leaves_dev, int32_t *leaf_count_dev, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  return launch_rows(h, leaves_dev, leaf_count_dev, (hipStream_t)stream, true);
}

int spmcts_select(spmcts_arena *h, void *leaves_dev, int32_t *leaf_count_dev, spmcts_stream stream) {
  const int rc = spmcts_select_tree(h, stream);
  if (rc) return rc;
  return spmcts_leaf_rows(h, leaves_dev, leaf_count_dev, stream);
}

int spmcts_expand2(spmcts_arena *h, const float *probs0_dev, const float *values0_dev, const float *probs1_dev,
                   const float *values1_dev, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  if (h->peer_step) return fail(-4, "a follower lane's simulation step needs spmcts_peer_push before its expand");
  if (h->v.seg1 < h->v.NS && (!probs1_dev || !values1_dev))
    return fail(-1, "two-network arena needs network-1 outputs");
  if (h->cache_step) {  // the rows of this step consulted the evaluation cache: fills and inserts first
    View v = h->v;
    if (h->cache_shared_step) cache_view(h, v);
    if (v.crec != h->cache_tab) return fail(-4, "the evaluation cache table changed between a step's rows and its expand");
    DISPATCH(h, hipLaunchKernelGGL(k_cache_io<GG>, dim3(nblk(h->v.NS, 256)), dim3(256), 0, (hipStream_t)stream, v,
                                   (float *)probs0_dev, (float *)values0_dev, (float *)probs1_dev,
                                   (float *)values1_dev));
    h->cache_step = false;
  }
  const int gpb = 64 / h->P;
  if (h->v.K > 1) {
    const int tb = h->tree_block, tpb = tb / h->P;
#ifdef SPMCTS_AB
    static int co = -1;  // A/B library only: the 96-register co-resident expand (measured slower)
    if (co < 0) {
      const char *e = getenv("SPMCTS_EXPAND_CO");
      co = e && atoi(e) ? 1 : 0;
    }
    if (co && tb == 64)
      DISPATCH(h, hipLaunchKernelGGL(k_expand_vl_co<GG>, dim3(nblk(h->v.T, tpb)), dim3(tb), 0, (hipStream_t)stream,
                                     h->v, probs0_dev, values0_dev, probs1_dev, values1_dev));
    else if (tb > 64)
      DISPATCH(h, hipLaunchKernelGGL((k_expand_vl<GG, 512>), dim3(nblk(h->v.T, tpb)), dim3(tb), 0, (hipStream_t)stream,
                                     h->v, probs0_dev, values0_dev, probs1_dev, values1_dev));
    else if (tree_copies())
      DISPATCH(h, hipLaunchKernelGGL((k_expand_vl<GG, 64, 16>), dim3(nblk(h->v.T, tpb)), dim3(tb), 0, (hipStream_t)stream,
                                     h->v, probs0_dev, values0_dev, probs1_dev, values1_dev));
    else
#endif
      DISPATCH(h, hipLaunchKernelGGL(k_expand_vl<GG>, dim3(nblk(h->v.T, tpb)), dim3(tb), 0, (hipStream_t)stream, h->v,
                                     probs0_dev, values0_dev, probs1_dev, values1_dev));
  } else {
    DISPATCH(h, hipLaunchKernelGGL(k_expand<GG>, dim3(nblk(h->v.T, gpb)), dim3(64), 0, (hipStream_t)stream, h->v,
                                   probs0_dev, values0_dev, probs1_dev, values1_dev));
  }
  LAUNCH_CHECK();
  return 0;
}

int spmcts_expand(spmcts_arena *h, const float *probs_dev, const float *values_dev, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  // one buffer indexed by row: network-1 rows (if any) sit at their own row index
  const size_t s1 = (size_t)h->v.seg1;
  const bool dual = h->v.seg1 < h->v.NS;
  return spmcts_expand2(h, probs_dev, values_dev, dual ? probs_dev + s1 * h->A : nullptr,
                        dual ? values_dev + s1 : nullptr, stream);
}

int spmcts_set_tree_players(spmcts_arena *h, const uint8_t *nets, const uint8_t *kinds, const int32_t *budgets) {
  if (!h) return fail(-1, "null arena");
  const int T = h->v.T;
  std::vector<uint8_t> nt(T, 0), kd(T, SPMCTS_PLAYER_MCTS);
  std::vector<int32_t> bd(T, 0x7fffffff);
  int n0 = 0;
  for (int t = 0; t < T; ++t) {
    if (nets) nt[t] = nets[t] ? 1 : 0;
    if (kinds) {
      if (kinds[t] > SPMCTS_PLAYER_LOOKAHEAD) return fail(-3, "unknown player kind");
      kd[t] = kinds[t];
    }
    if (budgets) bd[t] = budgets[t] < 0 ? 0x7fffffff : budgets[t];
    n0 += nt[t] ? 0 : 1;
  }
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(h->v.tnet, nt.data(), T, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->v.tkind, kd.data(), T, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->v.budget, bd.data(), 4 * (size_t)T, hipMemcpyHostToDevice));
  h->v.seg1 = n0 * h->v.K;  // network-0 trees never have more than n0 * K pending leaves
  return 0;
}

int spmcts_set_tree_search(spmcts_arena *h, const double *alpha, const uint8_t *strong_play,
                           const int32_t *search_threads) {
  if (!h) return fail(-1, "null arena");
  const int T = h->v.T;
  if (alpha) {
    for (int t = 0; t < T; ++t)
      if (!(alpha[t] > 0.0)) return fail(-3, "alpha must be > 0");
  }
  if (search_threads) {
    for (int t = 0; t < T; ++t)
      if (search_threads[t] < 1 || search_threads[t] > h->v.K)
        return fail(-3, "per-tree search_threads must be in [1, the arena's search_threads]");
  }
  HIP_TRY(hipDeviceSynchronize());
  if (alpha) HIP_TRY(hipMemcpy(h->v.talpha, alpha, sizeof(double) * (size_t)T, hipMemcpyHostToDevice));
  if (strong_play) {
    std::vector<uint8_t> st(T);
    for (int t = 0; t < T; ++t) st[t] = strong_play[t] ? 1 : 0;
    HIP_TRY(hipMemcpy(h->v.tstrong, st.data(), (size_t)T, hipMemcpyHostToDevice));
  }
  if (search_threads) HIP_TRY(hipMemcpy(h->v.tK, search_threads, 4 * (size_t)T, hipMemcpyHostToDevice));
  return 0;
}

int spmcts_arena_segments(const spmcts_arena *h, int32_t *seg1) {
  if (!h) return fail(-1, "null arena");
  if (seg1) *seg1 = h->v.seg1;
  return 0;
}

int spmcts_set_root_prior_net(spmcts_arena *h, int32_t net, const float *probs_dev, spmcts_stream stream) {
  if (!h || !probs_dev) return fail(-1, "null argument");
  if (net < 0 || net > 1) return fail(-3, "network index must be 0 or 1");
  HIP_TRY(hipMemcpyAsync(h->v.root_prior + 16 * net, probs_dev, sizeof(float) * h->A, hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return 0;
}

int spmcts_set_leaf_dedup(spmcts_arena *h, int32_t on) {
  if (!h) return fail(-1, "null arena");
  h->v.dedup = (on && h->v.K > 1) ? 1 : 0;  // K = 1 keeps one row per tree (k_expand walks rows)
  return 0;
}

int spmcts_set_eval_cache(spmcts_arena *h, int32_t window, int32_t capacity_log2) {
  if (!h) return fail(-1, "null arena");
  if (window < 0 || window > (1 << 20)) return fail(-3, "eval cache window out of range");
  if (capacity_log2 != 0 && (capacity_log2 < 10 || capacity_log2 > 28)) return fail(-3, "eval cache capacity_log2: 10..28 (0 = sized from the arena)");
  if (h->cache_step) return fail(-4, "a step that consulted the evaluation cache has not been expanded yet");
  for (const spmcts_arena *f : h->followers)
    if (f->cache_step && f->cache_shared_step)
      return fail(-4, "a follower lane's step that uses this arena's evaluation cache has not been expanded yet");
  HIP_TRY(hipSetDevice(h->device));
  HIP_TRY(hipDeviceSynchronize());  // no launch of this arena reads the old table any more
  for (void *p : h->cache_allocs) (void)hipFree(p);
  h->cache_allocs.clear();
  View &v = h->v;
  v.crec = nullptr;
  v.xc = nullptr;
  v.cwin = 0;
  v.cmask = 0;
  h->cache_step = h->cache_shared_step = false;
  if (window == 0) return 0;
  if (v.K < 2) return fail(-3, "the evaluation cache needs search_threads > 1 (it extends leaf dedup)");
  int L = capacity_log2;
  if (L == 0) {
    // entries held: window + 1 generations (the slack one) of at most one row per searching tree per sim, plus
    // the end-of-ply rows; a leader's table also takes a follower lane's rows (cache_view): twice one lane's, and
    // twice that again so probe chains stay short
    const long long searching = std::max<long long>(v.G > 0 ? v.G : v.T, 1);
    const long long held = (long long)(window + 1) * searching * ((long long)v.iters + 2);
    L = 10;
    while (L < 26 && (1ll << L) < 4 * held) ++L;
  }
  const size_t E = (size_t)1 << L;
  void *p[2] = {};
  const size_t bytes[2] = {E * CACHE_REC * 8, (size_t)v.NS * 4};
  for (int i = 0; i < 2; ++i) {
    const hipError_t e = hipMalloc(&p[i], bytes[i]);
    if (e != hipSuccess) {
      for (int j = 0; j < i; ++j) (void)hipFree(p[j]);
      return fail(-1000 - (int)e, std::string("eval cache hipMalloc: ") + hipGetErrorString(e));
    }
    h->cache_allocs.push_back(p[i]);
  }
  HIP_TRY(hipMemset(p[0], 0, bytes[0]));  // every entry never used
  v.crec = (uint64_t *)p[0];
  v.xc = (int32_t *)p[1];
  v.cmask = (int)(E - 1);
  v.cwin = window;
  v.cgen = (uint32_t)window + 1;  // generation 0 never read as live
  HIP_TRY(hipDeviceSynchronize());
  return 0;
}

int spmcts_eval_cache_clear(spmcts_arena *h) {
  if (!h) return fail(-1, "null arena");
  if (h->v.cwin) h->v.cgen += (uint32_t)h->v.cwin + 1;  // every entry leaves the window
  return 0;
}

int spmcts_games_set_record(spmcts_arena *h, int32_t record) {
  if (!h) return fail(-1, "null arena");
  h->v.record = record ? 1 : 0;
  return 0;
}

int spmcts_search_end(spmcts_arena *h, double temp, int32_t *actions_dev, int8_t *states_dev, float *tree_probs_dev,
                      double *q_dev, uint8_t *q_f64_dev, uint8_t *recorded_dev, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  const int n = h->n_active;
  if (n <= 0) return 0;
  DISPATCH(h, hipLaunchKernelGGL(k_search_end<GG>, dim3(nblk(n, 64)), dim3(64), 0, (hipStream_t)stream, h->v, n,
                                 temp, actions_dev, states_dev, tree_probs_dev, q_dev, q_f64_dev, recorded_dev));
  LAUNCH_CHECK();
  return 0;
}

int spmcts_play_action(spmcts_arena *h, const int32_t *trees_dev, const int32_t *actions_dev, int32_t n,
                       void *leaves_dev, int32_t *leaf_count_dev, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  hipStream_t s = (hipStream_t)stream;
  if (n > 0)
    DISPATCH(h, hipLaunchKernelGGL(k_play_action<GG>, dim3(nblk(n, 64)), dim3(64), 0, s, h->v, trees_dev,
                                   actions_dev, n));
  LAUNCH_CHECK();
  return launch_rows(h, leaves_dev, leaf_count_dev, s, false);
}

int spmcts_leaf_trees(spmcts_arena *h, int32_t *trees_dev, spmcts_stream stream) {
  if (!h || !trees_dev) return fail(-1, "null argument");
  HIP_TRY(hipMemcpyAsync(trees_dev, h->v.row_tree, sizeof(int32_t) * h->v.NS, hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return 0;
}

int spmcts_root_stats(spmcts_arena *h, int32_t tree, int32_t *child_n, double *child_w, float *child_p,
                      int32_t *root_n, double *root_w, int32_t *root_player, int8_t *board) {
  if (!h) return fail(-1, "null arena");
  if (tree < 0 || tree >= h->v.T) return fail(-3, "tree out of range");
  HIP_TRY(hipDeviceSynchronize());
  const size_t nb = (size_t)tree * h->v.cap * h->P;
  int32_t root = 0, cb = -1;
  int8_t rp = 0;
  uint64_t pos = 0, neg = 0;
  HIP_TRY(hipMemcpy(&root, h->v.root + tree, 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&cb, node_field(h, 8, 4, nb + root), 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&rp, h->v.rplayer + tree, 1, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&pos, h->v.rpos + tree, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&neg, h->v.rneg + tree, 8, hipMemcpyDeviceToHost));
  if (root_n) HIP_TRY(hipMemcpy(root_n, node_field(h, 0, 4, nb + root), 4, hipMemcpyDeviceToHost));
  if (root_w) HIP_TRY(hipMemcpy(root_w, node_field(h, 16, 8, nb + root), 8, hipMemcpyDeviceToHost));
  if (root_player) *root_player = rp;
  if (cb >= 0) {
    const size_t ci = nb + (size_t)cb * h->P;
    if (child_n) HIP_TRY(hipMemcpy(child_n, node_field(h, 0, 4, ci), 4 * h->A, hipMemcpyDeviceToHost));
    if (child_w) HIP_TRY(hipMemcpy(child_w, node_field(h, 16, 8, ci), 8 * h->A, hipMemcpyDeviceToHost));
    if (child_p) HIP_TRY(hipMemcpy(child_p, node_field(h, 12, 4, ci), 4 * h->A, hipMemcpyDeviceToHost));
  } else {
    for (int j = 0; j < h->A; ++j) {
      if (child_n) child_n[j] = 0;
      if (child_w) child_w[j] = 0.0;
      if (child_p) child_p[j] = 0.f;
    }
  }
  if (board) {
    for (int x = 0; x < h->W; ++x)
      for (int y = 0; y < h->H; ++y) {
        const uint64_t bit = 1ull << (x * (h->H + 1) + y);
        board[x * h->H + y] = (pos & bit) ? 1 : ((neg & bit) ? -1 : 0);
      }
  }
  return 0;
}

int spmcts_games_start(spmcts_arena *h, const int32_t *slots_dev, const float *priors_dev, int32_t n,
                       spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  if (h->v.G <= 0) return fail(-4, "arena has no game slots");
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  DISPATCH(h, hipLaunchKernelGGL(k_games_start<GG>, dim3(nblk(n, 128)), dim3(128), 0, s, h->v, slots_dev, priors_dev, n));
  hipLaunchKernelGGL(k_games_bump_id, dim3(1), dim3(1), 0, s, h->v, n);
  LAUNCH_CHECK();
  return 0;
}

int spmcts_games_set_limit(spmcts_arena *h, int64_t max_games) {
  if (!h) return fail(-1, "null arena");
  HIP_TRY(hipMemcpy(h->v.gcnt + 8, &max_games, 8, hipMemcpyHostToDevice));
  return 0;
}

int spmcts_games_begin_ply(spmcts_arena *h, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  if (h->v.G <= 0) return fail(-4, "arena has no game slots");
  h->n_active = h->v.G;
  h->v.sim = 0;
  if (h->v.cwin) ++h->v.cgen;  // a new evaluation-cache generation per ply
  DISPATCH(h, hipLaunchKernelGGL(k_games_begin_ply<GG>, dim3(nblk(h->v.G, 128)), dim3(128), 0, (hipStream_t)stream,
                                 h->v));
  if (h->v.gc)
    DISPATCH(h, hipLaunchKernelGGL(k_compact<GG>, dim3(h->v.G), dim3(256), 0, (hipStream_t)stream, h->v, h->v.G));
  LAUNCH_CHECK();
  return 0;
}

int spmcts_games_end_ply(spmcts_arena *h, void *leaves_dev, int32_t *leaf_count_dev, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  hipStream_t s = (hipStream_t)stream;
  DISPATCH(h, hipLaunchKernelGGL(k_games_end_ply<GG>, dim3(nblk(h->v.G, 64)), dim3(64), 0, s, h->v));
  LAUNCH_CHECK();
  return launch_rows(h, leaves_dev, leaf_count_dev, s, false);
}

int spmcts_games_finish_ply(spmcts_arena *h, int32_t refill, int32_t *out_dev, spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  hipStream_t s = (hipStream_t)stream;
  DISPATCH(h, hipLaunchKernelGGL(k_games_finish_scan<GG>, dim3(1), dim3(1024), 0, s, h->v, refill, out_dev));
  DISPATCH(h, hipLaunchKernelGGL(k_games_finish_apply<GG>, dim3(nblk(h->v.G, 64)), dim3(64), 0, s, h->v));
  LAUNCH_CHECK();
  return 0;
}

int spmcts_export_moves(spmcts_arena *h, int8_t *states_dev, float *tree_probs_dev, double *q_dev, uint8_t *q_f64_dev,
                        float *z_dev, int64_t *game_dev, int32_t max_records, int32_t *count_dev,
                        spmcts_stream stream) {
  if (!h) return fail(-1, "null arena");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_export, dim3(nblk(std::max(1, max_records), 256)), dim3(256), 0, s, h->v, h->A, h->cells,
                     states_dev, tree_probs_dev, q_dev, q_f64_dev, z_dev, game_dev, max_records, count_dev);
  hipLaunchKernelGGL(k_export_clear, dim3(1), dim3(1), 0, s, h->v);
  LAUNCH_CHECK();
  return 0;
}

int spmcts_games_state(spmcts_arena *h, uint8_t *active, int32_t *ply, uint8_t *swap, int64_t *game_id) {
  if (!h) return fail(-1, "null arena");
  HIP_TRY(hipDeviceSynchronize());
  const size_t G = h->v.G;
  if (active) HIP_TRY(hipMemcpy(active, h->v.gstate, G, hipMemcpyDeviceToHost));
  if (ply) HIP_TRY(hipMemcpy(ply, h->v.gply, 4 * G, hipMemcpyDeviceToHost));
  if (swap) HIP_TRY(hipMemcpy(swap, h->v.gswap, G, hipMemcpyDeviceToHost));
  if (game_id) HIP_TRY(hipMemcpy(game_id, h->v.gid, 8 * G, hipMemcpyDeviceToHost));
  return 0;
}

int spmcts_get_counters(spmcts_arena *h, spmcts_counters *out) {
  if (!h || !out) return fail(-1, "null argument");
  HIP_TRY(hipDeviceSynchronize());
  memset(out, 0, sizeof(*out));
  std::vector<int64_t> c((size_t)h->v.T * C_NCNT);
  HIP_TRY(hipMemcpy(c.data(), h->v.cnt, c.size() * 8, hipMemcpyDeviceToHost));
  for (int t = 0; t < h->v.T; ++t) {
    const int64_t *ct = c.data() + (size_t)t * C_NCNT;
    out->sims += ct[C_SIMS];
    out->nn_leaves += ct[C_NN];
    out->terminal_leaves += ct[C_TERM];
    out->depth_sum += ct[C_DEPTH];
    out->set_node_expansions += ct[C_SETNODE];
    out->moves += ct[C_MOVES];
    out->leaked_sims += ct[C_LEAK];
    out->compactions += ct[C_GC];
    out->blocks_in_use_max = std::max<int64_t>(out->blocks_in_use_max, ct[C_HWM]);
  }
  std::vector<int32_t> used(h->v.T);
  HIP_TRY(hipMemcpy(used.data(), h->v.used, 4 * used.size(), hipMemcpyDeviceToHost));
  for (int32_t u : used) out->blocks_in_use_max = std::max<int64_t>(out->blocks_in_use_max, u);
  int64_t g[16];
  HIP_TRY(hipMemcpy(g, h->v.gcnt, sizeof(g), hipMemcpyDeviceToHost));
  out->games_finished = g[0];
  for (int k = 0; k < 6; ++k) out->results[k / 3][k % 3] = g[1 + k];
  out->positions_exported = g[9];
  out->nn_rows = g[10];
  out->cache_rows = g[11];
  HIP_TRY(hipMemcpy(&out->error_flags, h->v.err, 4, hipMemcpyDeviceToHost));
  return 0;
}

int spmcts_check(spmcts_arena *h) {
  if (!h) return fail(-1, "null arena");
  HIP_TRY(hipDeviceSynchronize());
  uint32_t e = 0;
  HIP_TRY(hipMemcpy(&e, h->v.err, 4, hipMemcpyDeviceToHost));
  if (e) {
    char buf[128];
    snprintf(buf, sizeof(buf), "device error flags 0x%x", e);
    return fail(-5, buf);
  }
  return 0;
}

int spmcts_env_step(int32_t game, int32_t width, int32_t height, const int8_t *boards_dev, const int32_t *actions_dev,
                    const int8_t *players_dev, const uint8_t *over_dev, int32_t n, int8_t *out_boards_dev,
                    int8_t *reward_dev, uint8_t *done_dev, int8_t *status_dev, uint8_t *valid_dev,
                    spmcts_stream stream) {
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (game == SPMCTS_CONNECT4 && width == 7 && height == 6)
    hipLaunchKernelGGL(k_env_step<C4>, dim3(nblk(n, 256)), dim3(256), 0, s, boards_dev, actions_dev, players_dev,
                       over_dev, n, out_boards_dev, reward_dev, done_dev, status_dev, valid_dev);
  else if (game == SPMCTS_TICTACTOE && width == 3 && height == 3)
    hipLaunchKernelGGL(k_env_step<TTT>, dim3(nblk(n, 256)), dim3(256), 0, s, boards_dev, actions_dev, players_dev,
                       over_dev, n, out_boards_dev, reward_dev, done_dev, status_dev, valid_dev);
  else
    return fail(-2, "unsupported game/board size");
  LAUNCH_CHECK();
  return 0;
}

int spmcts_env_step_host(int32_t game, int32_t width, int32_t height, int8_t *board, int32_t action, int32_t player,
                         int32_t *reward, int32_t *done) {
  if (game == SPMCTS_CONNECT4 && width == 7 && height == 6) {
    if (action < 0 || action >= C4::A) return fail(-3, "action out of range");
    return env_step_host_t<C4>(board, action, player, reward, done);
  }
  if (game == SPMCTS_TICTACTOE && width == 3 && height == 3) {
    if (action < 0 || action >= TTT::A) return fail(-3, "action out of range");
    return env_step_host_t<TTT>(board, action, player, reward, done);
  }
  return fail(-2, "unsupported game/board size");
}

int spmcts_valid_moves_host(int32_t game, int32_t width, int32_t height, const int8_t *board, uint8_t *valid) {
  if (game == SPMCTS_CONNECT4 && width == 7 && height == 6) {
    const uint32_t m = legal_mask<C4>(from_cells<C4>(board));
    for (int a = 0; a < C4::A; ++a) valid[a] = (m >> a) & 1u;
    return 0;
  }
  if (game == SPMCTS_TICTACTOE && width == 3 && height == 3) {
    const uint32_t m = legal_mask<TTT>(from_cells<TTT>(board));
    for (int a = 0; a < TTT::A; ++a) valid[a] = (m >> a) & 1u;
    return 0;
  }
  return fail(-2, "unsupported game/board size");
}

int spmcts_table_net(int32_t game, int32_t width, int32_t height, const void *leaves_dev, int32_t leaf_format,
                     int32_t leaf_layout, int32_t n, uint64_t salt, const uint64_t *salts_dev, float *probs_dev,
                     float *values_dev, spmcts_stream stream) {
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (game == SPMCTS_CONNECT4 && width == 7 && height == 6)
    hipLaunchKernelGGL(k_table_net<C4>, dim3(nblk(n, 128)), dim3(128), 0, s, leaves_dev, leaf_format, leaf_layout, n,
                       salt, salts_dev, probs_dev, values_dev);
  else if (game == SPMCTS_TICTACTOE && width == 3 && height == 3)
    hipLaunchKernelGGL(k_table_net<TTT>, dim3(nblk(n, 128)), dim3(128), 0, s, leaves_dev, leaf_format, leaf_layout,
                       n, salt, salts_dev, probs_dev, values_dev);
  else
    return fail(-2, "unsupported game/board size");
  LAUNCH_CHECK();
  return 0;
}

int spmcts_copy_probe(const void *src_dev, void *dst_dev, uint64_t bytes, spmcts_stream stream) {
  const size_t n4 = bytes / 16;
  hipLaunchKernelGGL(k_copy_probe, dim3(4096), dim3(256), 0, (hipStream_t)stream, (const float4 *)src_dev,
                     (float4 *)dst_dev, n4);
  LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
