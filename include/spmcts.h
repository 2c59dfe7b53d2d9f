/*
 * spmcts.h — C ABI of the MI355X-native batched self-play MCTS arena.
 *
 * The arena replaces the per-process Python object tree of the reference
 * (reubenvanammers/self_play_reinforcement_learning, games/algos/mcts.py) and
 * the per-game episode loop that drives it (games/algos/selfplayworker.py
 * SelfPlayer, fed by games/algos/self_play_parallel.py SelfPlayScheduler).
 * Thousands of trees live in one device-resident struct-of-arrays node store;
 * every entry point below launches HIP kernels for gfx950 on the caller's
 * stream.  The reference is pure Python, so there is no C FFI to bind: the
 * drop-in boundary is the reference's own Python policy API (MCTreeSearch /
 * SelfPlayScheduler / Memory), re-implemented in
 * self_play_reinforcement_learning_amd/ on top of these functions via ctypes.
 * Each function cites the reference interface it replaces.
 *
 * Conventions
 *   - All array arguments named *_dev are DEVICE pointers owned by the caller
 *     (torch tensors); the arena owns only its node store and game state.
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  Calls are
 *     stream-ordered; none synchronises unless stated ("(sync)").
 *   - Return value: 0 on success, < 0 on error; spmcts_last_error() returns a
 *     thread-local message.  Errors raised on the device (node-pool
 *     exhaustion, RNG tape exhaustion, invalid action) are sticky flags read by
 *     spmcts_check() / spmcts_get_counters().
 *   - No exceptions cross the ABI.  One arena per device per process; calls on
 *     one arena must be serialised by the host (single writer).
 *
 * Board frame: +1 = the tree's owner (each MCTreeSearch sees itself as +1,
 * selfplayworker.py:175-176).  Boards are int8/int64 [W][H] = [column][row],
 * row 0 = bottom (connect4env.py:22).
 */
#ifndef SPMCTS_H
#define SPMCTS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct spmcts_arena spmcts_arena; /* opaque */
typedef void *spmcts_stream;              /* hipStream_t */

enum spmcts_game { SPMCTS_CONNECT4 = 0, SPMCTS_TICTACTOE = 1 };
enum spmcts_rng_mode {
  SPMCTS_RNG_PHILOX = 0, /* rocRAND Philox4x32-10, one subsequence per tree          */
  SPMCTS_RNG_TAPE = 1    /* replay injected per-tree double streams (parity mode)     */
};
enum spmcts_leaf_format {
  SPMCTS_LEAF_F32 = 0,      /* float  planes [B,3,W,H] (empty, own, enemy)  modules.py:115-125 */
  SPMCTS_LEAF_F16 = 1,      /* half   planes                                                   */
  SPMCTS_LEAF_BF16 = 2,     /* bf16   planes                                                   */
  SPMCTS_LEAF_BOARD_I64 = 3 /* int64 boards [B,W,H] = state * mover, for net.forward(s)        */
};
enum spmcts_layout { SPMCTS_NCHW = 0, SPMCTS_NHWC = 1 };
/* What plays a tree's moves in games mode (games/general/hardcoded_players.py) */
enum spmcts_player_kind {
  SPMCTS_PLAYER_MCTS = 0,     /* MCTreeSearch (the default)                                 */
  SPMCTS_PLAYER_RANDOM = 1,   /* Random: uniform over valid moves (hardcoded_players.py:36-56) */
  SPMCTS_PLAYER_LOOKAHEAD = 2 /* OneStepLookahead: win / block / random (:8-33)               */
};

/* return code of the tower entry points (spmcts_tower_forward*, spmcts_tower_heads*) and of
 * spmcts_arena_create: an environment switch of the A/B library (SPMCTS_TOWER_CG, SPMCTS_TOWER_RING,
 * SPMCTS_TOWER_C256, SPMCTS_WIDE_TAILS, SPMCTS_HEADS, SPMCTS_HEADS_C256, SPMCTS_TREE_BLOCK,
 * SPMCTS_EXPAND_CO, SPMCTS_TOWER_M16, SPMCTS_TREE_COPIES, SPMCTS_PEER_PUSH -- whatever its value; `make ab` builds libspmcts_ab.so, which
 * reads them) is set while the product library is loaded: refused instead of silently ignored */
#define SPMCTS_ERR_AB_SWITCH (-5)

/* device error flags (sticky) */
#define SPMCTS_ERR_POOL 0x1u      /* a tree ran out of node blocks                 */
#define SPMCTS_ERR_TAPE 0x2u      /* RNG tape exhausted                            */
#define SPMCTS_ERR_NOCHILD 0x4u   /* select reached a node whose children are all invalid */
#define SPMCTS_ERR_ACTION 0x8u    /* play_action on an illegal action              */
#define SPMCTS_ERR_STATE 0x10u    /* inconsistent tree state                       */
#define SPMCTS_ERR_EXPORT 0x20u   /* move export ring overflow                     */

typedef struct spmcts_config {
  int32_t game;            /* enum spmcts_game                                               */
  int32_t width, height;   /* 7x6 Connect4, 3x3 TicTacToe (only these are instantiated)      */
  int32_t n_trees;         /* tree slots (games mode needs >= 2*n_games)                     */
  int32_t n_games;         /* game slots for the self-play state machine (0 = tree mode only) */
  int32_t iterations;      /* simulations per move (mcts.py:125, sizes the node pool)        */
  int32_t blocks_per_tree; /* node blocks per tree; 0 = worst case from iterations          */
  int32_t rng_mode;        /* enum spmcts_rng_mode                                            */
  int32_t strong_play;     /* mcts.py:133, :307-311                                           */
  int32_t evaluate;        /* mcts.py:273-274 (temp / 20)                                     */
  int32_t leaf_format;     /* enum spmcts_leaf_format                                         */
  int32_t leaf_layout;     /* enum spmcts_layout (planes only)                                */
  int32_t compact;         /* 1: leaf rows compacted in tree order; 0: one row per active slot */
  int32_t search_threads;  /* K simulations in flight per tree with virtual loss (the reference's
                              thread_count, mcts.py:328-331, :345); 0 or 1 = sequential search.
                              Leaf rows per select = n_trees * K; K > 1 keeps a per-node vl.  */
  double cpuct;            /* MCNode.cpuct = 4 (mcts.py:25)                                   */
  double x_noise;          /* MCNode.x = 0.25 (mcts.py:25)                                    */
  double alpha;            /* Dirichlet alpha (mcts.py:135)                                   */
  uint64_t seed;           /* Philox key                                                      */
  uint64_t subsequence0;   /* Philox subsequence of tree 0 (rank * n_trees for multi-GPU)     */
} spmcts_config;

typedef struct spmcts_counters {
  int64_t sims;                /* simulations completed (search_node calls)                  */
  int64_t nn_leaves;           /* leaves sent to the network (search + play_action)          */
  int64_t terminal_leaves;     /* simulations that ended on a terminal leaf (no NN)          */
  int64_t depth_sum;           /* sum over sims of edges descended (select depth D)          */
  int64_t set_node_expansions; /* play_action expansions (mcts.py:203-208)                   */
  int64_t moves;               /* moves played by searching trees (= Move records)           */
  int64_t games_finished;
  int64_t positions_exported;  /* Move records exported                                      */
  int64_t results[2][3];       /* [swap_sides][win, draw, loss] (self_play_parallel.py:302-327) */
  int64_t blocks_in_use_max;   /* peak node blocks used by any tree (high-water since creation) */
  uint32_t error_flags;
  uint32_t reserved;
  int64_t leaked_sims;         /* threaded mode: sims that found every child invalid or locked and
                                  ended without a backup, their virtual loss left in place
                                  (mcts.py:349-354); sims + leaked_sims = searches x iterations */
  int64_t compactions;         /* subtree recyclings (node-store compactions before a search; only
                                  when blocks_per_tree is below the worst case)                 */
  int64_t nn_rows;             /* network rows emitted (= nn_leaves unless leaf dedup is on)  */
  int64_t cache_rows;          /* leaf rows served from the evaluation cache (spmcts_set_eval_cache) */
} spmcts_counters;

/* ---- library ------------------------------------------------------------ */
int spmcts_version(void);
const char *spmcts_last_error(void);
/* (sync) size of the device allocation an arena with this config needs */
int spmcts_arena_bytes(const spmcts_config *cfg, uint64_t *bytes_out);

/* ---- arena lifetime ------------------------------------------------------ */
/* Replaces MCTreeSearch.__init__ (mcts.py:119-164) for many trees at once. */
int spmcts_arena_create(const spmcts_config *cfg, int device, spmcts_arena **out);
int spmcts_arena_destroy(spmcts_arena *h);
/* geometry: A = actions, W, H, blocks per tree, lanes per tree */
int spmcts_arena_geometry(const spmcts_arena *h, int32_t *A, int32_t *W, int32_t *H, int32_t *blocks_per_tree,
                          int32_t *n_trees, int32_t *n_games);

/* Priors of the empty-board root: `self.network(base_state)` in MCTreeSearch.reset
 * (mcts.py:167-170).  Constant per network weights; used by every tree/game reset. */
int spmcts_set_root_prior(spmcts_arena *h, const float *probs_dev /*[A]*/, spmcts_stream stream);
/* Parity mode: per-tree flat double streams, consumed in the reference's call
 * order (dirichlet(A) per search, rand(A) per select level, one uniform per
 * np.random.choice).  offsets_dev[T+1] (int64) index into tape_dev. */
int spmcts_set_tape(spmcts_arena *h, const double *tape_dev, const int64_t *offsets_dev, spmcts_stream stream);

/* ---- tree-level API (the MCTreeSearch policy protocol) -------------------- */
/* MCTreeSearch.reset(player) (mcts.py:166-174): new root on the empty board.
 * priors_dev: NULL = the arena's root prior, else [n][A] per tree. */
int spmcts_tree_reset(spmcts_arena *h, const int32_t *trees_dev, const int8_t *root_player_dev,
                      const float *priors_dev, int32_t n, spmcts_stream stream);
/* MCTreeSearch.search prologue (mcts.py:323-327): Dirichlet noise on the roots of
 * the listed trees; they become the active set for spmcts_select. */
int spmcts_search_begin(spmcts_arena *h, const int32_t *trees_dev, int32_t n, spmcts_stream stream);
/* One search_node (mcts.py:340-367) for every active tree: PUCT select with
 * jitter, terminal leaves backed up in place, other leaves written to the leaf
 * batch (rows in tree order).  leaf_count_dev int32[3] = {rows, network-0 rows,
 * network-1 rows}: network-0 leaves occupy rows [0, n0), network-1 leaves rows
 * [seg1, seg1 + n1) (see spmcts_set_tree_players; single-network arenas: n1 = 0). */
int spmcts_select(spmcts_arena *h, void *leaves_dev, int32_t *leaf_count_dev, spmcts_stream stream);
/* spmcts_select in two launches (for per-kernel timing): the tree walk alone,
 * then the leaf-row compaction + encode of whatever is pending. */
int spmcts_select_tree(spmcts_arena *h, spmcts_stream stream);
int spmcts_leaf_rows(spmcts_arena *h, void *leaves_dev, int32_t *leaf_count_dev, spmcts_stream stream);
/* _expand_node tail + backup (mcts.py:316-321, :94-98, :361-364) for the rows of
 * the last select / play_action: create children with the network's priors,
 * back the value up the path.  probs_dev [rows][A] f32, values_dev [rows] f32
 * (network outputs from the mover's perspective, modules.py:109-112). */
int spmcts_expand(spmcts_arena *h, const float *probs_dev, const float *values_dev, spmcts_stream stream);
/* Two-network arenas: network-0 outputs indexed by row, network-1 outputs by row - seg1. */
int spmcts_expand2(spmcts_arena *h, const float *probs0_dev, const float *values0_dev, const float *probs1_dev,
                   const float *values1_dev, spmcts_stream stream);
/* (sync) Per-tree players, for evaluation games between two networks or against a
 * hard-coded player (SelfPlayWorker.set_up_policies evaluate=True, selfplayworker.py:68-94;
 * compare_models, self_play_parallel.py:355-379).  Host arrays of n_trees entries, each
 * may be NULL (default): nets = network id 0/1 of the tree's leaves; kinds = enum
 * spmcts_player_kind; budgets = simulations per search (MCTreeSearch.iterations of that
 * player; < 0 = unlimited).  Network-1 leaves are placed from row seg1 = #network-0 trees. */
int spmcts_set_tree_players(spmcts_arena *h, const uint8_t *nets, const uint8_t *kinds, const int32_t *budgets);
/* (sync) Per-tree search settings: each side of an evaluation game searches with its own
 * MCTreeSearch kwargs (selfplayworker.py:71-81 builds the opponent from its own container;
 * mcts.py:119-136): alpha = Dirichlet alpha of the root noise (mcts.py:49-53, > 0),
 * strong_play = terminal-value shaping (mcts.py:305-311), search_threads = sims in flight
 * (thread_count, mcts.py:328-331; 1 .. the arena's search_threads).  Host arrays of n_trees
 * entries; NULL = unchanged (defaults: the arena config's values). */
int spmcts_set_tree_search(spmcts_arena *h, const double *alpha, const uint8_t *strong_play,
                           const int32_t *search_threads);
int spmcts_arena_segments(const spmcts_arena *h, int32_t *seg1);
/* Empty-board root prior of network `net` (0 / 1), used by resets of that network's trees. */
int spmcts_set_root_prior_net(spmcts_arena *h, int32_t net, const float *probs_dev, spmcts_stream stream);
/* Games mode: keep Move records (play_episode update=True, the default) or not (evaluation games). */
int spmcts_games_set_record(spmcts_arena *h, int32_t record);
/* Batch leaf dedup (search_threads > 1 only; no effect with 1): pending leaves whose
 * network input is the same ((own, opp) stones from the mover's view, same network) share one
 * leaf row, so each distinct position of a simulation step is evaluated once and every leaf reads
 * its row's outputs.  The reference evaluates each leaf separately (InferenceWorker,
 * inference_worker.py:89-119); with a deterministic, batch-independent evaluator the outputs each
 * leaf receives are unchanged.  Off by default; leave it off for evaluators that give rows of
 * different trees different networks (per-row salts).  Leaf counts then count rows, not leaves. */
int spmcts_set_leaf_dedup(spmcts_arena *h, int32_t on);
/* Cross-lane leaf dedup (round 6).  Pair `h` (a follower lane) with `leader` (another arena of the same game,
 * device and search_threads > 1, both single-network; NULL unpairs): in each simulation step
 * (spmcts_select / spmcts_leaf_rows, with leaf dedup on in both) a follower's pending leaf whose network input
 * the leader evaluates in the SAME step takes the leader's row instead of one of its own -- the lanes of
 * engine.LanedEngine run in lock step, and the reference evaluates every leaf (inference_worker.py:89-119),
 * so with a deterministic, batch-independent evaluator each leaf's outputs are unchanged.  Contract: per step
 * the leader's rows are built before the follower's (host order), and the follower's expand is
 * preceded by spmcts_peer_push; the end-of-ply expansions (spmcts_play_action / spmcts_games_end_ply) stay lane-local.
 * Leaf counts of the follower count its own rows (the leader-served rows follow them). */
int spmcts_set_leaf_peer(spmcts_arena *h, spmcts_arena *leader);
/* Before a follower's expand of a simulation step: on leader_stream (after the leader's network outputs of
 * the step) the leader's rows are copied into the follower's leader-served rows of probs_dev / values_dev
 * (k_peer_push), and `stream` waits for them (events).  A no-op when the step had no leader-served rows
 * (unpaired, dedup off, an end-of-ply step); a follower's spmcts_expand / spmcts_expand2 after a
 * leader-served step without it fails (-4). */
int spmcts_peer_push(spmcts_arena *h, float *probs_dev, float *values_dev, const float *leader_probs_dev,
                     const float *leader_values_dev, spmcts_stream stream, spmcts_stream leader_stream);
/* Evaluation cache (round 6; search_threads > 1 with leaf dedup on): the network
 * outputs of the arena's own leaf rows are kept, keyed like leaf dedup ((own, opp) stones from the mover's
 * view), for `window` generations -- one generation per spmcts_games_begin_ply / spmcts_search_begin, so
 * window 1 = within the ply (search) that evaluated them.  An owner leaf whose key is cached takes a row
 * after the network rows (and a follower's leader-served rows) and, at spmcts_expand / spmcts_expand2, the
 * cached outputs are written into that row of probs / values (k_cache_io), and the rows the network (or the
 * leader) filled go into the cache.  Two-network arenas keep the networks' keys apart (served rows follow each
 * segment's network rows); a follower lane whose leader runs a cache of the same window uses the leader's
 * table.  The reference evaluates every leaf (inference_worker.py:89-119); with
 * a deterministic, batch-independent evaluator every leaf still receives exactly its own outputs.  After the
 * network's weights change call spmcts_eval_cache_clear.  window 0 turns it off; capacity_log2 = log2 of the
 * table's entries (10..28; 0 = four times the rows window + 1 plies can hold, at most 2^26), allocated here
 * (one 64-byte record per entry + 4 bytes per pending slot, outside spmcts_arena_bytes).  (sync) */
int spmcts_set_eval_cache(spmcts_arena *h, int32_t window, int32_t capacity_log2);
/* Every cached output leaves the window (host-side generation step; no device work). */
int spmcts_eval_cache_clear(spmcts_arena *h);
/* MCTreeSearch._play (mcts.py:272-299) for the active trees + remove_noise:
 * visit-count^(1/temp) distribution, np.random.choice semantics, Move record.
 * Outputs per active tree i: actions_dev[i], states_dev[i][W*H] (int8, tree
 * frame), tree_probs_dev[i][A], q_dev[i] (double; exported as a float32 tensor
 * unless q_f64_dev[i]), recorded_dev[i] (0 = numpy ValueError fallback). */
int spmcts_search_end(spmcts_arena *h, double temp, int32_t *actions_dev, int8_t *states_dev, float *tree_probs_dev,
                      double *q_dev, uint8_t *q_f64_dev, uint8_t *recorded_dev, spmcts_stream stream);
/* MCTreeSearch.play_action/_set_node (mcts.py:188-209): advance each listed
 * root; an unvisited child is expanded (rows for the network) and backed up. */
int spmcts_play_action(spmcts_arena *h, const int32_t *trees_dev, const int32_t *actions_dev, int32_t n,
                       void *leaves_dev, int32_t *leaf_count_dev, spmcts_stream stream);
/* Tree id of every leaf row of the last select / play_action / games_end_ply
 * (rows in tree order; trees_dev has room for n_trees entries). */
int spmcts_leaf_trees(spmcts_arena *h, int32_t *trees_dev, spmcts_stream stream);
/* (sync) root statistics of one tree: children n/w/p (A each), root n/w, player, board */
int spmcts_root_stats(spmcts_arena *h, int32_t tree, int32_t *child_n, double *child_w, float *child_p,
                      int32_t *root_n, double *root_w, int32_t *root_player, int8_t *board /*[W*H]*/);

/* ---- games-level API (SelfPlayer.play_episode state machine) -------------- */
/* Start games in the listed slots (selfplayworker.py:172-179): both trees reset,
 * swap_sides = game id odd (self_play_parallel.py:237).  Game ids continue from
 * the arena's counter. */
int spmcts_games_start(spmcts_arena *h, const int32_t *slots_dev, const float *priors_dev /* NULL or [n][2][A] */,
                       int32_t n, spmcts_stream stream);
/* Cap on games started by automatic refill (< 0 = unlimited). */
int spmcts_games_set_limit(spmcts_arena *h, int64_t max_games);
/* Each active game's player to move begins its search (noise); active set = movers. */
int spmcts_games_begin_ply(spmcts_arena *h, spmcts_stream stream);
/* Each active game: _play on the mover, Move recorded, env.step, play_action on
 * both trees (selfplayworker.py:209-224); expansions go to the leaf batch. */
int spmcts_games_end_ply(spmcts_arena *h, void *leaves_dev, int32_t *leaf_count_dev, spmcts_stream stream);
/* Finished games: result, push_to_queue of both trees' Moves into the export
 * ring (mcts.py:225-232, selfplayworker.py:185-190), refill (if `refill`).
 * out_dev[0] = games finished this ply, out_dev[1] = records in the ring. */
int spmcts_games_finish_ply(spmcts_arena *h, int32_t refill, int32_t *out_dev /*[2]*/, spmcts_stream stream);
/* Copy the export ring out and clear it: states int8 [n][W*H], tree_probs f32
 * [n][A], q f64 [n], q_f64 u8 [n], z f32 [n] (actual_val), game ids i64 [n]. */
int spmcts_export_moves(spmcts_arena *h, int8_t *states_dev, float *tree_probs_dev, double *q_dev, uint8_t *q_f64_dev,
                        float *z_dev, int64_t *game_dev, int32_t max_records, int32_t *count_dev,
                        spmcts_stream stream);
/* (sync) per-slot game state: active flag, ply, swap, game id */
int spmcts_games_state(spmcts_arena *h, uint8_t *active, int32_t *ply, uint8_t *swap, int64_t *game_id);

/* ---- diagnostics --------------------------------------------------------- */
int spmcts_get_counters(spmcts_arena *h, spmcts_counters *out); /* (sync) */
int spmcts_check(spmcts_arena *h);                                /* (sync) <0 if a device error flag is set */

/* ---- stand-alone kernels -------------------------------------------------- */
/* Batched env step (Connect4Env.step connect4env.py:29-43 / TicTacToeEnv.step
 * tictactoe_env.py:23-33) on device: boards int8 [n][W][H]. status: 0 ok,
 * 1 ValueError (full column), 2 GameOver (over_dev[i] set). */
int spmcts_env_step(int32_t game, int32_t width, int32_t height, const int8_t *boards_dev, const int32_t *actions_dev,
                    const int8_t *players_dev, const uint8_t *over_dev, int32_t n, int8_t *out_boards_dev,
                    int8_t *reward_dev, uint8_t *done_dev, int8_t *status_dev, uint8_t *valid_dev,
                    spmcts_stream stream);
/* Host-compiled twin of the same bitboard code (single board, host pointers), used
 * by the Python env facade for interactive play (not on the self-play path). */
int spmcts_env_step_host(int32_t game, int32_t width, int32_t height, int8_t *board /*[W][H] in/out*/,
                         int32_t action, int32_t player, int32_t *reward, int32_t *done);
int spmcts_valid_moves_host(int32_t game, int32_t width, int32_t height, const int8_t *board, uint8_t *valid);
/* Deterministic table network (oracle/table_net.py) over leaf rows, for bit-exact
 * search parity tests: leaves in any spmcts_leaf_format/layout; per-row salts optional. */
int spmcts_table_net(int32_t game, int32_t width, int32_t height, const void *leaves_dev, int32_t leaf_format,
                     int32_t leaf_layout, int32_t n, uint64_t salt, const uint64_t *salts_dev /* [n] or NULL */,
                     float *probs_dev, float *values_dev, spmcts_stream stream);
/* Fused residual-tower trunk for leaf evaluation (games/general/modules.py:43-107
 * with BatchNorm folded): stem conv3x3 + num_blocks BasicBlocks + the policy/value
 * 1x1 head convs, bias + ReLU (+ residual) fused, activations resident in LDS,
 * bf16 (or, with SPMCTS_TOWER_F16, fp16 = the reference's autocast dtype,
 * inference_worker.py:117) MFMA with fp32 accumulation.  planes_dev: bf16 [batch][W][H][3]
 * (NHWC leaf rows, 0/1 planes); weights and features_dev [batch][W*H][channels/2] (policy |
 * value head channels, cell-major) in the flags' element type.  Packed weight/bias layout:
 * csrc/tower.hip.  Instantiated for 7x6 and 3x3 boards with channels 128 or 256. */
#define SPMCTS_TOWER_F16 2
int spmcts_tower_forward(int32_t width, int32_t height, int32_t channels, int32_t n_blocks, const void *planes_dev,
                         int32_t batch, const void *weights_dev, const float *bias_dev, void *features_dev,
                         int32_t flags, spmcts_stream stream);
/* The linear heads on the trunk features (modules.py:96-105), fused: policy softmax over
 * `actions` and tanh value.  head_w: bf16 rows [32 (policy, zero-padded)] ++ [8ff] over K = W*H*ff
 * columns in (cell, channel) order, fragment-swizzled: for 32-row tile j and 16-column step s, one
 * contiguous 1 KiB block whose 16-byte lane l holds row 32j + (l % 32), columns 16s + 8(l / 32) .. +8;
 * head_b: f32 bp[32] ++ bv[8ff] ++ wo[8ff] ++ bo.  flags: SPMCTS_TOWER_F16 = features and head_w
 * are fp16 (else bf16). */
int spmcts_tower_heads(int32_t width, int32_t height, int32_t channels, int32_t actions, const void *features_dev,
                       int32_t batch, const void *head_w_dev, const float *head_b_dev, float *probs_dev,
                       float *values_dev, int32_t flags, spmcts_stream stream);
/* Head epilogue after one GEMM Z = features @ Wc^T (Wc rows: value hidden [hidden] then
 * policy [actions]): value = tanh(relu(Z[:hidden] + bv) . wo + bo), probs = softmax(Z[hidden:] + bp).
 * z_dev bf16 [batch][ldz]; head_b: f32 bv[hidden] ++ wo[hidden] ++ bo ++ bp[actions]. */
int spmcts_head_epilogue(int32_t hidden, int32_t actions, const void *z_dev, int32_t ldz, int32_t batch,
                         const float *head_b_dev, float *probs_dev, float *values_dev, spmcts_stream stream);
int spmcts_tower_supported(int32_t width, int32_t height, int32_t channels);
/* The packed weight blob layout the trunk of this shape expects (replaces nothing in the reference: the
 * blob is this library's own format, built by evaluator.HipTowerEvaluator.refresh from the module's
 * state_dict, modules.py:88-107).  SPMCTS_WLAYOUT_32X32: every conv as [Cout/32][taps][Cin/16][64 lanes][8],
 * block and head convs' input channels in the phys_off order.  SPMCTS_WLAYOUT_M16 (the 7x6 C = 128 and
 * C = 256 trunks, tower_m16.h / tower_wide16.h): the stem as 32X32; the block convs as [Cout/16][taps][Cin/32][64 lanes][8] (lane 16q + n:
 * output channel 16 ct + n, input channels 32 k + 8 q ..) and the block and head convs' input channels in
 * the phys16 order.  Returns -2 for an unsupported shape. */
#define SPMCTS_WLAYOUT_32X32 0
#define SPMCTS_WLAYOUT_M16 1
int spmcts_tower_weight_layout(int32_t width, int32_t height, int32_t channels);
/* Device-count variants: the batch size is read from count_dev (e.g. the leaf-row count written by
 * spmcts_select) so no host synchronisation is needed; max_batch bounds the grid.
 * flags: SPMCTS_TOWER_PACK = the launch shares the chip with concurrent launches on other streams
 * (engine.LanedEngine): every board goes in full-size tiles and only the last few boards in one
 * smaller tile, instead of whole chip rounds of full tiles plus one round of smaller tiles;
 * SPMCTS_TOWER_F16 = fp16 weights / activations / features. */
#define SPMCTS_TOWER_PACK 1
int spmcts_tower_forward_dev(int32_t width, int32_t height, int32_t channels, int32_t n_blocks, const void *planes_dev,
                             const int32_t *count_dev, int32_t max_batch, const void *weights_dev,
                             const float *bias_dev, void *features_dev, int32_t flags, spmcts_stream stream);
int spmcts_tower_heads_dev(int32_t width, int32_t height, int32_t channels, int32_t actions, const void *features_dev,
                           const int32_t *count_dev, int32_t max_batch, const void *head_w_dev,
                           const float *head_b_dev, float *probs_dev, float *values_dev, int32_t flags,
                           spmcts_stream stream);
/* The trainer's 3x3 residual-block convolutions (stride 1, padding 1) on the matrix cores, fp16 NCHW tensors
 * as torch autocast hands them to conv2d (replaces MIOpen's conv2d forward / backward-data / backward-weight
 * calls that the UpdateWorker's autocast SGD step makes, updateworker.py:141-149 -> mcts.py:254-270 ->
 * modules.py:13-40); fp32 accumulation, deterministic (no atomics).
 *   _supported: 1 if the (board, channels) shape is handled, in both directions (forward and input grad).
 *   _pack: the fp32 parameter w [cout][cin][3][3], rounded to fp16 -> wf [cout][9][cin] (forward) and
 *          wb [cin][9][cout] (taps flipped: the input-gradient convolution's weights).
 *   _fwd: y [n][cout][W][H] (fp16) = fp16(bias) + conv(x [n][cin][W][H] fp16, wpk = wf of _pack); bias is the
 *         fp32 parameter or NULL.  The input gradient is _fwd(dy, wb) with cin and cout swapped and no bias.
 *   _wgrad: dw [cout][cin][3][3] = fp16(sum over the batch of dy x x-patches) stored as f32, one slice of 8
 *           boards per partial sum (splits must be ceil(n / 8)) into part [splits][cout][9][cin] (f32 scratch),
 *           summed in order; db [cout] (f32 of the fp16 sum, may be NULL) = sum of dy over the batch and cells.
 * Return 0, -1 bad argument, -2 unsupported shape, -3 launch error. */
int spmcts_conv3x3_supported(int32_t width, int32_t height, int32_t cin, int32_t cout);
int spmcts_conv3x3_pack(int32_t cin, int32_t cout, const void *w, void *wf, void *wb, spmcts_stream stream);
int spmcts_conv3x3_fwd(int32_t n, int32_t width, int32_t height, int32_t cin, int32_t cout, const void *x,
                       const void *wpk, const void *bias, void *y, spmcts_stream stream);
int spmcts_conv3x3_wgrad(int32_t n, int32_t width, int32_t height, int32_t cin, int32_t cout, const void *x,
                         const void *dy, float *part, int32_t splits, void *dw, void *db, spmcts_stream stream);
/* Memory-roofline helper: device copy bandwidth probe (bytes each way). */
int spmcts_copy_probe(const void *src_dev, void *dst_dev, uint64_t bytes, spmcts_stream stream);

#ifdef __cplusplus
}
#endif
#endif /* SPMCTS_H */
