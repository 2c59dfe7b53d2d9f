// board.h — bitboard game rules shared by the HIP kernels and their host twins.
//
// Bit-exact restatement of the reference environments:
//   Connect4Env  games/connect4/connect4env.py:29-92 (step, valid_moves, get_reward)
//   TicTacToeEnv games/tictactoe/tictactoe_env.py:23-82
// Layout: one bit per cell, bit(x, y) = x * (H + 1) + y (x = column = board dim 0,
// y = row = board dim 1, row 0 = bottom).  Each column carries one always-zero
// sentinel bit, so shifted run detection never wraps between columns; every bit
// at or above W * (H + 1) is zero too.  A board is two masks: pieces of +1 and
// pieces of -1, in whatever frame the caller uses.
#pragma once
#include <stdint.h>

#ifndef SPM_HD
#define SPM_HD __host__ __device__ __forceinline__
#endif

namespace spm {

template <int W_, int H_, int L_, bool GRAVITY_>
struct Geo {
  static constexpr int W = W_, H = H_, L = L_;
  static constexpr bool GRAVITY = GRAVITY_;          // Connect4: piece drops to the column height
  static constexpr int A = GRAVITY_ ? W_ : W_ * H_;  // action_space.n
  static constexpr int APAD = A <= 8 ? 8 : 16;       // lanes per tree (power of two)
  static constexpr int CB = H_ + 1;                  // bits per column incl. sentinel
  static constexpr int CELLS = W_ * H_;
  static constexpr int MAXD = W_ * H_ + 2;           // max path length (root .. leaf)
  static constexpr int MAXM = (W_ * H_ + 1) / 2 + 1; // max Move records per tree per game
  static_assert(W_ * (H_ + 1) <= 64, "board does not fit a 64-bit mask");
  static_assert(A <= 16, "too many actions for one lane group");
};

using C4 = Geo<7, 6, 4, true>;
using TTT = Geo<3, 3, 3, false>;

struct Board {
  uint64_t pos;  // pieces of +1
  uint64_t neg;  // pieces of -1
};

SPM_HD int popc(uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popcll(v);
#else
  return __builtin_popcountll(v);
#endif
}

template <class G>
SPM_HD int cell_bit(int x, int y) { return x * G::CB + y; }

template <class G>
SPM_HD uint64_t col_mask(int x) { return ((1ull << G::H) - 1ull) << (x * G::CB); }

// All cells of the maximal board line through (x, y) along (dx, dy).
template <class G>
SPM_HD uint64_t line_mask(int x, int y, int dx, int dy) {
  while (x - dx >= 0 && x - dx < G::W && y - dy >= 0 && y - dy < G::H) {
    x -= dx;
    y -= dy;
  }
  uint64_t m = 0;
  while (x >= 0 && x < G::W && y >= 0 && y < G::H) {
    m |= 1ull << cell_bit<G>(x, y);
    x += dx;
    y += dy;
  }
  return m;
}

// get_reward (connect4env.py:72-84, tictactoe_env.py:63-75): the reference folds a
// saturating run counter over the whole row, column and both diagonals through
// (x, y) and reports a win iff any of those four lines holds a run of >= L of
// `mine`.  Runs: r has bit i set iff cells i, i+s, ..., i+(L-1)s are all set;
// a run lies on the line through (x, y) iff its first cell does.
template <class G>
SPM_HD bool win_through(uint64_t mine, int x, int y) {
  const int dxs[4] = {1, 0, 1, 1};
  const int dys[4] = {0, 1, 1, -1};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int s = dxs[d] * G::CB + dys[d];
    uint64_t r = mine;
#pragma unroll
    for (int k = 1; k < G::L; ++k) r &= mine >> (k * s);
    if (r & line_mask<G>(x, y, dxs[d], dys[d])) return true;
  }
  return false;
}

// valid_moves: Connect4 heights < height (heights = column |piece| sums,
// connect4env.py:47-48, :56-58); TicTacToe empty cells (tictactoe_env.py:42-43).
template <class G>
SPM_HD uint32_t legal_mask(Board b) {
  const uint64_t occ = b.pos | b.neg;
  uint32_t m = 0;
  if (G::GRAVITY) {
#pragma unroll
    for (int x = 0; x < G::W; ++x)
      if (popc(occ & col_mask<G>(x)) < G::H) m |= 1u << x;
  } else {
#pragma unroll
    for (int a = 0; a < G::A; ++a)
      if (!((occ >> cell_bit<G>(a / G::H, a % G::H)) & 1ull)) m |= 1u << a;
  }
  return m;
}

enum StepStatus { STEP_OK = 0, STEP_VALUE_ERROR = 1, STEP_GAME_OVER = 2 };

// step(action, player) (connect4env.py:29-43, tictactoe_env.py:23-33).
// Connect4: drop at row = number of pieces in the column, ValueError when full.
// TicTacToe: (x, y) = unravel_index(a, (W, H)); an occupied cell is a silent no-op
// but the reward/done check still runs.  done = win or board full.
template <class G>
SPM_HD int step(Board &b, int a, int player, int *reward, int *done) {
  const uint64_t occ = b.pos | b.neg;
  int x, y;
  if (G::GRAVITY) {
    x = a;
    y = popc(occ & col_mask<G>(x));
    if (y >= G::H) {
      *reward = 0;
      *done = 0;
      return STEP_VALUE_ERROR;
    }
  } else {
    x = a / G::H;
    y = a % G::H;
  }
  const uint64_t bit = 1ull << cell_bit<G>(x, y);
  if (!(occ & bit)) {
    if (player > 0)
      b.pos |= bit;
    else
      b.neg |= bit;
  }
  const uint64_t mine = player > 0 ? b.pos : b.neg;
  const int r = win_through<G>(mine, x, y) ? 1 : 0;
  *reward = r;
  *done = (r != 0) || (popc(b.pos | b.neg) == G::CELLS);
  return STEP_OK;
}

// Apply a move already known to be legal and non-terminal (tree descent).
template <class G>
SPM_HD void play(Board &b, int a, int player) {
  const uint64_t occ = b.pos | b.neg;
  int x, y;
  if (G::GRAVITY) {
    x = a;
    y = popc(occ & col_mask<G>(x));
  } else {
    x = a / G::H;
    y = a % G::H;
  }
  const uint64_t bit = 1ull << cell_bit<G>(x, y);
  if (player > 0)
    b.pos |= bit;
  else
    b.neg |= bit;
}

template <class G>
SPM_HD Board from_cells(const int8_t *c) {  // int8 [W][H] values in {-1, 0, 1}
  Board b{0, 0};
  for (int x = 0; x < G::W; ++x)
    for (int y = 0; y < G::H; ++y) {
      const int v = c[x * G::H + y];
      if (v > 0) b.pos |= 1ull << cell_bit<G>(x, y);
      if (v < 0) b.neg |= 1ull << cell_bit<G>(x, y);
    }
  return b;
}

template <class G>
SPM_HD int8_t cell_value(Board b, int x, int y) {
  const uint64_t bit = 1ull << cell_bit<G>(x, y);
  return (b.pos & bit) ? int8_t(1) : ((b.neg & bit) ? int8_t(-1) : int8_t(0));
}

// ---- deterministic table network (oracle/table_net.py) ----------------------
SPM_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace spm
