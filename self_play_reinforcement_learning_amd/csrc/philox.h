// philox.h — per-lane Philox4x32-10 draws on rocRAND's state, without rocRAND's run-time indexing.
//
// The search draws one double per child lane from a shared tree stream: lane j takes the 2 words at
// position 2j past the state (skipahead(2j) + rocrand_uniform_double), then the state advances by
// 2A words.  rocRAND's engine reads its 4-word output block at a run-time `substate` index, which
// puts the whole state in scratch memory on every draw (a private-memory round trip per tree level
// in k_select_vl / k_expand_vl).  These helpers compute the same words from the counter, key and
// substate directly — the two output blocks a draw can touch, words picked by select — and leave
// rocRAND's invariant `result == philox10(counter)` to the caller's final store (philox_sync).
// Bit-identical to the rocRAND calls they replace (tests/test_philox.py checks them on the host
// against rocRAND itself over random states and offsets).
#pragma once
#include <hip/hip_runtime.h>
#include <rocrand/rocrand_philox4x32_10.h>
#include <rocrand/rocrand_uniform.h>

namespace spm {

// rocrand_state_philox4x32_10's leading fields (the engine keeps its state protected; it is the
// engine's only data member and these are its first four fields, in this order).
struct PhiloxFields {
  uint4 counter;
  uint4 result;
  uint2 key;
  unsigned int substate;
};
static_assert(sizeof(rocrand_state_philox4x32_10) >= sizeof(PhiloxFields), "rocRAND Philox state layout");

__host__ __device__ __forceinline__ PhiloxFields philox_fields(const rocrand_state_philox4x32_10 &s) {
  PhiloxFields f;
  __builtin_memcpy(&f, &s, sizeof f);
  return f;
}

__host__ __device__ __forceinline__ void philox_put(rocrand_state_philox4x32_10 &s, const PhiloxFields &f) {
  __builtin_memcpy(&s, &f, sizeof f);
}

// counter + off, with rocRAND's carry rule (discard_state)
__host__ __device__ __forceinline__ uint4 philox_add(uint4 c, unsigned long long off) {
  const unsigned int lo = (unsigned int)off, hi = (unsigned int)(off >> 32);
  const uint4 t = c;
  c.x += lo;
  c.y += hi + (c.x < t.x ? 1u : 0u);
  c.z += (c.y < t.y ? 1u : 0u);
  c.w += (c.z < t.z ? 1u : 0u);
  return c;
}

// counter + 1 (rocRAND's bump_counter, taken when a draw crosses into the next block)
__host__ __device__ __forceinline__ uint4 philox_bump(uint4 c) {
  c.x += 1u;
  unsigned int add = c.x == 0u ? 1u : 0u;
  c.y += add;
  add = c.y == 0u ? add : 0u;
  c.z += add;
  add = c.z == 0u ? add : 0u;
  c.w += add;
  return c;
}

// the 4-word output block of a counter: 10 Philox4x32 rounds (Random123 constants)
__host__ __device__ __forceinline__ uint4 philox10(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const unsigned long long m0 = (unsigned long long)ROCRAND_PHILOX_M4x32_0 * c.x;
    const unsigned long long m1 = (unsigned long long)ROCRAND_PHILOX_M4x32_1 * c.z;
    c = uint4{(unsigned int)(m1 >> 32) ^ c.y ^ k.x, (unsigned int)m1, (unsigned int)(m0 >> 32) ^ c.w ^ k.y,
              (unsigned int)m0};
    k.x += ROCRAND_PHILOX_W32_0;
    k.y += ROCRAND_PHILOX_W32_1;
  }
  return c;
}

__host__ __device__ __forceinline__ unsigned int philox_word(uint4 b, unsigned int w) {
  return w == 0u ? b.x : w == 1u ? b.y : w == 2u ? b.z : b.w;
}

// skipahead(off) without regenerating `result` (rocRAND's discard_impl)
__host__ __device__ __forceinline__ void philox_skip(PhiloxFields &f, unsigned long long off) {
  unsigned int sub = f.substate + (unsigned int)(off & 3u);
  unsigned long long co = off >> 2;
  if (sub >= 4u) {
    co += 1u;
    sub -= 4u;
  }
  f.substate = sub;
  f.counter = philox_add(f.counter, co);
}

// rocrand_uniform_double(state after skipahead(off)): the words at offsets off and off + 1
__host__ __device__ __forceinline__ double philox_uniform_at(PhiloxFields f, unsigned long long off) {
  philox_skip(f, off);
  const uint4 b0 = philox10(f.counter, f.key);
  const uint4 b1 = philox10(philox_bump(f.counter), f.key);
  const unsigned int w = f.substate;
  const unsigned int v1 = philox_word(b0, w);
  const unsigned int v2 = w < 3u ? philox_word(b0, w + 1u) : b1.x;
  return rocrand_device::detail::uniform_distribution_double(v1, v2);
}

// The same draws for a whole group of lanes at once: lane j's words sit at positions sub + 2j and
// sub + 2j + 1 past the state's block, i.e. in output blocks (sub + 2j) >> 2 and the next one, so the
// group computes each block once (lane b: block b) and every lane picks its words from the lane that
// holds them, instead of every lane computing two blocks.  Host-testable pieces:
__host__ __device__ __forceinline__ void philox_group_src(unsigned int sub, int j, int &blk, unsigned int &w) {
  const unsigned int p = sub + 2u * (unsigned int)j;
  blk = (int)(p >> 2);
  w = p & 3u;
}

// the draw from block `b` (word w, and w + 1 or the next block's first word)
__host__ __device__ __forceinline__ double philox_group_value(uint4 b, unsigned int next_x, unsigned int w) {
  const unsigned int v1 = philox_word(b, w);
  const unsigned int v2 = w < 3u ? philox_word(b, w + 1u) : next_x;
  return rocrand_device::detail::uniform_distribution_double(v1, v2);
}

// Device form: every lane of the P-lane group (gbase = its first lane in the wave) must call it;
// lane j's result equals philox_uniform_at(f, 2j).  Blocks up to (3 + 2P) / 4 + 1 < P are needed.
template <int P>
__device__ __forceinline__ double philox_uniform_group(const PhiloxFields &f, int j, int gbase) {
  static_assert((3 + 2 * P) / 4 + 1 < P, "the group holds every block its draws touch");
  const uint4 mine = philox10(philox_add(f.counter, (unsigned long long)j), f.key);  // block j
  int blk;
  unsigned int w;
  philox_group_src(f.substate, j, blk, w);
  const int src = gbase + (blk < P ? blk : P - 1);
  const int nxt = gbase + (blk + 1 < P ? blk + 1 : P - 1);
  const uint4 b = uint4{(unsigned int)__shfl((int)mine.x, src, 64), (unsigned int)__shfl((int)mine.y, src, 64),
                        (unsigned int)__shfl((int)mine.z, src, 64), (unsigned int)__shfl((int)mine.w, src, 64)};
  const unsigned int nx = (unsigned int)__shfl((int)mine.x, nxt, 64);
  return philox_group_value(b, nx, w);
}

// restore rocRAND's invariant result == philox10(counter) before the state is stored or handed to
// rocRAND's own functions
__host__ __device__ __forceinline__ void philox_sync(PhiloxFields &f) { f.result = philox10(f.counter, f.key); }

}  // namespace spm
