// Host-side check of csrc/philox.h against rocRAND's own Philox engine (compiled by
// tests/test_philox.py with hipcc; runs on the CPU, no GPU calls).  For random states (seed,
// subsequence, offset, so every substate and counter carries occur) and every lane offset the
// search uses, the direct draw must equal skipahead(2j) + rocrand_uniform_double bit for bit, and
// advance + sync must reproduce skipahead(2k)'s whole state.
#include <stdio.h>
#include <string.h>

#include "philox.h"

using namespace spm;

static unsigned long long lcg(unsigned long long &x) {
  x = x * 6364136223846793005ull + 1442695040888963407ull;
  return x;
}

int main() {
  unsigned long long seed = 12345;
  long checks = 0, bad = 0;
  for (int it = 0; it < 4000; ++it) {
    rocrand_state_philox4x32_10 s;
    const unsigned long long sd = lcg(seed), sub = lcg(seed) >> (it % 3 == 0 ? 0 : 40);
    unsigned long long off = lcg(seed) >> (it % 2 ? 58 : 20);
    if (it % 7 == 0) off = 0xfffffffcull * 4 + (it & 3);  // counter.x carry into .y
    rocrand_init(sd, sub, off, &s);
    // a few rocRAND draws first: substate anywhere in 0..3
    for (int d = 0; d < it % 5; ++d) (void)rocrand(&s);
    for (int j = 0; j < 16; ++j) {
      rocrand_state_philox4x32_10 a = s;
      skipahead(2ull * j, &a);
      const double want = rocrand_uniform_double(&a);
      const double got = philox_uniform_at(philox_fields(s), 2ull * j);
      ++checks;
      if (memcmp(&want, &got, sizeof want) != 0) {
        if (bad < 5) printf("draw mismatch it=%d j=%d %.17g %.17g\n", it, j, want, got);
        ++bad;
      }
    }
    // the group form's index math: lane j's draw from the blocks b = 0, 1, ... (block b = counter + b)
    {
      const PhiloxFields f = philox_fields(s);
      uint4 blocks[12];
      for (int b = 0; b < 12; ++b) blocks[b] = philox10(philox_add(f.counter, (unsigned long long)b), f.key);
      for (int j = 0; j < 16; ++j) {
        int blk;
        unsigned int w;
        philox_group_src(f.substate, j, blk, w);
        const double got = philox_group_value(blocks[blk], blocks[blk + 1].x, w);
        const double want = philox_uniform_at(f, 2ull * j);
        ++checks;
        if (memcmp(&want, &got, sizeof want) != 0) {
          if (bad < 5) printf("group draw mismatch it=%d j=%d\n", it, j);
          ++bad;
        }
      }
    }
    for (int k = 1; k <= 16; k += 3) {
      rocrand_state_philox4x32_10 a = s;
      skipahead(2ull * k, &a);
      PhiloxFields f = philox_fields(s);
      philox_skip(f, 2ull * k);
      philox_sync(f);
      const PhiloxFields w = philox_fields(a);
      ++checks;
      if (memcmp(&w, &f, sizeof f) != 0) {
        if (bad < 5) printf("advance mismatch it=%d k=%d\n", it, k);
        ++bad;
      }
      // and rocRAND continues identically from the synced state
      rocrand_state_philox4x32_10 b = s;
      philox_put(b, f);
      const unsigned int ra = rocrand(&a), rb = rocrand(&b);
      ++checks;
      if (ra != rb) ++bad;
    }
  }
  printf("checks %ld mismatches %ld\n", checks, bad);
  return bad ? 1 : 0;
}
