// Host build of coa_lehmer.h (tests/test_lehmer_host.py): exposes one Lehmer
// step to Python, which checks every state it reaches against an exact
// big-integer Euclidean algorithm.  Test infrastructure only.
#include <stdint.h>
#define COA_LH inline
#include "coa_lehmer.h"

extern "C" int lehmer_step(uint32_t* a, uint32_t* b, uint32_t* ta, uint32_t* tb, int stop_bits) {
  return coa_lehmer::step(a, b, ta, tb, stop_bits);
}
