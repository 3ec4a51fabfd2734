// Exactness of ksa_sim::isqrt64 (csrc/sim/queue_sim.h) on the host: floor(sqrt(x)) for powers of
// two and their neighbours, squares and their neighbours across the single-precision range
// (r < 2^24), both sides of the 2^48 switch to the double-precision estimate, 2^64 - 1, and
// random values of every magnitude. Prints the failures; exit status 1 when there are any.
// Built and run by tests/test_isqrt.py.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../sim/queue_sim.h"

namespace {

long failures = 0;

void check(uint64_t x) {
  const uint64_t r = ksa_sim::isqrt64(x);
  const unsigned __int128 lo = static_cast<unsigned __int128>(r) * r;
  const unsigned __int128 hi = static_cast<unsigned __int128>(r + 1) * (r + 1);
  if (lo > x || hi <= x) {
    if (failures < 10) std::printf("isqrt64(%llu) = %llu\n", static_cast<unsigned long long>(x), static_cast<unsigned long long>(r));
    ++failures;
  }
}

}  // namespace

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 2000000;
  for (int k = 0; k < 64; ++k)
    for (int d = -3; d <= 3; ++d) check((uint64_t(1) << k) + static_cast<uint64_t>(static_cast<int64_t>(d)));
  for (uint64_t r = 1; r < (uint64_t(1) << 24); r += 997)
    for (int d = -1; d <= 1; ++d) check(r * r + static_cast<uint64_t>(static_cast<int64_t>(d)));
  for (uint64_t r = (uint64_t(1) << 24) - 64; r < (uint64_t(1) << 24) + 64; ++r)
    for (int d = -1; d <= 1; ++d) check(r * r + static_cast<uint64_t>(static_cast<int64_t>(d)));
  check(~uint64_t(0));
  std::mt19937_64 g(1);
  for (long i = 0; i < n; ++i) check(g() >> (g() % 64));
  std::printf("%ld failures\n", failures);
  return failures ? 1 : 0;
}
