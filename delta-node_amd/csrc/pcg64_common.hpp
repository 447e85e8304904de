// pcg64_common.hpp — PCG64 (numpy's default bit generator) constants and the
// closed-form jump tables, shared by host and device code.
//   step:   s <- a s + inc (mod 2^128), a = 0x2360ED051FC65DA4_4385DF649FCCF645
//   output: XSL-RR 128/64 of the new state (numpy pcg64.h)
//   T^r(s) = A_r s + inc G_r with A_r = a^r, G_r = sum_{i<r} a^i (mod 2^128)
#pragma once

#include <stdint.h>

namespace dn {

typedef unsigned __int128 u128;

__host__ __device__ inline u128 to_u128(uint64_t hi, uint64_t lo) { return (static_cast<u128>(hi) << 64) | lo; }

__host__ __device__ inline u128 pcg64_mult() { return to_u128(0x2360ED051FC65DA4ull, 0x4385DF649FCCF645ull); }

// jA[k], jG[k] = (A, G) of T^(2^k), k = 0..63.
inline void pcg64_jump_tables(u128 jA[64], u128 jG[64]) {
  u128 A = pcg64_mult(), G = 1;
  for (int k = 0; k < 64; ++k) {
    jA[k] = A;
    jG[k] = G;
    G = G * (A + 1);  // G_{2n} = G_n (A_n + 1)
    A = A * A;        // A_{2n} = A_n^2
  }
}

}  // namespace dn
