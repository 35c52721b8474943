// s3dg_jump.h — Xoshiro256 jump-ahead polynomials (see s3dg_jump.cpp).
#pragma once
#include <stdint.h>

namespace s3dg {
// Degree of the recovered characteristic polynomial (256 when healthy).
int xoshiro_poly_degree();
// J = x^n mod P as 4 little-endian words; false if P could not be recovered.
bool jump_poly(uint64_t n, uint64_t out[4]);
// s <- T^n s for the n that produced J (host reference of the device jump).
void apply_jump(uint64_t s[4], const uint64_t J[4]);
// out = a * b mod P: the jump by n + m from the jumps by n and by m
bool jump_mul(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]);
}  // namespace s3dg
