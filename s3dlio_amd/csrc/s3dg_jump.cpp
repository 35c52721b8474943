// s3dg_jump.cpp — Xoshiro256++ jump-ahead polynomials (host side).
//
// The Xoshiro256 state transition T is linear over GF(2).  Its
// characteristic polynomial P (degree 256) is recovered once with
// Berlekamp-Massey from one state bit's sequence; then "advance n steps" is
// J(T)·s with J = x^n mod P, which a lane applies in 256 steps:
//   acc = 0; for i in 0..255: if J_i: acc ^= s;  s = T(s)
// (Vigna's jump() with a precomputed polynomial, generalised to any n).
// Used by the K2 keystream kernel, which gives every lane of a chunk its
// own starting draw (src/data_formats/npz.rs:381-382 fills one chunk with
// one sequential stream).
#include "s3dg_jump.h"

#include <cstring>
#include <mutex>
#include <vector>

namespace s3dg {
namespace {

inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

// State step without output (the output function does not feed back).
inline void step(uint64_t s[4]) {
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
}

// GF(2)[x] polynomials as little-endian 64-bit words.
using Poly = std::vector<uint64_t>;

int degree(const Poly &p) {
    for (int w = (int)p.size() - 1; w >= 0; --w)
        if (p[w]) return w * 64 + 63 - __builtin_clzll(p[w]);
    return -1;
}
bool bit(const Poly &p, int i) { return (size_t)(i >> 6) < p.size() && ((p[i >> 6] >> (i & 63)) & 1); }
void setbit(Poly &p, int i) {
    if ((size_t)(i >> 6) >= p.size()) p.resize((i >> 6) + 1, 0);
    p[i >> 6] ^= 1ull << (i & 63);
}

// Berlekamp-Massey over GF(2): connection polynomial C of sequence s[0..n).
Poly berlekamp_massey(const std::vector<uint8_t> &s) {
    const int n = (int)s.size();
    std::vector<uint8_t> C(n + 1, 0), B(n + 1, 0), T;
    C[0] = B[0] = 1;
    int L = 0, m = 1;
    for (int i = 0; i < n; ++i) {
        uint8_t d = s[i];
        for (int k = 1; k <= L; ++k) d ^= (uint8_t)(C[k] & s[i - k]);
        if (d == 0) { ++m; continue; }
        T = C;
        for (int k = 0; k + m <= n; ++k) C[k + m] ^= B[k];
        if (2 * L <= i) { L = i + 1 - L; B = T; m = 1; } else ++m;
    }
    // characteristic polynomial = reciprocal of C: P(x) = x^L C(1/x)
    Poly P;
    for (int k = 0; k <= L; ++k)
        if (C[k]) setbit(P, L - k);
    return P;
}

// r ^= p * x^sh (word-wise shift-xor; r long enough)
void xor_shifted(Poly &r, const Poly &p, int sh) {
    const int wo = sh >> 6, bo = sh & 63;
    for (size_t j = 0; j < p.size(); ++j) {
        if (!p[j]) continue;
        r[wo + j] ^= p[j] << bo;
        if (bo) r[wo + j + 1] ^= p[j] >> (64 - bo);
    }
}

// a * b mod P over GF(2): one shift-xor of b per set bit of a, then one of P
// per set bit at or above x^dP (round 5: word-wise, ~40x faster than bit by
// bit: 0.08 ms per jump polynomial instead of 3 ms)
Poly mulmod(const Poly &a, const Poly &b, const Poly &P, int dP) {
    const int da = degree(a), db = degree(b);
    Poly r((size_t)((da > 0 ? da : 0) + (db > 0 ? db : 0) + 64) / 64 + 2 + P.size(), 0);
    if (da >= 0 && db >= 0)
        for (int i = 0; i <= da; ++i)
            if (bit(a, i)) xor_shifted(r, b, i);
    for (int i = degree(r); i >= dP; --i)
        if (bit(r, i)) xor_shifted(r, P, i - dP);
    r.resize((dP + 63) / 64, 0);
    return r;
}

struct Engine {
    Poly P;
    int dP = -1;
};

const Engine &engine() {
    static Engine E;
    static std::once_flag once;
    std::call_once(once, [] {
        uint64_t s[4] = {0x0123456789ABCDEFull, 0x9E3779B97F4A7C15ull, 0xDEADBEEFCAFEF00Dull, 7ull};
        std::vector<uint8_t> seq(1024);
        for (auto &b : seq) { b = (uint8_t)(s[0] & 1); step(s); }
        E.P = berlekamp_massey(seq);
        E.dP = degree(E.P);
    });
    return E;
}

}  // namespace

int xoshiro_poly_degree() { return engine().dP; }

bool jump_poly(uint64_t n, uint64_t out[4]) {
    const Engine &E = engine();
    if (E.dP != 256) return false;
    Poly result(4, 0), base(4, 0);
    result[0] = 1;                      // x^0
    base[0] = 2;                        // x^1
    while (n) {
        if (n & 1) result = mulmod(result, base, E.P, E.dP);
        base = mulmod(base, base, E.P, E.dP);
        n >>= 1;
    }
    for (int k = 0; k < 4; ++k) out[k] = k < (int)result.size() ? result[k] : 0;
    return true;
}

bool jump_mul(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    const Engine &E = engine();
    if (E.dP != 256) return false;
    const Poly r = mulmod(Poly(a, a + 4), Poly(b, b + 4), E.P, E.dP);
    for (int k = 0; k < 4; ++k) out[k] = k < (int)r.size() ? r[k] : 0;
    return true;
}

void apply_jump(uint64_t s[4], const uint64_t J[4]) {
    uint64_t acc[4] = {0, 0, 0, 0};
    for (int i = 0; i < 256; ++i) {
        if ((J[i >> 6] >> (i & 63)) & 1)
            for (int k = 0; k < 4; ++k) acc[k] ^= s[k];
        step(s);
    }
    std::memcpy(s, acc, sizeof(acc));
}

}  // namespace s3dg
