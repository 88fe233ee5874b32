// Host build of csrc/field29.h (its functions are host+device): prints
// operands and results of the 29-bit-limb primitives for tests/test_field29.py
// to check against Python integers.
#include <stdio.h>

#include "../../quill-zkvm_amd/csrc/field29.h"
using namespace qg;

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  s ^= s << 13;
  s ^= s >> 7;
  s ^= s << 17;
  return (uint32_t)(s >> 16);
}

template <class C>
static Fp<C> rnd_below(int top_bits) {
  Fp<C> x;
  for (int i = 0; i < 8; i++) x.v[i] = rnd();
  x.v[7] &= (1u << (top_bits - 224)) - 1;
  return x;
}

static void pr(const char* k, const Fp<FqP>& x) {
  printf("%s=", k);
  for (int i = 7; i >= 0; i--) printf("%08x", x.v[i]);
  printf(" ");
}

int main() {
  for (int it = 0; it < 2000; it++) {
    // a, b < 2p-ish (254 bits), c < p (253 bits)
    Fp<FqP> a = rnd_below<FqP>(254), b = rnd_below<FqP>(254), c = rnd_below<FqP>(253);
    if (it == 0) a = Fp<FqP>::zero();
    F29<FqP> A = to29(a), B = to29(b), Cc = to29(c);
    F29<FqP> m = mul29(A, B);                       // a b 2^-261 mod p, < 2p
    F29<FqP> d = sub29(A, B);                       // a + 4p - b
    F29<FqP> md = mul29(norm29(d), Cc);             // (a - b) c 2^-261
    F29<FqP> r = red2p29(add29(m, Cc));             // (m + c) < 2p
    F29<FqP> lz = mul29(add29(A, B), Cc);           // lazy operand
    F29<FqP> sq = sqr29(norm29(sub29(A, B)));       // (a - b)^2 2^-261
    F29<FqP> ms = mulsub29(A, norm29(sub29(B, Cc)), Cc, m);  // a (b - c) - c m
    pr("a", a);
    pr("b", b);
    pr("c", c);
    pr("m", from29(m));
    pr("md", from29(md));
    pr("r", from29(r));
    pr("cm", from29(canon29(red2p29(m))));
    pr("lz", from29(lz));
    pr("sq", from29(sq));
    pr("ms", from29(ms));
    printf("\n");
  }
  // is_zero_mod29_fast: k p (k < 20) is zero, k p + 1 and random values are not
  int ok = 1;
  for (uint32_t k = 0; k < 20; k++) {
    F29<FqP> z = F29<FqP>::from_l9(l9_mul_small(F29P<FqP>::P, k));
    ok &= is_zero_mod29_fast<FqP, 20>(z) ? 1 : 0;
    ok &= is_zero_mod29_fast<FqP, 8>(z) == (k < 8) ? 1 : 0;
    F29<FqP> z1 = z;
    z1.l[0] += 1;
    ok &= !is_zero_mod29_fast<FqP, 20>(normfull29(z1)) ? 1 : 0;
  }
  for (int it = 0; it < 20000; it++) {
    const F29<FqP> a = to29(rnd_below<FqP>(254));
    ok &= is_zero_mod29_fast<FqP, 20>(a) == is_zero_mod29_20(a) ? 1 : 0;
  }
  printf("zerotest=%x\n", ok);
  return 0;
}
