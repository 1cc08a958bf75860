// Host build of the BN254 9 x 29-bit Montgomery field (geth-sharding_amd/csrc/bn254_fe9.cuh; plain
// C++ when __HIPCC__ is not defined), exported for tests/test_bn9.py.  Every export reports the
// (limb bound, value bound) its result type claims, so the test can hold the arithmetic to the
// magnitudes the compile-time checks rely on.
#include "../../geth-sharding_amd/csrc/bn254_fe9.cuh"
using namespace gsv::bn;

template <int L, int V>
static fqm<L, V> ld(const uint32_t* a) {
    fqm<L, V> r;
    for (int i = 0; i < 9; i++) r.v[i] = a[i];
    return r;
}
template <int L, int V>
static void st(uint32_t* r, int* lv, const fqm<L, V>& x) {
    for (int i = 0; i < 9; i++) r[i] = x.v[i];
    lv[0] = L;
    lv[1] = V;
}
#define MUL(La, Va, Lb, Vb)                                                                     \
    extern "C" void h_mul_##La##_##Va##_##Lb##_##Vb(uint32_t* r, int* lv, const uint32_t* a, \
                                                    const uint32_t* b) {                      \
        st(r, lv, fq_mul(ld<La, Va>(a), ld<Lb, Vb>(b)));                                       \
    }
MUL(1, 1, 1, 1)
MUL(1, 32, 1, 32)
MUL(2, 48, 3, 48)
MUL(6, 8, 1, 160)
MUL(3, 64, 2, 36)
MUL(8, 4, 8, 4)
#define MUL2(La, Va, Lb, Vb, Lc, Vc, Ld, Vd)                                                                    \
    extern "C" void h_mul2_##La##_##Va##_##Lb##_##Vb##_##Lc##_##Vc##_##Ld##_##Vd(                            \
        uint32_t* r, int* lv, const uint32_t* a, const uint32_t* b, const uint32_t* c, const uint32_t* d) {   \
        st(r, lv, fq_mul2(ld<La, Va>(a), ld<Lb, Vb>(b), ld<Lc, Vc>(c), ld<Ld, Vd>(d)));                       \
    }
MUL2(1, 32, 1, 32, 1, 32, 2, 34)
MUL2(2, 40, 1, 32, 2, 40, 2, 36)
MUL2(1, 3, 3, 3, 1, 3, 3, 3)
#define ADDSUB(La, Va, Lb, Vb)                                                                                  \
    extern "C" void h_add_##La##_##Va##_##Lb##_##Vb(uint32_t* r, int* lv, const uint32_t* a, const uint32_t* b) { \
        st(r, lv, fq_add(ld<La, Va>(a), ld<Lb, Vb>(b)));                                                       \
    }                                                                                                           \
    extern "C" void h_sub_##La##_##Va##_##Lb##_##Vb(uint32_t* r, int* lv, const uint32_t* a, const uint32_t* b) { \
        st(r, lv, fq_sub(ld<La, Va>(a), ld<Lb, Vb>(b)));                                                       \
    }
ADDSUB(1, 32, 1, 32)
ADDSUB(3, 40, 5, 48)
ADDSUB(7, 100, 6, 60)
ADDSUB(2, 160, 1, 160)
extern "C" void h_reduce(uint32_t* r, int* lv, const uint32_t* a) { st(r, lv, fq_reduce(ld<8, 160>(a))); }
extern "C" void h_canon(uint32_t* r, int* lv, const uint32_t* a) { st(r, lv, fq_canon(ld<8, 160>(a))); }
extern "C" void h_normalize(uint32_t* r, int* lv, const uint32_t* a) { st(r, lv, fq_normalize(ld<8, 160>(a))); }
extern "C" void h_neg(uint32_t* r, int* lv, const uint32_t* a) { st(r, lv, fq_neg(ld<6, 48>(a))); }
extern "C" void h_inv(uint32_t* r, int* lv, const uint32_t* a) { st(r, lv, fq_inv(ld<1, VS>(a))); }
extern "C" void h_mul_small8(uint32_t* r, int* lv, const uint32_t* a) { st(r, lv, fq_mul_small<8>(ld<1, 16>(a))); }
// tower: stored operands (fq = fqm<1, VS>), results stored
static fp2 ld2(const uint32_t* a) { return fp2{ld<1, VS>(a), ld<1, VS>(a + 9)}; }
static void st2(uint32_t* r, const fp2& x) { for (int i = 0; i < 9; i++) { r[i] = x.x.v[i]; r[9 + i] = x.y.v[i]; } }
static fp6 ld6(const uint32_t* a) { return fp6{ld2(a), ld2(a + 18), ld2(a + 36)}; }
template <class E>
static void st6(uint32_t* r, const fp6t<E>& x0) {
    fp6 x = fp6_store(x0);
    st2(r, x.x);
    st2(r + 18, x.y);
    st2(r + 36, x.z);
}
extern "C" int h_vs() { return VS; }
extern "C" void h_fp2_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) { st2(r, fp2_store(fp2_mul(ld2(a), ld2(b)))); }
extern "C" void h_fp2_sqr(uint32_t* r, const uint32_t* a) { st2(r, fp2_store(fp2_sqr(ld2(a)))); }
extern "C" void h_fp2_mul_xi(uint32_t* r, const uint32_t* a) { st2(r, fp2_store(fp2_mul_xi(ld2(a)))); }
extern "C" void h_fp2_inv(uint32_t* r, const uint32_t* a) { st2(r, fp2_inv(ld2(a))); }
extern "C" void h_fp6_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) { st6(r, fp6_mul(ld6(a), ld6(b))); }
extern "C" void h_fp6_sqr(uint32_t* r, const uint32_t* a) { st6(r, fp6_sqr(ld6(a))); }
extern "C" void h_fp6_sparse(uint32_t* r, const uint32_t* a, const uint32_t* by, const uint32_t* bz) {
    st6(r, fp6_mul_sparse(ld6(a), ld2(by), ld2(bz)));
}
extern "C" void h_fp6_inv(uint32_t* r, const uint32_t* a) { st6(r, fp6_inv(ld6(a))); }
extern "C" void h_fp6_frob(uint32_t* r, const uint32_t* a) { st6(r, fp6_frob(ld6(a))); }
extern "C" void h_fp6_frob_p2(uint32_t* r, const uint32_t* a) { st6(r, fp6_frob_p2(ld6(a))); }
extern "C" void h_fp6_mul_tau(uint32_t* r, const uint32_t* a) { st6(r, fp6_mul_tau(ld6(a))); }
// lazy operands: F_p^6 products of sums (value bound 64, limb bound 2) and a six-term dot product
// at its largest admissible bounds
extern "C" void h_fp6_mul_sums(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* c, const uint32_t* d) {
    st6(r, fp6_mul(fp6_add(ld6(a), ld6(b)), fp6_add(ld6(c), ld6(d))));
}
extern "C" void h_fp6_sparse_sum(uint32_t* r, const uint32_t* a, const uint32_t* b, const uint32_t* by, const uint32_t* bz) {
    st6(r, fp6_mul_sparse(fp6_add(ld6(a), ld6(b)), ld2(by), fp2_add(ld2(by), ld2(bz))));
}
extern "C" void h_fp6_sub_tau(uint32_t* r, const uint32_t* a, const uint32_t* b) {
    st6(r, fp6_sub(fp6_mul_tau(ld6(a)), fp6_neg(ld6(b))));
}
extern "C" void h_dot6(uint32_t* r, int* lv, const uint32_t* x) {
    st(r, lv, fq_dot(ld<1, 64>(x), ld<1, 64>(x + 9), ld<1, 64>(x + 18), ld<1, 64>(x + 27), ld<1, 64>(x + 36),
                     ld<1, 64>(x + 45), ld<1, 64>(x + 54), ld<1, 64>(x + 63), ld<1, 64>(x + 72), ld<1, 64>(x + 81),
                     ld<1, 64>(x + 90), ld<1, 64>(x + 99)));
}
