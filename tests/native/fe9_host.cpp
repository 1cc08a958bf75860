// Host build of the device field/group arithmetic in secp256k1_fe9.cuh (plain C++: the header
// compiles for the host when __HIPCC__ is not defined), exported for tests/test_fe9.py.
#include "../../geth-sharding_amd/csrc/secp256k1_fe9.cuh"
using namespace gsv;
extern "C" {
void h_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) { fe9 x, y, z; for (int i = 0; i < 9; i++) { x.v[i] = a[i]; y.v[i] = b[i]; } fe9_mul(z, x, y); for (int i = 0; i < 9; i++) r[i] = z.v[i]; }
void h_sqr(uint32_t* r, const uint32_t* a) { fe9 x, z; for (int i = 0; i < 9; i++) x.v[i] = a[i]; fe9_sqr(z, x); for (int i = 0; i < 9; i++) r[i] = z.v[i]; }
void h_sub(uint32_t* r, const uint32_t* a, const uint32_t* b, int m) {
    fe9 x, y, z; for (int i = 0; i < 9; i++) { x.v[i] = a[i]; y.v[i] = b[i]; }
    switch (m) { case 1: fe9_sub<1>(z, x, y); break; case 2: fe9_sub<2>(z, x, y); break; case 3: fe9_sub<3>(z, x, y); break;
                 case 4: fe9_sub<4>(z, x, y); break; case 5: fe9_sub<5>(z, x, y); break; case 6: fe9_sub<6>(z, x, y); break; default: fe9_sub<7>(z, x, y); }
    for (int i = 0; i < 9; i++) r[i] = z.v[i];
}
void h_norm_weak(uint32_t* r) { fe9 x; for (int i = 0; i < 9; i++) x.v[i] = r[i]; fe9_normalize_weak(x); for (int i = 0; i < 9; i++) r[i] = x.v[i]; }
int h_is_zero_weak(const uint32_t* r) { fe9 x; for (int i = 0; i < 9; i++) x.v[i] = r[i]; return fe9_is_zero_weak(x) ? 1 : 0; }
void h_norm_full(uint32_t* r) { fe9 x; for (int i = 0; i < 9; i++) x.v[i] = r[i]; fe9_normalize_full(x); for (int i = 0; i < 9; i++) r[i] = x.v[i]; }
void h_inv(uint32_t* r, const uint32_t* a) { fe9 x, z; for (int i = 0; i < 9; i++) x.v[i] = a[i]; fe9_inv(z, x); for (int i = 0; i < 9; i++) r[i] = z.v[i]; }
void h_pow_pm3_4(uint32_t* r, const uint32_t* a) { fe9 x, z; for (int i = 0; i < 9; i++) x.v[i] = a[i]; fe9_pow_pm3_4(z, x); for (int i = 0; i < 9; i++) r[i] = z.v[i]; }
int h_sqrt(uint32_t* r, const uint32_t* a) { fe9 x, z; for (int i = 0; i < 9; i++) x.v[i] = a[i]; int ok = fe9_sqrt(z, x); for (int i = 0; i < 9; i++) r[i] = z.v[i]; return ok; }
void h_from_words(uint32_t* r, const uint32_t* w) { fe9 x; fe9_from_words(x, w); for (int i = 0; i < 9; i++) r[i] = x.v[i]; }
void h_to_words(uint32_t* w, const uint32_t* a) { fe9 x; for (int i = 0; i < 9; i++) x.v[i] = a[i]; fe9_to_words(w, x); }
// point ops: p = 27 words (X, Y, Z), q = 18 words (x, y)
void h_dbl(uint32_t* r, const uint32_t* p) { gej9 a, o; for (int i = 0; i < 9; i++) { a.x.v[i] = p[i]; a.y.v[i] = p[9 + i]; a.z.v[i] = p[18 + i]; } gej9_dbl(o, a); for (int i = 0; i < 9; i++) { r[i] = o.x.v[i]; r[9 + i] = o.y.v[i]; r[18 + i] = o.z.v[i]; } }
void h_add_ge(uint32_t* r, uint32_t* h, uint32_t* rr, const uint32_t* p, const uint32_t* q) {
    gej9 a, o; ge9 b; fe9 hh, r2;
    for (int i = 0; i < 9; i++) { a.x.v[i] = p[i]; a.y.v[i] = p[9 + i]; a.z.v[i] = p[18 + i]; b.x.v[i] = q[i]; b.y.v[i] = q[9 + i]; }
    gej9_add_ge_core(o, hh, r2, a, b);
    for (int i = 0; i < 9; i++) { r[i] = o.x.v[i]; r[9 + i] = o.y.v[i]; r[18 + i] = o.z.v[i]; h[i] = hh.v[i]; rr[i] = r2.v[i]; }
}
static void ld(gej9& a, const uint32_t* p) { for (int i = 0; i < 9; i++) { a.x.v[i] = p[i]; a.y.v[i] = p[9 + i]; a.z.v[i] = p[18 + i]; } }
static void st(uint32_t* r, const gej9& o) { for (int i = 0; i < 9; i++) { r[i] = o.x.v[i]; r[9 + i] = o.y.v[i]; r[18 + i] = o.z.v[i]; } }
int h_add_ge_full(uint32_t* r, const uint32_t* p, int pinf, const uint32_t* q) {
    gej9 a, o; ge9 b; ld(a, p);
    for (int i = 0; i < 9; i++) { b.x.v[i] = q[i]; b.y.v[i] = q[9 + i]; }
    bool inf = pinf != 0; gej9_add_ge(o, inf, a, b); st(r, o); return inf;
}
int h_add(uint32_t* r, const uint32_t* p, int pinf, const uint32_t* q, int qinf) {
    gej9 a, b, o; ld(a, p); ld(b, q); bool rinf; gej9_add(o, rinf, a, pinf != 0, b, qinf != 0); st(r, o); return rinf;
}
void h_build_table(uint32_t* T, uint32_t* zfac, const uint32_t* x, const uint32_t* y) {
    ge9 t[4]; fe9 z, X, Y; for (int i = 0; i < 9; i++) { X.v[i] = x[i]; Y.v[i] = y[i]; }
    build_r_table9(t, z, X, Y);
    for (int e = 0; e < 4; e++) for (int i = 0; i < 9; i++) { T[18 * e + i] = t[e].x.v[i]; T[18 * e + 9 + i] = t[e].y.v[i]; }
    for (int i = 0; i < 9; i++) zfac[i] = z.v[i];
}
}
#include "../../geth-sharding_amd/csrc/modinv30.cuh"
extern "C" void h_modinv(uint32_t* out, const uint32_t* x, int which) { modinv30_words(out, x, which == 2 ? MI30_BN : which ? MI30_P : MI30_N); }
