// Deterministic float sin/cos for rBRIEF steering, identical on host and gfx950.
//
// The reference steers the BRIEF pattern with `a = cos(angle), b = sin(angle)` on a
// float angle (src/ORBextractor.cc:155-157); g++ -O3 turns the pair into one glibc
// `sincosf` call.  glibc 2.35's sincosf is not correctly rounded, and the GPU's
// libm differs again, so neither can be used directly for bit-exact descriptors.
//
// Instead: evaluate sin/cos of the float argument in IEEE double with a fixed
// operation order (Cody-Waite reduction by pi/2, degree-17/18 Taylor polynomials),
// round to float.  Every operation is a single IEEE-754 double +, *, or rint, so the
// result is bit-identical on x86 (g++ -ffp-contract=off) and on gfx950
// (hipcc -ffp-contract=off).  Exhaustively over all 1,135,869,952 float degree angles
// in [0, 360), this differs from glibc sincosf on ~1.5M inputs, of which only the
// entries of orb_sincos_exceptions.inc change any of the 512 rounded pattern offsets;
// those angles take glibc's values from that table (tools/gen_sincos_exceptions.cpp).
#pragma once
#include <stdint.h>

#ifndef ORB_HD
#if defined(__HIPCC__)
#define ORB_HD __host__ __device__
#else
#define ORB_HD
#endif
#endif

ORB_HD static inline void orb_det_sincosf(float xf, float* s_out, float* c_out) {
    const double x = (double)xf;
    const double kTwoOverPi = 6.36619772367581382433e-01;
    const double kPio2Hi = 1.57079632673412561417e+00;   // first 33 bits of pi/2
    const double kPio2Lo = 6.07710050650619224932e-11;   // pi/2 - kPio2Hi
    const double n = __builtin_rint(x * kTwoOverPi);
    const double r = (x - n * kPio2Hi) - n * kPio2Lo;
    const double r2 = r * r;
    double sp = 2.81145725434552076319e-15;            //  1/17!
    sp = sp * r2 + -7.64716373181981647590e-13;         // -1/15!
    sp = sp * r2 + 1.60590438368216145994e-10;          //  1/13!
    sp = sp * r2 + -2.50521083854417187751e-08;         // -1/11!
    sp = sp * r2 + 2.75573192239858906526e-06;          //  1/9!
    sp = sp * r2 + -1.98412698412698412526e-04;         // -1/7!
    sp = sp * r2 + 8.33333333333333321769e-03;          //  1/5!
    sp = sp * r2 + -1.66666666666666657415e-01;         // -1/3!
    const double sn = r + r * (r2 * sp);
    double cp = 1.56192069685862264622e-16;             //  1/18!
    cp = cp * r2 + -4.77947733238738529744e-14;         // -1/16!
    cp = cp * r2 + 1.14707455977297247139e-11;          //  1/14!
    cp = cp * r2 + -2.08767569878680989792e-09;         // -1/12!
    cp = cp * r2 + 2.75573192239858906526e-07;          //  1/10!
    cp = cp * r2 + -2.48015873015873015658e-05;         // -1/8!
    cp = cp * r2 + 1.38888888888888894189e-03;          //  1/6!
    cp = cp * r2 + -4.16666666666666643537e-02;         // -1/4!
    cp = cp * r2 + 5.00000000000000000000e-01;          //  1/2!
    const double cs = 1.0 - r2 * cp;
    const int q = ((int)n) & 3;
    double s, c;
    if (q == 0)      { s = sn;  c = cs;  }
    else if (q == 1) { s = cs;  c = -sn; }
    else if (q == 2) { s = -sn; c = -cs; }
    else             { s = -cs; c = sn;  }
    *s_out = (float)s;
    *c_out = (float)c;
}
