/* gm_math.h -- fp64 sine / cosine shared by the device kernels and the CPU oracle.
 *
 * The physics needs sin / cos in three places (hinge rotations in mj_kinematics, the free
 * joint's quaternion update in mj_Euler, the gauge's joint points); libm (glibc) and the
 * device math library (ocml) round differently in the last bit, and a contact-rich grasp
 * amplifies a last-bit difference over a 63-substep env-step.  Both sides therefore use
 * this one implementation, so identical inputs give identical bits: Cody-Waite reduction
 * by pi/2 (33 + 53 bit split; exact for |x| < 2^20) and the fdlibm __kernel_sin /
 * __kernel_cos minimax polynomials (tail term zero), about 1 ulp.  Every operation is a
 * separately rounded IEEE-754 double operation written out explicitly (callers build with
 * FMA contraction off), so the result does not depend on the compiler or the target.
 */
#ifndef GM_MATH_H
#define GM_MATH_H

#if defined(__HIPCC__)
#define GM_MATH_FN __host__ __device__ static inline
#else
#define GM_MATH_FN static inline
#endif

#if defined(GM_LIBM_TRIG) && !defined(__HIPCC__)
/* the oracle's libm variant (oracle/Makefile liboracle_libm.so, test infrastructure):
 * glibc's own sin / cos, to show the shared kernel below is not what makes device and
 * oracle agree (tests/test_physics_independent.py) */
#include <math.h>
GM_MATH_FN void gm_sincos(double x, double* s, double* c) { *s = sin(x); *c = cos(x); }
#else
GM_MATH_FN void gm_sincos(double x, double* s, double* c) {
  const double invpio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00;   /* first 33 bits of pi/2 */
  const double pio2_1t = 6.07710050650619224932e-11;  /* pi/2 - pio2_1 */
  const double toint = 6755399441055744.0;            /* 1.5 * 2^52: round to nearest */
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double t = x * invpio2 + toint;
  const double fn = t - toint;
  const int n = (int)fn;
  const double r = (x - fn * pio2_1) - fn * pio2_1t;
  const double z = r * r;
  const double ps = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  const double sn = r + (z * r) * (S1 + z * ps);
  const double pc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  const double cs = 1.0 - (0.5 * z - z * pc);
  switch (n & 3) {
    case 0: *s = sn; *c = cs; break;
    case 1: *s = cs; *c = -sn; break;
    case 2: *s = -sn; *c = -cs; break;
    default: *s = -cs; *c = sn; break;
  }
}
#endif

GM_MATH_FN double gm_sin(double x) { double s, c; gm_sincos(x, &s, &c); return s; }
GM_MATH_FN double gm_cos(double x) { double s, c; gm_sincos(x, &s, &c); return c; }

#endif
