// dune-hdd_amd/csrc/kernels/trig_phase.hh -- sin / cos of the coefficient phases (OS2014 sinusoid
// kappa = a + b sin(kx x + ky y), problems/OS2014.hh:63-76; ESV2007 force a cos(kx x) cos(ky y),
// problems/ESV2007.hh:78), evaluated at every quadrature point of the smooth-coefficient kernels.
//
// Two-term Cody-Waite reduction by pi/2 with fma (the split's residual |pi/2 - P1 - P2| ~ 4e-33 keeps the
// reduced argument exact to rounding for |x| < 2^40), the fdlibm minimax kernels on [-pi/4, pi/4] and the
// quadrant by select: branch-free, max |error| vs libm 2.2e-16 (tests/test_trig_phase.py), and none of
// libm's Payne-Hanek large-argument path, whose registers cost the P1 smooth kernel its second wave per
// SIMD's worth of latency hiding (C3 0.38 -> 0.30 ms, profiles/r01/s3/ab_sin_phase.log).
// Host-compilable (the CPU accuracy test includes it with the HIP qualifiers defined away).
#pragma once
#include <cmath>
#include <cstdint>

namespace hdd {
namespace dev {

// value at quadrant offset `shift` (0: sin, 1: cos)
__host__ __device__ __forceinline__ double trig_phase(double x, int shift)
{
  const double k = rint(x * 0.63661977236758134308);
  double r = fma(-k, 1.57079632679489655800e+00, x);
  r = fma(-k, 6.12323399573676603587e-17, r);
  const double z = r * r;
  const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                          2.75573137070700676789e-06), -1.98412698298579493134e-04),
                               8.33333333332248946124e-03), -1.66666666666666324348e-01);
  const double sr = fma(r * z, ps, r);
  const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                          -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                               -1.38888888888741095749e-03), 4.16666666666666019037e-02);
  const double cr = fma(z * z, pc, fma(-0.5, z, 1.0));
  const int q = int((int64_t(k) + shift) & 3);
  const double v = (q & 1) ? cr : sr;
  return (q & 2) ? -v : v;
}
__host__ __device__ __forceinline__ double sin_phase(double x) { return trig_phase(x, 0); }
__host__ __device__ __forceinline__ double cos_phase(double x) { return trig_phase(x, 1); }

// sin and cos of one phase from one reduction (the two kernels trig_phase evaluates anyway)
__host__ __device__ __forceinline__ void sincos_phase(double x, double& s, double& c)
{
  const double k = rint(x * 0.63661977236758134308);
  double r = fma(-k, 1.57079632679489655800e+00, x);
  r = fma(-k, 6.12323399573676603587e-17, r);
  const double z = r * r;
  const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                          2.75573137070700676789e-06), -1.98412698298579493134e-04),
                               8.33333333332248946124e-03), -1.66666666666666324348e-01);
  const double sr = fma(r * z, ps, r);
  const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                          -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                               -1.38888888888741095749e-03), 4.16666666666666019037e-02);
  const double cr = fma(z * z, pc, fma(-0.5, z, 1.0));
  const int q = int(int64_t(k) & 3);
  const double sv = (q & 1) ? cr : sr, cv = (q & 1) ? sr : cr;
  s = (q & 2) ? -sv : sv;
  c = ((q + 1) & 2) ? -cv : cv;
}

// Small offsets from a reference phase: a quadrature point's phase is phi0 + d with |d| <= |grad phase| h, so
// on meshes fine against the coefficient's wavelength sin(phi0 + d) = s0 cos d + c0 sin d with one reduction
// per element (sincos_phase(phi0)) and Taylor polynomials in d per point: for |d| <= SMALL_PHASE the
// truncation (d^13 / 13!, d^12 / 12!) is below 2^-60 relative, i.e. the values equal sin_phase's to rounding.
constexpr double SMALL_PHASE = 0.125;
__host__ __device__ __forceinline__ void sincos_small(double d, double& s, double& c)
{
  const double z = d * d;
  s = d * fma(z, fma(z, fma(z, fma(z, fma(z, -2.5052108385441718775e-08, 2.7557319223985890653e-06),
                                   -1.9841269841269841270e-04), 8.3333333333333333333e-03),
                         -1.6666666666666666667e-01), 1.0);
  c = fma(z, fma(z, fma(z, fma(z, fma(z, -2.7557319223985890653e-07, 2.4801587301587301587e-05),
                               -1.3888888888888888889e-03), 4.1666666666666666667e-02), -0.5), 1.0);
}
// Tiny offsets (|d| <= TINY_PHASE = 1/64: meshes ~10x finer than SMALL_PHASE needs, e.g. the ESV2007 force on
// the C2 mesh, |d| <= 0.004): sin to d^7, cos to d^6 -- truncation d^9 / 9! < 1e-20 relative, d^8 / 8! < 1e-19
// absolute -- two multiply-adds fewer per value than sincos_small
constexpr double TINY_PHASE = 0.015625;
__host__ __device__ __forceinline__ void sincos_tiny(double d, double& s, double& c)
{
  const double z = d * d;
  s = d * fma(z, fma(z, fma(z, -1.9841269841269841270e-04, 8.3333333333333333333e-03), -1.6666666666666666667e-01), 1.0);
  c = fma(z, fma(z, fma(z, -1.3888888888888888889e-03, 4.1666666666666666667e-02), -0.5), 1.0);
}
__host__ __device__ __forceinline__ double cos_tiny(double s0, double c0, double d)
{
  double sd, cd;
  sincos_tiny(d, sd, cd);
  return fma(c0, cd, -(s0 * sd));
}
__host__ __device__ __forceinline__ double sin_tiny(double s0, double c0, double d)
{
  double sd, cd;
  sincos_tiny(d, sd, cd);
  return fma(s0, cd, c0 * sd);
}
__host__ __device__ __forceinline__ double sin_near(double s0, double c0, double d)
{
  double sd, cd;
  sincos_small(d, sd, cd);
  return fma(s0, cd, c0 * sd);
}
__host__ __device__ __forceinline__ double cos_near(double s0, double c0, double d)
{
  double sd, cd;
  sincos_small(d, sd, cd);
  return fma(c0, cd, -(s0 * sd));
}

}  // namespace dev
}  // namespace hdd
