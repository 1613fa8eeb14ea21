// dune-hdd_amd/csrc/kernels/swipdg_device.hh -- shared by the swipdg_*.hip translation units (one per kernel
// family, so the template instantiations compile in parallel).
//
// CDNA4 (gfx950) kernels of the SWIPDG stiffness assembly -- the MI355X replacement of dune-gdt's
// SystemAssembler::walk() over Operators::EllipticSWIPDG (reference call sites:
// dune/hdd/linearelliptic/discretizations/swipdg.hh:218-249, 485; block-swipdg.hh:1136-1179, 1270-1326).
//
// Design:
//   * owner-computes: the rows of an element are written by the lanes that own the element; every face
//     term is evaluated by the row owner on its side (entity/entity + entity/neighbour blocks), so each
//     CSR value is written exactly once, with no atomics and no zero-fill, in one pass over the mesh;
//   * a workgroup = one tile of 64 consecutive owned elements; WPE waves per tile, wave w owns the local
//     test functions (rows) [w*RPT, (w+1)*RPT) of the 64 elements, lane = element (coalesced SoA loads);
//   * the row block of an element is contiguous in the CSR value array (sorted blocks, element-blocked
//     DoFs), so each wave stages one row of its 64 elements in LDS and streams it out with consecutive
//     lanes on consecutive values (6-12 cache lines per store instruction instead of 64);
//   * reference-element basis/quadrature tables are compile-time constants (immediates), not LDS: at
//     p = 1 they are a handful of numbers per rule;
//   * the neighbour geometry is rebuilt from the shared face vertices plus the neighbour's non-face
//     vertices (twin face / orientation from face_info), so a face gathers 2 (triangle) or 4 (quad)
//     coordinates, the neighbour's tensor and coefficient;
//   * XCD-aware tile order: consecutive tiles run on one XCD so the neighbour rows above/below a tile
//     hit that XCD's L2.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "hdd.h"
#include "hdd_internal.hh"
#include "swipdg_kernels.hh"
#include "flattop.hh"
#include "trig_phase.hh"

#ifndef HDD_MIN_WAVES_PER_EU
#define HDD_MIN_WAVES_PER_EU 4
#endif
// profiling ablations (HDD_DEBUG_FLAGS at run time) exist only in a library built with -DHDD_ABLATION
// (scripts/ablate.py): 1 = skip compute, 2 = drop the value stores, 4 = skip the neighbour gathers
#ifdef HDD_ABLATION
#define HDD_ABL(a, bit) (((a).debug_flags & (bit)) != 0)
#else
#define HDD_ABL(a, bit) false
#endif

namespace hdd {
namespace dev {

// ------------------------------------------------------------------------------------------------
// reference elements (Dune numbering) and shape functions
// ------------------------------------------------------------------------------------------------
struct Simplex {
  static constexpr int NV = 3, NF = 3, NB = 3;
  // vertex k of the reference simplex: (0,0), (1,0), (0,1)
  __host__ __device__ static constexpr double rv(int k, int d) { return (k == 1 + d) ? 1.0 : 0.0; }
  // faces 0:(0,1) 1:(0,2) 2:(1,2)
  __host__ __device__ static constexpr int fv(int f, int k) { return f == 0 ? k : (f == 1 ? 2 * k : 1 + k); }
  // orientation of (t_y, -t_x) w.r.t. the outer normal on the reference element
  __host__ __device__ static constexpr double face_sign(int f) { return f == 1 ? -1.0 : 1.0; }
  __device__ static inline void shape(double x, double y, double* phi, double* gx, double* gy)
  {
    phi[0] = 1.0 - x - y; phi[1] = x; phi[2] = y;
    gx[0] = -1.0; gy[0] = -1.0;
    gx[1] = 1.0;  gy[1] = 0.0;
    gx[2] = 0.0;  gy[2] = 1.0;
  }
};

struct Cube {
  static constexpr int NV = 4, NF = 4, NB = 4;
  // vertex k: (k & 1, k >> 1)
  __host__ __device__ static constexpr double rv(int k, int d) { return double((k >> d) & 1); }
  // faces 0:(0,2) 1:(1,3) 2:(0,1) 3:(2,3)
  __host__ __device__ static constexpr int fv(int f, int k)
  {
    return f == 0 ? 2 * k : (f == 1 ? 1 + 2 * k : (f == 2 ? k : 2 + k));
  }
  __host__ __device__ static constexpr double face_sign(int f) { return (f == 0 || f == 3) ? -1.0 : 1.0; }
  __device__ static inline void shape(double x, double y, double* phi, double* gx, double* gy)
  {
    phi[0] = (1 - x) * (1 - y); phi[1] = x * (1 - y); phi[2] = (1 - x) * y; phi[3] = x * y;
    gx[0] = -(1 - y); gy[0] = -(1 - x);
    gx[1] = (1 - y);  gy[1] = -x;
    gx[2] = -y;       gy[2] = (1 - x);
    gx[3] = y;        gy[3] = x;
  }
};

// ------------------------------------------------------------------------------------------------
// quadrature (compile-time): Gauss-Legendre on [0,1]; simplex centroid / 3-point / Dunavant-6
// ------------------------------------------------------------------------------------------------
template <int N>
struct Gauss01;
template <>
struct Gauss01<1> {
  __device__ static constexpr double s(int) { return 0.5; }
  __device__ static constexpr double w(int) { return 1.0; }
};
template <>
struct Gauss01<2> {
  __device__ static constexpr double s(int q) { return q == 0 ? 0.21132486540518711775 : 0.78867513459481288225; }
  __device__ static constexpr double w(int) { return 0.5; }
};
template <>
struct Gauss01<3> {
  __device__ static constexpr double s(int q)
  {
    return q == 0 ? 0.11270166537925831148 : (q == 1 ? 0.5 : 0.88729833462074168852);
  }
  __device__ static constexpr double w(int q) { return q == 1 ? 8.0 / 18.0 : 5.0 / 18.0; }
};

template <class E, int NQ>
struct VolRule;
template <>
struct VolRule<Simplex, 1> {
  __device__ static constexpr double x(int) { return 1.0 / 3.0; }
  __device__ static constexpr double y(int) { return 1.0 / 3.0; }
  __device__ static constexpr double w(int) { return 0.5; }
};
template <>
struct VolRule<Simplex, 3> {
  __device__ static constexpr double x(int q) { return q == 1 ? 2.0 / 3.0 : 1.0 / 6.0; }
  __device__ static constexpr double y(int q) { return q == 2 ? 2.0 / 3.0 : 1.0 / 6.0; }
  __device__ static constexpr double w(int) { return 1.0 / 6.0; }
};
template <>
struct VolRule<Simplex, 6> {  // Dunavant degree 4 (used for integrand orders 3 and 4)
  static constexpr double A = 0.44594849091596488632, WA = 0.22338158967801146570;
  static constexpr double B = 0.091576213509770743460, WB = 0.10995174365532186764;
  __device__ static constexpr double pa(int k, int d) { return k == 0 ? A : ((k == 1) == (d == 0) ? 1 - 2 * A : A); }
  __device__ static constexpr double pb(int k, int d) { return k == 0 ? B : ((k == 1) == (d == 0) ? 1 - 2 * B : B); }
  __device__ static constexpr double x(int q) { return q < 3 ? pa(q, 0) : pb(q - 3, 0); }
  __device__ static constexpr double y(int q) { return q < 3 ? pa(q, 1) : pb(q - 3, 1); }
  __device__ static constexpr double w(int q) { return q < 3 ? 0.5 * WA : 0.5 * WB; }
};
template <int NQ>
struct VolRule<Cube, NQ> {   // tensor Gauss, NQ = n*n, point q = j*n + i
  static constexpr int N = NQ == 1 ? 1 : (NQ == 4 ? 2 : 3);
  __device__ static constexpr double x(int q) { return Gauss01<N>::s(q % N); }
  __device__ static constexpr double y(int q) { return Gauss01<N>::s(q / N); }
  __device__ static constexpr double w(int q) { return Gauss01<N>::w(q % N) * Gauss01<N>::w(q / N); }
};

// ------------------------------------------------------------------------------------------------
// coefficients
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double kappa_elem(const KappaArg& k, int64_t e)
{
  return k.kind == HDD_FN_PER_ELEM ? k.per_elem[e] : k.c;
}
// |F|^-beta for beta != 1 (the 2d default is beta = 1/(d-1) = 1, taken inline as 1/|F|): out of line, so
// libm's pow and its registers stay out of the closed-form kernels' main path (P1 226 -> 191 VGPRs, Q1
// 62 -> 26 AGPR spill slots)
__device__ __attribute__((noinline)) double inv_pow(double len, double beta) { return 1.0 / pow(len, beta); }
__device__ __forceinline__ double kappa_at(const KappaArg& k, double pe, double x, double y)
{
  if (k.kind == HDD_FN_FLATTOP) return flattop_sum(k.table, k.n_table, k.c, k.b, x, y);
  return k.kind == HDD_FN_SINUSOID ? k.c + k.b * sin_phase(k.kx * x + k.ky * y) : pe;
}

typedef double dvec2 __attribute__((ext_vector_type(2)));

struct Tensor {
  double a00, a01, a11;
};
__device__ __forceinline__ Tensor tensor_of(const AssembleArgs& a, int64_t e)
{
  Tensor t;
  if (a.tkind == HDD_TENSOR_ISO_PER_ELEM) {
    const double v = a.tper[e];
    t.a00 = v; t.a01 = 0.0; t.a11 = v;
  } else if (a.tkind == HDD_TENSOR_SYM_PER_ELEM) {
    t.a00 = a.tper[e]; t.a01 = a.tper[a.n_local + e]; t.a11 = a.tper[2 * a.n_local + e];
  } else {
    t.a00 = a.tc0; t.a01 = a.tc1; t.a11 = a.tc2;
  }
  return t;
}
// (A g) . n
__device__ __forceinline__ double agn(const Tensor& A, double gx, double gy, double nx, double ny)
{
  return (A.a00 * gx + A.a01 * gy) * nx + (A.a01 * gx + A.a11 * gy) * ny;
}

// affine geometry x = v0 + J xh;  J^{-T} for the gradients
struct Geom {
  double x0, y0, j00, j01, j10, j11, det, i00, i01, i10, i11;   // i = J^{-1}
  __device__ __forceinline__ void init(double ax, double ay, double bx, double by, double cx, double cy)
  {
    x0 = ax; y0 = ay;
    j00 = bx - ax; j01 = cx - ax; j10 = by - ay; j11 = cy - ay;
    det = j00 * j11 - j01 * j10;
    const double id = 1.0 / det;
    i00 = j11 * id; i01 = -j01 * id; i10 = -j10 * id; i11 = j00 * id;
  }
  __device__ __forceinline__ void grad(double ghx, double ghy, double& gx, double& gy) const
  {
    gx = i00 * ghx + i10 * ghy;
    gy = i01 * ghx + i11 * ghy;
  }
  __device__ __forceinline__ void global(double xh, double yh, double& x, double& y) const
  {
    x = x0 + j00 * xh + j01 * yh;
    y = y0 + j10 * xh + j11 * yh;
  }
};

// ------------------------------------------------------------------------------------------------
// per-thread element context (loaded once, shared by all components)
// ------------------------------------------------------------------------------------------------
template <class E>
struct ElemCtx {
  double X[E::NV], Y[E::NV];
  int32_t nbr[E::NF];
  uint32_t finfo;
  Tensor A;
  Geom G;
  double adet, osgn;
  int64_t e;
  int pos_self, pos[E::NF], rowlen;
  double* img;   // LDS image of this element's row block
};

// geometry of the neighbour across face f: shared face vertices + the neighbour's non-face vertices
template <class E>
struct NbrFace {
  Geom H;
  Tensor A;
  int ta, tb, to;   // neighbour local vertices on the face (matching my fv(f,0) / fv(f,1) unless rev)
  bool rev;
};

template <class E, int F>
__device__ __forceinline__ void load_neighbor(const AssembleArgs& a, const ElemCtx<E>& c, int32_t n, NbrFace<E>& nf)
{
  const int64_t ne = a.n_local;
  constexpr int fa = E::fv(F, 0), fb = E::fv(F, 1);
  const uint32_t inf = (c.finfo >> (4 * F)) & 15u;
  const int tw = int(inf & 7u);
  nf.rev = (inf & 8u) != 0u;
  nf.ta = E::fv(tw, 0);
  nf.tb = E::fv(tw, 1);
  const double PAx = nf.rev ? c.X[fb] : c.X[fa], PAy = nf.rev ? c.Y[fb] : c.Y[fa];
  const double PBx = nf.rev ? c.X[fa] : c.X[fb], PBy = nf.rev ? c.Y[fa] : c.Y[fb];
  double NX[E::NV], NY[E::NV];
  if constexpr (E::NV == 3) {
    nf.to = 3 - nf.ta - nf.tb;
    const double Ox = a.coords[(2 * nf.to) * ne + n], Oy = a.coords[(2 * nf.to + 1) * ne + n];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      NX[k] = k == nf.ta ? PAx : (k == nf.tb ? PBx : Ox);
      NY[k] = k == nf.ta ? PAy : (k == nf.tb ? PBy : Oy);
    }
  } else {
    nf.to = -1;
    const int tc = E::fv(tw ^ 1, 0), td = E::fv(tw ^ 1, 1);
    const double Cx = a.coords[(2 * tc) * ne + n], Cy = a.coords[(2 * tc + 1) * ne + n];
    const double Dx = a.coords[(2 * td) * ne + n], Dy = a.coords[(2 * td + 1) * ne + n];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      NX[k] = k == nf.ta ? PAx : (k == nf.tb ? PBx : (k == tc ? Cx : Dx));
      NY[k] = k == nf.ta ? PAy : (k == nf.tb ? PBy : (k == tc ? Cy : Dy));
    }
  }
  nf.H.init(NX[0], NY[0], NX[1], NY[1], NX[2], NY[2]);
  nf.A = tensor_of(a, n);
}

struct FaceGeo {
  double len, nx, ny, hpow, tx, ty, xa, ya;
};

template <class E, int F>
__device__ __forceinline__ FaceGeo face_geo(const AssembleArgs& a, const ElemCtx<E>& c)
{
  constexpr int fa = E::fv(F, 0), fb = E::fv(F, 1);
  FaceGeo g;
  g.xa = c.X[fa];
  g.ya = c.Y[fa];
  g.tx = c.X[fb] - c.X[fa];
  g.ty = c.Y[fb] - c.Y[fa];
  g.len = sqrt(g.tx * g.tx + g.ty * g.ty);
  const double nsc = E::face_sign(F) * c.osgn / g.len;
  g.nx = g.ty * nsc;
  g.ny = -g.tx * nsc;
  g.hpow = a.beta == 1.0 ? g.len : pow(g.len, a.beta);
  return g;
}

// ------------------------------------------------------------------------------------------------
// row I of one component, P1 simplex with piecewise-constant coefficients: closed-form face integrals
// (exactly what the reference's order-2 Gauss rule integrates: int phi = |F|/2, int phi phi = |F|/6 (1+d_ij))
// ------------------------------------------------------------------------------------------------
template <int I>
__device__ __forceinline__ void row_simplex_pwc(const AssembleArgs& a, const ElemCtx<Simplex>& c, const KappaArg& K)
{
  using E = Simplex;
  const double ke = kappa_elem(K, c.e);
  double g[3][2];
  {
    double phi[3], ghx[3], ghy[3];
    E::shape(1.0 / 3.0, 1.0 / 3.0, phi, ghx, ghy);
#pragma unroll
    for (int k = 0; k < 3; ++k) c.G.grad(ghx[k], ghy[k], g[k][0], g[k][1]);
  }
  double self[3];
  {
    const double fac = 0.5 * c.adet;   // 1-point rule: weight 1/2 * |det J|
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double Agx = c.A.a00 * g[j][0] + c.A.a01 * g[j][1];
      const double Agy = c.A.a01 * g[j][0] + c.A.a11 * g[j][1];
      self[j] = fac * ke * (Agx * g[I][0] + Agy * g[I][1]);
    }
  }
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const int32_t n = c.nbr[f];
    if (n <= HDD_NBR_NEUMANN) continue;
    FaceGeo fg;
    double Ae[3];
    // face f as a compile-time constant for the helpers
    if (f == 0) fg = face_geo<E, 0>(a, c);
    else if (f == 1) fg = face_geo<E, 1>(a, c);
    else fg = face_geo<E, 2>(a, c);
#pragma unroll
    for (int k = 0; k < 3; ++k) Ae[k] = agn(c.A, g[k][0], g[k][1], fg.nx, fg.ny);
    const int fa = E::fv(f, 0), fb = E::fv(f, 1), fc = 3 - fa - fb;
    const double half = 0.5 * fg.len, third = fg.len / 3.0, sixth = fg.len / 6.0;
    const double M1I = I == fc ? 0.0 : half;
    const double dm = agn(c.A, fg.nx, fg.ny, fg.nx, fg.ny);
    if (n >= 0) {
      NbrFace<E> nf;
      if (f == 0) load_neighbor<E, 0>(a, c, n, nf);
      else if (f == 1) load_neighbor<E, 1>(a, c, n, nf);
      else load_neighbor<E, 2>(a, c, n, nf);
      const double kn = kappa_elem(K, n);
      const double dp = agn(nf.A, fg.nx, fg.ny, fg.nx, fg.ny);
      const double gamma = (dp * dm) / (dp + dm);
      const double w_plus = dm / (dp + dm);
      const double w_minus = dp / (dp + dm);
      const double pen = (ke * kn * a.sigma_inner * gamma) / fg.hpow;
      double An[3];
      {
        double phi[3], ghx[3], ghy[3];
        E::shape(1.0 / 3.0, 1.0 / 3.0, phi, ghx, ghy);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          double hx, hy;
          nf.H.grad(ghx[k], ghy[k], hx, hy);
          An[k] = agn(nf.A, hx, hy, fg.nx, fg.ny);
        }
      }
      // neighbour vertex matching my vertex I (only meaningful if I is on the face)
      const int mI = (I == fa) ? (nf.rev ? nf.tb : nf.ta) : (nf.rev ? nf.ta : nf.tb);
      double* out = c.img + c.pos[f] * 3;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double M1j = j == nf.to ? 0.0 : half;
        const double Mx = I == fc ? 0.0 : (j == mI ? third : (j == nf.to ? 0.0 : sixth));
        out[j] = -w_plus * kn * An[j] * M1I + w_minus * ke * Ae[I] * M1j - pen * Mx;
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double M1j = j == fc ? 0.0 : half;
        const double Mm = (I == fc || j == fc) ? 0.0 : (I == j ? third : sixth);
        self[j] += -w_minus * ke * (Ae[j] * M1I + Ae[I] * M1j) + pen * Mm;
      }
    } else {   // Dirichlet: SWIPDG::BoundaryLHS
      const double pen = (a.sigma_boundary * ke * dm) / fg.hpow;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double M1j = j == fc ? 0.0 : half;
        const double Mm = (I == fc || j == fc) ? 0.0 : (I == j ? third : sixth);
        self[j] += -ke * (Ae[j] * M1I + Ae[I] * M1j) + pen * Mm;
      }
    }
  }
  double* out = c.img + c.pos_self * 3;
#pragma unroll
  for (int j = 0; j < 3; ++j) out[j] = self[j];
}

// ------------------------------------------------------------------------------------------------
// row I of one component, generic quadrature (Q1 quads; smooth coefficients on either element)
// ------------------------------------------------------------------------------------------------
template <class E, int NQV, int NQF, int I>
__device__ __forceinline__ void row_quadrature(const AssembleArgs& a, const ElemCtx<E>& c, const KappaArg& K)
{
  constexpr int NB = E::NB, NF = E::NF;
  const double ke = kappa_elem(K, c.e);
  double self[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) self[j] = 0.0;
  // ---- LocalEvaluation::Elliptic ----
#pragma unroll
  for (int q = 0; q < NQV; ++q) {
    double phi[NB], ghx[NB], ghy[NB], gx[NB], gy[NB];
    E::shape(VolRule<E, NQV>::x(q), VolRule<E, NQV>::y(q), phi, ghx, ghy);
#pragma unroll
    for (int k = 0; k < NB; ++k) c.G.grad(ghx[k], ghy[k], gx[k], gy[k]);
    double px = 0.0, py = 0.0;
    if (smooth_kind(K.kind)) c.G.global(VolRule<E, NQV>::x(q), VolRule<E, NQV>::y(q), px, py);
    const double kap = kappa_at(K, ke, px, py);
    const double fac = VolRule<E, NQV>::w(q) * c.adet;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const double Agx = c.A.a00 * gx[j] + c.A.a01 * gy[j];
      const double Agy = c.A.a01 * gx[j] + c.A.a11 * gy[j];
      self[j] += fac * kap * (Agx * gx[I] + Agy * gy[I]);
    }
  }
  // ---- faces ----
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int32_t n = c.nbr[f];
    if (n <= HDD_NBR_NEUMANN) continue;
    FaceGeo fg;
    if (f == 0) fg = face_geo<E, 0>(a, c);
    else if (f == 1) fg = face_geo<E, 1>(a, c);
    else if (f == 2) fg = face_geo<E, 2 % NF>(a, c);
    else fg = face_geo<E, 3 % NF>(a, c);
    const int fa = E::fv(f, 0), fb = E::fv(f, 1);
    const double rax = E::rv(fa, 0), ray = E::rv(fa, 1), rbx = E::rv(fb, 0), rby = E::rv(fb, 1);
    const double dm = agn(c.A, fg.nx, fg.ny, fg.nx, fg.ny);
    if (n >= 0) {
      NbrFace<E> nf;
      if (f == 0) load_neighbor<E, 0>(a, c, n, nf);
      else if (f == 1) load_neighbor<E, 1>(a, c, n, nf);
      else if (f == 2) load_neighbor<E, 2 % NF>(a, c, n, nf);
      else load_neighbor<E, 3 % NF>(a, c, n, nf);
      const double kn = kappa_elem(K, n);
      const double dp = agn(nf.A, fg.nx, fg.ny, fg.nx, fg.ny);
      const double gamma = (dp * dm) / (dp + dm);
      const double w_plus = dm / (dp + dm);
      const double w_minus = dp / (dp + dm);
      const double sax = E::rv(nf.ta, 0), say = E::rv(nf.ta, 1), sbx = E::rv(nf.tb, 0), sby = E::rv(nf.tb, 1);
      double nbv[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) nbv[j] = 0.0;
#pragma unroll
      for (int q = 0; q < NQF; ++q) {
        const double s = Gauss01<NQF>::s(q);
        double pe[NB], ghx[NB], ghy[NB], gex[NB], gey[NB];
        E::shape(rax + s * (rbx - rax), ray + s * (rby - ray), pe, ghx, ghy);
#pragma unroll
        for (int k = 0; k < NB; ++k) c.G.grad(ghx[k], ghy[k], gex[k], gey[k]);
        const double sn = nf.rev ? 1.0 - s : s;
        double pn[NB], hhx[NB], hhy[NB], gnx[NB], gny[NB];
        E::shape(sax + sn * (sbx - sax), say + sn * (sby - say), pn, hhx, hhy);
#pragma unroll
        for (int k = 0; k < NB; ++k) nf.H.grad(hhx[k], hhy[k], gnx[k], gny[k]);
        double kme = ke, knb = kn;
        if (smooth_kind(K.kind)) {
          kme = kappa_at(K, ke, fg.xa + s * fg.tx, fg.ya + s * fg.ty);
          knb = kme;
        }
        const double pen = (kme * knb * a.sigma_inner * gamma) / fg.hpow;
        const double fac = Gauss01<NQF>::w(q) * fg.len;
        double Ae[NB], An[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          Ae[k] = agn(c.A, gex[k], gey[k], fg.nx, fg.ny);
          An[k] = agn(nf.A, gnx[k], gny[k], fg.nx, fg.ny);
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          self[j] += fac * (-w_minus * kme * Ae[j] * pe[I] - w_minus * kme * pe[j] * Ae[I] + pen * pe[j] * pe[I]);
          nbv[j] += fac * (-w_plus * knb * An[j] * pe[I] + w_minus * kme * pn[j] * Ae[I] - pen * pn[j] * pe[I]);
        }
      }
      double* out = c.img + c.pos[f] * NB;
#pragma unroll
      for (int j = 0; j < NB; ++j) out[j] = nbv[j];
    } else {   // Dirichlet
#pragma unroll
      for (int q = 0; q < NQF; ++q) {
        const double s = Gauss01<NQF>::s(q);
        double pe[NB], ghx[NB], ghy[NB], gex[NB], gey[NB];
        E::shape(rax + s * (rbx - rax), ray + s * (rby - ray), pe, ghx, ghy);
#pragma unroll
        for (int k = 0; k < NB; ++k) c.G.grad(ghx[k], ghy[k], gex[k], gey[k]);
        double kme = ke;
        if (smooth_kind(K.kind)) kme = kappa_at(K, ke, fg.xa + s * fg.tx, fg.ya + s * fg.ty);
        const double pen = (a.sigma_boundary * kme * dm) / fg.hpow;
        const double fac = Gauss01<NQF>::w(q) * fg.len;
        double Ae[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) Ae[k] = agn(c.A, gex[k], gey[k], fg.nx, fg.ny);
#pragma unroll
        for (int j = 0; j < NB; ++j) self[j] += fac * (-kme * Ae[j] * pe[I] - kme * pe[j] * Ae[I] + pen * pe[j] * pe[I]);
      }
    }
  }
  double* out = c.img + c.pos_self * NB;
#pragma unroll
  for (int j = 0; j < NB; ++j) out[j] = self[j];
}

template <class E, int NQV, int NQF, bool PWC, int I>
__device__ __forceinline__ void row(const AssembleArgs& a, const ElemCtx<E>& c, const KappaArg& K)
{
  if constexpr (PWC && std::is_same<E, Simplex>::value && NQV == 1 && NQF == 2)
    row_simplex_pwc<I>(a, c, K);
  else
    row_quadrature<E, NQV, NQF, I>(a, c, K);
}

// ------------------------------------------------------------------------------------------------
// the kernel: one workgroup = 64 consecutive owned elements x NB waves (wave w = local row w)
// ------------------------------------------------------------------------------------------------
template <class E, int NQV, int NQF, bool PWC>
__global__ void __launch_bounds__(64 * E::NB, HDD_MIN_WAVES_PER_EU)
swipdg_assemble_kernel(const AssembleArgs a)
{
  constexpr int NB = E::NB, NF = E::NF, NV = E::NV;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // XCD-aware tile order (bijective): hardware block b runs on XCD b % 8; each XCD gets a contiguous
  // range of tiles so the element rows above / below a tile sit in the same L2.
  const int64_t nwg = gridDim.x;
  const int64_t b = blockIdx.x;
  const int64_t q8 = nwg >> 3, r8 = nwg & 7, xcd = b & 7;
  const int64_t tile = xcd * q8 + (xcd < r8 ? xcd : r8) + (b >> 3);

  const int64_t t0 = a.own_begin + tile * 64;
  const int64_t tend = t0 + 64 < a.own_end ? t0 + 64 : a.own_end;
  const int64_t e = t0 + lane;
  const bool active = e < tend;
  const int64_t ne = a.n_local;
  const int64_t* eptr = a.elem_ptr - a.own_begin;
  const int64_t base = eptr[t0];
  const int64_t base_al = base & ~int64_t(1);          // 16-byte aligned image origin
  const int64_t tile_end = eptr[tend];

  ElemCtx<E> c;
  c.e = active ? e : t0;   // inactive tail lanes shadow a valid element; their LDS writes are skipped
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    c.X[k] = a.coords[(2 * k) * ne + c.e];
    c.Y[k] = a.coords[(2 * k + 1) * ne + c.e];
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) c.nbr[f] = a.nbrs[f * ne + c.e];
  c.finfo = a.finfo[c.e];
  c.A = tensor_of(a, c.e);
  const int64_t my_off = eptr[c.e];
  c.G.init(c.X[0], c.Y[0], c.X[1], c.Y[1], c.X[2], c.Y[2]);
  c.adet = fabs(c.G.det);
  c.osgn = c.G.det > 0.0 ? 1.0 : -1.0;
  int nblk = 1;
  c.pos_self = 0;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    nblk += c.nbr[f] >= 0;
    c.pos_self += (c.nbr[f] >= 0 && c.nbr[f] < c.e);
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    int p = (c.e < c.nbr[f]) ? 1 : 0;
#pragma unroll
    for (int g = 0; g < NF; ++g) p += (c.nbr[g] >= 0 && c.nbr[g] < c.nbr[f]);
    c.pos[f] = p;
  }
  c.rowlen = nblk * NB;
  // lanes past the tile end write to a scratch row after the image
  c.img = active ? lds + (my_off - base_al) + int64_t(wave) * c.rowlen
                 : lds + 64 * NB * (NF + 1) * NB + 2;

  // one component per launch (the host loops over the affine components): a component loop in here
  // would let the compiler hoist every component-invariant face quantity of all faces above the loop
  {
    const KappaArg K = a.kappa[0];
    double* out = a.vals[0];
    switch (wave) {
      case 0: row<E, NQV, NQF, PWC, 0>(a, c, K); break;
      case 1: row<E, NQV, NQF, PWC, 1>(a, c, K); break;
      case 2: row<E, NQV, NQF, PWC, 2>(a, c, K); break;
      default: if constexpr (NB > 3) row<E, NQV, NQF, PWC, NB - 1>(a, c, K); break;
    }
    __syncthreads();
    // stream the tile's contiguous row blocks [base, tile_end) out of LDS, 16 bytes per lane
    const int64_t lo = base_al, hi = tile_end;
    const int64_t n2 = (hi - lo) >> 1;
    for (int64_t k = threadIdx.x; k < n2; k += blockDim.x) {
      const int64_t gi = lo + 2 * k;
      const dvec2 v = *reinterpret_cast<const dvec2*>(lds + 2 * k);
      if (gi >= base) {
        __builtin_nontemporal_store(v, reinterpret_cast<dvec2*>(out + gi));
      } else {   // first pair straddles the tile start: only the upper value is ours
        out[gi + 1] = v.y;
      }
    }
    if (((hi - lo) & 1) && threadIdx.x == 0) out[hi - 1] = lds[hi - 1 - lo];
  }
}

// ------------------------------------------------------------------------------------------------
// P1 simplex, piecewise-constant coefficients: one thread per element computes all 3 rows.
//
// Face terms in "role" form: for face f with my vertices a = fv(f,0), b = fv(f,1), the neighbour's
// vertices are named by their physical position (role A = position of my a, B = position of my b,
// O = the neighbour's opposite vertex).  Then every coefficient of the entity/entity and
// entity/neighbour blocks is orientation-free, and the twin face / reversal only decides the three LDS
// column slots j(A), j(B), j(O) the entity/neighbour values are stored to.  The neighbour gradients come
// from the triangle (A, B, O) (barycentric gradients), so a face gathers only O (2 doubles), the
// neighbour tensor and, if per element, its diffusion factor.
//
// fp64 reciprocals / rsqrt use the hardware estimate + two Newton steps (< 1 ulp off the IEEE result);
// the oracle comparison tolerance is 1e-12 of the row maximum.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double rcp_nr(double x)
{
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}
__device__ __forceinline__ double rsq_nr(double x)
{
  double y = __builtin_amdgcn_rsq(x);
  double h = 0.5 * x;
  y = y * fma(-h * y, y, 1.5);
  y = y * fma(-h * y, y, 1.5);
  return y;
}

// ------------------------------------------------------------------------------------------------
// Persistent, software-pipelined variant of the P1 kernel.
//
// gfx950's vmcnt is in order and counts stores: a wave that waits for a load issued after its stores
// also waits for those stores.  So each wave walks a sequence of tiles and orders its memory operations
//   [prefetch own data of tile t+1] [compute tile t -> LDS] [gathers of tile t+1] [stores of tile t]
// The loads of tile t+1 are in flight while tile t computes, the neighbour gathers are issued before the
// store burst, and the stores are branch-free buffer stores (fixed count, out-of-range ones dropped by
// the descriptor's range check), so the next wait can stay counted instead of draining the stores.
// ------------------------------------------------------------------------------------------------
struct P1Own {
  double X[3], Y[3];
  int32_t nbr[3];
  uint32_t finfo;
  Tensor A;
  double ke;
  int32_t vid[3];   // vertex-indexed geometry (VX): local vertex ids; X / Y then arrive with the gathers
};
struct P1Gat {
  double Ox[3], Oy[3];
  Tensor Ap[3];
  double kn[3];
  int32_t ov[3];    // VX: the neighbour's off-face vertex id; Ox / Oy arrive in the second gather stage
};

// vertex (x, y) of the vertex-indexed geometry: one 16-byte load
__device__ __forceinline__ void vertex_xy(const AssembleArgs& a, int32_t v, double& x, double& y)
{
  const dvec2 p = *reinterpret_cast<const dvec2*>(a.vxy + 2 * int64_t(v));
  x = p.x;
  y = p.y;
}

template <int TK>
__device__ __forceinline__ Tensor tensor_k(const AssembleArgs& a, int64_t e)
{
  Tensor t;
  if constexpr (TK == HDD_TENSOR_ISO_PER_ELEM) {
    const double v = a.tper[e];
    t.a00 = v; t.a01 = 0.0; t.a11 = v;
  } else if constexpr (TK == HDD_TENSOR_SYM_PER_ELEM) {
    t.a00 = a.tper[e]; t.a01 = a.tper[a.n_local + e]; t.a11 = a.tper[2 * a.n_local + e];
  } else {
    t.a00 = a.tc0; t.a01 = a.tc1; t.a11 = a.tc2;
  }
  return t;
}
template <int KK>
__device__ __forceinline__ double kappa_k(const AssembleArgs& a, int64_t e)
{
  if constexpr (KK == HDD_FN_PER_ELEM) return a.kappa[0].per_elem[e];
  else return a.kappa[0].c;
}

// ------------------------------------------------------------------------------------------------
// 32-bit offset loads (vertex-indexed P1 meshes).  Each SoA array is read through a buffer resource made from its
// base pointer (wave-uniform SGPRs, hoisted out of the tile loop), the row of a [rows][n_local] array in the
// instruction's SGPR soffset and the element part in a 32-bit VGPR offset: no 64-bit VALU address arithmetic (the
// global loads cost a v_lshl_add_u64 each, the neighbours' vertex-id gathers a 64-bit multiply-add; round 5 counted
// 461 integer / select instructions beside 359 f64 ones in the C2 kernel).  The host enables vertex-indexed
// geometry only while every byte offset fits in 32 bits (n_local * 48 < 2^32, hdd_swipdg_assemble); the resources
// carry no range (num_records = 2^32 - 1).
// ------------------------------------------------------------------------------------------------
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc32(const void* p)
{
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, -1, 0x00020000);
}
__device__ __forceinline__ uint32_t ld32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff = 0)
{
  return __builtin_amdgcn_raw_buffer_load_b32(r, int(voff), int(soff), 0);
}
__device__ __forceinline__ double ld64f(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff = 0)
{
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, int(voff), int(soff), 0));
}
__device__ __forceinline__ dvec2 ld128f(__amdgpu_buffer_rsrc_t r, uint32_t voff)
{
  return __builtin_bit_cast(dvec2, __builtin_amdgcn_raw_buffer_load_b128(r, int(voff), 0, 0));
}
// the tensor / kappa of local element e (byte offset e8 = 8 e)
template <int TK>
__device__ __forceinline__ Tensor tensor_o32(const AssembleArgs& a, uint32_t e8)
{
  Tensor t;
  if constexpr (TK == HDD_TENSOR_ISO_PER_ELEM) {
    const double v = ld64f(rsrc32(a.tper), e8);
    t.a00 = v; t.a01 = 0.0; t.a11 = v;
  } else if constexpr (TK == HDD_TENSOR_SYM_PER_ELEM) {
    const __amdgpu_buffer_rsrc_t r = rsrc32(a.tper);
    const uint32_t row = uint32_t(a.n_local) * 8u;
    t.a00 = ld64f(r, e8); t.a01 = ld64f(r, e8, row); t.a11 = ld64f(r, e8, 2u * row);
  } else {
    t.a00 = a.tc0; t.a01 = a.tc1; t.a11 = a.tc2;
  }
  return t;
}
template <int KK>
__device__ __forceinline__ double kappa_o32(const AssembleArgs& a, uint32_t e8)
{
  if constexpr (KK == HDD_FN_PER_ELEM) return ld64f(rsrc32(a.kappa[0].per_elem), e8);
  else return a.kappa[0].c;
}
__device__ __forceinline__ void vertex_xy_o32(const AssembleArgs& a, int32_t v, double& x, double& y)
{
  const dvec2 p = ld128f(rsrc32(a.vxy), uint32_t(v) * 16u);
  x = p.x;
  y = p.y;
}

// Own-data loads of a tile (coalesced SoA).  VX: vertex ids instead of coordinates -- the vertex
// coordinates are then gathered with the neighbour data (p1_load_gat), the neighbour's off-face vertex in a
// second stage (p1_load_gat2) that the persistent driver issues after the tile's stores.  VX reads go through the
// 32-bit offset loads above.
template <int TK, int KK, bool VX = false>
__device__ __forceinline__ void p1_load_own(const AssembleArgs& a, int64_t e, P1Own& o)
{
  const int64_t ne = a.n_local;
  if constexpr (VX) {
    const uint32_t e4 = uint32_t(e) * 4u, row = uint32_t(ne) * 4u;
    const __amdgpu_buffer_rsrc_t rv = rsrc32(a.ev), rn = rsrc32(a.nbrs);
#pragma unroll
    for (int k = 0; k < 3; ++k) o.vid[k] = int32_t(ld32(rv, e4, uint32_t(k) * row));
#pragma unroll
    for (int f = 0; f < 3; ++f) o.nbr[f] = int32_t(ld32(rn, e4, uint32_t(f) * row));
    o.finfo = ld32(rsrc32(a.finfo), e4);
    o.A = tensor_o32<TK>(a, 2u * e4);
    o.ke = kappa_o32<KK>(a, 2u * e4);
    return;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    o.X[k] = a.coords[(2 * k) * ne + e];
    o.Y[k] = a.coords[(2 * k + 1) * ne + e];
  }
#pragma unroll
  for (int f = 0; f < 3; ++f) o.nbr[f] = a.nbrs[f * ne + e];
  o.finfo = a.finfo[e];
  o.A = tensor_k<TK>(a, e);
  o.ke = kappa_k<KK>(a, e);
}

template <int TK, int KK, bool VX = false>
__device__ __forceinline__ void p1_load_gat(const AssembleArgs& a, int64_t e, P1Own& o, P1Gat& g)
{
  const int64_t ne = a.n_local;
  if constexpr (VX) {
#pragma unroll
    for (int k = 0; k < 3; ++k) vertex_xy_o32(a, o.vid[k], o.X[k], o.Y[k]);
    const uint32_t row = uint32_t(ne) * 4u;
    const __amdgpu_buffer_rsrc_t rv = rsrc32(a.ev);
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const uint32_t n = o.nbr[f] >= 0 ? uint32_t(o.nbr[f]) : uint32_t(e);   // boundary faces: harmless own reload
      // the neighbour's vertex opposite its twin face tw (Simplex faces (0,1), (0,2), (1,2)): 2 - tw (clamped, so
      // whatever a boundary face's info bits hold the offset stays inside the array)
      const uint32_t to = min(2u - ((o.finfo >> (4 * f)) & 7u), 2u);
      g.ov[f] = int32_t(ld32(rv, to * row + 4u * n));
      g.Ap[f] = tensor_o32<TK>(a, 8u * n);
      g.kn[f] = kappa_o32<KK>(a, 8u * n);
    }
    return;
  }
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const int64_t n = o.nbr[f] >= 0 ? int64_t(o.nbr[f]) : e;   // boundary faces: harmless own reload
    const uint32_t inf = (o.finfo >> (4 * f)) & 15u;
    const int tw = int(inf & 7u);
    const int to = 3 - Simplex::fv(tw, 0) - Simplex::fv(tw, 1);
    g.Ox[f] = a.coords[(2 * to) * ne + n];
    g.Oy[f] = a.coords[(2 * to + 1) * ne + n];
    g.Ap[f] = tensor_k<TK>(a, n);
    g.kn[f] = kappa_k<KK>(a, n);
  }
}
template <bool VX>
__device__ __forceinline__ void p1_load_gat2(const AssembleArgs& a, P1Gat& g)
{
  if constexpr (VX) {
#pragma unroll
    for (int f = 0; f < 3; ++f) vertex_xy_o32(a, g.ov[f], g.Ox[f], g.Oy[f]);
  }
}

// P1 closed-form per-element math on preloaded data (role form, see above); writes the row block into `img`.
// PEN: only the interior-penalty terms (the SWIPDG penalty product, swipdg.hh:462-508), no volume and no
// consistency / symmetry terms.
// the element's own block from one face: S_ij += -c (Ae_j [i != fc] + Ae_i [j != fc]) + (pen / 3 or pen / 6 on the
// face's vertex pairs), c = |F| / 2 times the consistency weight (fc: the vertex opposite the face)
__device__ __forceinline__ void p1_face_self(double (&S)[3][3], const double (&Ae)[3], int fc, double c, double penT,
                                             double penS)
{
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = i; j < 3; ++j) {   // the block is symmetric: the upper triangle (p1_compute mirrors it)
      if (i == fc && j == fc) continue;
      const double v = i == fc ? Ae[i] : (j == fc ? Ae[j] : Ae[i] + Ae[j]);
      S[i][j] = fma(-c, v, S[i][j] + (i == fc || j == fc ? 0.0 : (i == j ? penT : penS)));
    }
}

// ALLIN: the caller guarantees three interior faces (every element of a full interior tile, see the persistent
// driver): no per-face branches, the row length and block count compile-time constants
template <bool PEN = false, bool ALLIN = false>
__device__ __forceinline__ void p1_compute(const AssembleArgs& a, int64_t e, const P1Own& o, const P1Gat& gt,
                                           double* img)
{
  using E = Simplex;
  const double j00 = o.X[1] - o.X[0], j01 = o.X[2] - o.X[0], j10 = o.Y[1] - o.Y[0], j11 = o.Y[2] - o.Y[0];
  const double det = j00 * j11 - j01 * j10;
  const double id = rcp_nr(det);
  const double i00 = j11 * id, i01 = -j01 * id, i10 = -j10 * id, i11 = j00 * id;
  double g[3][2];
  g[1][0] = i00; g[1][1] = i01;
  g[2][0] = i10; g[2][1] = i11;
  g[0][0] = -i00 - i10; g[0][1] = -i01 - i11;
  double Ag[3][2];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    Ag[k][0] = o.A.a00 * g[k][0] + o.A.a01 * g[k][1];
    Ag[k][1] = o.A.a01 * g[k][0] + o.A.a11 * g[k][1];
  }
  const double adet = fabs(det);
  const double osgn = det > 0.0 ? 1.0 : -1.0;
  const int32_t ei = int32_t(e);   // local ids are int32 (hdd_mesh neighbors): 32-bit compares
  int nblk = 1, pos_self = 0, pos[3];
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    nblk += ALLIN || o.nbr[f] >= 0;
    pos_self += ((ALLIN || o.nbr[f] >= 0) && o.nbr[f] < ei);
  }
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    int p = (ei < o.nbr[f]) ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) p += ((ALLIN || o.nbr[q] >= 0) && o.nbr[q] < o.nbr[f]);
    pos[f] = p;
  }
  const int rowlen = ALLIN ? 12 : nblk * 3;
  const double ke = o.ke;
  double S[3][3];
  {
    const double fac = PEN ? 0.0 : 0.5 * adet * ke;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = i; j < 3; ++j) S[i][j] = fac * (Ag[j][0] * g[i][0] + Ag[j][1] * g[i][1]);   // symmetric A
  }
  constexpr double CS = PEN ? 0.0 : 1.0;   // consistency / symmetry terms on (stiffness) or off (penalty)
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const int32_t n = o.nbr[f];
    if (!ALLIN && n <= HDD_NBR_NEUMANN) continue;
    const int fa = E::fv(f, 0), fb = E::fv(f, 1), fc = 3 - fa - fb;
    const double tx = o.X[fb] - o.X[fa], ty = o.Y[fb] - o.Y[fa];
    const double il = rsq_nr(tx * tx + ty * ty);
    const double len = (tx * tx + ty * ty) * il;
    const double nsc = E::face_sign(f) * osgn * il;
    const double nx = ty * nsc, ny = -tx * nsc;
    double Ae[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) Ae[k] = Ag[k][0] * nx + Ag[k][1] * ny;
    const double dm = agn(o.A, nx, ny, nx, ny);
    const double ihp = a.beta == 1.0 ? il : inv_pow(len, a.beta);
    const double half = 0.5 * len, third = len * (1.0 / 3.0), sixth = len * (1.0 / 6.0);
    if (ALLIN || n >= 0) {
      const uint32_t inf = (o.finfo >> (4 * f)) & 15u;
      const int tw = int(inf & 7u);
      const bool rev = (inf & 8u) != 0u;
      const int ta = E::fv(tw, 0), tb = E::fv(tw, 1), to = 3 - ta - tb;
      const double Ox = gt.Ox[f], Oy = gt.Oy[f];
      const Tensor Ap = gt.Ap[f];
      const double kn = gt.kn[f];
      const double dp = agn(Ap, nx, ny, nx, ny);
      const double rs = rcp_nr(dp + dm);
      const double gamma = (dp * dm) * rs;
      const double w_plus = dm * rs, w_minus = dp * rs;
      const double pen = (ke * kn * a.sigma_inner * gamma) * ihp;
      const double Ax = o.X[fa], Ay = o.Y[fa], Bx = o.X[fb], By = o.Y[fb];
      const double iD = rcp_nr((Bx - Ax) * (Oy - Ay) - (By - Ay) * (Ox - Ax));
      const double mx = Ap.a00 * nx + Ap.a01 * ny, my = Ap.a01 * nx + Ap.a11 * ny;
      const double AnA = ((By - Oy) * mx + (Ox - Bx) * my) * iD;
      const double AnB = ((Oy - Ay) * mx + (Ax - Ox) * my) * iD;
      const double AnO = ((Ay - By) * mx + (Bx - Ax) * my) * iD;
      const int jA = rev ? tb : ta, jB = rev ? ta : tb;
      // the face's constants folded once (half = |F| / 2, third, sixth = the P1 trace mass entries), so every entry
      // is a two-FMA chain (fc, fa, fb are compile-time per unrolled face)
      const double cplh = -w_plus * kn * CS * half;
      const double symh = w_minus * ke * CS * half;
      const double penT = pen * third, penS = pen * sixth;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        double* row = img + i * rowlen + pos[f] * 3;
        if (i == fc) {
          row[jA] = symh * Ae[i];
          row[jB] = symh * Ae[i];
          row[to] = 0.0;
        } else {
          row[jA] = fma(cplh, AnA, fma(symh, Ae[i], -(i == fa ? penT : penS)));
          row[jB] = fma(cplh, AnB, fma(symh, Ae[i], -(i == fb ? penT : penS)));
          row[to] = cplh * AnO;
        }
      }
      p1_face_self(S, Ae, fc, symh, penT, penS);
    } else {
      const double pen = (a.sigma_boundary * ke * dm) * ihp;
      p1_face_self(S, Ae, fc, ke * CS * half, pen * third, pen * sixth);
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) img[i * rowlen + pos_self * 3 + j] = j >= i ? S[i][j] : S[j][i];
}

typedef int ivec4 __attribute__((ext_vector_type(4)));
typedef int ivec2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------------------------------------
// Generic thread-per-element policy (Q1 parallelograms, smooth coefficients): quadrature at compile-time
// points on my side, "role" coordinates on the neighbour side.  Roles are named by physical position
// (A = my fv(f,0), B = my fv(f,1), third role = the neighbour vertex next to A off the face, fourth
// (cubes) = next to B) and numbered like the reference element, so the neighbour's basis in role
// coordinates is E::shape at the compile-time point (s, 0) and only the LDS column slots depend on the
// twin face / reversal.  Gathers per face: one neighbour vertex (2 doubles), its tensor, its kappa.
// ------------------------------------------------------------------------------------------------
template <class E>
struct GOwn {
  double X[E::NV], Y[E::NV];
  int32_t nbr[E::NF];
  uint32_t finfo;
  Tensor A;
  double ke;
  int32_t vid[E::NV];   // VX: local vertex ids (as P1Own)
};
template <class E>
struct GGat {
  double Cx[E::NF], Cy[E::NF];
  Tensor Ap[E::NF];
  double kn[E::NF];
  int32_t ov[E::NF];    // VX: the neighbour's third-role vertex id
};

template <class E>
__device__ __forceinline__ int role_slot(uint32_t finfo, int f, int r)
{
  const uint32_t inf = (finfo >> (4 * f)) & 15u;
  const int tw = int(inf & 7u);
  const bool rev = (inf & 8u) != 0u;
  const int ka = rev ? 1 : 0;
  if (r == 0) return E::fv(tw, ka);
  if (r == 1) return E::fv(tw, 1 - ka);
  if constexpr (E::NV == 3) return 3 - E::fv(tw, 0) - E::fv(tw, 1);
  else return r == 2 ? E::fv(tw ^ 1, ka) : E::fv(tw ^ 1, 1 - ka);
}

// One lane's row block in the LDS tile image, written at index i -> (i + rot) mod RB (rot = 0: plain).
// Uniform Q1 tiles use rot = 2 ((lane >> 1) & 15): see the persistent kernel's image comment.
template <int RB>
struct RotImg {
  double* p;
  int rot;
  __device__ __forceinline__ double& operator[](int i) const
  {
    const unsigned q = unsigned(i + rot);
    return p[q < unsigned(RB) ? q : q - unsigned(RB)];
  }
};

template <class E, int NQV, int NQF, int TK, int KK, bool VX = false>
struct GenericPolicy {
  static constexpr int NB = E::NB, NF = E::NF, NV = E::NV;
  static constexpr int RB = (NF + 1) * NB * NB;
  // workgroups (single-wave tiles) per CU and the register cap: simplices (18 KB tiles) run 8 per CU at
  // <= 256 registers (2 waves / SIMD hide the sinusoid's VALU latency: C3 0.278 -> 0.241 ms per component,
  // profiles/r01/s2/ab1.log); quads are LDS-bound at 4 per CU (40 KB rotated image) and keep the full
  // register file (capping them at 256 spills: 0.84 -> 1.30 ms)
  static constexpr int WGCU = NB == 4 ? 4 : 8;
  static constexpr int MINW = NB == 4 ? 1 : 2;
  static constexpr bool PAD = NB == 4;   // rotated LDS image for uniform tiles (see the persistent kernel)
  using Own = GOwn<E>;
  using Gat = GGat<E>;

  __device__ static void load_own(const AssembleArgs& a, int64_t e, Own& o)
  {
    const int64_t ne = a.n_local;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if constexpr (VX) {
        o.vid[k] = a.ev[k * ne + e];
      } else {
        o.X[k] = a.coords[(2 * k) * ne + e];
        o.Y[k] = a.coords[(2 * k + 1) * ne + e];
      }
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) o.nbr[f] = a.nbrs[f * ne + e];
    o.finfo = a.finfo[e];
    o.A = tensor_k<TK>(a, e);
    o.ke = smooth_kind(KK) ? 0.0 : kappa_k<KK == HDD_FN_PER_ELEM ? HDD_FN_PER_ELEM : HDD_FN_CONST>(a, e);
  }

  __device__ static void load_gat(const AssembleArgs& a, int64_t e, Own& o, Gat& g)
  {
    const int64_t ne = a.n_local;
    if constexpr (VX) {
#pragma unroll
      for (int k = 0; k < NV; ++k) vertex_xy(a, o.vid[k], o.X[k], o.Y[k]);
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int64_t n = o.nbr[f] >= 0 ? int64_t(o.nbr[f]) : e;
      const int c = role_slot<E>(o.finfo, f, 2);
      if constexpr (VX) {
        g.ov[f] = a.ev[c * ne + n];
      } else {
        g.Cx[f] = a.coords[(2 * c) * ne + n];
        g.Cy[f] = a.coords[(2 * c + 1) * ne + n];
      }
      g.Ap[f] = tensor_k<TK>(a, n);
      g.kn[f] = smooth_kind(KK) ? 0.0 : kappa_k<KK == HDD_FN_PER_ELEM ? HDD_FN_PER_ELEM : HDD_FN_CONST>(a, n);
    }
  }

  __device__ static void load_gat2(const AssembleArgs& a, Gat& g)
  {
    if constexpr (VX) {
#pragma unroll
      for (int f = 0; f < NF; ++f) vertex_xy(a, g.ov[f], g.Cx[f], g.Cy[f]);
    }
  }

  __device__ static double kap(const AssembleArgs& a, double x, double y)
  {
    const KappaArg& K = a.kappa[0];
    if constexpr (KK == HDD_FN_FLATTOP) return flattop_sum(K.table, K.n_table, K.c, K.b, x, y);
    return K.c + K.b * sin_phase(K.kx * x + K.ky * y);
  }

  __device__ static int n_interior(const Own& o)
  {
    int c = 0;
#pragma unroll
    for (int f = 0; f < NF; ++f) c += o.nbr[f] >= 0;
    return c;
  }

  template <class IMG>
  __device__ static void compute(const AssembleArgs& a, int64_t e, const Own& o, const Gat& gt, IMG img)
  {
    Geom G;
    G.init(o.X[0], o.Y[0], o.X[1], o.Y[1], o.X[2], o.Y[2]);
    const double adet = fabs(G.det);
    const double osgn = G.det > 0.0 ? 1.0 : -1.0;
    int pos_self = 0, pos[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) pos_self += (o.nbr[f] >= 0 && o.nbr[f] < e);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      int p = (e < o.nbr[f]) ? 1 : 0;
#pragma unroll
      for (int q = 0; q < NF; ++q) p += (o.nbr[q] >= 0 && o.nbr[q] < o.nbr[f]);
      pos[f] = p;
    }
    const int rowlen = (n_interior(o) + 1) * NB;
    double S[NB][NB];
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) S[i][j] = 0.0;
    // ---- LocalEvaluation::Elliptic ----
#pragma unroll
    for (int q = 0; q < NQV; ++q) {
      double phi[NB], ghx[NB], ghy[NB], gx[NB], gy[NB];
      E::shape(VolRule<E, NQV>::x(q), VolRule<E, NQV>::y(q), phi, ghx, ghy);
#pragma unroll
      for (int k = 0; k < NB; ++k) G.grad(ghx[k], ghy[k], gx[k], gy[k]);
      double kq = o.ke;
      if constexpr (smooth_kind(KK)) {
        double px, py;
        G.global(VolRule<E, NQV>::x(q), VolRule<E, NQV>::y(q), px, py);
        kq = kap(a, px, py);
      }
      const double fac = VolRule<E, NQV>::w(q) * adet * kq;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const double Agx = o.A.a00 * gx[j] + o.A.a01 * gy[j];
        const double Agy = o.A.a01 * gx[j] + o.A.a11 * gy[j];
#pragma unroll
        for (int i = 0; i < NB; ++i) S[i][j] += fac * (Agx * gx[i] + Agy * gy[i]);
      }
    }
    // ---- faces ----
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int32_t n = o.nbr[f];
      if (n <= HDD_NBR_NEUMANN) continue;
      const int fa = E::fv(f, 0), fb = E::fv(f, 1);
      const double Ax = o.X[fa], Ay = o.Y[fa], Bx = o.X[fb], By = o.Y[fb];
      const double tx = Bx - Ax, ty = By - Ay;
      const double il = rsq_nr(tx * tx + ty * ty);
      const double len = (tx * tx + ty * ty) * il;
      const double nsc = E::face_sign(f) * osgn * il;
      const double nx = ty * nsc, ny = -tx * nsc;
      const double dm = agn(o.A, nx, ny, nx, ny);
      const double ihp = a.beta == 1.0 ? il : inv_pow(len, a.beta);
      const double rax = E::rv(fa, 0), ray = E::rv(fa, 1), rbx = E::rv(fb, 0), rby = E::rv(fb, 1);
      if (n >= 0) {
        Geom Hn;   // neighbour in role coordinates: A = (0,0), B = (1,0), third role = (0,1)
        Hn.init(Ax, Ay, Bx, By, gt.Cx[f], gt.Cy[f]);
        const Tensor Ap = gt.Ap[f];
        const double dp = agn(Ap, nx, ny, nx, ny);
        const double rs = rcp_nr(dp + dm);
        const double gamma = (dp * dm) * rs;
        const double w_plus = dm * rs, w_minus = dp * rs;
        double EN[NB][NB];
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
          for (int j = 0; j < NB; ++j) EN[i][j] = 0.0;
#pragma unroll
        for (int q = 0; q < NQF; ++q) {
          const double s = Gauss01<NQF>::s(q);
          double pe[NB], ghx[NB], ghy[NB], gex[NB], gey[NB];
          E::shape(rax + s * (rbx - rax), ray + s * (rby - ray), pe, ghx, ghy);
#pragma unroll
          for (int k = 0; k < NB; ++k) G.grad(ghx[k], ghy[k], gex[k], gey[k]);
          double pn[NB], hhx[NB], hhy[NB];
          E::shape(s, 0.0, pn, hhx, hhy);
          double kme = o.ke, knb = gt.kn[f];
          if constexpr (smooth_kind(KK)) {
            kme = kap(a, Ax + s * tx, Ay + s * ty);
            knb = kme;
          }
          const double pen = (kme * knb * a.sigma_inner * gamma) * ihp;
          const double fac = Gauss01<NQF>::w(q) * len;
          double Ae[NB], An[NB];
#pragma unroll
          for (int k = 0; k < NB; ++k) {
            double hx, hy;
            Hn.grad(hhx[k], hhy[k], hx, hy);
            Ae[k] = agn(o.A, gex[k], gey[k], nx, ny);
            An[k] = agn(Ap, hx, hy, nx, ny);
          }
#pragma unroll
          for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) {
              S[i][j] += fac * (-w_minus * kme * Ae[j] * pe[i] - w_minus * kme * pe[j] * Ae[i] + pen * pe[j] * pe[i]);
              EN[i][j] += fac * (-w_plus * knb * An[j] * pe[i] + w_minus * kme * pn[j] * Ae[i] - pen * pn[j] * pe[i]);
            }
        }
        int slot[NB];
#pragma unroll
        for (int r = 0; r < NB; ++r) slot[r] = role_slot<E>(o.finfo, f, r);
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
          for (int r = 0; r < NB; ++r) img[i * rowlen + pos[f] * NB + slot[r]] = EN[i][r];
      } else {   // Dirichlet: SWIPDG::BoundaryLHS
#pragma unroll
        for (int q = 0; q < NQF; ++q) {
          const double s = Gauss01<NQF>::s(q);
          double pe[NB], ghx[NB], ghy[NB], gex[NB], gey[NB];
          E::shape(rax + s * (rbx - rax), ray + s * (rby - ray), pe, ghx, ghy);
#pragma unroll
          for (int k = 0; k < NB; ++k) G.grad(ghx[k], ghy[k], gex[k], gey[k]);
          double kme = o.ke;
          if constexpr (smooth_kind(KK)) kme = kap(a, Ax + s * tx, Ay + s * ty);
          const double pen = (a.sigma_boundary * kme * dm) * ihp;
          const double fac = Gauss01<NQF>::w(q) * len;
          double Ae[NB];
#pragma unroll
          for (int k = 0; k < NB; ++k) Ae[k] = agn(o.A, gex[k], gey[k], nx, ny);
#pragma unroll
          for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j)
              S[i][j] += fac * (-kme * Ae[j] * pe[i] - kme * pe[j] * Ae[i] + pen * pe[j] * pe[i]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) img[i * rowlen + pos_self * NB + j] = S[i][j];
  }
};

// ------------------------------------------------------------------------------------------------
// Q1 on parallelograms, piecewise-constant coefficients: closed-form face integrals.
//
// On an affine quadrilateral the trace of a Q1 function on a face is linear in the face parameter s and
// so is (A grad phi) . n, so every face integrand of SWIPDG::Inner / BoundaryLHS is a quadratic in s: the
// reference's 2-point Gauss rule integrates it exactly, and so does the closed form used here,
//   int (A grad phi_j . n) phi_i = |F| (p_i alpha_j + q_i beta_j),  int phi_i phi_j = |F| M_ij,
// with alpha_j / beta_j the values at the face's first / second vertex, (p, q) = (1/3, 1/6) for the first
// face vertex and (1/6, 1/3) for the second, M = [[1/3, 1/6], [1/6, 1/3]] on the face vertices.  The
// vertex values are ghat_j(v) . m with m = J^{-1} A n (one 2-vector per face and side) and the reference
// gradients ghat_j(v) compile-time constants in {0, +-1}.  The volume term keeps the reference's 1-point
// rule (integrand order 0 for piecewise-constant data): S_ij = |det J| kappa ghat_i(c)^T J^{-1} A J^{-T}
// ghat_j(c).  Results equal the quadrature form up to rounding (GPU parity tolerance 1e-12 of the row
// maximum).  Neighbour quantities are in role coordinates (A = my face vertex a, B = b, C = the
// neighbour vertex next to A), as in GenericPolicy.
// ------------------------------------------------------------------------------------------------
// PEN: penalty terms only (the SWIPDG penalty product).  H2: half images (see the persistent kernel): the tile's
// two 32-element halves are computed and streamed in turn through a 20 KB image, so 8 tiles fit per CU and the
// kernel runs two waves per SIMD (<= 256 registers) instead of one.
template <int TK, int KK, bool PEN = false, bool VX = false, bool H2 = false>
struct Q1PwcPolicy : GenericPolicy<Cube, 1, 2, TK, KK, VX> {
  using Base = GenericPolicy<Cube, 1, 2, TK, KK, VX>;
  using E = Cube;
  static constexpr int NB = 4, NF = 4;
  static constexpr bool HALF = H2;
  static constexpr bool EMIT = true;   // emit(): the row block one 4 x 4 block at a time (the sharded SoA fixup)
  static constexpr int WGCU = H2 ? 8 : 4, MINW = H2 ? 2 : 1;
  using Own = typename Base::Own;
  using Gat = typename Base::Gat;

  // reference Q1 gradient of basis k at the reference point (x, y): component d
  __host__ __device__ static constexpr double gh(int k, int d, double x, double y)
  {
    return d == 0 ? ((k & 1) ? 1.0 : -1.0) * ((k & 2) ? y : 1.0 - y)
                  : ((k & 2) ? 1.0 : -1.0) * ((k & 1) ? x : 1.0 - x);
  }

  // Canonical register order of one element's values: V[i * VR + b * NB + c], row i, block b (0: the element
  // itself, column c = basis j; 1 + f: the neighbour across face f, column c = role r).  VR = 20 values per row.
  static constexpr int VR = (NF + 1) * NB, NV80 = NB * VR;

  // block positions inside the element's row block (blocks sorted by element id): the element's own, face f's
  __device__ static void positions(int64_t e, const Own& o, int& pos_self, int* pos)
  {
    pos_self = 0;
#pragma unroll
    for (int f = 0; f < NF; ++f) pos_self += (o.nbr[f] >= 0 && o.nbr[f] < e);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      int p = (e < o.nbr[f]) ? 1 : 0;
#pragma unroll
      for (int q = 0; q < NF; ++q) p += (o.nbr[q] >= 0 && o.nbr[q] < o.nbr[f]);
      pos[f] = p;
    }
  }

  // the element's row block into an LDS image (row length (1 + interior faces) * NB, blocks sorted by element id)
  template <class IMG>
  __device__ static void compute(const AssembleArgs& a, int64_t e, const Own& o, const Gat& gt, IMG img)
  {
    int pos_self, pos[NF];
    positions(e, o, pos_self, pos);
    const int rowlen = (Base::n_interior(o) + 1) * NB;
    emit(a, o, gt, [&](int b, const double (&blk)[NB][NB]) {
      if (b > 0 && o.nbr[b - 1] < 0) return;
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int c = 0; c < NB; ++c)
          img[i * rowlen + (b == 0 ? pos_self * NB + c : pos[b - 1] * NB + role_slot<E>(o.finfo, b - 1, c))] = blk[i][c];
    });
  }

  // The closed forms.  sink(b, blk) receives the row block one 4 x 4 block at a time, blk[i][c] = row i, column c: the
  // neighbour blocks face by face (b = 1 + f, column c = role r; called for every face in uniform control flow,
  // zeros when face f has no neighbour), the element's own block last (b = 0, column c = basis j).
  template <class SINK>
  __device__ static void emit(const AssembleArgs& a, const Own& o, const Gat& gt, SINK&& sink)
  {
    const double j00 = o.X[1] - o.X[0], j01 = o.X[2] - o.X[0], j10 = o.Y[1] - o.Y[0], j11 = o.Y[2] - o.Y[0];
    const double det = j00 * j11 - j01 * j10;
    const double id = rcp_nr(det);
    const double i00 = j11 * id, i01 = -j01 * id, i10 = -j10 * id, i11 = j00 * id;   // J^{-1}
    const double adet = fabs(det);
    const double osgn = det > 0.0 ? 1.0 : -1.0;
    const Tensor A = o.A;
    const double ke = o.ke;
    double S[NB][NB];
    {   // LocalEvaluation::Elliptic, 1-point rule: K = J^{-1} A J^{-T}
      const double p00 = i00 * A.a00 + i01 * A.a01, p01 = i00 * A.a01 + i01 * A.a11;
      const double p10 = i10 * A.a00 + i11 * A.a01, p11 = i10 * A.a01 + i11 * A.a11;
      const double k00 = p00 * i00 + p01 * i01, k01 = p00 * i10 + p01 * i11, k11 = p10 * i10 + p11 * i11;
      const double fac = PEN ? 0.0 : adet * ke;
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const double gix = gh(i, 0, 0.5, 0.5), giy = gh(i, 1, 0.5, 0.5);
          const double gjx = gh(j, 0, 0.5, 0.5), gjy = gh(j, 1, 0.5, 0.5);
          S[i][j] = fac * (gix * (k00 * gjx + k01 * gjy) + giy * (k01 * gjx + k11 * gjy));
        }
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int32_t n = o.nbr[f];
      double EN[NB][NB];
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int r = 0; r < NB; ++r) EN[i][r] = 0.0;
      if (n > HDD_NBR_NEUMANN) {
        const int fa = E::fv(f, 0), fb = E::fv(f, 1);
        const double ax = E::rv(fa, 0), ay = E::rv(fa, 1), bx = E::rv(fb, 0), by = E::rv(fb, 1);
        const double Ax = o.X[fa], Ay = o.Y[fa], Bx = o.X[fb], By = o.Y[fb];
        const double tx = Bx - Ax, ty = By - Ay;
        const double il = rsq_nr(tx * tx + ty * ty);
        const double len = (tx * tx + ty * ty) * il;
        const double nsc = E::face_sign(f) * osgn * il;
        const double nx = ty * nsc, ny = -tx * nsc;
        const double anx = A.a00 * nx + A.a01 * ny, any = A.a01 * nx + A.a11 * ny;
        const double dm = anx * nx + any * ny;
        const double ihp = a.beta == 1.0 ? il : inv_pow(len, a.beta);
        const double mx = i00 * anx + i01 * any, my = i10 * anx + i11 * any;   // J^{-1} A n
        double al[NB], be[NB];   // (A grad phi_k . n) at my face vertices a, b
#pragma unroll
        for (int k = 0; k < NB; ++k) {
          al[k] = gh(k, 0, ax, ay) * mx + gh(k, 1, ax, ay) * my;
          be[k] = gh(k, 0, bx, by) * mx + gh(k, 1, bx, by) * my;
        }
        const double L3 = len * (1.0 / 3.0), L6 = len * (1.0 / 6.0);
        // int (A grad phi_j . n) phi_i  and  int phi_i phi_j
        auto I1 = [&](int j, int i) { return i == fa ? L3 * al[j] + L6 * be[j] : (i == fb ? L6 * al[j] + L3 * be[j] : 0.0); };
        auto MM = [&](int i, int j) {
          return (i == fa || i == fb) && (j == fa || j == fb) ? (i == j ? L3 : L6) : 0.0;
        };
        if (n >= 0) {
          const double Cx = gt.Cx[f], Cy = gt.Cy[f];
          const Tensor Ap = gt.Ap[f];
          const double kn = gt.kn[f];
          // neighbour in role coordinates: A = (0,0), B = (1,0), C = (0,1)
          const double h00 = Bx - Ax, h01 = Cx - Ax, h10 = By - Ay, h11 = Cy - Ay;
          const double hid = rcp_nr(h00 * h11 - h01 * h10);
          const double anpx = Ap.a00 * nx + Ap.a01 * ny, anpy = Ap.a01 * nx + Ap.a11 * ny;
          const double dp = anpx * nx + anpy * ny;
          const double mpx = (h11 * anpx - h01 * anpy) * hid, mpy = (-h10 * anpx + h00 * anpy) * hid;
          double alp[NB], bep[NB];   // (A+ grad phi+_r . n) at A (0,0) and B (1,0)
#pragma unroll
          for (int r = 0; r < NB; ++r) {
            alp[r] = gh(r, 0, 0.0, 0.0) * mpx + gh(r, 1, 0.0, 0.0) * mpy;
            bep[r] = gh(r, 0, 1.0, 0.0) * mpx + gh(r, 1, 1.0, 0.0) * mpy;
          }
          const double rs = rcp_nr(dp + dm);
          const double gamma = (dp * dm) * rs;
          const double w_plus = dm * rs, w_minus = dp * rs;
          const double pen = (ke * kn * a.sigma_inner * gamma) * ihp;
          constexpr double CS = PEN ? 0.0 : 1.0;
          const double cs = -w_minus * ke * CS, cp = -w_plus * kn * CS, cm = w_minus * ke * CS;
#pragma unroll
          for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) S[i][j] += cs * (I1(j, i) + I1(i, j)) + pen * MM(i, j);
#pragma unroll
          for (int i = 0; i < NB; ++i) {
            // int phi+_r phi_i: phi+_A = 1 - s, phi+_B = s (roles 0, 1); int phi+_r (A grad phi_i . n) likewise
            const double pi = i == fa ? L3 : (i == fb ? L6 : 0.0), qi = i == fa ? L6 : (i == fb ? L3 : 0.0);
#pragma unroll
            for (int r = 0; r < NB; ++r) {
              const double anr = pi * alp[r] + qi * bep[r];
              const double ai = r == 0 ? L3 * al[i] + L6 * be[i] : (r == 1 ? L6 * al[i] + L3 * be[i] : 0.0);
              const double mr = r == 0 ? pi : (r == 1 ? qi : 0.0);
              EN[i][r] = cp * anr + cm * ai - pen * mr;
            }
          }
        } else {   // Dirichlet: SWIPDG::BoundaryLHS
          const double pen = (a.sigma_boundary * ke * dm) * ihp;
#pragma unroll
          for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) S[i][j] += -ke * (PEN ? 0.0 : 1.0) * (I1(j, i) + I1(i, j)) + pen * MM(i, j);
        }
      }   // a neighbour or Dirichlet
      sink(1 + f, EN);
    }
    sink(0, S);
  }
};

// P1 simplex, piecewise-constant coefficients: the closed-form policy (p1_compute above)
template <int TK, int KK, bool PEN = false, bool VX = false>
struct P1PwcPolicy {
  static constexpr int NB = 3, NF = 3;
  static constexpr int RB = 36;
  // store-bound.  Element-major geometry: 8 tiles per CU since the out-of-line pow (191 VGPRs, 2 waves per
  // SIMD): C2 0.310 / 0.305 vs 0.312 / 0.314 ms at 4 (profiles/r01/s3/sweep_wgcu_s3.log).  Vertex-indexed
  // geometry: 4 (one wave per SIMD): C2 0.230-0.237 ms vs 0.246-0.247 at 8, 0.242 at 6, 0.256 at 3
  // (same box, profiles/r02/s2/ab_wgcu_vx*)
  static constexpr int WGCU = VX ? 4 : 8, MINW = 1;
  static constexpr bool PAD = false;          // store-bound: its 4-way write conflicts stay hidden
  using Own = P1Own;
  using Gat = P1Gat;
  __device__ static void load_own(const AssembleArgs& a, int64_t e, Own& o) { p1_load_own<TK, KK, VX>(a, e, o); }
  __device__ static void load_gat(const AssembleArgs& a, int64_t e, Own& o, Gat& g) { p1_load_gat<TK, KK, VX>(a, e, o, g); }
  __device__ static void load_gat2(const AssembleArgs& a, Gat& g) { p1_load_gat2<VX>(a, g); }
  __device__ static int n_interior(const Own& o) { return int(o.nbr[0] >= 0) + int(o.nbr[1] >= 0) + int(o.nbr[2] >= 0); }
  __device__ static void compute(const AssembleArgs& a, int64_t e, const Own& o, const Gat& g, double* img)
  {
    p1_compute<PEN>(a, e, o, g, img);
  }
  // full interior tiles (64 elements, three interior faces each: tile length 64 RB): branch-free faces, the image
  // layout static (lane l's row block at l RB)
  static constexpr bool FULLTILE = true;
  __device__ static void compute_full(const AssembleArgs& a, int64_t e, const Own& o, const Gat& g, double* img)
  {
    p1_compute<PEN, true>(a, e, o, g, img);
  }
};

// ------------------------------------------------------------------------------------------------
// P1 with a smooth diffusion factor (OS2014 sinusoid, C3): kappa moments.
//
// P1 gradients, and hence (A grad phi) . n, are constant on an element, so every integrand is kappa (or
// kappa^2 in the interior penalty, kappa^- kappa^+ with one smooth kappa) times a polynomial of the trace:
//   volume   int kappa grad phi_j . A grad phi_i  = |det J| (sum_q w_q kappa(x_q)) g_i . A g_j      (Dunavant 6)
//   face     int kappa phi_i        = |F| sum_q w_q kappa(x_q) phi_i(s_q)                         (Gauss 3)
//            int kappa^m phi_i phi_j = |F| sum_q w_q kappa(x_q)^m phi_i(s_q) phi_j(s_q)  (m = 2 inner, 1 Dirichlet)
// The moments use the reference's points and weights (the same rules as GenericPolicy: integrand orders
// ord kappa + 0 / ord kappa + 2 with ord kappa = 3), so the entries equal the quadrature form up to
// rounding, at 15 kappa evaluations and the P1 closed-form entry count per element.
// ------------------------------------------------------------------------------------------------
template <int TK, bool VX = false, int KK = HDD_FN_SINUSOID>   // KK: the smooth kind (SINUSOID, FLATTOP)
struct P1SmoothPolicy {
  static constexpr int NB = 3, NF = 3;
  static constexpr int RB = 36;
  // 8 tiles per CU at <= 256 registers: 0.201 ms per C3 component vs 0.231 at 4 (and 0.230 for the
  // quadrature policy at 8; profiles/r01/s2/ab_p1s.log)
  static constexpr int WGCU = 8, MINW = 2;
  static constexpr bool PAD = false;
  using Own = P1Own;
  using Gat = P1Gat;
  __device__ static void load_own(const AssembleArgs& a, int64_t e, Own& o) { p1_load_own<TK, HDD_FN_CONST, VX>(a, e, o); }
  __device__ static void load_gat(const AssembleArgs& a, int64_t e, Own& o, Gat& g)
  {
    p1_load_gat<TK, HDD_FN_CONST, VX>(a, e, o, g);
  }
  __device__ static void load_gat2(const AssembleArgs& a, Gat& g) { p1_load_gat2<VX>(a, g); }
  __device__ static int n_interior(const Own& o) { return int(o.nbr[0] >= 0) + int(o.nbr[1] >= 0) + int(o.nbr[2] >= 0); }

  __device__ static void compute(const AssembleArgs& a, int64_t e, const Own& o, const Gat& gt, double* img)
  {
    const KappaArg& K = a.kappa[0];
    auto kap = [&](double x, double y) {
      if constexpr (KK == HDD_FN_FLATTOP) return flattop_sum(K.table, K.n_table, K.c, K.b, x, y);
      return K.c + K.b * sin_phase(K.kx * x + K.ky * y);
    };
    const double j00 = o.X[1] - o.X[0], j01 = o.X[2] - o.X[0], j10 = o.Y[1] - o.Y[0], j11 = o.Y[2] - o.Y[0];
    double kv = 0.0;   // sum_q w_q kappa(x_q), Dunavant 6
    if constexpr (KK == HDD_FN_SINUSOID) {   // small elements: one reduction per element (see the fused policy)
      const double d1 = K.kx * j00 + K.ky * j10, d2 = K.kx * j01 + K.ky * j11;
      if (__all(fabs(d1) + fabs(d2) <= SMALL_PHASE)) {
        double s0, c0;
        sincos_phase(K.kx * o.X[0] + K.ky * o.Y[0], s0, c0);
#pragma unroll
        for (int q = 0; q < 6; ++q)
          kv += VolRule<Simplex, 6>::w(q) *
                (K.c + K.b * sin_near(s0, c0, VolRule<Simplex, 6>::x(q) * d1 + VolRule<Simplex, 6>::y(q) * d2));
        const double dv[3] = {0.0, d1, d2};
        emit(a, e, o, gt, img, kv, [&](int f, double, double, int q) {
          const double da = dv[Simplex::fv(f, 0)], db = dv[Simplex::fv(f, 1)];
          return K.c + K.b * sin_near(s0, c0, da + Gauss01<3>::s(q) * (db - da));
        });
        return;
      }
    }
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const double xh = VolRule<Simplex, 6>::x(q), yh = VolRule<Simplex, 6>::y(q);
      kv += VolRule<Simplex, 6>::w(q) * kap(o.X[0] + j00 * xh + j01 * yh, o.Y[0] + j10 * xh + j11 * yh);
    }
    emit(a, e, o, gt, img, kv, [&](int f, double x, double y, int) { return kap(x, y); });
  }

  // the entries from the volume moment kv = sum_q w_q kappa(x_q) and kappa at the face Gauss points,
  // KF(f, x, y, q) (point q of face f at (x, y), from vertex a to b); ALLIN: three interior faces (full tiles of the
  // persistent driver, as p1_compute)
  template <bool ALLIN = false, class KFace>
  __device__ static void emit(const AssembleArgs& a, int64_t e, const Own& o, const Gat& gt, double* img, double kv,
                              KFace KF)
  {
    double* imgs[1] = {img};
    const double kvs[1] = {kv};
    emitN<1, ALLIN>(a, e, o, gt, imgs, kvs, [&](int, int f, double x, double y, int q) { return KF(f, x, y, q); });
  }

  // NC components at once (the fused C3 policy): the geometry -- Jacobian, gradients, face normals and lengths, the
  // neighbour's gradients, the harmonic weights -- is evaluated once and each component's entries (its own kappa
  // moments) written into its image img[c]; per component the arithmetic is exactly that of emit (NC = 1).
  // KF(c, f, x, y, q): component c's kappa at point q of face f.
  template <int NC, bool ALLIN = false, class KFace>
  __device__ static void emitN(const AssembleArgs& a, int64_t e, const Own& o, const Gat& gt, double* const (&img)[NC],
                               const double (&kv)[NC], KFace KF)
  {
    using E = Simplex;
    const double j00 = o.X[1] - o.X[0], j01 = o.X[2] - o.X[0], j10 = o.Y[1] - o.Y[0], j11 = o.Y[2] - o.Y[0];
    const double det = j00 * j11 - j01 * j10;
    const double id = rcp_nr(det);
    const double i00 = j11 * id, i01 = -j01 * id, i10 = -j10 * id, i11 = j00 * id;
    double g[3][2];
    g[1][0] = i00; g[1][1] = i01;
    g[2][0] = i10; g[2][1] = i11;
    g[0][0] = -i00 - i10; g[0][1] = -i01 - i11;
    double Ag[3][2];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      Ag[k][0] = o.A.a00 * g[k][0] + o.A.a01 * g[k][1];
      Ag[k][1] = o.A.a01 * g[k][0] + o.A.a11 * g[k][1];
    }
    const double adet = fabs(det);
    const double osgn = det > 0.0 ? 1.0 : -1.0;
    const int32_t ei = int32_t(e);   // 32-bit compares (local ids are int32)
    int nblk = 1, pos_self = 0, pos[3];
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      nblk += ALLIN || o.nbr[f] >= 0;
      pos_self += ((ALLIN || o.nbr[f] >= 0) && o.nbr[f] < ei);
    }
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      int p = (ei < o.nbr[f]) ? 1 : 0;
#pragma unroll
      for (int q = 0; q < 3; ++q) p += ((ALLIN || o.nbr[q] >= 0) && o.nbr[q] < o.nbr[f]);
      pos[f] = p;
    }
    const int rowlen = ALLIN ? 12 : nblk * 3;
    // the own block is symmetric (volume g_i.A g_j, face terms symmetric in i, j): its upper triangle, mirrored at
    // the end
    double S[NC][3][3];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const double vol = adet * kv[c];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = i; j < 3; ++j) S[c][i][j] = vol * (Ag[j][0] * g[i][0] + Ag[j][1] * g[i][1]);
    }
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const int32_t n = o.nbr[f];
      if (!ALLIN && n <= HDD_NBR_NEUMANN) continue;
      const int fa = E::fv(f, 0), fb = E::fv(f, 1), fc = 3 - fa - fb;
      const double Ax = o.X[fa], Ay = o.Y[fa], Bx = o.X[fb], By = o.Y[fb];
      const double tx = Bx - Ax, ty = By - Ay;
      const double il = rsq_nr(tx * tx + ty * ty);
      const double len = (tx * tx + ty * ty) * il;
      const double nsc = E::face_sign(f) * osgn * il;
      const double nx = ty * nsc, ny = -tx * nsc;
      double Ae[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) Ae[k] = Ag[k][0] * nx + Ag[k][1] * ny;
      const double dm = agn(o.A, nx, ny, nx, ny);
      const double ihp = a.beta == 1.0 ? il : inv_pow(len, a.beta);
      const bool inner = ALLIN || n >= 0;
      // moments over the face's Gauss 3 points (s from vertex a to vertex b), per component
      double k1a[NC], k1b[NC], qaa[NC], qab[NC], qbb[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        k1a[c] = k1b[c] = qaa[c] = qab[c] = qbb[c] = 0.0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const double sq = Gauss01<3>::s(q), wq = Gauss01<3>::w(q) * len;
          const double k = KF(c, f, Ax + sq * tx, Ay + sq * ty, q);
          const double kk = inner ? k * k : k;
          k1a[c] += wq * k * (1.0 - sq);
          k1b[c] += wq * k * sq;
          qaa[c] += wq * kk * (1.0 - sq) * (1.0 - sq);
          qab[c] += wq * kk * sq * (1.0 - sq);
          qbb[c] += wq * kk * sq * sq;
        }
      }
      auto M1 = [&](int c, int i) { return i == fa ? k1a[c] : (i == fb ? k1b[c] : 0.0); };
      auto MM = [&](int c, int i, int j) {
        return (i == fc || j == fc) ? 0.0 : (i != j ? qab[c] : (i == fa ? qaa[c] : qbb[c]));
      };
      if (inner) {
        const uint32_t inf = (o.finfo >> (4 * f)) & 15u;
        const int tw = int(inf & 7u);
        const bool rev = (inf & 8u) != 0u;
        const int ta = E::fv(tw, 0), tb = E::fv(tw, 1), to = 3 - ta - tb;
        const double Ox = gt.Ox[f], Oy = gt.Oy[f];
        const Tensor Ap = gt.Ap[f];
        const double dp = agn(Ap, nx, ny, nx, ny);
        const double rs = rcp_nr(dp + dm);
        const double gamma = (dp * dm) * rs;
        const double w_plus = dm * rs, w_minus = dp * rs;
        const double pc = (a.sigma_inner * gamma) * ihp;
        const double iD = rcp_nr((Bx - Ax) * (Oy - Ay) - (By - Ay) * (Ox - Ax));
        const double mx = Ap.a00 * nx + Ap.a01 * ny, my = Ap.a01 * nx + Ap.a11 * ny;
        const double AnA = ((By - Oy) * mx + (Ox - Bx) * my) * iD;
        const double AnB = ((Oy - Ay) * mx + (Ax - Ox) * my) * iD;
        const double AnO = ((Ay - By) * mx + (Bx - Ax) * my) * iD;
        const int jA = rev ? tb : ta, jB = rev ? ta : tb;
        // per-face products once: each entry a two-FMA chain
        const double wA = -w_plus * AnA, wB = -w_plus * AnB, wO = -w_plus * AnO;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const double wka = w_minus * k1a[c], wkb = w_minus * k1b[c];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            double* row = img[c] + i * rowlen + pos[f] * 3;
            const double m1i = M1(c, i);
            row[jA] = fma(wA, m1i, fma(Ae[i], wka, -pc * MM(c, i, fa)));
            row[jB] = fma(wB, m1i, fma(Ae[i], wkb, -pc * MM(c, i, fb)));
            row[to] = wO * m1i;
          }
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = i; j < 3; ++j)
              S[c][i][j] += -w_minus * (Ae[j] * M1(c, i) + Ae[i] * M1(c, j)) + pc * MM(c, i, j);
        }
      } else {   // Dirichlet: SWIPDG::BoundaryLHS, penalty sigma_b kappa (n.An) / |F|^beta
        const double pc = (a.sigma_boundary * dm) * ihp;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = i; j < 3; ++j) S[c][i][j] += -(Ae[j] * M1(c, i) + Ae[i] * M1(c, j)) + pc * MM(c, i, j);
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) img[c][i * rowlen + pos_self * 3 + j] = j >= i ? S[c][i][j] : S[c][j][i];
  }
};

// C3 fused: the affine part and the components of an OS2014-type diffusion factor share the phase of their
// sinusoid (kappa_c = a_c + b_c sin(kx x + ky y), problems/OS2014.hh:63-76), so one launch evaluates the 15
// sines of an element ONCE and emits every component from them: per tile, the sines (the volume sum
// sum_q w_q sin and the 3 x 3 face values) stay in registers and the component loop of the persistent
// driver builds each component's LDS image and streams it to that component's value array.  The mesh and
// the gathers are read once instead of once per component.  Entries equal the per-component kernel's up to
// rounding (kappa's volume sum is a_c sum w + b_c sum w sin instead of sum w (a_c + b_c sin)).
// TWO: exactly two components (C3), emitted in one pass over the geometry into two LDS images (emit_two)
template <int TK, bool VX = false, bool TWO_ = false>
struct P1SmoothFusedPolicy : P1SmoothPolicy<TK, VX> {
  using Base = P1SmoothPolicy<TK, VX>;
  using Own = typename Base::Own;
  using Gat = typename Base::Gat;
  static constexpr bool FUSED = true;
  static constexpr bool TWO = TWO_;
  // one wave per SIMD with the whole register file: at two (<= 256 registers) the shared sines, the tile's
  // records and the next tile's in-flight data spill (160-400 B of scratch per lane)
  static constexpr int WGCU = 4, MINW = 1;
  struct Shared {
    double sv;            // sum_q w_q sin(phase(x_q)) (Dunavant 6)
    double sf[3][3];      // sin at the Gauss 3 points of every face
  };
  __device__ static constexpr double wv()   // sum_q w_q = 1/2, the reference triangle's area
  {
    double w = 0.0;
    for (int q = 0; q < 6; ++q) w += VolRule<Simplex, 6>::w(q);
    return w;
  }
  __device__ static void prepare(const AssembleArgs& a, const Own& o, Shared& sh)
  {
    using E = Simplex;
    const KappaArg& K = a.kappa[0];   // the phase (kx, ky) every fused component shares
    const double j00 = o.X[1] - o.X[0], j01 = o.X[2] - o.X[0], j10 = o.Y[1] - o.Y[0], j11 = o.Y[2] - o.Y[0];
    sh.sv = 0.0;
    // phase = p0 + xh d1 + yh d2 on the element; when every lane's element is small against the wavelength
    // (|d1| + |d2| <= SMALL_PHASE, wave-uniform), one reduction per element (sincos of p0) and Taylor offsets
    // per point (trig_phase.hh) instead of 15 full reductions
    const double d1 = K.kx * j00 + K.ky * j10, d2 = K.kx * j01 + K.ky * j11;
    if (__all(fabs(d1) + fabs(d2) <= SMALL_PHASE)) {
      double s0, c0;
      sincos_phase(K.kx * o.X[0] + K.ky * o.Y[0], s0, c0);
#pragma unroll
      for (int q = 0; q < 6; ++q)
        sh.sv += VolRule<Simplex, 6>::w(q) * sin_near(s0, c0, VolRule<Simplex, 6>::x(q) * d1 + VolRule<Simplex, 6>::y(q) * d2);
      const double dv[3] = {0.0, d1, d2};
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        const double da = dv[E::fv(f, 0)], db = dv[E::fv(f, 1)];
#pragma unroll
        for (int q = 0; q < 3; ++q) sh.sf[f][q] = sin_near(s0, c0, da + Gauss01<3>::s(q) * (db - da));
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const double xh = VolRule<Simplex, 6>::x(q), yh = VolRule<Simplex, 6>::y(q);
      const double x = o.X[0] + j00 * xh + j01 * yh, y = o.Y[0] + j10 * xh + j11 * yh;
      sh.sv += VolRule<Simplex, 6>::w(q) * sin_phase(K.kx * x + K.ky * y);
    }
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      const int fa = E::fv(f, 0), fb = E::fv(f, 1);
      const double Ax = o.X[fa], Ay = o.Y[fa], tx = o.X[fb] - Ax, ty = o.Y[fb] - Ay;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const double sq = Gauss01<3>::s(q);
        sh.sf[f][q] = sin_phase(K.kx * (Ax + sq * tx) + K.ky * (Ay + sq * ty));
      }
    }
  }
  template <bool ALLIN = false>
  __device__ static void emit_component(const AssembleArgs& a, int c, int64_t e, const Own& o, const Gat& gt,
                                        const Shared& sh, double* img)
  {
    const KappaArg& K = a.kappa[c];
    Base::template emit<ALLIN>(a, e, o, gt, img, K.c * wv() + K.b * sh.sv,
                               [&](int f, double, double, int q) { return K.c + K.b * sh.sf[f][q]; });
  }
  // both components of a two-component call in one pass over the geometry (the C3 case: OS2014's affine part and
  // its mu-component), into the images img0 / img1
  template <bool ALLIN = false>
  __device__ static void emit_two(const AssembleArgs& a, int64_t e, const Own& o, const Gat& gt, const Shared& sh,
                                  double* img0, double* img1)
  {
    const KappaArg& K0 = a.kappa[0];
    const KappaArg& K1 = a.kappa[1];
    double* const imgs[2] = {img0, img1};
    const double kvs[2] = {K0.c * wv() + K0.b * sh.sv, K1.c * wv() + K1.b * sh.sv};
    Base::template emitN<2, ALLIN>(a, e, o, gt, imgs, kvs, [&](int c, int f, double, double, int q) {
      return c == 0 ? K0.c + K0.b * sh.sf[f][q] : K1.c + K1.b * sh.sf[f][q];
    });
  }
  // (no FULLTILE path: a branch-free second copy of the two-component emission measured slower -- C3 0.249 vs 0.234
  // ms per assembly, rocprof averages on one box, profiles/r06/c_c3/; the kernel is one wave per SIMD and larger code
  // / register allocation across both copies cost more than the branches save)
};

// ------------------------------------------------------------------------------------------------
// Element-local products on the element-diagonal (volume) pattern (swipdg.hh:358-461: L2, H1Semi,
// Elliptic, BoundaryL2 with over_integrate = 2), P1 triangles / Q1 parallelograms, piecewise-constant
// data.  The reference's rules (orders 2p + 2, 2(p-1) + 2 [+ ord kappa]) integrate these polynomial
// integrands exactly, so the closed forms below equal them up to rounding:
//   P1:  l2 |det| (1 + d_ij) / 24;  h1 / elliptic  (|det| / 2) ghat_i^T K ghat_j
//   Q1:  l2 |det| M(i0,j0) M(i1,j1);  h1 / elliptic  sum_ab K_ab F^ab(i,j) with the 1D integrals
//        M = int L_i L_j, D = int L_i' L_j', C = int L_i' L_j (F^00 = D x M, F^01 = C x C^T, F^10 = C^T x C,
//        F^11 = M x D);  K = |det J| kappa J^-1 A J^-T (A = I for h1)
//   boundary l2: sum over boundary faces of |F| (1/3, 1/6) on the face vertices.
// Row block = nb x nb (no neighbour blocks), so tiles are 64 nb^2 doubles and no gathers are needed.
// ------------------------------------------------------------------------------------------------
template <class E, int KIND, int TK, int KK, int VX = 0>   // VX: vertex-indexed geometry (P1 / Q1 kernels' VX)
struct VolProductPolicy {
  static constexpr int NB = E::NB, NF = E::NF, NV = E::NV;
  static constexpr int RB = NB * NB;
  static constexpr int WGCU = 4, MINW = 1;
  static constexpr bool PAD = false;
  struct Own {
    double X[NV], Y[NV];
    int32_t nbr[NF];
    Tensor A;
    double ke;
    int32_t vid[NV];
  };
  struct Gat {};
  static constexpr int NVL = KIND == HDD_PRODUCT_BOUNDARY_L2 ? NV : 3;   // vertices read (0, 1, 2 span the map)
  __device__ static void load_own(const AssembleArgs& a, int64_t e, Own& o)
  {
    const int64_t ne = a.n_local;
#pragma unroll
    for (int k = 0; k < NVL; ++k) {
      if constexpr (VX != 0) {
        o.vid[k] = a.ev[k * ne + e];
      } else {
        o.X[k] = a.coords[(2 * k) * ne + e];
        o.Y[k] = a.coords[(2 * k + 1) * ne + e];
      }
    }
    if constexpr (KIND == HDD_PRODUCT_BOUNDARY_L2) {
#pragma unroll
      for (int f = 0; f < NF; ++f) o.nbr[f] = a.nbrs[f * ne + e];
    }
    if constexpr (KIND == HDD_PRODUCT_ELLIPTIC) {
      o.A = tensor_k<TK>(a, e);
      o.ke = kappa_k<KK>(a, e);
    }
  }
  __device__ static void load_gat(const AssembleArgs& a, int64_t, Own& o, Gat&)
  {
    if constexpr (VX != 0) {
#pragma unroll
      for (int k = 0; k < NVL; ++k) vertex_xy(a, o.vid[k], o.X[k], o.Y[k]);
    }
  }
  __device__ static void load_gat2(const AssembleArgs&, Gat&) {}
  __device__ static int n_interior(const Own&) { return 0; }

  __host__ __device__ static constexpr double m1(int i, int j) { return i == j ? 1.0 / 3.0 : 1.0 / 6.0; }
  __host__ __device__ static constexpr double d1(int i, int j) { return i == j ? 1.0 : -1.0; }
  __host__ __device__ static constexpr double c1(int i, int) { return i ? 0.5 : -0.5; }   // int L_i' L_j

  __device__ static void compute(const AssembleArgs&, int64_t, const Own& o, const Gat&, double* img)
  {
    const double j00 = o.X[1] - o.X[0], j01 = o.X[2] - o.X[0], j10 = o.Y[1] - o.Y[0], j11 = o.Y[2] - o.Y[0];
    const double det = j00 * j11 - j01 * j10;
    const double adet = fabs(det);
    double S[NB][NB];
    if constexpr (KIND == HDD_PRODUCT_L2) {
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          S[i][j] = std::is_same<E, Simplex>::value ? adet * (i == j ? 1.0 / 12.0 : 1.0 / 24.0)
                                                     : adet * (m1(i & 1, j & 1) * m1(i >> 1, j >> 1));
    } else if constexpr (KIND == HDD_PRODUCT_BOUNDARY_L2) {
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) S[i][j] = 0.0;
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        if (o.nbr[f] >= 0) continue;
        const int fa = E::fv(f, 0), fb = E::fv(f, 1);
        const double tx = o.X[fb] - o.X[fa], ty = o.Y[fb] - o.Y[fa];
        const double len = sqrt(tx * tx + ty * ty);
        S[fa][fa] += len * (1.0 / 3.0);
        S[fb][fb] += len * (1.0 / 3.0);
        S[fa][fb] += len * (1.0 / 6.0);
        S[fb][fa] += len * (1.0 / 6.0);
      }
    } else {   // H1_SEMI / ELLIPTIC: K = |det| kappa J^-1 A J^-T
      const double id = rcp_nr(det);
      const double i00 = j11 * id, i01 = -j01 * id, i10 = -j10 * id, i11 = j00 * id;
      double a00 = 1.0, a01 = 0.0, a11 = 1.0, fac = adet;
      if constexpr (KIND == HDD_PRODUCT_ELLIPTIC) {
        a00 = o.A.a00; a01 = o.A.a01; a11 = o.A.a11;
        fac *= o.ke;
      }
      const double p00 = i00 * a00 + i01 * a01, p01 = i00 * a01 + i01 * a11;
      const double p10 = i10 * a00 + i11 * a01, p11 = i10 * a01 + i11 * a11;
      const double k00 = fac * (p00 * i00 + p01 * i01), k01 = fac * (p00 * i10 + p01 * i11);
      const double k11 = fac * (p10 * i10 + p11 * i11);
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if constexpr (std::is_same<E, Simplex>::value) {
            const double gix = i == 1 ? 1.0 : (i == 0 ? -1.0 : 0.0), giy = i == 2 ? 1.0 : (i == 0 ? -1.0 : 0.0);
            const double gjx = j == 1 ? 1.0 : (j == 0 ? -1.0 : 0.0), gjy = j == 2 ? 1.0 : (j == 0 ? -1.0 : 0.0);
            S[i][j] = 0.5 * (gix * (k00 * gjx + k01 * gjy) + giy * (k01 * gjx + k11 * gjy));
          } else {
            const int i0 = i & 1, i1 = i >> 1, jj0 = j & 1, jj1 = j >> 1;
            S[i][j] = k00 * d1(i0, jj0) * m1(i1, jj1) + k01 * c1(i0, jj0) * c1(jj1, i1) +
                      k01 * c1(jj0, i0) * c1(i1, jj1) + k11 * m1(i0, jj0) * d1(i1, jj1);
          }
        }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) img[i * NB + j] = S[i][j];
  }
};

// offset of this lane's row block inside the tile: NB^2 * sum over the active lanes below of (1 + interior
// faces) -- the pattern's elem_ptr rule -- from ballots + mbcnt instead of a per-element elem_ptr load
template <int NB>
__device__ __forceinline__ int tile_offset(int c, bool active)
{
  auto below = [](uint64_t m) {
    return int(__builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u)));
  };
  int sum = below(__ballot(active));
  sum += below(__ballot(active && (c & 1)));
  sum += 2 * below(__ballot(active && (c & 2)));
  sum += 4 * below(__ballot(active && (c & 4)));
  return NB * NB * sum;
}

// ------------------------------------------------------------------------------------------------
// Persistent, software-pipelined driver (see the P1 comment above): per wave a sequence of 64-element
// tiles, memory order [prefetch own data t+1][compute t -> LDS][gathers t+1][stores t].
// ------------------------------------------------------------------------------------------------
//
// LDS image.  Contiguous (element i at its CSR offset inside the tile, streamed with aligned 16-byte reads)
// puts the lanes' row blocks RB doubles apart: for Q1 (RB = 80 = 160 dwords) a ds_write_b64 meets only
// two bank pairs per 32 lanes, a 16-way conflict (80 such writes per tile).  Policies with P::PAD stage
// *uniform* tiles (every element with all NF faces interior: tile length = nact * RB, the bulk of a mesh)
// rotated instead: lane i's value j at lds[i RB + (j + 2 ((i >> 1) & 15)) mod RB] -- 2-way conflicts (the
// floor for a layout that keeps value pairs 16-byte aligned), no padding, so the image is exactly 64 RB
// doubles (40 KB for Q1: 4 tiles per CU instead of 3), and the reader fetches each 16-byte chunk of the
// tile's CSR range with one ds_read_b128.  Other tiles use the contiguous image; for P::PAD policies their
// tail lanes dump into the image's last row block (free: a non-uniform tile with < 64 elements holds at
// most 63 RB - NB^2 values).

// FUSED policies emit several components per tile from one prepare() (P1SmoothFusedPolicy): the driver
// builds and streams one LDS image per component (a.n_comp of them, into a.vals[c])
template <class P, class = void>
struct fused_of : std::false_type {
  struct Shared {};
};
template <class P>
struct fused_of<P, std::void_t<decltype(P::FUSED)>> : std::bool_constant<P::FUSED> {
  using Shared = typename P::Shared;
};
// HALF policies (Q1PwcPolicy<.., H2>) stage a tile through an image of 32 row blocks, one half after the other
template <class P, class = void>
struct half_of : std::false_type {};
template <class P>
struct half_of<P, std::void_t<decltype(P::HALF)>> : std::bool_constant<P::HALF> {};
template <class P>
constexpr int image_blocks() { return half_of<P>::value ? 32 : 64; }
// TWO policies (P1SmoothFusedPolicy<.., true>) emit two components per tile into two images (the LDS holds both)
template <class P, class = void>
struct two_of : std::false_type {};
template <class P>
struct two_of<P, std::void_t<decltype(P::TWO)>> : std::bool_constant<P::TWO> {};
// FULLTILE policies (P1PwcPolicy) have a compute_full for tiles of 64 elements with every face interior
template <class P, class = void>
struct fulltile_of : std::false_type {};
template <class P>
struct fulltile_of<P, std::void_t<decltype(P::FULLTILE)>> : std::bool_constant<P::FULLTILE> {};
template <class P, class = void>
struct emit_of : std::false_type {};
template <class P>
struct emit_of<P, std::void_t<decltype(P::EMIT)>> : std::bool_constant<P::EMIT> {};

// TL: tiles come from a.tile_list, else 0..n_tiles-1; SKIP: the sharded step's full-range launch, which leaves
// the row blocks of elements with a ghost face neighbour to the concurrent element pass (a.skip_ghost)
template <class P, bool TL, bool SKIP = false>
__global__ void __launch_bounds__(64, P::MINW)
swipdg_persistent_kernel(const AssembleArgs a, int64_t n_tiles)
{
  constexpr bool FUSED = fused_of<P>::value;
  constexpr bool HALF = half_of<P>::value;
  constexpr int RB = P::RB;
  constexpr int IMG = image_blocks<P>() * RB;
  constexpr int STORES = (IMG / 2 + 63) / 64;
  constexpr bool TWO = two_of<P>::value;
  constexpr int IMGS = IMG + 2 + RB;   // TWO: doubles per image (+ the alignment slot and the tail lanes' scratch row)
  static_assert(!HALF || (P::PAD && !FUSED && RB == 80), "half images: the Q1 closed-form policy");
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x;
  const int64_t G = gridDim.x, b = blockIdx.x;
  int64_t t, t_end, t_step;
  if (G >= n_tiles) {
    t = b; t_end = b + 1; t_step = 1;
  } else {   // XCD-aware: the 8 XCDs sweep contiguous eighths of the tile range
    const int64_t x = b & 7, w = b >> 3, gx = G >> 3;
    const int64_t s0 = (n_tiles * x) / 8, s1 = (n_tiles * (x + 1)) / 8;
    if (HDD_ABL(a, 32)) {          // study: each wave a contiguous block of its XCD's eighth
      t = s0 + ((s1 - s0) * w) / gx;
      t_end = s0 + ((s1 - s0) * (w + 1)) / gx;
      t_step = 1;
    } else if (HDD_ABL(a, 64)) {   // study: global round robin
      t = b; t_end = n_tiles; t_step = G;
    } else {
      t = s0 + w;
      t_end = s1;
      t_step = gx;
    }
  }
  if (t >= t_end) return;
  double* scratch = P::PAD ? lds + IMG - RB : lds + IMG + 2;
  // Loads whose values must be wave-uniform (tile ids of a tile list, the tiles' CSR bounds elem_ptr[]) are
  // vector loads (the compiler cannot prove elem_ptr unaliased by the value stores, so no s_load); a
  // readfirstlane right after such a load waits for it -- and, vmcnt being in order, for the previous tile's
  // stores issued before it.  So they are issued one tile ahead as raw values and made uniform only in the
  // next iteration, where the wait is a counted one behind the stores.
  // Tile list (interior / halo-boundary split of a sharded assembly): position -> tile.
  auto tile_raw = [&](int64_t pos) -> int64_t {
    if constexpr (TL) return int64_t(a.tile_list[pos]);
    return pos;
  };
  // Full uniform tiles of HALF policies (see the HALF branch below): tile-invariant LDS byte addresses of the lane's
  // two row bases (writer) and of its chunks 0..4 (reader; chunk k + 5 j lies 5120 j bytes further)
  [[maybe_unused]] uint32_t hrow[2] = {0u, 0u}, hrd[5] = {0u, 0u, 0u, 0u, 0u};
  if constexpr (HALF) {
    const int m = lane & 31, hi = lane >> 5;
#pragma unroll
    for (int i = 0; i < 2; ++i) hrow[i] = uint32_t(m * RB + 20 * ((i + 2 * hi + ((m & 7) >> 1)) & 3)) * 8u;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int c = lane + 64 * k, mc = c / 40, u = c % 40, r = u / 10, x = 2 * (u % 10);
      const int rot2 = 2 * (mc & 1), rho = (mc & 7) >> 1;
      const int w = x + rot2;
      hrd[k] = uint32_t(mc * RB + 20 * ((r + rho) & 3) + (w >= 20 ? w - 20 : w)) * 8u;
    }
  }
  auto uni64 = [](int64_t v) -> int64_t { return __builtin_amdgcn_readfirstlane(v); };
  auto elem_of_tile = [&](int64_t tile) {
    const int64_t t0 = a.own_begin + tile * 64;
    const int64_t e0 = t0 + lane;
    return e0 < a.own_end ? e0 : t0;
  };
  auto bounds_raw = [&](int64_t tile, int64_t& base_r, int64_t& end_r) {
    const int64_t t0 = a.own_begin + tile * 64;
    const int64_t tend = t0 + 64 < a.own_end ? t0 + 64 : a.own_end;
    base_r = a.elem_ptr[t0 - a.own_begin];
    end_r = a.elem_ptr[tend - a.own_begin];
  };
  auto next = [&](int64_t pos) { return pos + t_step < t_end ? pos + t_step : pos; };
  int64_t tile = uni64(tile_raw(t));
  int64_t e = elem_of_tile(tile);
  typename P::Own own;
  typename P::Gat gat;
  P::load_own(a, e, own);
  P::load_gat(a, e, own, gat);
  P::load_gat2(a, gat);
  int64_t base_r, tile_end_r;
  bounds_raw(tile, base_r, tile_end_r);
  int64_t tile_n_r = tile_raw(next(t));
  // Drain the prologue's loads before entering the loop.  The compiler's wait counts at the loop head are
  // the minimum over the entry paths: entered straight from the prologue, the first tile's vertex rows
  // are followed by only ~7 memory operations, so the first compute of EVERY iteration waited with
  // vmcnt(7) -- i.e. for all but the last two of the previous tile's 20 stores.  With nothing outstanding
  // on entry only the back edge counts, and that wait skips the stores (in-order vmcnt).
  __builtin_amdgcn_s_waitcnt(0);
  double* out = a.vals[0];
  [[maybe_unused]] typename fused_of<P>::Shared shv;
  for (;;) {
    const bool has_next = t + t_step < t_end;
    const int64_t tn = has_next ? t + t_step : t;
    // own data of the next tile; its id was loaded one iteration ago
    const int64_t tile_n = uni64(tile_n_r);
    const int64_t en = elem_of_tile(tile_n);
    typename P::Own own_n;
    P::load_own(a, en, own_n);
    int64_t base_n_r, tile_end_n_r;
    bounds_raw(tile_n, base_n_r, tile_end_n_r);   // CSR bounds of tile t+1
    const int64_t tile_nn_r = tile_raw(next(tn));
    const int64_t base = uni64(base_r), tile_end = uni64(tile_end_r);   // loaded one iteration ago

    const int64_t t0 = a.own_begin + tile * 64;
    const bool active = t0 + lane < a.own_end;
    const int64_t base_al = base & ~int64_t(1);
    const int tlen = int(tile_end - base);
    // FULLTILE policies: a tile of 64 elements whose row blocks all have the maximum length (every face interior) --
    // the bulk of a mesh -- has a static image layout (lane l at l RB) and takes the branch-free compute_full
    const bool fullt = fulltile_of<P>::value && tlen == 64 * RB;   // wave-uniform
    int off;
    if (fullt) off = lane * RB + int(base - base_al);
    else off = tile_offset<P::NB>(P::n_interior(own), active) + int(base - base_al);
    // sharded step (a.skip_ghost): the row blocks of elements with a ghost face neighbour are written by the
    // element pass on the transfer stream, concurrently -- this tile must not store them (wave-uniform mask)
    uint64_t gmask = 0;
    if constexpr (SKIP) {
      bool g = false;
#pragma unroll
      for (int f = 0; f < P::NF; ++f) g |= own.nbr[f] >= 0 && (own.nbr[f] < a.own_begin || own.nbr[f] >= a.own_end);
      gmask = __ballot(active && g);
    }
    const bool uni = P::PAD && tlen == RB * int(a.own_end - t0 < 64 ? a.own_end - t0 : 64);   // wave-uniform
    typename P::Gat gat_n;
    if constexpr (HALF) {
      // Half images (Q1): the tile's row blocks reach HBM in two halves, elements 0-31 and then 32-63, each half's
      // 32 row blocks staged in a 20 KB LDS image and streamed out as one contiguous CSR range ([base, base + len0),
      // then [base + len0, tile_end); Q1 row blocks are multiples of 16 values and base is even, so both ranges are
      // 16-byte aligned).  20 KB images fit 8 tiles per CU: two waves per SIMD at <= 256 registers.
      //
      // Every lane computes its element's 80 values ONCE, into registers (all 64 lanes busy), and
      // v_permlane32_swap regroups them by half: afterwards V[0..39] hold, in lanes 0-31, rows 0-1 of elements
      // 0-31 and, in lanes 32-63, rows 2-3 of elements 0-31 (lane l - 32's); V[40..79] the same for elements 32-63.
      // So a half's image takes 40 full-width ds_write_b64, and no element is computed twice (round 4 computed each
      // half under a 32-lane exec mask: +57 % VALU instructions for the same output).  The placement of
      // a value (row offsets, column offsets, which blocks exist) is computed by the lane that owns the element and
      // swapped the same way.
      //
      // Full uniform tiles (64 elements with four interior faces each: the bulk of a mesh) use a rotated image:
      // element m of the half, value (row r, column x) of its row block at
      //   m * 80 + 20 ((r + rho_m) & 3) + ((x + rot_m) mod 20),  rot_m = 2 (m & 1), rho_m = (m & 7) >> 1,
      // so the 16 lanes of a ds_write_b64 group (elements m and m + 8 share (rot, rho)) hit 8 distinct 8-byte bank
      // pairs for every (r, x): 2-way, the floor while value pairs stay 16-byte aligned for the reader (an
      // exhaustive search over per-element (row, column) rotations; rotating columns alone mod 20 gives at most 4
      // conflict-free elements).  Other tiles (partial, boundary elements, sharded SKIP tiles) use the contiguous
      // image (CSR order) with per-block predicates.
      constexpr int STH = IMG / 128;   // 16-byte chunks per lane per half (20)
      constexpr int NH = P::NV80 / 2;  // values per lane per half (40)
      static_assert(STH % 4 == 0, "SKIP tiles store a half in 4 KB windows");
      const int nact = int(a.own_end - t0 < 64 ? a.own_end - t0 : 64);
      // (sharded SKIP tiles stay on the rotated image: their skipped elements' chunks are dropped at the store)
      const bool full = uni && nact == 64;   // wave-uniform
      int ps, pf[P::NF];
      P::positions(e, own, ps, pf);
      // column byte offsets of the lane's own element: (x + rot) mod 20 (rotated image) or x (contiguous), x = block
      // position * 4 + column; 8 bits each, four per register
      const int rot2 = full ? 2 * (lane & 1) : 0;
      auto col8 = [&](int x) {
        const int w = x + rot2;
        return uint32_t(w >= P::VR ? w - P::VR : w) * 8u;
      };
      uint32_t W0[P::VR / 4], W1[P::VR / 4];
#pragma unroll
      for (int g = 0; g < P::VR / 4; ++g) {
        uint32_t w = 0;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int q = 4 * g + s, b = q / P::NB, c = q % P::NB;
          const int x = b == 0 ? ps * P::NB + c : pf[b - 1] * P::NB + role_slot<Cube>(own.finfo, b - 1, c);
          w |= col8(x) << (8 * s);
        }
        W0[g] = w;
      }
      // contiguous image: the element block's byte offset in the tile image, the row length in bytes, and which of
      // its blocks exist (bit 0: the element is active, bit 1 + f: face f has a neighbour)
      uint32_t ob0 = uint32_t(off) * 8u, rl0 = uint32_t(P::NB * (P::n_interior(own) + 1)) * 8u, pk0 = active ? 1u : 0u;
#pragma unroll
      for (int f = 0; f < P::NF; ++f) pk0 |= (active && own.nbr[f] >= 0 ? 2u : 0u) << f;
      // the element a lane writes in half h is (lane & 31) + 32 h: after the swaps X0 holds half 0's, X1 half 1's
      auto swap32 = [](uint32_t& x0, uint32_t& x1) {
        const auto r = __builtin_amdgcn_permlane32_swap(x0, x1, false, false);
        x0 = r[0];
        x1 = r[1];
      };
#pragma unroll
      for (int g = 0; g < P::VR / 4; ++g) {
        W1[g] = W0[g];
        swap32(W0[g], W1[g]);
      }
      uint32_t ob1 = ob0, rl1 = rl0, pk1 = pk0;
      swap32(ob0, ob1);
      swap32(rl0, rl1);
      swap32(pk0, pk1);
      const int len0 = full ? 32 * RB : (nact > 32 ? __builtin_amdgcn_readlane(off, 32) : tlen);
      // LDS byte address of the lane's two rows (rows i + 2 (lane >> 5) of its element) in each half's image
      uint32_t row0[2], row1[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t ri = uint32_t(i + 2 * (lane >> 5));
        row0[i] = full ? hrow[i] : ob0 + ri * rl0;
        row1[i] = full ? hrow[i] : ob1 - uint32_t(len0) * 8u + ri * rl1;
      }
      char* const ldsb = reinterpret_cast<char*>(lds);
      auto wcol = [](const uint32_t* Wh, int q) { return (Wh[q / 4] >> (8 * (q % 4))) & 255u; };
      // The values, one 4 x 4 block at a time as the closed forms complete it: rows (0, 1) and (2, 3) swapped
      // between the wave's halves, half 0's part straight into the image, half 1's part kept in registers
      double V1[NH];
      auto put0 = [&](int b, const double (&blk)[P::NB][P::NB]) {
        double lo[2][P::NB];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int c = 0; c < P::NB; ++c) {
            ivec2 x = __builtin_bit_cast(ivec2, blk[i][c]), y = __builtin_bit_cast(ivec2, blk[i + 2][c]);
#pragma unroll
            for (int d = 0; d < 2; ++d) {
              const auto r = __builtin_amdgcn_permlane32_swap(unsigned(x[d]), unsigned(y[d]), false, false);
              x[d] = int(r[0]);
              y[d] = int(r[1]);
            }
            lo[i][c] = __builtin_bit_cast(double, x);
            V1[i * P::VR + b * P::NB + c] = __builtin_bit_cast(double, y);
          }
        if ((pk0 >> b) & 1u) {
#pragma unroll
          for (int c = 0; c < P::NB; ++c) {
            const uint32_t w = wcol(W0, b * P::NB + c);
#pragma unroll
            for (int i = 0; i < 2; ++i) *reinterpret_cast<double*>(ldsb + row0[i] + w) = lo[i][c];
          }
        }
      };
      // (ablation bit 8192: tiles off the rotated-image path skip their compute and stores -- what they cost)
      const bool abl_nf = HDD_ABL(a, 8192) && !full;
      if (!HDD_ABL(a, 1) && !abl_nf) P::emit(a, own, gat, put0);
      // sharded step: image ranges of the skipped elements, tile coordinates (as in stores_skip below)
      constexpr int NR = 4;
      int rb[NR], re[NR];
      uint64_t mrest = gmask;
      const int bo = off, be = off + P::NB * P::NB * (P::n_interior(own) + 1);
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        rb[i] = re[i] = 0;
        if (SKIP && mrest) {
          const int l = __builtin_ctzll(mrest);
          mrest &= mrest - 1;
          rb[i] = __builtin_amdgcn_readlane(bo, l);
          re[i] = __builtin_amdgcn_readlane(be, l);
        }
      }
      auto skipped = [&](int d) {
        bool r = false;
#pragma unroll
        for (int i = 0; i < NR; ++i) r |= d >= rb[i] && d < re[i];
        for (uint64_t mm = mrest; mm; mm &= mm - 1) {
          const int l = __builtin_ctzll(mm);
          r |= d >= __builtin_amdgcn_readlane(bo, l) && d < __builtin_amdgcn_readlane(be, l);
        }
        return r;
      };
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int hb = h ? len0 : 0, hl = (h ? tlen : len0) - hb;   // wave-uniform
        if (h == 1) {   // half 1's values from registers
#pragma unroll
          for (int b = 0; b < P::NF + 1; ++b) {
            if (!((pk1 >> b) & 1u)) continue;
#pragma unroll
            for (int c = 0; c < P::NB; ++c) {
              const uint32_t w = wcol(W1, b * P::NB + c);
#pragma unroll
              for (int i = 0; i < 2; ++i) *reinterpret_cast<double*>(ldsb + row1[i] + w) = V1[i * P::VR + b * P::NB + c];
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (h == 1 && !HDD_ABL(a, 4)) P::load_gat(a, en, own_n, gat_n);   // first gather stage of tile t+1
        if (hl <= 0 || abl_nf) continue;
        const int nb = HDD_ABL(a, 2) ? 0 : hl * 8;
        const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(out + base + hb, (short)0, nb, 0x00020000);
        const uint32_t gm = SKIP ? uint32_t(gmask >> (32 * h)) : 0u;   // this half's skipped elements
        if (full && !gm) {   // 2560 values: every chunk in range, the lane part of the offset in voffset
#pragma unroll
          for (int k = 0; k < STH; ++k) {
            // lane l's chunk k + 5 j (CSR chunk l + 64 (k + 5 j)) sits at hrd[k] + 5120 j in the rotated image
            const dvec2 v = *reinterpret_cast<const dvec2*>(ldsb + hrd[k % 5] + 5120 * (k / 5));
            // (ablation bit 8: default-policy stores instead of non-temporal ones)
            // soffset 1024 k: an SGPR, no VALU per store.  hipcc does not pad the hazard of a VALU write to a
            // > 8-byte store's data registers right after a store with a register soffset, and gfx950 then stores
            // a stale first dword (round 5, the SKIP branch below in its first form); nothing but LDS reads follows
            // these stores -- tests/test_isa_hazards.py scans the built library for the pattern.
            // Cache policy nt (aux 2).  nt + sc1 (aux 18) measured 0.5350 -> 0.5208 ms in interleaved 10-launch
            // loops but +1.0 % in the bench's own 20 / 5 window against the nt library (same box, 3 alternations):
            // kept nt (profiles/r05/f_aux/).  Ablation bits 8 / 1024 / 2048 / 4096: default policy, nt + sc1, sc1,
            // sc0 + nt.
            if (HDD_ABL(a, 8)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rh, 16 * lane, 1024 * k, 0);
            else if (HDD_ABL(a, 1024)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rh, 16 * lane, 1024 * k, 18);
            else if (HDD_ABL(a, 2048)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rh, 16 * lane, 1024 * k, 16);
            else if (HDD_ABL(a, 4096)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rh, 16 * lane, 1024 * k, 3);
            else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rh, 16 * lane, 1024 * k, 2);
          }
        } else if (full) {   // a sharded SKIP tile: chunk l + 64 k belongs to element (l + 64 k) / 40 of the half (40
          // chunks per 640-byte row block); a skipped element's chunks get a voffset beyond the window and are
          // dropped.  The predicate's VALU follows the stores, so no register soffset here: 4 KB windows, one buffer
          // resource each, the offset inside in voffset + the instruction's immediate.
#pragma unroll
          for (int j = 0; j < STH / 4; ++j) {
            const int nbj = nb - 4096 * j;
            const __amdgpu_buffer_rsrc_t rj =
                __builtin_amdgcn_make_buffer_rsrc(out + base + hb + 512 * j, (short)0, nbj > 0 ? nbj : 0, 0x00020000);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int k = 4 * j + q;
              const dvec2 v = *reinterpret_cast<const dvec2*>(ldsb + hrd[k % 5] + 5120 * (k / 5));
              const uint32_t vo = (gm >> ((lane + 64 * k) / 40)) & 1u ? 0x40000000u : 16u * lane;
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rj, vo + 1024 * q, 0, 2);
            }
          }
        } else {      // the range check drops the chunks beyond the half; skipped elements' chunks go out of range
#pragma unroll
          for (int k = 0; k < STH; ++k) {
            const int d = 2 * (lane + 64 * k);
            const dvec2 v = *reinterpret_cast<const dvec2*>(lds + d);
            const int o8 = SKIP && gmask && skipped(hb + d) ? nb : d * 8;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rh, o8, 0, 2);
          }
        }
      }
    } else {
    if constexpr (P::PAD) {
      const RotImg<RB> img{uni ? lds + lane * RB : (active ? lds + off : scratch), uni ? 2 * ((lane >> 1) & 15) : 0};
      if (!HDD_ABL(a, 1)) P::compute(a, e, own, gat, img);
    } else {
      double* img = active ? lds + off : scratch;
      if constexpr (TWO) {   // the shared part once, then both components into their images
        P::prepare(a, own, shv);
        if (!HDD_ABL(a, 1)) P::emit_two(a, e, own, gat, shv, img, img + IMGS);
      } else if constexpr (FUSED) {   // the shared part once, then component 0 (the others after its stores)
        P::prepare(a, own, shv);
        if (!HDD_ABL(a, 1)) P::emit_component(a, 0, e, own, gat, shv, img);
      } else if constexpr (fulltile_of<P>::value) {
        if (HDD_ABL(a, 1)) {
        } else if (fullt) {
          P::compute_full(a, e, own, gat, lds + off);
        } else {
          P::compute(a, e, own, gat, img);
        }
      } else {
        if (!HDD_ABL(a, 1)) P::compute(a, e, own, gat, img);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    double* img_base = lds;   // the image the non-PAD store paths read (TWO: lds + IMGS for component 1)
    const int64_t start = (base + 1) & ~int64_t(1);
    const int64_t stop = tile_end & ~int64_t(1);
    const int nbytes = stop > start && !HDD_ABL(a, 2) ? int(stop - start) * 8 : 0;
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(out + start, (short)0, nbytes, 0x00020000);
    // store chunks k < ksplit go out before the gathers of tile t+1, the rest after them (production: all
    // after; the HDD_ABLATION study bits 128 / 256 move half / all of them in front)
    const int ksplit = HDD_ABL(a, 128) ? STORES / 2 : (HDD_ABL(a, 256) ? STORES : 0);
    // tiles with skipped elements: uniform rotated tiles drop the skipped elements' chunks (element blocks are RB
    // doubles apart and RB is even, so no 16-byte chunk straddles two elements); contiguous images test each
    // chunk against the skipped elements' ranges
    auto stores_skip = [&]() {
      if (P::PAD && uni) {   // (Q1 row blocks are multiples of 16 doubles: base is even, start == base)
        auto at = [](int d) {
          const int l = d / RB, j = d - l * RB;
          const int q = j + 2 * ((l >> 1) & 15);
          return l * RB + (q < RB ? q : q - RB);
        };
        if (!(gmask & 1)) out[base] = lds[at(0)];
        if (!((gmask >> ((tlen - 1) / RB)) & 1)) out[tile_end - 1] = lds[at(tlen - 1)];
        const int dmax = tlen - 2;
#pragma unroll 1   // (a rolled loop: the unrolled form's 40 offsets cost the main path 90 AGPRs)
        for (int k = 0; k < STORES; ++k) {
          const int d = 2 * (lane + 64 * k);
          const dvec2 v = *reinterpret_cast<const dvec2*>(lds + at(d <= dmax ? d : 0));
          const int o8 = ((gmask >> (d <= dmax ? d / RB : 0)) & 1) ? nbytes : d * 8;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rsrc, o8, 0, 2);
        }
      } else if (!uni) {
        // contiguous image: the image ranges [b, e) of the skipped elements (a tile holds one or two -- a strip's
        // row end and the next row's start) go to scalar registers, and each chunk tests its two doubles against
        // them: one 16-byte store when neither is skipped, one 8-byte store when exactly one is
        const int bo = off, be = off + P::NB * P::NB * (P::n_interior(own) + 1);
        constexpr int NR = 4;
        int rb[NR], re[NR];
        uint64_t m = gmask;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          rb[i] = re[i] = 0;
          if (m) {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            rb[i] = __builtin_amdgcn_readlane(bo, l);
            re[i] = __builtin_amdgcn_readlane(be, l);
          }
        }
        auto skipped = [&](int d) {   // image position d inside a skipped element's block
          bool r = false;
#pragma unroll
          for (int i = 0; i < NR; ++i) r |= d >= rb[i] && d < re[i];
          for (uint64_t mm = m; mm; mm &= mm - 1) {   // more than NR skipped elements (uniform loop)
            const int l = __builtin_ctzll(mm);
            r |= d >= __builtin_amdgcn_readlane(bo, l) && d < __builtin_amdgcn_readlane(be, l);
          }
          return r;
        };
        const int a0 = int(start - base_al);   // image position of the first chunk
        if (!skipped(int(base - base_al))) out[base] = img_base[base - base_al];
        if (!skipped(int(tile_end - 1 - base_al))) out[tile_end - 1] = img_base[tile_end - 1 - base_al];
#pragma unroll
        for (int k = 0; k < STORES; ++k) {
          const int idx = 2 * (lane + 64 * k);
          const int li = idx < IMG ? idx : 0;
          const dvec2 v = *reinterpret_cast<const dvec2*>(img_base + a0 + li);
          // (even blocks, Q1: a chunk's two doubles always share an element)
          const bool s0 = skipped(a0 + li), s1 = (P::NB * P::NB) % 2 == 1 ? skipped(a0 + li + 1) : s0;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rsrc, s0 || s1 ? nbytes : idx * 8, 0, 2);
          if constexpr ((P::NB * P::NB) % 2 == 1) {   // odd blocks (P1): a mixed chunk's unskipped half alone
            const int o8 = s0 == s1 ? nbytes : (s0 ? idx * 8 + 8 : idx * 8);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(ivec2, s0 ? v.y : v.x), rsrc, o8, 0, 2);
          }
        }
      }
    };
    // uniform-tile 16-byte stores (ablation bits 1024 / 2048 / 4096: nt + sc1, sc1, sc0 + nt instead of nt; C2
    // measured within noise of nt for each, 20 interleaved rounds, profiles/r05/f_aux/)
    auto st128 = [&](const dvec2& v, int off) {
      if (HDD_ABL(a, 1024)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rsrc, off, 0, 18);
      else if (HDD_ABL(a, 2048)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rsrc, off, 0, 16);
      else if (HDD_ABL(a, 4096)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rsrc, off, 0, 3);
      else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rsrc, off, 0, 2);
    };
    auto stores = [&](bool front) {
      if (gmask) {
        if (!front) stores_skip();
        return;
      }
      if (P::PAD && uni) {
        auto at = [](int d) {   // rotated slot of the tile's CSR value d
          const int l = d / RB, j = d - l * RB;
          const int q = j + 2 * ((l >> 1) & 15);
          return l * RB + (q < RB ? q : q - RB);
        };
        if (!front) {
          const double head = lds[at(0)];
          const double tail = lds[at(tlen - 1)];
          out[base] = head;
          out[tile_end - 1] = tail;
        }
        const int d0 = int(start - base), dmax = tlen - 2;
        if (d0 == 0) {   // element blocks start on even d: every 16-byte chunk is one aligned LDS pair
#pragma unroll
          for (int k = 0; k < STORES; ++k) {
            if ((k < ksplit) != front) continue;
            const int d = 2 * (lane + 64 * k);
            const dvec2 v = *reinterpret_cast<const dvec2*>(lds + at(d <= dmax ? d : 0));
            st128(v, d * 8);
          }
        } else {
#pragma unroll
          for (int k = 0; k < STORES; ++k) {
            if ((k < ksplit) != front) continue;
            const int m2 = 2 * (lane + 64 * k);
            const int d = m2 + 1 <= dmax ? m2 + 1 : 0;
            dvec2 v;
            v.x = lds[at(d)];
            v.y = lds[at(d + 1)];
            st128(v, m2 * 8);
          }
        }
      } else {
        if (!front) {
          const double head = img_base[base - base_al];
          const double tail = img_base[tile_end - 1 - base_al];
          out[base] = head;
          out[tile_end - 1] = tail;
        }
        const double* src = img_base + (start - base_al);
#pragma unroll
        for (int k = 0; k < STORES; ++k) {
          if ((k < ksplit) != front) continue;
          const int idx = 2 * (lane + 64 * k);
          const int li = idx < IMG ? idx : 0;
          const dvec2 v = *reinterpret_cast<const dvec2*>(src + li);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), rsrc, idx * 8, 0, 2);
        }
      }
    };
    if (ksplit > 0) stores(true);
    if (!HDD_ABL(a, 4)) P::load_gat(a, en, own_n, gat_n);
    stores(false);
    if constexpr (TWO) {   // component 1 from the second image
      img_base = lds + IMGS;
      out = a.vals[1];
      rsrc = __builtin_amdgcn_make_buffer_rsrc(out + start, (short)0, nbytes, 0x00020000);
      stores(false);
      img_base = lds;
      out = a.vals[0];
    } else if constexpr (FUSED) {   // the other components: same image slots, their own value arrays
      for (int c = 1; c < a.n_comp; ++c) {
        double* img = active ? lds + off : scratch;
        if (!HDD_ABL(a, 1)) P::emit_component(a, c, e, own, gat, shv, img);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        out = a.vals[c];
        rsrc = __builtin_amdgcn_make_buffer_rsrc(out + start, (short)0, nbytes, 0x00020000);
        stores(false);
      }
      out = a.vals[0];
    }
    }   // !HALF
    // second gather stage of tile t+1 (vertex-indexed geometry: the neighbours' off-face vertices by the
    // ids the first stage brought): its wait covers the first stage only, which was issued before the
    // stores of tile t (vmcnt is in order), so it never waits for those stores
    if (!HDD_ABL(a, 4)) P::load_gat2(a, gat_n);   // (ablation 4: no stage-1 ids to follow)
    if (!has_next) break;
    t = tn;
    tile_n_r = tile_nn_r;
    base_r = base_n_r;
    tile_end_r = tile_end_n_r;
    tile = tile_n;
    e = en;
    own = own_n;
    gat = gat_n;
  }
}

// ------------------------------------------------------------------------------------------------
// Element-list pass (a.list_elements): one lane per listed owned element -- the fixup of a sharded step, which
// assembles every tile while the halo is in flight and then recomputes only the elements that read a ghost
// (a few thousand: one lane each, its row block built in the lane's own LDS slot and written by that lane).
// ------------------------------------------------------------------------------------------------
template <class P>
__global__ void __launch_bounds__(64) swipdg_elements_kernel(const AssembleArgs a, int64_t n)
{
  constexpr int RB = P::RB;
  constexpr bool FUSED = fused_of<P>::value;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x;
  double* img = lds + lane * RB;
  for (int64_t i0 = int64_t(blockIdx.x) * 64; i0 < n; i0 += int64_t(gridDim.x) * 64) {
    const int64_t i = i0 + lane;
    const bool act = i < n;
    const int64_t e = a.own_begin + int64_t(a.tile_list[act ? i : i0]);
    typename P::Own own;
    typename P::Gat gat;
    P::load_own(a, e, own);
    P::load_gat(a, e, own, gat);
    P::load_gat2(a, gat);
    const int64_t base = a.elem_ptr[e - a.own_begin];
    const int len = P::NB * P::NB * (P::n_interior(own) + 1);
    [[maybe_unused]] typename fused_of<P>::Shared shv;
    if constexpr (FUSED) P::prepare(a, own, shv);
    const int ncomp = FUSED ? a.n_comp : 1;
    for (int c = 0; c < ncomp; ++c) {
      if constexpr (FUSED) {
        P::emit_component(a, c, e, own, gat, shv, img);
      } else if constexpr (P::PAD) {
        P::compute(a, e, own, gat, RotImg<RB>{img, 0});
      } else {
        P::compute(a, e, own, gat, img);
      }
      double* out = a.vals[c];
      if (act)
        for (int k = 0; k < len; ++k) __builtin_nontemporal_store(img[k], out + base + k);
    }
  }
}

// Element-list pass without LDS, so that it runs on the transfer stream beside a persistent assembly that holds
// the LDS (sharded step, shard.hip).  a.list_elements == 3: lane i writes the row block of listed element i in
// place (the concurrent assembly runs with a.skip_ghost and leaves those blocks alone; inactive lanes repeat
// lane 0's element); == 2: into side buffers a.vals[c] + i RB (slot n: the inactive lanes' dummy), which
// fix_scatter_kernel copies into place after the join (round-3 A/B variant).
template <class P>
__global__ void __launch_bounds__(64) swipdg_elements_buf_kernel(const AssembleArgs a, int64_t n)
{
  constexpr int RB = P::RB;
  constexpr bool FUSED = fused_of<P>::value;
  const int lane = threadIdx.x;
  for (int64_t i0 = int64_t(blockIdx.x) * 64; i0 < n; i0 += int64_t(gridDim.x) * 64) {
    const int64_t i = i0 + lane;
    const bool act = i < n;
    const int64_t e = a.own_begin + int64_t(a.tile_list[act ? i : i0]);
    const int64_t slot = act ? i : n;
    typename P::Own own;
    typename P::Gat gat;
    P::load_own(a, e, own);
    P::load_gat(a, e, own, gat);
    P::load_gat2(a, gat);
    if constexpr (emit_of<P>::value) {
      if (a.list_elements == 4) {   // value-major side buffer: canonical value k of list entry i at vals[0][k fix_ld + i]
        double* const buf = a.vals[0] + i;
        P::emit(a, own, gat, [&](int b, const double (&blk)[P::NB][P::NB]) {
          if (!act) return;
#pragma unroll
          for (int r = 0; r < P::NB; ++r)
#pragma unroll
            for (int c = 0; c < P::NB; ++c) buf[int64_t(r * P::VR + b * P::NB + c) * a.fix_ld] = blk[r][c];
        });
        continue;
      }
    }
    [[maybe_unused]] typename fused_of<P>::Shared shv;
    if constexpr (FUSED) P::prepare(a, own, shv);
    const int ncomp = FUSED ? a.n_comp : 1;
    const int64_t dst = a.list_elements == 3 ? a.elem_ptr[e - a.own_begin] : slot * RB;
    for (int c = 0; c < ncomp; ++c) {
      double* img = a.vals[c] + dst;
      if constexpr (FUSED) P::emit_component(a, c, e, own, gat, shv, img);
      else if constexpr (P::PAD) P::compute(a, e, own, gat, RotImg<RB>{img, 0});
      else P::compute(a, e, own, gat, img);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host-side launch
// ------------------------------------------------------------------------------------------------
template <class E, int NQV, int NQF, bool PWC>
static hipError_t launch_t(const AssembleArgs& a, hipStream_t s)
{
  const int64_t n_own = a.own_end - a.own_begin;
  if (n_own <= 0) return hipSuccess;
  static const std::string name = [] {   // "swipdg_assemble_kernel<E, NQV, NQF, PWC>" (hdd_last_tile_kernel)
    const std::string f = __PRETTY_FUNCTION__;
    const size_t i = f.find('['), j = f.rfind(']');
    return "swipdg_assemble_kernel<" + (i == std::string::npos ? std::string("?") : f.substr(i + 1, j - i - 1)) + ">";
  }();
  hdd::last_tile_kernel_slot() = name.c_str();
  const int64_t tiles = (n_own + 63) / 64;
  // tile image (64 elements x full row blocks) + 1 alignment slot + a scratch row for tail lanes
  const size_t lds = (size_t(64) * E::NB * (E::NF + 1) * E::NB + 2 + (E::NF + 1) * E::NB) * sizeof(double);
  for (int c = 0; c < a.n_comp; ++c) {
    AssembleArgs ac = a;
    ac.n_comp = 1;
    ac.kappa[0] = a.kappa[c];
    ac.vals[0] = a.vals[c];
    hipLaunchKernelGGL((swipdg_assemble_kernel<E, NQV, NQF, PWC>), dim3(unsigned(tiles)), dim3(64 * E::NB), lds, s, ac);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// "swipdg_persistent_kernel<Policy<...>, TL, SKIP>" from the template argument's pretty name (host, once per policy)
template <class P>
static std::string kernel_name(const char* flags)
{
  const std::string f = __PRETTY_FUNCTION__;   // "... [P = hdd::dev::Q1PwcPolicy<1, 0, false, true, true>]"
  const size_t a = f.find("P = "), b = f.rfind(']');
  std::string p = a == std::string::npos ? "?" : f.substr(a + 4, b - a - 4);
  if (p.rfind("hdd::dev::", 0) == 0) p = p.substr(10);
  return "swipdg_persistent_kernel<" + p + ", " + flags + ">";
}

template <class P>
static hipError_t launch_persistent(const AssembleArgs& a, hipStream_t s)
{
  const int64_t n_own = a.own_end - a.own_begin;
  if (n_own <= 0) return hipSuccess;
  const int64_t tiles = a.tile_list ? a.n_tile_list : (n_own + 63) / 64;
  if (tiles <= 0) return hipSuccess;
  const size_t lds = (P::PAD ? size_t(image_blocks<P>()) * P::RB : size_t(64) * P::RB + 2 + P::RB) * sizeof(double) *
                     (two_of<P>::value ? 2 : 1);
  if (two_of<P>::value && a.n_comp != 2) return hipErrorInvalidValue;
  const int cus = a.n_cu;
  // tiles per CU measured per policy (profiles/r01/sweep_wg_per_cu.log, profiles/r01/s2/); a.wgcu > 0 is the
  // HDD_P1_WGCU sweep override, read once per context
  int wgcu = a.wgcu > 0 ? a.wgcu : P::WGCU;
#ifdef HDD_ABLATION
  // HDD_P1_WGCU = W + 16 C (C > 0): W tiles per CU with at most C resident per CU -- the dynamic LDS padded to
  // 160 KB / C, so the dispatcher cannot stack more workgroups on one CU than C (residency study)
  const size_t lds_launch = a.wgcu >= 16 ? std::max(lds, size_t((160 * 1024) / (a.wgcu >> 4)) & ~size_t(15)) : lds;
  if (a.wgcu >= 16) wgcu = (a.wgcu & 15) ? (a.wgcu & 15) : P::WGCU;
#define HDD_LDS_LAUNCH lds_launch
#else
#define HDD_LDS_LAUNCH lds
#endif
  wgcu = std::max(1, std::min<int>(wgcu, int((160 * 1024) / HDD_LDS_LAUNCH)));   // resident by LDS (Q1 tiles: 3 per CU)
  // The sharded step's full-range launch (SKIP, or every tile beside the SoA side-buffer pass) runs beside the
  // element pass: the grid is shortened
  // by the pass's workgroups (a multiple of 8 keeps the XCD eighths even), so the pass gets SIMDs of its own
  // instead of slowing the persistent waves it would share them with.  C4 N = 8 middle rank +9.2 -> +7.8 %, C2 N = 8
  // end rank +4.9 -> +2.0 % over one launch (profiles/r04/e_reserve/; ablation bit 4194304: no reserve).
  int64_t slots = int64_t(cus) * wgcu;
  const bool reserve = a.reserve_wg > 0 && !HDD_ABL(a, 4194304);
  if (reserve) slots = std::max<int64_t>(8, (slots - a.reserve_wg) & ~int64_t(7));
  const int64_t G = std::min<int64_t>(tiles, slots);
  const int n_launch = fused_of<P>::value ? 1 : a.n_comp;   // a FUSED policy emits every component per tile
  if (a.list_elements) {   // element-list fixup pass: one lane per element
    const size_t lds_e = size_t(64) * P::RB * sizeof(double);
    const int64_t ge = std::min<int64_t>((a.n_tile_list + 63) / 64, int64_t(cus) * 4);
    if (a.list_elements >= 2) {   // no LDS: into the side buffers (2: slot RB doubles) or in place (3)
      if (a.list_elements == 2 && a.fix_rb != P::RB) return hipErrorInvalidValue;
      if (a.list_elements == 4 && (!emit_of<P>::value || a.fix_ld < a.n_tile_list + 1)) return hipErrorInvalidValue;
      for (int c = 0; c < n_launch; ++c) {
        AssembleArgs ac = a;
        if (!fused_of<P>::value) {
          ac.n_comp = 1;
          ac.kappa[0] = a.kappa[c];
          ac.vals[0] = a.vals[c];
        }
        hipLaunchKernelGGL((swipdg_elements_buf_kernel<P>), dim3(unsigned(ge)), dim3(64), 0, s, ac, a.n_tile_list);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
      }
      return hipSuccess;
    }
    for (int c = 0; c < n_launch; ++c) {
      AssembleArgs ac = a;
      if (!fused_of<P>::value) {
        ac.n_comp = 1;
        ac.kappa[0] = a.kappa[c];
        ac.vals[0] = a.vals[c];
      }
      hipLaunchKernelGGL((swipdg_elements_kernel<P>), dim3(unsigned(ge)), dim3(64), lds_e, s, ac, a.n_tile_list);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // the dispatch's choice, readable through hdd_last_tile_kernel(): "swipdg_persistent_kernel<P, TL, SKIP>"
  static const std::string names[3] = {kernel_name<P>("true, false"), kernel_name<P>("false, true"),
                                       kernel_name<P>("false, false")};
  hdd::last_tile_kernel_slot() = names[a.tile_list ? 0 : (a.skip_ghost ? 1 : 2)].c_str();
  for (int c = 0; c < n_launch; ++c) {
    AssembleArgs ac = a;
    if (!fused_of<P>::value) {
      ac.n_comp = 1;
      ac.kappa[0] = a.kappa[c];
      ac.vals[0] = a.vals[c];
    }
    if (a.tile_list)
      hipLaunchKernelGGL((swipdg_persistent_kernel<P, true>), dim3(unsigned(G)), dim3(64), HDD_LDS_LAUNCH, s, ac, tiles);
    else if (a.skip_ghost)
      hipLaunchKernelGGL((swipdg_persistent_kernel<P, false, true>), dim3(unsigned(G)), dim3(64), HDD_LDS_LAUNCH, s, ac, tiles);
    else
      hipLaunchKernelGGL((swipdg_persistent_kernel<P, false>), dim3(unsigned(G)), dim3(64), HDD_LDS_LAUNCH, s, ac, tiles);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
#undef HDD_LDS_LAUNCH

// instantiate a policy for the runtime (tensor kind, piecewise-constant kappa kind) pair
template <template <int, int> class PT>
static hipError_t dispatch_pwc(const AssembleArgs& a, hipStream_t s)
{
  const int tk = a.tkind;
  const bool pe = a.kappa[0].kind == HDD_FN_PER_ELEM;
  if (tk == HDD_TENSOR_CONST)
    return pe ? launch_persistent<PT<HDD_TENSOR_CONST, HDD_FN_PER_ELEM>>(a, s) : launch_persistent<PT<HDD_TENSOR_CONST, HDD_FN_CONST>>(a, s);
  if (tk == HDD_TENSOR_ISO_PER_ELEM)
    return pe ? launch_persistent<PT<HDD_TENSOR_ISO_PER_ELEM, HDD_FN_PER_ELEM>>(a, s) : launch_persistent<PT<HDD_TENSOR_ISO_PER_ELEM, HDD_FN_CONST>>(a, s);
  return pe ? launch_persistent<PT<HDD_TENSOR_SYM_PER_ELEM, HDD_FN_PER_ELEM>>(a, s) : launch_persistent<PT<HDD_TENSOR_SYM_PER_ELEM, HDD_FN_CONST>>(a, s);
}

// instantiate a policy for the runtime (tensor kind, kappa kind) pair; VX: vertex-indexed geometry
template <template <int, int, bool> class PT, bool VX>
static hipError_t dispatch_kinds_vx(const AssembleArgs& a, hipStream_t s, bool smooth)
{
  const int tk = a.tkind, kk = a.kappa[0].kind;
  if (smooth && kk == HDD_FN_FLATTOP) {
    if (tk == HDD_TENSOR_CONST) return launch_persistent<PT<HDD_TENSOR_CONST, HDD_FN_FLATTOP, VX>>(a, s);
    if (tk == HDD_TENSOR_ISO_PER_ELEM) return launch_persistent<PT<HDD_TENSOR_ISO_PER_ELEM, HDD_FN_FLATTOP, VX>>(a, s);
    return launch_persistent<PT<HDD_TENSOR_SYM_PER_ELEM, HDD_FN_FLATTOP, VX>>(a, s);
  }
  if (smooth) {
    if (tk == HDD_TENSOR_CONST) return launch_persistent<PT<HDD_TENSOR_CONST, HDD_FN_SINUSOID, VX>>(a, s);
    if (tk == HDD_TENSOR_ISO_PER_ELEM) return launch_persistent<PT<HDD_TENSOR_ISO_PER_ELEM, HDD_FN_SINUSOID, VX>>(a, s);
    return launch_persistent<PT<HDD_TENSOR_SYM_PER_ELEM, HDD_FN_SINUSOID, VX>>(a, s);
  }
  const bool pe = kk == HDD_FN_PER_ELEM;
  if (tk == HDD_TENSOR_CONST)
    return pe ? launch_persistent<PT<HDD_TENSOR_CONST, HDD_FN_PER_ELEM, VX>>(a, s)
              : launch_persistent<PT<HDD_TENSOR_CONST, HDD_FN_CONST, VX>>(a, s);
  if (tk == HDD_TENSOR_ISO_PER_ELEM)
    return pe ? launch_persistent<PT<HDD_TENSOR_ISO_PER_ELEM, HDD_FN_PER_ELEM, VX>>(a, s)
              : launch_persistent<PT<HDD_TENSOR_ISO_PER_ELEM, HDD_FN_CONST, VX>>(a, s);
  return pe ? launch_persistent<PT<HDD_TENSOR_SYM_PER_ELEM, HDD_FN_PER_ELEM, VX>>(a, s)
            : launch_persistent<PT<HDD_TENSOR_SYM_PER_ELEM, HDD_FN_CONST, VX>>(a, s);
}
// Vertex-indexed geometry pays on triangles (C2 0.323 -> 0.245 ms, same box: 2 waves per SIMD hide the
// second gather stage); the Q1 tiles run one wave per SIMD (40 KB image), where that stage's latency is
// exposed (C4 0.600 -> 0.690 ms), so quads keep the element-major coords.
template <template <int, int, bool> class PT>
static hipError_t dispatch_kinds(const AssembleArgs& a, hipStream_t s, bool smooth)
{
  if constexpr (PT<HDD_TENSOR_CONST, HDD_FN_CONST, false>::NB == 4) {   // quads: element-major only
    return dispatch_kinds_vx<PT, false>(a, s, smooth);
  } else {
    return a.ev && a.elem_type == HDD_SIMPLEX ? dispatch_kinds_vx<PT, true>(a, s, smooth)
                                              : dispatch_kinds_vx<PT, false>(a, s, smooth);
  }
}

template <int TK, int KK, bool VX> using P1Pwc = P1PwcPolicy<TK, KK, false, VX>;
template <int TK, int KK, bool VX> using Q1Pwc = Q1PwcPolicy<TK, KK, false, VX>;
template <int TK, int KK, bool VX> using Q1PwcH2 = Q1PwcPolicy<TK, KK, false, VX, true>;
template <int TK, int KK, bool VX> using Q1Smooth3 = GenericPolicy<Cube, 4, 3, TK, KK, VX>;
template <int TK, int KK, bool VX> using P1Smooth3 = GenericPolicy<Simplex, 6, 3, TK, KK, VX>;


// per-family entry points (one translation unit each)
hipError_t launch_p1_pwc(const AssembleArgs& a, hipStream_t s);       // swipdg_p1.hip
hipError_t launch_p1_smooth(const AssembleArgs& a, hipStream_t s);
hipError_t launch_p1_penalty(const AssembleArgs& a, hipStream_t s);
hipError_t launch_p1_smooth_fused(const AssembleArgs& a, hipStream_t s);   // all components in one launch
hipError_t launch_q1_pwc(const AssembleArgs& a, hipStream_t s);       // swipdg_q1.hip
hipError_t launch_q1_smooth(const AssembleArgs& a, hipStream_t s);
hipError_t launch_q1_penalty(const AssembleArgs& a, hipStream_t s);
hipError_t launch_vol_products(const AssembleArgs& a, int product, hipStream_t s);   // swipdg_vol.hip

}  // namespace dev
}  // namespace hdd
