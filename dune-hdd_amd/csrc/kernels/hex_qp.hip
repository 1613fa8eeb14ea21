// dune-hdd_amd/csrc/kernels/hex_qp.hip
//
// SWIPDG stiffness assembly for discontinuous Q_p (p = 1..3) on affine hexahedra -- the C5 configuration
// (ESV2007 3d structured, SWIPDG p=3; BASELINE.json configs[4]).  Replaces, for HDD_HEX meshes, the
// SystemAssembler walk of SWIPDG::init() (dune/hdd/linearelliptic/discretizations/swipdg.hh:218-249, 485)
// over LocalEvaluation::Elliptic (volume), SWIPDG::Inner and SWIPDG::BoundaryLHS.
//
// At p=3 every local matrix is a dense 64x64 contraction over quadrature points, so it runs on the f64
// matrix cores (v_mfma_f64_16x16x4_f64):
//   volume   S  = Dhat * R,             Dhat[i][(q,a)] = d_a phi_i(x_q),  R[(q,a)][j] = sum_b G_q[a][b] d_b phi_j(x_q),
//            G_q = w_q |det J| kappa(x_q) J^{-1} A J^{-T}                        (K = 3 nq)
//   face f   S += [V- | N-] * [[eta V- - alpha N-]^T ; [-alpha V-]^T]           (K = 2 nqf)
//            E_f = [V- | N-] * [[-beta N+ - eta V+]^T ; [alpha V+]^T]          (entity/neighbour block)
//   with V[i][q] = phi_i(x_q), N[i][q] = (A grad phi_i . n)(x_q), alpha = w|F| omega^- kappa^-,
//   beta = w|F| omega^+ kappa^+, eta = w|F| sigma kappa^- kappa^+ gamma / |F|^beta  (Dirichlet faces:
//   alpha = w|F| kappa, eta = w|F| sigma_b kappa (n.An) / |F|^beta).
// Rows are owner-computed (each element writes its own 64 rows: the self block and one block per
// interior face), so no atomics and every value is written exactly once.
//
// One workgroup = NT wavefronts per element (NT = ceil(nb/16): 4 at p=3); wave w owns output column
// tile w and all row tiles.  Operand fragments are generated into LDS from 1D tables (the basis and the
// Gauss rules are tensor products on the reference cube), in MFMA fragment order so that every operand
// read is one conflict-free ds_read_b64 per lane.  Faces must be aligned (twin face f^1, no flip): the
// structured grids hdd_grid_create_structured_3d builds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "hdd_internal.hh"
#include "swipdg_kernels.hh"
#include "trig_phase.hh"

namespace hdd {
namespace dev {

typedef double dbl4 __attribute__((ext_vector_type(4)));

#ifdef HDD_ABLATION   // profiling ablations (HDD_DEBUG_FLAGS): 2 = drop the value stores
#define HDD_HEX_ABL(a, bit) (((a).debug_flags & (bit)) != 0)
#else
#define HDD_HEX_ABL(a, bit) false
#endif

template <int P, int SM>
struct HexCfg {
  static constexpr int NP = P + 1;
  static constexpr int NB = NP * NP * NP;
  static constexpr int NBP = (NB + 15) / 16 * 16;
  static constexpr int NT = NBP / 16;                 // 16-wide tiles per block side = waves per element
  static constexpr int THREADS = 64 * NT;
  static constexpr int NV1 = P + SM, NF1 = P + 1 + SM;  // Gauss points per direction (SM: smooth kappa, order 3)
  static constexpr int NQV = NV1 * NV1 * NV1, NQF = NF1 * NF1;
  static constexpr int KV = 3 * NQV, KVS = (KV + 3) / 4;   // volume k-steps
  static constexpr int KF = 2 * NQF, KFS = (KF + 3) / 4;   // face k-steps
  static constexpr int KC = KVS < 16 ? KVS : 16;           // volume k-steps per LDS chunk
  static constexpr int CHUNK = KC * NT * 64;               // doubles per fragment table chunk
  static constexpr int FACE = KFS * NT * 64;
  static constexpr int BUF = (2 * CHUNK > 3 * FACE) ? 2 * CHUNK : 3 * FACE;
};

struct HexLds1D {
  double Lv[4][8], Dv[4][8], Lf[4][8], Df[4][8], Le[4][2], De[4][2];
  double sv[8], wv[8], sf[8], wf[8];
};

__device__ __forceinline__ dbl4 mfma(double a, double b, dbl4 c)
{
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <int NP>
__device__ __forceinline__ void split3(int i, int& i0, int& i1, int& i2)
{
  i0 = i % NP;
  i1 = (i / NP) % NP;
  i2 = i / (NP * NP);
}

// volume reference gradient component a of basis i at volume point (q0, q1, q2)
template <int NP>
__device__ __forceinline__ double dhat(const HexLds1D& t, int i, int a, int q0, int q1, int q2)
{
  int i0, i1, i2;
  split3<NP>(i, i0, i1, i2);
  const double f0 = a == 0 ? t.Dv[i0][q0] : t.Lv[i0][q0];
  const double f1 = a == 1 ? t.Dv[i1][q1] : t.Lv[i1][q1];
  const double f2 = a == 2 ? t.Dv[i2][q2] : t.Lv[i2][q2];
  return f0 * f1 * f2;
}

// value and reference gradient of basis i at the face point (qs, qt) of the face (axis af, side sd);
// selects instead of runtime-indexed local arrays (those would live in scratch)
template <int NP>
__device__ __forceinline__ void face_eval(const HexLds1D& t, int i, int af, int sd, int qs, int qt, double& v,
                                          double& g0, double& g1, double& g2)
{
  int i0, i1, i2;
  split3<NP>(i, i0, i1, i2);
  const int ia = af == 0 ? i0 : (af == 1 ? i1 : i2);
  const int ib0 = af == 0 ? i1 : i0;            // first free axis
  const int ib1 = af == 2 ? i1 : i2;            // second free axis
  const double le = t.Le[ia][sd], de = t.De[ia][sd];
  const double l0 = t.Lf[ib0][qs], d0 = t.Df[ib0][qs];
  const double l1 = t.Lf[ib1][qt], d1 = t.Df[ib1][qt];
  v = le * l0 * l1;
  const double ga = de * l0 * l1, gb0 = le * d0 * l1, gb1 = le * l0 * d1;
  g0 = af == 0 ? ga : gb0;
  g1 = af == 1 ? ga : (af == 0 ? gb0 : gb1);
  g2 = af == 2 ? ga : gb1;
}

struct ElemGeo {
  double v0[3], J[3][3], Ji[3][3], det;
};

__device__ __forceinline__ void elem_geo(const HexArgs& a, int64_t e, ElemGeo& G)
{
  const int64_t n = a.n_local;
  const double* c = a.coords;
  // vertices 0, 1, 2, 4 of the Dune cube: rows 3k + comp
  for (int d = 0; d < 3; ++d) {
    G.v0[d] = c[d * n + e];
    G.J[d][0] = c[(3 + d) * n + e] - G.v0[d];
    G.J[d][1] = c[(6 + d) * n + e] - G.v0[d];
    G.J[d][2] = c[(12 + d) * n + e] - G.v0[d];
  }
  const double(*J)[3] = G.J;
  const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
  const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
  const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
  G.det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
  const double id = 1.0 / G.det;
  G.Ji[0][0] = c00 * id;
  G.Ji[1][0] = c01 * id;
  G.Ji[2][0] = c02 * id;
  G.Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * id;
  G.Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * id;
  G.Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * id;
  G.Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * id;
  G.Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * id;
  G.Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * id;
}

__device__ __forceinline__ void elem_tensor(const HexArgs& a, int64_t e, double A[3][3])
{
  double c[6];
  if (a.tkind == HDD_TENSOR_ISO_PER_ELEM) {
    const double k = a.tper[e];
    c[0] = k; c[1] = 0.0; c[2] = 0.0; c[3] = k; c[4] = 0.0; c[5] = k;
  } else if (a.tkind == HDD_TENSOR_SYM_PER_ELEM) {
    for (int r = 0; r < 6; ++r) c[r] = a.tper[r * a.n_local + e];
  } else {
    for (int r = 0; r < 6; ++r) c[r] = a.tc[r];
  }
  A[0][0] = c[0]; A[0][1] = A[1][0] = c[1]; A[0][2] = A[2][0] = c[2];
  A[1][1] = c[3]; A[1][2] = A[2][1] = c[4]; A[2][2] = c[5];
}

__device__ __forceinline__ double kappa_at(const HexArgs& a, int64_t e, const double* x)
{
  if (a.kkind == HDD_FN_PER_ELEM) return a.kper[e];
  if (a.kkind == HDD_FN_SINUSOID) return a.kc + a.kb * sin_phase(a.kx * x[0] + a.ky * x[1]);
  return a.kc;
}

template <int P, int SM>
__global__ __launch_bounds__((HexCfg<P, SM>::THREADS)) void hex_qp_kernel(HexArgs a)
{
  using C = HexCfg<P, SM>;
  constexpr int NP = C::NP, NB = C::NB, NT = C::NT, NQV = C::NQV, NQF = C::NQF;
  __shared__ HexLds1D t1;
  __shared__ double Gq[NQV][6];
  __shared__ double fq[3][NQF];
  __shared__ double buf[C::BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);

  if (tid == 0) {   // constant-index copies of the by-value kernel argument tables
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        t1.Lv[r][q] = a.tab.Lv[r][q]; t1.Dv[r][q] = a.tab.Dv[r][q];
        t1.Lf[r][q] = a.tab.Lf[r][q]; t1.Df[r][q] = a.tab.Df[r][q];
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) { t1.Le[r][q] = a.tab.Le[r][q]; t1.De[r][q] = a.tab.De[r][q]; }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      t1.sv[q] = a.tab.sv[q]; t1.wv[q] = a.tab.wv[q]; t1.sf[q] = a.tab.sf[q]; t1.wf[q] = a.tab.wf[q];
    }
  }

  const int64_t n_own = a.own_end - a.own_begin;
  for (int64_t k = blockIdx.x; k < n_own; k += gridDim.x) {
    const int64_t e = a.own_begin + k;
    ElemGeo G;
    elem_geo(a, e, G);
    double A[3][3];
    elem_tensor(a, e, A);
    int32_t nbr[6];
#pragma unroll
    for (int f = 0; f < 6; ++f) nbr[f] = a.nbrs[f * a.n_local + e];
    // block positions (columns sorted by element id) and row length
    int nblk = 1;
#pragma unroll
    for (int f = 0; f < 6; ++f) nblk += nbr[f] >= 0;
    const int64_t rl = int64_t(NB) * nblk;
    auto pos_of = [&](int64_t x) {
      int p = e < x;
#pragma unroll
      for (int f = 0; f < 6; ++f) p += (nbr[f] >= 0 && nbr[f] < x);
      return p;
    };
    double* out = a.vals + a.elem_ptr[k];

    __syncthreads();   // previous element finished with the LDS tables
    // G_q = w_q |det J| kappa(x_q) J^{-1} A J^{-T}
    if (tid < NQV) {
      const int q0 = tid % C::NV1, q1 = (tid / C::NV1) % C::NV1, q2 = tid / (C::NV1 * C::NV1);
      const double xh[3] = {t1.sv[q0], t1.sv[q1], t1.sv[q2]};
      double x[3];
      for (int d = 0; d < 3; ++d) x[d] = G.v0[d] + G.J[d][0] * xh[0] + G.J[d][1] * xh[1] + G.J[d][2] * xh[2];
      const double fac = t1.wv[q0] * t1.wv[q1] * t1.wv[q2] * fabs(G.det) * kappa_at(a, e, x);
      double JA[3][3];
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) JA[r][c] = G.Ji[r][0] * A[0][c] + G.Ji[r][1] * A[1][c] + G.Ji[r][2] * A[2][c];
      const int ab[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
      for (int m = 0; m < 6; ++m) {
        const int r = ab[m][0], c = ab[m][1];
        Gq[tid][m] = fac * (JA[r][0] * G.Ji[c][0] + JA[r][1] * G.Ji[c][1] + JA[r][2] * G.Ji[c][2]);
      }
    }
    dbl4 S[NT];
    for (int I = 0; I < NT; ++I) S[I] = dbl4{0.0, 0.0, 0.0, 0.0};

    // ---- volume: S = Dhat * R, K = 3 NQV in LDS chunks of KC k-steps ----
    for (int s0 = 0; s0 < C::KVS; s0 += C::KC) {
      const int ns = min(C::KC, C::KVS - s0);
      __syncthreads();
      double* AV = buf;
      double* BV = buf + C::CHUNK;
      for (int idx = tid; idx < ns * NT * 64; idx += C::THREADS) {
        const int s = idx / (NT * 64), T = (idx / 64) % NT, l = idx & 63;
        const int kk = 4 * (s0 + s) + (l >> 4);
        const int rc = T * 16 + (l & 15);
        double av = 0.0, bv = 0.0;
        if (kk < C::KV && rc < NB) {
          const int q = kk / 3, ax = kk % 3;
          const int q0 = q % C::NV1, q1 = (q / C::NV1) % C::NV1, q2 = q / (C::NV1 * C::NV1);
          av = dhat<NP>(t1, rc, ax, q0, q1, q2);
          const double g0 = dhat<NP>(t1, rc, 0, q0, q1, q2);
          const double g1 = dhat<NP>(t1, rc, 1, q0, q1, q2);
          const double g2 = dhat<NP>(t1, rc, 2, q0, q1, q2);
          const double* g = Gq[q];
          // row ax of the symmetric G: (00 01 02 / 11 12 / 22)
          const double ga = ax == 0 ? g[0] : (ax == 1 ? g[1] : g[2]);
          const double gb = ax == 0 ? g[1] : (ax == 1 ? g[3] : g[4]);
          const double gc = ax == 0 ? g[2] : (ax == 1 ? g[4] : g[5]);
          bv = ga * g0 + gb * g1 + gc * g2;
        }
        AV[idx] = av;   // A fragment: row rc, k = kk  (T = row tile)
        BV[idx] = bv;   // B fragment: k = kk, column rc (T = column tile)
      }
      __syncthreads();
      for (int s = 0; s < ns; ++s) {
        const double b = BV[(s * NT + w) * 64 + lane];
#pragma unroll
        for (int I = 0; I < NT; ++I) S[I] = mfma(AV[(s * NT + I) * 64 + lane], b, S[I]);
      }
    }

    // ---- faces (unrolled: face axis / side are compile-time constants) ----
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      const int32_t nf = nbr[f];
      if (nf == HDD_NBR_NEUMANN) continue;
      const bool inner = nf >= 0;
      const int af = f >> 1, sd = f & 1;
      // unit outer normal n = J^{-T} n_ref / |.|, face volume |det J| |J^{-T} n_ref| (Nanson)
      const double sg = sd ? 1.0 : -1.0;
      double n[3] = {sg * G.Ji[af][0], sg * G.Ji[af][1], sg * G.Ji[af][2]};
      const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
      n[0] /= nn; n[1] /= nn; n[2] /= nn;
      const double fvol = fabs(G.det) * nn;
      const double hpow = pow(fvol, a.beta);
      double An[3], cm[3];
      for (int r = 0; r < 3; ++r) An[r] = A[r][0] * n[0] + A[r][1] * n[1] + A[r][2] * n[2];
      for (int r = 0; r < 3; ++r) cm[r] = G.Ji[r][0] * An[0] + G.Ji[r][1] * An[1] + G.Ji[r][2] * An[2];
      const double dm = n[0] * An[0] + n[1] * An[1] + n[2] * An[2];
      double cp[3] = {0.0, 0.0, 0.0}, wm = 1.0, wp = 0.0, gam = dm, sig = a.sigma_boundary;
      if (inner) {
        ElemGeo Gn;
        elem_geo(a, nf, Gn);
        double Ao[3][3], Ano[3];
        elem_tensor(a, nf, Ao);
        for (int r = 0; r < 3; ++r) Ano[r] = Ao[r][0] * n[0] + Ao[r][1] * n[1] + Ao[r][2] * n[2];
        for (int r = 0; r < 3; ++r) cp[r] = Gn.Ji[r][0] * Ano[0] + Gn.Ji[r][1] * Ano[1] + Gn.Ji[r][2] * Ano[2];
        const double dp = n[0] * Ano[0] + n[1] * Ano[1] + n[2] * Ano[2];
        gam = dp * dm / (dp + dm);
        wp = dm / (dp + dm);
        wm = dp / (dp + dm);
        sig = a.sigma_inner;
      }
      __syncthreads();   // previous users of fq / buf are done
      if (tid < NQF) {
        const int qs = tid % C::NF1, qt = tid / C::NF1;
        const double ss = t1.sf[qs], st = t1.sf[qt];
        const double xh[3] = {af == 0 ? double(sd) : ss, af == 1 ? double(sd) : (af == 0 ? ss : st),
                              af == 2 ? double(sd) : st};
        double x[3];
        for (int d = 0; d < 3; ++d) x[d] = G.v0[d] + G.J[d][0] * xh[0] + G.J[d][1] * xh[1] + G.J[d][2] * xh[2];
        const double fac = t1.wf[qs] * t1.wf[qt] * fvol;
        const double ke = kappa_at(a, e, x);
        const double kn = inner ? kappa_at(a, nf, x) : 0.0;
        fq[0][tid] = fac * wm * ke;                                           // alpha
        fq[1][tid] = fac * wp * kn;                                           // beta
        fq[2][tid] = fac * sig * (inner ? ke * kn : ke) * gam / hpow;        // eta
      }
      __syncthreads();
      double* AF = buf;
      double* BE = buf + C::FACE;
      double* BN = buf + 2 * C::FACE;
      for (int idx = tid; idx < C::FACE; idx += C::THREADS) {
        const int s = idx / (NT * 64), T = (idx / 64) % NT, l = idx & 63;
        const int kk = 4 * s + (l >> 4);
        const int rc = T * 16 + (l & 15);
        double af_ = 0.0, be = 0.0, bn = 0.0;
        if (kk < C::KF && rc < NB) {
          const bool vpart = kk < NQF;
          const int q = vpart ? kk : kk - NQF;
          const int qs = q % C::NF1, qt = q / C::NF1;
          double vm, gm0, gm1, gm2;
          face_eval<NP>(t1, rc, af, sd, qs, qt, vm, gm0, gm1, gm2);
          const double Nm = cm[0] * gm0 + cm[1] * gm1 + cm[2] * gm2;
          const double al = fq[0][q], be_ = fq[1][q], et = fq[2][q];
          af_ = vpart ? vm : Nm;
          be = vpart ? et * vm - al * Nm : -al * vm;
          if (inner) {
            double vp, gp0, gp1, gp2;
            face_eval<NP>(t1, rc, af, 1 - sd, qs, qt, vp, gp0, gp1, gp2);
            const double Np = cp[0] * gp0 + cp[1] * gp1 + cp[2] * gp2;
            bn = vpart ? -be_ * Np - et * vp : al * vp;
          }
        }
        AF[idx] = af_;
        BE[idx] = be;
        BN[idx] = bn;
      }
      __syncthreads();
      dbl4 E[NT];
      for (int I = 0; I < NT; ++I) E[I] = dbl4{0.0, 0.0, 0.0, 0.0};
      for (int s = 0; s < C::KFS; ++s) {
        const double be = BE[(s * NT + w) * 64 + lane];
#pragma unroll
        for (int I = 0; I < NT; ++I) S[I] = mfma(AF[(s * NT + I) * 64 + lane], be, S[I]);
      }
      if (inner) {
        for (int s = 0; s < C::KFS; ++s) {
          const double bn = BN[(s * NT + w) * 64 + lane];
#pragma unroll
          for (int I = 0; I < NT; ++I) E[I] = mfma(AF[(s * NT + I) * 64 + lane], bn, E[I]);
        }
        const int64_t cofs = int64_t(pos_of(nf)) * NB;
        const int col = w * 16 + (lane & 15);
#pragma unroll
        for (int I = 0; I < NT; ++I)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = I * 16 + (lane >> 4) + 4 * r;
            if (row < NB && col < NB) out[row * rl + cofs + col] = E[I][r];
          }
      }
    }
    const int64_t sofs = int64_t(pos_of(e)) * NB;
    const int col = w * 16 + (lane & 15);
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = I * 16 + (lane >> 4) + 4 * r;
        if (row < NB && col < NB) out[row * rl + sofs + col] = S[I][r];
      }
  }
}

// ---------------------------------------------------------------------------------------------------
// p = 3, reference integrand orders, piecewise-constant kappa (the C5 configuration): register-only
// fragment generation.  With lane l = 16 g + r, r = i0 + 4 i1 and row tile I = i2, every MFMA operand value
// is (per-lane factor) x (wave-uniform factor): the lane group g carries one quadrature coordinate
// (q0 in the volume, qs on faces) and the k-step the others (compile-time after unrolling).  No LDS
// tables, no barriers in the element loop; each wave (column tile w) is independent.
//   volume K: k-step s = (a, q1, q2) (27 steps, g = q0 with q0 = 3 a zero-weight pad), faces K: 8 steps,
//   s < 4: [V] with qt = s, s >= 4: [N] with qt = s - 4 (qs = g).
// ---------------------------------------------------------------------------------------------------
// value and (c . reference gradient) of the basis function with lane indices (i0, i1) and third index
// T (factors lT*, uniform) at the face point (qs = g, qt) of a face with axis AF, side value table column
template <int AF>
__device__ __forceinline__ void q3_face_eval(double Le0, double De0, double Le1, double De1,   // [i0][sd], [i1][sd]
                                             double Lfg0, double Dfg0, double Lfg1, double Dfg1, // [i0][g], [i1][g]
                                             double Lf1q, double Df1q,                         // [i1][qt]
                                             double lTf, double dTf, double lTe, double dTe,   // [T][qt], [T][sd]
                                             double c0, double c1, double c2, double& V, double& N)
{
  if (AF == 0) {          // x face: x <-> i0 (side), y <-> i1 (qs), z <-> T (qt)
    const double b = Le0 * Lfg1;
    V = b * lTf;
    N = (c0 * De0 * Lfg1 + c1 * Le0 * Dfg1) * lTf + c2 * b * dTf;
  } else if (AF == 1) {   // y face: x <-> i0 (qs), y <-> i1 (side), z <-> T (qt)
    const double b = Lfg0 * Le1;
    V = b * lTf;
    N = (c0 * Dfg0 * Le1 + c1 * Lfg0 * De1) * lTf + c2 * b * dTf;
  } else {                // z face: x <-> i0 (qs), y <-> i1 (qt), z <-> T (side)
    const double b = Lfg0 * Lf1q;
    V = b * lTe;
    N = (c0 * Dfg0 * Lf1q + c1 * Lfg0 * Df1q) * lTe + c2 * b * dTe;
  }
}

// Per-element coefficient record (HEX_REC doubles), written by hex_q3_setup_kernel (one thread per
// element: geometry, neighbour geometry, normals, |F|^beta, weights, penalties, block positions) and read
// by hex_q3_kernel with scalar loads, so the MFMA waves carry no dependent global-load chains:
//   [0] value offset of the element's row block (int64)   [1] nblk (lo 32) | position of the self block (hi 32)
//   [2..7] M = |det J| kappa J^{-1} A J^{-T} (xx xy xz yy yz zz)
//   [8 + 10 f + 0..8] face f: cm[3] = J^{-1} A^- n, cp[3] = J^{-1}_+ A^+ n, ca, cb, ce (alpha / beta / eta
//   without the quadrature weight);  [8 + 10 f + 9]: kind (lo 32: -2 Neumann, -1 Dirichlet, 1 inner) | block position (hi 32)
__device__ __forceinline__ double i2d(int64_t v) { return __longlong_as_double(v); }
__device__ __forceinline__ int64_t d2i(double v) { return __double_as_longlong(v); }

__global__ __launch_bounds__(256) void hex_q3_setup_kernel(HexArgs a)
{
  const int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  const int64_t n_own = a.own_end - a.own_begin;
  if (k >= n_own) return;
  const int64_t e = a.own_begin + k;
  double* R = a.ws + k * HEX_REC;
  ElemGeo G;
  elem_geo(a, e, G);
  double A[3][3];
  elem_tensor(a, e, A);
  const double ke = a.kkind == HDD_FN_PER_ELEM ? a.kper[e] : a.kc;
  int32_t nbr[6];
#pragma unroll
  for (int f = 0; f < 6; ++f) nbr[f] = a.nbrs[f * a.n_local + e];
  int nblk = 1;
#pragma unroll
  for (int f = 0; f < 6; ++f) nblk += nbr[f] >= 0;
  auto pos_of = [&](int64_t x) {
    int p = e < x;
#pragma unroll
    for (int f = 0; f < 6; ++f) p += (nbr[f] >= 0 && nbr[f] < x);
    return p;
  };
  R[0] = i2d(a.elem_ptr[k]);
  R[1] = i2d(int64_t(uint32_t(nblk)) | (int64_t(pos_of(e)) << 32));
  {
    double JA[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) JA[i][j] = G.Ji[i][0] * A[0][j] + G.Ji[i][1] * A[1][j] + G.Ji[i][2] * A[2][j];
    const double gf = fabs(G.det) * ke;
    const int ij[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
#pragma unroll
    for (int m = 0; m < 6; ++m) {
      const int i = ij[m][0], j = ij[m][1];
      R[2 + m] = gf * (JA[i][0] * G.Ji[j][0] + JA[i][1] * G.Ji[j][1] + JA[i][2] * G.Ji[j][2]);
    }
  }
#pragma unroll
  for (int f = 0; f < 6; ++f) {
    double* F = R + 8 + 10 * f;
    const int32_t nf = nbr[f];
    const int af = f >> 1, sd = f & 1;
    const bool inner = nf >= 0;
    const double sg = sd ? 1.0 : -1.0;
    double n[3] = {sg * G.Ji[af][0], sg * G.Ji[af][1], sg * G.Ji[af][2]};
    const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    n[0] /= nn; n[1] /= nn; n[2] /= nn;
    const double fvol = fabs(G.det) * nn;
    const double hpow = pow(fvol, a.beta);
    double An[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) An[i] = A[i][0] * n[0] + A[i][1] * n[1] + A[i][2] * n[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) F[i] = G.Ji[i][0] * An[0] + G.Ji[i][1] * An[1] + G.Ji[i][2] * An[2];
    const double dm = n[0] * An[0] + n[1] * An[1] + n[2] * An[2];
    double cp[3] = {0.0, 0.0, 0.0}, wm = 1.0, wp = 0.0, gam = dm, sig = a.sigma_boundary, kn = 0.0;
    if (inner) {
      ElemGeo Gn;
      elem_geo(a, nf, Gn);
      double Ao[3][3], Ano[3];
      elem_tensor(a, nf, Ao);
#pragma unroll
      for (int i = 0; i < 3; ++i) Ano[i] = Ao[i][0] * n[0] + Ao[i][1] * n[1] + Ao[i][2] * n[2];
#pragma unroll
      for (int i = 0; i < 3; ++i) cp[i] = Gn.Ji[i][0] * Ano[0] + Gn.Ji[i][1] * Ano[1] + Gn.Ji[i][2] * Ano[2];
      const double dp = n[0] * Ano[0] + n[1] * Ano[1] + n[2] * Ano[2];
      gam = dp * dm / (dp + dm);
      wp = dm / (dp + dm);
      wm = dp / (dp + dm);
      sig = a.sigma_inner;
      kn = a.kkind == HDD_FN_PER_ELEM ? a.kper[nf] : a.kc;
    }
    F[3] = cp[0]; F[4] = cp[1]; F[5] = cp[2];
    F[6] = fvol * wm * ke;
    F[7] = fvol * wp * kn;
    F[8] = fvol * sig * (inner ? ke * kn : ke) * gam / hpow;
    const int32_t kind = inner ? 1 : nf;
    F[9] = i2d(int64_t(uint32_t(kind)) | (int64_t(inner ? pos_of(nf) : 0) << 32));
  }
}

typedef const double __attribute__((address_space(4)))* cdptr;   // constant AS: uniform loads -> s_load
typedef int32_t i32x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void hex_q3_kernel(HexArgs a)
{
  constexpr int NB = 64, XLD = 17;   // per-wave transpose buffer: 64 rows x 16 columns, padded rows
  __shared__ HexTables T;
  __shared__ double XT[4][NB * XLD];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  {   // flat parallel copy of the by-value tables
    const double* src = &a.tab.sv[0];
    double* dst = &T.sv[0];
    for (int i = tid; i < int(sizeof(HexTables) / sizeof(double)); i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const int r = lane & 15, g = lane >> 4, i0 = r & 3, i1 = r >> 2;
  // per-lane volume factors (q0 = g; g = 3 is a zero-weight pad)
  const bool gv = g < 3;
  const int gq = gv ? g : 0;
  const double Lv0g = gv ? T.Lv[i0][gq] : 0.0, Dv0g = gv ? T.Dv[i0][gq] : 0.0, wvg = gv ? T.wv[gq] : 0.0;
  double P01[3][3];
#pragma unroll
  for (int q1 = 0; q1 < 3; ++q1) {
    P01[0][q1] = Dv0g * T.Lv[i1][q1];
    P01[1][q1] = Lv0g * T.Dv[i1][q1];
    P01[2][q1] = Lv0g * T.Lv[i1][q1];
  }
  // per-lane face factors
  const double Lfg0 = T.Lf[i0][g], Dfg0 = T.Df[i0][g], Lfg1 = T.Lf[i1][g], Dfg1 = T.Df[i1][g], wfg = T.wf[g];
  const double Le0[2] = {T.Le[i0][0], T.Le[i0][1]}, De0[2] = {T.De[i0][0], T.De[i0][1]};
  const double Le1[2] = {T.Le[i1][0], T.Le[i1][1]}, De1[2] = {T.De[i1][0], T.De[i1][1]};

  const int64_t n_own = a.own_end - a.own_begin;
  for (int64_t k = blockIdx.x; k < n_own; k += gridDim.x) {
    // column tile of this wave, rotated per element: the z-face skips below then even out over the SIMDs
    const int wc = (w + int(k)) & 3;
    const double LeW[2] = {T.Le[wc][0], T.Le[wc][1]}, DeW[2] = {T.De[wc][0], T.De[wc][1]};
    const int col = wc * 16 + r;
    const cdptr R = (cdptr)(a.ws + k * HEX_REC);
    double* out = a.vals + d2i(R[0]);
    const int64_t hdr = d2i(R[1]);
    const int64_t rl = int64_t(NB) * int32_t(hdr & 0xffffffff);
    const int64_t sofs = (hdr >> 32) * NB;
    // the element's row block (<= 7 x 64 x 64 doubles = 229 KB) as one buffer: per-lane part of a store
    // address in voffset, the wave-uniform row / block part in soffset (no 64-bit VALU address math)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, int(rl * NB * 8), 0x00020000);
    const int rli = int(rl);
    const double M[3][3] = {{R[2], R[3], R[4]}, {R[3], R[5], R[6]}, {R[4], R[6], R[7]}};

    dbl4 S[4];
#pragma unroll
    for (int I = 0; I < 4; ++I) S[I] = dbl4{0.0, 0.0, 0.0, 0.0};

    // ---- faces, rows rotated to the face normal ----
    // A-operand rows of a face with normal axis n run in the layout (row tile = basis index along n, lane
    // r & 3 / r >> 2 = the basis indices along the face's qs / qt axes): the [V] rows (nonzero trace) then
    // sit on row tile 3 sd for every face, so the [V] part takes one MFMA per k-step instead of four.
    // Columns stay natural (coalesced 128-byte row stores).  S follows the faces' layouts: x faces ->
    // (LDS transpose, per wave) natural -> (register transpose, same lane) y layout -> y faces -> natural
    // -> volume and z faces.  x layout: row n = I + 4 g + 16 rr; y layout: n = g + 4 I + 16 rr.
    double* xt = XT[w];
    auto reg_transpose = [&]() __attribute__((always_inline)) {   // (tile, comp) -> (comp, tile), same lane
      dbl4 Tm[4];
#pragma unroll
      for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) Tm[rr][I] = S[I][rr];
#pragma unroll
      for (int I = 0; I < 4; ++I) S[I] = Tm[I];
    };
#pragma unroll 1
    for (int f = 0; f < 6; ++f) {
      if (f == 2) {   // x layout -> natural (cross-lane: via this wave's LDS buffer) -> y layout
#pragma unroll
        for (int I = 0; I < 4; ++I)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) xt[(I + 4 * g + 16 * rr) * XLD + r] = S[I][rr];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int I = 0; I < 4; ++I)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) S[I][rr] = xt[(16 * I + g + 4 * rr) * XLD + r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        reg_transpose();   // natural (tile i2, comp i1) -> y layout (tile i1, comp i2)
      }
      if (f == 4) {
        reg_transpose();   // y layout -> natural
        // ---- volume (natural layout) ----
#pragma unroll 1
        for (int q2 = 0; q2 < 3; ++q2) {
          const double lw = T.Lv[wc][q2], dw = T.Dv[wc][q2];
          const double lI[4] = {T.Lv[0][q2], T.Lv[1][q2], T.Lv[2][q2], T.Lv[3][q2]};
          const double dI[4] = {T.Dv[0][q2], T.Dv[1][q2], T.Dv[2][q2], T.Dv[3][q2]};
          const double w2 = T.wv[q2];
#pragma unroll
          for (int q1 = 0; q1 < 3; ++q1) {
            const double wq = wvg * T.wv[q1] * w2;
            const double D0 = P01[0][q1] * lw, D1 = P01[1][q1] * lw, D2 = P01[2][q1] * dw;
#pragma unroll
            for (int ax = 0; ax < 3; ++ax) {
              const double b = wq * (M[ax][0] * D0 + M[ax][1] * D1 + M[ax][2] * D2);
#pragma unroll
              for (int I = 0; I < 4; ++I) S[I] = mfma(P01[ax][q1] * (ax == 2 ? dI[I] : lI[I]), b, S[I]);
            }
          }
        }
      }
      const cdptr F = R + 8 + 10 * f;
      const int64_t fk = d2i(F[9]);
      const int kind = int32_t(fk & 0xffffffff);
      if (kind == HDD_NBR_NEUMANN) continue;
      const bool inner = kind > 0;
      const int af = f >> 1, sd = f & 1;
      const double cm[3] = {F[0], F[1], F[2]}, cp[3] = {F[3], F[4], F[5]};
      // coefficients of the rotated row operands: (qs axis, qt axis, normal)
      const double cr0 = af == 1 ? cm[0] : (af == 0 ? cm[1] : cm[0]);
      const double cr1 = af == 2 ? cm[1] : cm[2];
      const double cr2 = cm[af];
      const double ca = F[6], cb = F[7], ce = F[8];
      const double Le0o = sd ? Le0[1] : Le0[0], De0o = sd ? De0[1] : De0[0];
      const double Le1o = sd ? Le1[1] : Le1[0], De1o = sd ? De1[1] : De1[0];
      const double Le0n = sd ? Le0[0] : Le0[1], De0n = sd ? De0[0] : De0[1];
      const double Le1n = sd ? Le1[0] : Le1[1], De1n = sd ? De1[0] : De1[1];
      const double LeWo = sd ? LeW[1] : LeW[0], DeWo = sd ? DeW[1] : DeW[0];
      const double LeWn = sd ? LeW[0] : LeW[1], DeWn = sd ? DeW[0] : DeW[1];
      dbl4 E[4];
#pragma unroll
      for (int I = 0; I < 4; ++I) E[I] = dbl4{0.0, 0.0, 0.0, 0.0};
      // one face point row qt per iteration: k-step qt ([V] part) and k-step 4 + qt ([N] part) share every
      // basis evaluation
      // face side and inner / boundary are template parameters: no runtime branch around an accumulator
      // inside the face-point loop (such branches made the compiler route MFMA results through copies)
      auto face_steps = [&](auto afc, auto sdc, auto inc, auto dsc, auto dec) __attribute__((always_inline)) {
        constexpr int AF = decltype(afc)::value, SD = decltype(sdc)::value;
        constexpr bool IN = decltype(inc)::value, DS = decltype(dsc)::value, DE = decltype(dec)::value;
#pragma unroll   // (full unroll: 1.5 % over a rolled loop, profiles/r01/s2/c5/ab_qt_unroll.log)
        for (int qt = 0; qt < 4; ++qt) {
          const double wq = wfg * T.wf[qt];
          const double al = ca * wq, be = cb * wq, et = ce * wq;
          const double lf1 = T.Lf[i1][qt], df1 = T.Df[i1][qt];
          const double lfw = T.Lf[wc][qt], dfw = T.Df[wc][qt];
          double Vo, No, Vn = 0.0, Nn = 0.0;
          q3_face_eval<AF>(Le0o, De0o, Le1o, De1o, Lfg0, Dfg0, Lfg1, Dfg1, lf1, df1, lfw, dfw, LeWo, DeWo, cm[0],
                           cm[1], cm[2], Vo, No);
          if constexpr (IN)
            q3_face_eval<AF>(Le0n, De0n, Le1n, De1n, Lfg0, Dfg0, Lfg1, Dfg1, lf1, df1, lfw, dfw, LeWn, DeWn, cp[0],
                             cp[1], cp[2], Vn, Nn);
          const double bEv = et * Vo - al * No, bNv = -be * Nn - et * Vn;   // [V] rows of K
          const double bEn = -al * Vo, bNn = al * Vn;                       // [N] rows of K
          double Va[4], Na[4];   // rotated rows: tile I = normal index, lane (r & 3, r >> 2) = (qs, qt) axes
#pragma unroll
          for (int I = 0; I < 4; ++I)
            q3_face_eval<2>(0.0, 0.0, 0.0, 0.0, Lfg0, Dfg0, Lfg1, Dfg1, lf1, df1, 0.0, 0.0, T.Le[I][SD], T.De[I][SD],
                            cr0, cr1, cr2, Va[I], Na[I]);
          // [V] rows live on row tile 3 SD
          S[3 * SD] = mfma(Va[3 * SD], bEv, S[3 * SD]);
          if constexpr (IN) E[3 * SD] = mfma(Va[3 * SD], bNv, E[3 * SD]);
          // [N] rows of K: B = -alpha V- / alpha V+ at the columns; on z faces V vanishes off the face plane,
          // i.e. outside column tile 3 SD (own side) / 3 (1 - SD) (neighbour side): DS / DE false
          if constexpr (DS) {
#pragma unroll
            for (int I = 0; I < 4; ++I) S[I] = mfma(Na[I], bEn, S[I]);
          }
          if constexpr (IN && DE) {
#pragma unroll
            for (int I = 0; I < 4; ++I) E[I] = mfma(Na[I], bNn, E[I]);
          }
        }
      };
      // face kind -> compile-time loop variant (20 of them): side, inner / boundary, and on z faces
      // whether this wave's column tile meets the own / neighbour [N] part at all
      using BT = std::true_type;
      using BF = std::false_type;
      auto with_de = [&](auto afc, auto sdc, auto inc, auto dsc) __attribute__((always_inline)) {
        constexpr int AF = decltype(afc)::value, SD = decltype(sdc)::value;
        if (AF != 2 || wc == 3 * (1 - SD)) face_steps(afc, sdc, inc, dsc, BT{});
        else face_steps(afc, sdc, inc, dsc, BF{});
      };
      auto with_ds = [&](auto afc, auto sdc, auto inc) __attribute__((always_inline)) {
        constexpr int AF = decltype(afc)::value, SD = decltype(sdc)::value;
        constexpr bool IN = decltype(inc)::value;
        if constexpr (IN) {
          if (AF != 2 || wc == 3 * SD) with_de(afc, sdc, inc, BT{});
          else with_de(afc, sdc, inc, BF{});
        } else {
          if (AF != 2 || wc == 3 * SD) face_steps(afc, sdc, inc, BT{}, BF{});
          else face_steps(afc, sdc, inc, BF{}, BF{});
        }
      };
      auto by_kind = [&](auto afc) __attribute__((always_inline)) {
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        if (sd) {
          if (inner) with_ds(afc, I1{}, BT{});
          else with_ds(afc, I1{}, BF{});
        } else {
          if (inner) with_ds(afc, I0{}, BT{});
          else with_ds(afc, I0{}, BF{});
        }
      };
      if (af == 0) by_kind(std::integral_constant<int, 0>{});
      else if (af == 1) by_kind(std::integral_constant<int, 1>{});
      else by_kind(std::integral_constant<int, 2>{});
      if (inner) {
        const int64_t cofs = (fk >> 32) * NB;
        const int vo = ((af == 0 ? 4 * g : g) * rli + col) * 8;
#pragma unroll
        for (int I = 0; I < 4; ++I)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int urow = af == 0 ? I + 16 * rr : (af == 1 ? 4 * I + 16 * rr : 16 * I + 4 * rr);
            const double v = E[I][rr];   // (bit_cast of a vector element directly reads element 0)
            if (!HDD_HEX_ABL(a, 2))
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(i32x2, v), rs, vo,
                                                    (urow * rli + int(cofs)) * 8, 2);
          }
      }
    }
    const int vs = (g * rli + col) * 8;
#pragma unroll
    for (int I = 0; I < 4; ++I)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const double v = S[I][rr];
        if (!HDD_HEX_ABL(a, 2))
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(i32x2, v), rs, vs,
                                                ((I * 16 + 4 * rr) * rli + int(sofs)) * 8, 2);
      }
  }
}

// ---------------------------------------------------------------------------------------------------
// p = 3, piecewise-constant data: the local matrices as a dense GEMM over reference matrices.
//
// With kappa and A constant on an affine hexahedron, every integrand is a coefficient (element data) times a
// product of 1D factors, and the reference's tensor Gauss rules factorise the same way, so each block is a
// linear combination of element-independent 64 x 64 reference matrices (sums over the SAME quadrature
// points the reference uses: 3^3 volume, 4^2 face points):
//   self block  S = sum_ab M_ab V_ab                                (M = |det J| kappa J^-1 A J^-T, 6 terms)
//                 + sum_f [ ce_f I_V^f - ca_f sum_a cm_f,a (I_N^{f,a} + I_N^{f,a}^T) ]   (4 terms per face)
//   face block  E_f = -ce_f J_V^f - cb_f sum_a cp_f,a J_N^{f,a} + ca_f sum_a cm_f,a J_N'^{f,a}   (7 terms)
// (cm = J^-1 A^- n, cp = J_+^-1 A^+ n, ca / cb / ce = |F| omega^- kappa^- / |F| omega^+ kappa^+ / the
// penalty, as in the p=3 records; V_ab, I_V, I_N, J_V, J_N, J_N' = Kronecker products of the 1D Gauss sums
// of L L, L' L', L L', L' L and the trace values L(0|1), L'(0|1)).  So, for 16 elements at once,
//   [16 elements x 32 terms] x [32 terms x 4096 entries]  (self)    [16 x 8] x [8 x 4096] per face block,
// a dense f64 GEMM on v_mfma_f64_16x16x4_f64 with the reference matrices as the B operand.  A wave owns one
// matrix row i: its B fragments (row i of every reference matrix, 80 values per lane) stay in registers for
// the whole launch; it walks 16-element groups, reading each group's coefficient fragments (A) and writing
// row i of the 7 blocks of its 16 elements (16 lanes = 128 contiguous bytes per element row).  320 MFMAs per
// element instead of 1200, no operand generation on the VALU: the kernel is bound by the 229 KB per
// element of value stores.  XCD-aware: the 64 row waves of a group run on one XCD (its L2 holds the
// group's coefficients).
// ---------------------------------------------------------------------------------------------------
size_t hex_q3_workspace_doubles(int64_t n_own)
{
  const int64_t groups = (n_own + 15) / 16;
  return size_t(n_own) * HEX_REC + size_t(groups) * 16 * Q3G_K + size_t(n_own) * 2;
}

void hex_q3g_reference_tables(const HexTables& t, double* out)
{
  const int nv = 3, nf = 4;   // the reference's Gauss points per direction at p = 3 (orders 4 and 6)
  double Mm[4][4], Dd[4][4], Ca[4][4], Cb[4][4], Mf[4][4], Cfa[4][4], Cfb[4][4];
  for (int x = 0; x < 4; ++x)
    for (int y = 0; y < 4; ++y) {
      Mm[x][y] = Dd[x][y] = Ca[x][y] = Cb[x][y] = Mf[x][y] = Cfa[x][y] = Cfb[x][y] = 0.0;
      for (int q = 0; q < nv; ++q) {
        Mm[x][y] += t.wv[q] * t.Lv[x][q] * t.Lv[y][q];
        Dd[x][y] += t.wv[q] * t.Dv[x][q] * t.Dv[y][q];
        Ca[x][y] += t.wv[q] * t.Lv[x][q] * t.Dv[y][q];   // derivative on the ansatz function
        Cb[x][y] += t.wv[q] * t.Dv[x][q] * t.Lv[y][q];   // derivative on the test function
      }
      for (int q = 0; q < nf; ++q) {
        Mf[x][y] += t.wf[q] * t.Lf[x][q] * t.Lf[y][q];
        Cfa[x][y] += t.wf[q] * t.Lf[x][q] * t.Df[y][q];
        Cfb[x][y] += t.wf[q] * t.Df[x][q] * t.Lf[y][q];
      }
    }
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      const int ii[3] = {i & 3, (i >> 2) & 3, i >> 4}, jj[3] = {j & 3, (j >> 2) & 3, j >> 4};
      auto T = [&](int k) -> double& { return out[size_t(k) * 4096 + size_t(i) * 64 + j]; };
      auto mm = [&](int d) { return Mm[ii[d]][jj[d]]; };
      auto ca = [&](int d) { return Ca[ii[d]][jj[d]]; };
      auto cb = [&](int d) { return Cb[ii[d]][jj[d]]; };
      T(0) = Dd[ii[0]][jj[0]] * mm(1) * mm(2);
      T(1) = mm(0) * Dd[ii[1]][jj[1]] * mm(2);
      T(2) = mm(0) * mm(1) * Dd[ii[2]][jj[2]];
      T(3) = (cb(0) * ca(1) + ca(0) * cb(1)) * mm(2);
      T(4) = (cb(0) * ca(2) + ca(0) * cb(2)) * mm(1);
      T(5) = mm(0) * (cb(1) * ca(2) + ca(1) * cb(2));
      for (int f = 0; f < 6; ++f) {
        const int af = f >> 1, sd = f & 1;
        const int t1 = af == 0 ? 1 : 0, t2 = af == 2 ? 1 : 2;
        auto mf = [&](int d) { return Mf[ii[d]][jj[d]]; };
        const double mt = mf(t1) * mf(t2);
        // trace factors on my side (sd) and on the neighbour's (1 - sd)
        const double Lti = t.Le[ii[af]][sd], Ltj = t.Le[jj[af]][sd], Dti = t.De[ii[af]][sd];
        const double Lnj = t.Le[jj[af]][1 - sd], Dnj = t.De[jj[af]][1 - sd];
        // I_N^{f,a}(x, y) = sum phi_x d_a phi_y over the face (x, y basis indices)
        auto IN = [&](int a, const int* xi, const int* yi) {
          const double Lx = t.Le[xi[af]][sd], Ly = t.Le[yi[af]][sd], Dy = t.De[yi[af]][sd];
          if (a == af) return Lx * Dy * Mf[xi[t1]][yi[t1]] * Mf[xi[t2]][yi[t2]];
          const int o = a == t1 ? t2 : t1;
          return Lx * Ly * Cfa[xi[a]][yi[a]] * Mf[xi[o]][yi[o]];
        };
        T(6 + 4 * f) = Lti * Ltj * mt;
        for (int a = 0; a < 3; ++a) T(7 + 4 * f + a) = IN(a, ii, jj) + IN(a, jj, ii);
        const int kb = 32 + 8 * f;
        T(kb) = Lti * Lnj * mt;
        for (int a = 0; a < 3; ++a) {
          if (a == af) {
            T(kb + 1 + a) = Lti * Dnj * mt;
            T(kb + 4 + a) = Dti * Lnj * mt;
          } else {
            const int o = a == t1 ? t2 : t1;
            T(kb + 1 + a) = Lti * Lnj * Cfa[ii[a]][jj[a]] * mf(o);
            T(kb + 4 + a) = Lti * Lnj * Cfb[ii[a]][jj[a]] * mf(o);
          }
        }
        T(kb + 7) = 0.0;
      }
      T(30) = T(31) = 0.0;
    }
}

// element records -> the GEMM's coefficient fragments [group][term][16] and row-block layout per element
__global__ __launch_bounds__(256) void hex_q3g_coef_kernel(HexArgs a, int64_t n_groups)
{
  const int64_t n_own = a.own_end - a.own_begin;
  const int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;   // element slot (groups padded to 16)
  if (k >= n_groups * 16) return;
  double* C = a.q3g_coef + (k >> 4) * (Q3G_K * 16) + (k & 15);
  auto put = [&](int t, double v) { C[t * 16] = v; };
  if (k >= n_own) {
    for (int t = 0; t < Q3G_K; ++t) put(t, 0.0);
    return;
  }
  const double* R = a.ws + k * HEX_REC;
  put(0, R[2]); put(1, R[5]); put(2, R[7]); put(3, R[3]); put(4, R[4]); put(5, R[6]);   // M00 M11 M22 M01 M02 M12
  put(30, 0.0); put(31, 0.0);
  const int64_t hdr = d2i(R[1]);
  uint64_t info = uint64_t(hdr & 0xff) | (uint64_t((hdr >> 32) & 0xff) << 8);   // nblk | self position
#pragma unroll
  for (int f = 0; f < 6; ++f) {
    const double* F = R + 8 + 10 * f;
    const int64_t fk = d2i(F[9]);
    const int kind = int32_t(fk & 0xffffffff);
    const bool inner = kind > 0, neu = kind == HDD_NBR_NEUMANN;
    const double ca = F[6], cb = F[7], ce = F[8];
    put(6 + 4 * f, neu ? 0.0 : ce);
    for (int d = 0; d < 3; ++d) put(7 + 4 * f + d, neu ? 0.0 : -ca * F[d]);
    const int kb = 32 + 8 * f;
    put(kb, inner ? -ce : 0.0);
    for (int d = 0; d < 3; ++d) {
      put(kb + 1 + d, inner ? -cb * F[3 + d] : 0.0);
      put(kb + 4 + d, inner ? ca * F[d] : 0.0);
    }
    put(kb + 7, 0.0);
    info |= uint64_t(inner ? ((fk >> 32) & 0xff) : 0xff) << (16 + 8 * f);
  }
  a.q3g_meta[2 * k] = d2i(R[0]);
  a.q3g_meta[2 * k + 1] = int64_t(info);
}

__global__ __launch_bounds__(256) void hex_q3g_kernel(HexArgs a, int64_t n_groups)
{
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x;
  const int x = b & 7, kq = b >> 3, rq = kq & 15, rep = kq >> 4;   // XCD, row quad, replica
  const int row = rq * 4 + wv;                                       // matrix row i of every block
  const int kl = lane >> 4, cl = lane & 15;
  const int64_t n_own = a.own_end - a.own_begin;
  // B fragments: row `row` of every reference matrix (k = 4 kk + kl, entry = 64 row + 16 tc + cl)
  double bS[8][4], bE[6][2][4];
  {
    const double* T = a.q3g_tab + row * 64 + cl;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
      for (int tc = 0; tc < 4; ++tc) bS[kk][tc] = T[(4 * kk + kl) * 4096 + 16 * tc];
#pragma unroll
    for (int f = 0; f < 6; ++f)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int tc = 0; tc < 4; ++tc) bE[f][kk][tc] = T[(32 + 8 * f + 4 * kk + kl) * 4096 + 16 * tc];
  }
  double* const vals = a.vals;
  for (int64_t g = x + 8 * int64_t(rep); g < n_groups; g += 8 * int64_t(a.q3g_reps)) {
    const double* C = a.q3g_coef + g * (Q3G_K * 16) + cl;   // A fragments: element cl, term 4 kk + kl
    double aS[8], aE[6][2];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) aS[kk] = C[(4 * kk + kl) * 16];
#pragma unroll
    for (int f = 0; f < 6; ++f)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) aE[f][kk] = C[(32 + 8 * f + 4 * kk + kl) * 16];
    // the 4 output elements of this lane: D register r holds element kl + 4 r, entry 16 tc + cl
    double* rowp[4];
    uint64_t info[4];
    bool ok[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t k = g * 16 + kl + 4 * r;
      ok[r] = k < n_own;
      const int64_t kk = ok[r] ? k : 0;
      const int64_t off = a.q3g_meta[2 * kk];
      info[r] = uint64_t(a.q3g_meta[2 * kk + 1]);
      rowp[r] = vals + off + int64_t(row) * 64 * int64_t(info[r] & 0xff) + cl;
    }
    // self block
    dbl4 acc[4];
#pragma unroll
    for (int tc = 0; tc < 4; ++tc) acc[tc] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
      for (int tc = 0; tc < 4; ++tc) acc[tc] = mfma(aS[kk], bS[kk][tc], acc[tc]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pos = int((info[r] >> 8) & 0xff);
      if (ok[r]) {
#pragma unroll
        for (int tc = 0; tc < 4; ++tc) __builtin_nontemporal_store(acc[tc][r], rowp[r] + pos * 64 + 16 * tc);
      }
    }
    // face blocks
#pragma unroll
    for (int f = 0; f < 6; ++f) {
#pragma unroll
      for (int tc = 0; tc < 4; ++tc) {
        acc[tc] = mfma(aE[f][0], bE[f][0][tc], dbl4{0.0, 0.0, 0.0, 0.0});
        acc[tc] = mfma(aE[f][1], bE[f][1][tc], acc[tc]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pos = int((info[r] >> (16 + 8 * f)) & 0xff);
        if (ok[r] && pos != 0xff) {
#pragma unroll
          for (int tc = 0; tc < 4; ++tc) __builtin_nontemporal_store(acc[tc][r], rowp[r] + pos * 64 + 16 * tc);
        }
      }
    }
  }
}

static hipError_t launch_hex_q3(const HexArgs& a, hipStream_t s)
{
  const int64_t n_own = a.own_end - a.own_begin;
  if (n_own <= 0) return hipSuccess;
  hipLaunchKernelGGL(hex_q3_setup_kernel, dim3(unsigned((n_own + 255) / 256)), dim3(256), 0, s, a);
  if (a.variant & HDD_VARIANT_HEX_Q3_REGISTER) {   // the register-fragment MFMA kernel (operands generated per element)
    const int64_t grid = std::min<int64_t>(n_own, 1 << 20);
    hdd::last_tile_kernel_slot() = "hex_q3_kernel";
    hipLaunchKernelGGL(hex_q3_kernel, dim3(unsigned(grid)), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  hdd::last_tile_kernel_slot() = "hex_q3g_kernel";
  const int64_t n_groups = (n_own + 15) / 16;
  hipLaunchKernelGGL(hex_q3g_coef_kernel, dim3(unsigned((n_groups * 16 + 255) / 256)), dim3(256), 0, s, a, n_groups);
  // 16 row quads x 8 XCDs x reps workgroups of 4 row waves
  hipLaunchKernelGGL(hex_q3g_kernel, dim3(unsigned(128 * a.q3g_reps)), dim3(256), 0, s, a, n_groups);
  return hipGetLastError();
}

static bool hex_generic_forced()
{
#ifdef HDD_ABLATION
  static const bool generic = getenv("HDD_HEX_GENERIC") != nullptr;   // A/B against the LDS-table kernel
  return generic;
#else
  return false;   // (release builds read no kernel choice from the environment)
#endif
}

bool hex_uses_records(const HexArgs& a, int degree, int nq1v, int nq1f)
{
  return degree == 3 && nq1v == 3 && nq1f == 4 && a.kkind != HDD_FN_SINUSOID && !hex_generic_forced();
}

template <int P, int SM>
static hipError_t launch_hex_t(const HexArgs& a, hipStream_t s)
{
  using C = HexCfg<P, SM>;
  const int64_t n_own = a.own_end - a.own_begin;
  if (n_own <= 0) return hipSuccess;
  const int64_t grid = std::min<int64_t>(n_own, 1 << 20);
  static const std::string name = "hex_qp_kernel<" + std::to_string(P) + ", " + std::to_string(SM) + ">";
  hdd::last_tile_kernel_slot() = name.c_str();   // (hdd_last_tile_kernel)
  hipLaunchKernelGGL((hex_qp_kernel<P, SM>), dim3(unsigned(grid)), dim3(C::THREADS), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_hex(const HexArgs& a, int degree, int nq1v, int nq1f, hipStream_t s, bool* supported)
{
  *supported = true;
  const int sm = nq1v - degree;
  if (nq1f - degree - 1 != sm || (sm != 0 && sm != 1)) {
    *supported = false;
    return hipSuccess;
  }
  if (hex_uses_records(a, degree, nq1v, nq1f)) {
    if (!a.ws) return hipErrorInvalidValue;
    return launch_hex_q3(a, s);
  }
  switch (degree * 2 + sm) {
    case 2: return launch_hex_t<1, 0>(a, s);
    case 3: return launch_hex_t<1, 1>(a, s);
    case 4: return launch_hex_t<2, 0>(a, s);
    case 5: return launch_hex_t<2, 1>(a, s);
    case 6: return launch_hex_t<3, 0>(a, s);
    case 7: return launch_hex_t<3, 1>(a, s);
    default: *supported = false; return hipSuccess;
  }
}

// ---------------------------------------------------------------------------------------------------
// device pattern build (EllipticSWIPDG::pattern, swipdg.hh:169): counts -> scan (host side) -> fill
// ---------------------------------------------------------------------------------------------------
__global__ void pattern_counts_kernel(const int32_t* __restrict__ nbrs, int32_t nf, int64_t n_local,
                                      int64_t own_begin, int64_t n_own, int64_t nb2, int64_t* __restrict__ counts)
{
  const int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (k >= n_own) return;
  const int64_t e = own_begin + k;
  int blocks = 1;
  for (int f = 0; f < nf; ++f) blocks += nbrs[f * n_local + e] >= 0;
  counts[k] = nb2 * blocks;
}

// one wavefront per element row block: writes nb rows of nb*nblk sorted global columns
__global__ void pattern_fill_kernel(const int32_t* __restrict__ nbrs, int32_t nf, int32_t nb, int64_t n_local,
                                    int64_t own_begin, int64_t n_own, const int64_t* __restrict__ gid,
                                    const int64_t* __restrict__ elem_ptr, int64_t* __restrict__ row_ptr,
                                    int32_t* __restrict__ col)
{
  const int64_t k = blockIdx.x * int64_t(blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= n_own) return;
  const int64_t e = own_begin + k;
  int64_t blk[7];
  int nblk = 0;
  blk[nblk++] = gid ? gid[e] : e;
  for (int f = 0; f < nf; ++f) {
    const int32_t n = nbrs[f * n_local + e];
    if (n >= 0) blk[nblk++] = gid ? gid[n] : n;
  }
  for (int i = 1; i < nblk; ++i)   // insertion sort of <= 7 keys
    for (int j = i; j > 0 && blk[j - 1] > blk[j]; --j) {
      const int64_t t = blk[j]; blk[j] = blk[j - 1]; blk[j - 1] = t;
    }
  const int64_t base = elem_ptr[k];
  const int rl = nb * nblk;   // <= 7 * 64 columns per row
  for (int i = lane; i < nb; i += 64) row_ptr[k * nb + i] = base + int64_t(i) * rl;
  if (k == n_own - 1 && lane == 0) row_ptr[n_own * nb] = base + int64_t(nb) * rl;
  if (nb == 64) {   // Q3: one block row = one wave store, block ids uniform (no division, no indexed array)
    for (int i = 0; i < 64; ++i) {
      int32_t* crow = col + base + int64_t(i) * rl;
#pragma unroll
      for (int b = 0; b < 7; ++b)
        if (b < nblk) crow[b * 64 + lane] = int32_t(blk[b] * 64 + lane);
    }
    return;
  }
  for (int m = lane; m < nb * rl; m += 64) {
    const int c = m % rl;
    col[base + m] = int32_t(blk[c / nb] * nb + (c % nb));
  }
}

// P1 / Q1 (nb = nf = 3 or 4): one wave per 64-element tile, lane = element.  The lane sorts its <= nf + 1
// column blocks in registers, stages its row block of column ids in an LDS image of the tile (offsets from
// ballots, the elem_ptr rule) and the wave streams the tile's contiguous column range out with 16-byte
// stores: no 64-bit divisions, no per-entry block search (the wave-per-element kernel above keeps hexahedra).
__device__ __forceinline__ int lanes_below(uint64_t m)
{
  return int(__builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u)));
}

template <int NB, int NF>
struct PatTile {
  int32_t nb[NF];   // local neighbour ids (< 0: boundary)
  int64_t own;      // global id of the element
};

// Software-pipelined like swipdg_persistent_kernel (gfx950's vmcnt is in order and counts stores): per
// wave a sequence of tiles, memory order [own data of tile t+1][sort + LDS image of t][neighbour global ids
// of t+1][stores of t].  The tile's row_ptr entries are staged in LDS and written with coalesced 8-byte
// stores (a lane's three or four consecutive entries would be 24 / 32 bytes apart); the column range goes
// out as aligned 16-byte non-temporal buffer stores (head / tail ints separately, so no store straddles
// the range); uniform tiles (64 elements with NF interior faces: 16-byte aligned row blocks) are staged with
// 16-byte LDS writes.
template <int NB, int NF>
__global__ void __launch_bounds__(64) pattern_fill_tile_kernel(const int32_t* __restrict__ nbrs, int64_t n_local,
                                                               int64_t own_begin, int64_t n_own,
                                                               const int64_t* __restrict__ gid,
                                                               const int64_t* __restrict__ elem_ptr,
                                                               int64_t* __restrict__ row_ptr, int32_t* __restrict__ col,
                                                               int64_t n_tiles)
{
  constexpr int RB = (NF + 1) * NB * NB;
  constexpr int CH = (64 * RB + 3) / 4;           // 16-byte chunks of a full tile image
  constexpr int CPL = (CH + 63) / 64;             // chunk stores per lane
  __shared__ __attribute__((aligned(16))) int32_t img[64 * RB + 8 + RB];
  __shared__ int64_t rps[64 * NB];
  typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x;
  int64_t t = blockIdx.x;
  if (t >= n_tiles) return;
  const int64_t step = gridDim.x;
  auto load_own = [&](int64_t tt, PatTile<NB, NF>& p) {
    const int64_t k = tt * 64 + lane;
    const int64_t e = own_begin + (k < n_own ? k : tt * 64);
#pragma unroll
    for (int f = 0; f < NF; ++f) p.nb[f] = nbrs[f * n_local + e];
    p.own = gid ? gid[e] : e;
  };
  auto load_keys = [&](const PatTile<NB, NF>& p, int64_t* nk) {
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int32_t n = p.nb[f];
      nk[f] = n >= 0 ? (gid ? gid[n] : int64_t(n)) : INT64_MAX;
    }
  };
  PatTile<NB, NF> cur;
  int64_t nk[NF];
  load_own(t, cur);
  load_keys(cur, nk);
  for (;;) {
    const bool has_next = t + step < n_tiles;
    const int64_t tn = has_next ? t + step : t;
    PatTile<NB, NF> nxt;
    load_own(tn, nxt);

    const int64_t k0 = t * 64, k = k0 + lane;
    const bool active = k < n_own;
    const int64_t kend = k0 + 64 < n_own ? k0 + 64 : n_own;
    const int nact = int(kend - k0);
    const int64_t base = __builtin_amdgcn_readfirstlane(elem_ptr[k0]);
    const int64_t tend = __builtin_amdgcn_readfirstlane(elem_ptr[kend]);
    int64_t key[NF + 1];
    key[0] = cur.own;
    int nblk = 1;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      key[f + 1] = nk[f];
      nblk += cur.nb[f] >= 0;
    }
#pragma unroll
    for (int i = 0; i < NF; ++i)   // sorting network (bubble, compile-time)
#pragma unroll
      for (int j = 0; j < NF - i; ++j) {
        const int64_t lo = key[j] < key[j + 1] ? key[j] : key[j + 1];
        const int64_t hi = key[j] < key[j + 1] ? key[j + 1] : key[j];
        key[j] = lo;
        key[j + 1] = hi;
      }
    const int64_t al = base & ~int64_t(3);
    const int c = nblk - 1;
    int sum = lanes_below(__ballot(active));
    sum += lanes_below(__ballot(active && (c & 1)));
    sum += 2 * lanes_below(__ballot(active && (c & 2)));
    sum += 4 * lanes_below(__ballot(active && (c & 4)));
    const int off = NB * NB * sum;
    const int rl = NB * nblk;
    if (active) {
#pragma unroll
      for (int i = 0; i < NB; ++i) rps[lane * NB + i] = base + off + i * rl;
    }
    const bool uni = nact == 64 && tend - base == int64_t(64) * RB && base == al;   // wave-uniform
    if (uni) {   // row block of lane = 16-byte aligned at lane * RB: NB rows x (NF + 1) blocks x NB ints
      i32x4* my = reinterpret_cast<i32x4*>(img + lane * RB);
#pragma unroll
      for (int q = 0; q < RB / 4; ++q) {
        i32x4 v;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int m = 4 * q + u, j = m % NB, b = (m / NB) % (NF + 1);
          v[u] = int32_t(key[b] * NB + j);
        }
        my[q] = v;
      }
    } else {
      int32_t* my = active ? img + (base - al) + off : img + 64 * RB + 8;
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int b = 0; b <= NF; ++b)
          if (b < nblk)
#pragma unroll
            for (int j = 0; j < NB; ++j) my[i * rl + b * NB + j] = int32_t(key[b] * NB + j);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    int64_t nk_n[NF];
    load_keys(nxt, nk_n);

    // row_ptr of the tile's rows: contiguous, coalesced
#pragma unroll
    for (int m = 0; m < NB; ++m) {
      const int idx = lane + 64 * m;
      if (idx < nact * NB) row_ptr[k0 * NB + idx] = rps[idx];
    }
    if (k == n_own - 1) row_ptr[n_own * NB] = tend;
    // columns: head ints [base, a0), aligned middle [a0, a1) in 16-byte chunks, tail [a1, tend)
    const int64_t a0 = (base + 3) & ~int64_t(3), a1 = tend & ~int64_t(3);
    if (a0 >= a1) {   // short range (tiny tiles): plain ints
      for (int64_t g = base + lane; g < tend; g += 64) col[g] = img[g - al];
    } else {
      if (lane < a0 - base) col[base + lane] = img[base - al + lane];
      if (lane < tend - a1) col[a1 + lane] = img[a1 - al + lane];
      const int nbytes = int(a1 - a0) * 4;
      __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(col + a0, (short)0, nbytes, 0x00020000);
      const int32_t* src = img + (a0 - al);
#pragma unroll
      for (int u = 0; u < CPL; ++u) {
        const int m = lane + 64 * u;
        const int li = 4 * m < 64 * RB + 4 ? 4 * m : 0;
        const i32x4 v = *reinterpret_cast<const i32x4*>(src + li);
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, m * 16, 0, 2);   // out-of-range chunks dropped
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!has_next) break;
    t = tn;
    cur = nxt;
#pragma unroll
    for (int f = 0; f < NF; ++f) nk[f] = nk_n[f];
  }
}

// elem_ptr in three small launches instead of counts + a general-purpose device scan (which took 40 us of the
// C2 pattern's 200): per-block sums of 2048 elements' counts, one workgroup scanning the block sums, then each
// block re-counts its elements and writes their prefix (the neighbour ids are read twice: 2 x 4 B per face)
constexpr int PE_THREADS = 256, PE_PER = 8, PE_BLOCK = PE_THREADS * PE_PER;   // 8: 2,000 blocks at C2

__device__ __forceinline__ int64_t pe_count(const int32_t* __restrict__ nbrs, int32_t nf, int64_t n_local, int64_t e,
                                            int64_t nb2)
{
  int blocks = 1;
  for (int f = 0; f < nf; ++f) blocks += nbrs[f * n_local + e] >= 0;
  return nb2 * blocks;
}

// block-wide exclusive scan of one value per thread (PE_THREADS threads); returns the block total too
__device__ __forceinline__ int64_t pe_block_scan(int64_t v, int64_t* sh, int64_t& total)
{
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int64_t incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t u = __shfl_up(incl, off, 64);
    if (lane >= off) incl += u;
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  int64_t before = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < PE_THREADS / 64; ++k) {
    before += k < w ? sh[k] : 0;
    total += sh[k];
  }
  __syncthreads();
  return before + incl - v;
}

__global__ void __launch_bounds__(PE_THREADS) pattern_block_sums_kernel(const int32_t* __restrict__ nbrs, int32_t nf,
                                                                        int64_t n_local, int64_t own_begin,
                                                                        int64_t n_own, int64_t nb2,
                                                                        int64_t* __restrict__ sums)
{
  __shared__ int64_t sh[PE_THREADS / 64];
  const int64_t b0 = int64_t(blockIdx.x) * PE_BLOCK + threadIdx.x;   // coalesced: element b0 + i * PE_THREADS
  int64_t v = 0;
#pragma unroll
  for (int i = 0; i < PE_PER; ++i)
    if (b0 + i * PE_THREADS < n_own) v += pe_count(nbrs, nf, n_local, own_begin + b0 + i * PE_THREADS, nb2);
  int64_t total;
  (void)pe_block_scan(v, sh, total);
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// one workgroup: exclusive offsets of the block sums, in place (chunks of PE_THREADS x PE_PER with a carry)
__global__ void __launch_bounds__(PE_THREADS) pattern_sums_scan_kernel(int64_t* __restrict__ sums, int64_t n)
{
  __shared__ int64_t sh[PE_THREADS / 64];
  int64_t carry = 0;
  for (int64_t c0 = 0; c0 < n; c0 += PE_BLOCK) {
    const int64_t i0 = c0 + int64_t(threadIdx.x) * PE_PER;
    int64_t v[PE_PER], s = 0;
#pragma unroll
    for (int i = 0; i < PE_PER; ++i) {
      v[i] = i0 + i < n ? sums[i0 + i] : 0;
      s += v[i];
    }
    int64_t total;
    int64_t ex = carry + pe_block_scan(s, sh, total);
#pragma unroll
    for (int i = 0; i < PE_PER; ++i)
      if (i0 + i < n) {
        sums[i0 + i] = ex;
        ex += v[i];
      }
    carry += total;
  }
}

// BASE_SUM: the block's offset is the sum of the preceding blocks' totals, read by every block (L2-resident:
// 2,000 totals at C2, <= 8 loads per thread) -- no scan launch between the two passes; else offs[] holds the
// scanned offsets.  host_nnz (optional, a mapped pinned host word): the total, written by the last element's
// thread, so the caller reads nnz after a stream synchronisation without a copy launch.
template <bool BASE_SUM>
__global__ void __launch_bounds__(PE_THREADS) pattern_elem_ptr_kernel(const int32_t* __restrict__ nbrs, int32_t nf,
                                                                      int64_t n_local, int64_t own_begin,
                                                                      int64_t n_own, int64_t nb2,
                                                                      const int64_t* __restrict__ offs,
                                                                      int64_t* __restrict__ elem_ptr,
                                                                      int64_t* __restrict__ host_nnz)
{
  __shared__ int64_t sh[PE_THREADS / 64];
  __shared__ int64_t cnt[PE_BLOCK];
  int64_t base = 0;
  if constexpr (BASE_SUM) {
    int64_t part[4] = {0, 0, 0, 0};
    const int nb = int(blockIdx.x);
    int i = int(threadIdx.x);
    for (; i + 3 * PE_THREADS < nb; i += 4 * PE_THREADS) {
#pragma unroll
      for (int u = 0; u < 4; ++u) part[u] += offs[i + u * PE_THREADS];
    }
    for (; i < nb; i += PE_THREADS) part[0] += offs[i];
    int64_t tot;
    (void)pe_block_scan((part[0] + part[1]) + (part[2] + part[3]), sh, tot);
    base = tot;
  } else {
    base = offs[blockIdx.x];
  }
  // counts read coalesced (element b0 + i * PE_THREADS), transposed through LDS so that each thread scans
  // PE_PER consecutive elements, prefixes written back coalesced
  const int64_t blk0 = int64_t(blockIdx.x) * PE_BLOCK;
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < PE_PER; ++i) {
    const int64_t k = blk0 + t + i * PE_THREADS;
    cnt[t + i * PE_THREADS] = k < n_own ? pe_count(nbrs, nf, n_local, own_begin + k, nb2) : 0;
  }
  __syncthreads();
  int64_t c[PE_PER], s = 0;
#pragma unroll
  for (int i = 0; i < PE_PER; ++i) {
    c[i] = cnt[t * PE_PER + i];
    s += c[i];
  }
  int64_t total;
  int64_t p = base + pe_block_scan(s, sh, total);   // (its barriers order the cnt reads above)
#pragma unroll
  for (int i = 0; i < PE_PER; ++i) {
    p += c[i];
    cnt[t * PE_PER + i] = p;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < PE_PER; ++i) {
    const int64_t k = blk0 + t + i * PE_THREADS;
    if (k < n_own) elem_ptr[k + 1] = cnt[t + i * PE_THREADS];
    if (host_nnz && k == n_own - 1) *host_nnz = cnt[t + i * PE_THREADS];
  }
  if (blockIdx.x == 0 && t == 0) elem_ptr[0] = 0;
}

int64_t pattern_elem_ptr_scratch(int64_t n_own) { return (n_own + PE_BLOCK - 1) / PE_BLOCK; }

hipError_t launch_pattern_elem_ptr(const int32_t* nbrs, int32_t nf, int64_t n_local, int64_t own_begin,
                                   int64_t own_end, int64_t nb2, int64_t* d_elem_ptr, int64_t* d_scratch, hipStream_t s,
                                   int64_t* host_nnz, bool scan_launch)
{
  const int64_t n_own = own_end - own_begin;
  if (n_own <= 0) return hipMemsetAsync(d_elem_ptr, 0, sizeof(int64_t), s);
  const int64_t nblk = pattern_elem_ptr_scratch(n_own);
  hipLaunchKernelGGL(pattern_block_sums_kernel, dim3(unsigned(nblk)), dim3(PE_THREADS), 0, s, nbrs, nf, n_local,
                     own_begin, n_own, nb2, d_scratch);
  // the offsets summed per block up to 32 K blocks (67 M elements: <= 128 L2 loads per thread), else scanned
  if (scan_launch || nblk > 32768) {
    hipLaunchKernelGGL(pattern_sums_scan_kernel, dim3(1), dim3(PE_THREADS), 0, s, d_scratch, nblk);
    hipLaunchKernelGGL(pattern_elem_ptr_kernel<false>, dim3(unsigned(nblk)), dim3(PE_THREADS), 0, s, nbrs, nf,
                       n_local, own_begin, n_own, nb2, d_scratch, d_elem_ptr, host_nnz);
  } else {
    hipLaunchKernelGGL(pattern_elem_ptr_kernel<true>, dim3(unsigned(nblk)), dim3(PE_THREADS), 0, s, nbrs, nf,
                       n_local, own_begin, n_own, nb2, d_scratch, d_elem_ptr, host_nnz);
  }
  return hipGetLastError();
}

hipError_t launch_pattern_counts(const int32_t* nbrs, int32_t nf, int64_t n_local, int64_t own_begin, int64_t own_end,
                                 int64_t nb2, int64_t* d_counts, hipStream_t s)
{
  const int64_t n_own = own_end - own_begin;
  if (n_own <= 0) return hipSuccess;
  hipLaunchKernelGGL(pattern_counts_kernel, dim3(unsigned((n_own + 255) / 256)), dim3(256), 0, s, nbrs, nf, n_local,
                     own_begin, n_own, nb2, d_counts);
  return hipGetLastError();
}

hipError_t launch_pattern_fill(const int32_t* nbrs, int32_t nf, int32_t nb, int64_t n_local, int64_t own_begin,
                               int64_t own_end, const int64_t* gid, const int64_t* elem_ptr, int64_t* row_ptr,
                               int32_t* col, int cus, hipStream_t s)
{
  const int64_t n_own = own_end - own_begin;
  if (n_own <= 0) return hipSuccess;
  if ((nb == 3 && nf == 3) || (nb == 4 && nf == 4)) {
    const int64_t tiles = (n_own + 63) / 64;
    const unsigned grid = unsigned(std::min<int64_t>(tiles, int64_t(cus) * 8));
    if (nb == 3)
      hipLaunchKernelGGL((pattern_fill_tile_kernel<3, 3>), dim3(grid), dim3(64), 0, s, nbrs, n_local, own_begin, n_own,
                         gid, elem_ptr, row_ptr, col, tiles);
    else
      hipLaunchKernelGGL((pattern_fill_tile_kernel<4, 4>), dim3(grid), dim3(64), 0, s, nbrs, n_local, own_begin, n_own,
                         gid, elem_ptr, row_ptr, col, tiles);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(pattern_fill_kernel, dim3(unsigned((n_own + 3) / 4)), dim3(256), 0, s, nbrs, nf, nb, n_local,
                     own_begin, n_own, gid, elem_ptr, row_ptr, col);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hdd
