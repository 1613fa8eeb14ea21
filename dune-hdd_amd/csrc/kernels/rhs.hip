// dune-hdd_amd/csrc/kernels/rhs.hip
//
// SWIPDG right-hand side: the functionals SWIPDG::init() adds to its walk
// (dune/hdd/linearelliptic/discretizations/swipdg.hh:251-347):
//   L2Volume(f)                 b_i += int_K f phi_i
//   DirichletBoundarySWIPDG     b_i += int_F -kappa g_D (A grad phi_i).n + sigma_b kappa (n.A n) / |F|^beta g_D phi_i
//   L2Face(g_N) (Neumann faces) b_i += int_F g_N phi_i
// for P1 triangles, Q1 quadrilaterals and Q_p hexahedra.  One thread per (owned element, basis function):
// the vector has nb entries per element (work O(nb nq) per element, negligible next to the matrix), so
// the kernel is written for generality, not for a roofline.  Quadrature rules come from the host.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "swipdg_kernels.hh"

namespace hdd {
namespace dev {

__device__ __forceinline__ double rhs_fn(const KappaArg& f, int64_t e, const double* x, int dim)
{
  switch (f.kind) {
    case HDD_FN_PER_ELEM: return f.per_elem[e];
    case HDD_FN_SINUSOID: return f.c + f.b * sin(f.kx * x[0] + f.ky * x[1]);
    case HDD_FN_COS_PRODUCT:
      return f.c * cos(f.kx * x[0]) * cos(f.ky * x[1]) * ((dim == 3 && f.b != 0.0) ? cos(f.b * x[2]) : 1.0);
    default: return f.c;
  }
}

__device__ __forceinline__ void lagr(int p, int k, double x, double& v, double& d)
{
  double val = 1.0, der = 0.0;
  for (int m = 0; m <= p; ++m) {
    if (m == k) continue;
    const double den = double(k - m) / p, f = (x - double(m) / p) / den;
    der = der * f + val / den;
    val *= f;
  }
  v = val;
  d = der;
}

// basis function i and its reference gradient at the reference point xh
__device__ void rhs_basis(int et, int p, int i, const double* xh, double& v, double* g)
{
  if (et == HDD_SIMPLEX) {
    const double l[3] = {1.0 - xh[0] - xh[1], xh[0], xh[1]};
    const double gx[3] = {-1.0, 1.0, 0.0}, gy[3] = {-1.0, 0.0, 1.0};
    v = l[i];
    g[0] = gx[i];
    g[1] = gy[i];
    return;
  }
  const int dim = et == HDD_HEX ? 3 : 2;
  const int np = p + 1;
  double lv[3], ld[3];
  int r = i;
  for (int a = 0; a < dim; ++a) {
    lagr(p, r % np, xh[a], lv[a], ld[a]);
    r /= np;
  }
  v = 1.0;
  for (int a = 0; a < dim; ++a) v *= lv[a];
  for (int b = 0; b < dim; ++b) {
    double gb = 1.0;
    for (int a = 0; a < dim; ++a) gb *= a == b ? ld[a] : lv[a];
    g[b] = gb;
  }
}

__global__ __launch_bounds__(256) void rhs_kernel(RhsArgs a)
{
  const int dim = a.elem_type == HDD_HEX ? 3 : 2;
  const int nvpe = a.elem_type == HDD_SIMPLEX ? 3 : (a.elem_type == HDD_CUBE ? 4 : 8);
  const int nf = a.elem_type == HDD_SIMPLEX ? 3 : (a.elem_type == HDD_CUBE ? 4 : 6);
  const int64_t n_own = a.own_end - a.own_begin;
  const int64_t total = n_own * a.nb;
  for (int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    const int64_t k = t / a.nb;
    const int i = int(t - k * a.nb);
    const int64_t e = a.own_begin + k;
    const int64_t n = a.n_local;
    // affine geometry x = v0 + J xh (columns: vertices 1, 2 (, 4) minus vertex 0)
    const int vcol[3] = {1, 2, 4};
    double v0[3] = {0, 0, 0}, J[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int c = 0; c < dim; ++c) v0[c] = a.coords[c * n + e];
    for (int j = 0; j < dim; ++j)
      for (int c = 0; c < dim; ++c) J[c][j] = a.coords[(dim * vcol[j] + c) * n + e] - v0[c];
    (void)nvpe;
    double Ji[3][3], det;
    if (dim == 2) {
      det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
      Ji[0][0] = J[1][1] / det; Ji[0][1] = -J[0][1] / det;
      Ji[1][0] = -J[1][0] / det; Ji[1][1] = J[0][0] / det;
    } else {
      const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
      const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
      const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
      det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
      Ji[0][0] = c00 / det; Ji[1][0] = c01 / det; Ji[2][0] = c02 / det;
      Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / det;
      Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / det;
      Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / det;
      Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / det;
      Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / det;
      Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / det;
    }
    double acc = 0.0;
    double xh[3] = {0, 0, 0}, x[3] = {0, 0, 0}, v, gh[3];
    if (a.has_force) {
      for (int q = 0; q < a.nqv; ++q) {
        for (int c = 0; c < dim; ++c) xh[c] = a.qv[q][c];
        for (int c = 0; c < dim; ++c) {
          x[c] = v0[c];
          for (int j = 0; j < dim; ++j) x[c] += J[c][j] * xh[j];
        }
        rhs_basis(a.elem_type, a.degree, i, xh, v, gh);
        acc += a.qv[q][3] * fabs(det) * rhs_fn(a.force, e, x, dim) * v;
      }
    }
    if (a.has_dirichlet || a.has_neumann) {
      for (int f = 0; f < nf; ++f) {
        const int32_t nbr = a.nbrs[f * n + e];
        const bool dir = nbr == HDD_NBR_DIRICHLET && a.has_dirichlet;
        const bool neu = nbr == HDD_NBR_NEUMANN && a.has_neumann;
        if (!dir && !neu) continue;
        // reference face: corner r0 and spanning vectors t1 (, t2), reference outer normal nr
        double r0[3] = {0, 0, 0}, t1[3] = {0, 0, 0}, t2[3] = {0, 0, 0}, nr[3] = {0, 0, 0};
        if (a.elem_type == HDD_SIMPLEX) {
          // faces (v0,v1), (v0,v2), (v1,v2) of the reference triangle (0,0), (1,0), (0,1)
          const double P[3][2] = {{0, 0}, {1, 0}, {0, 1}};
          const int fv[3][2] = {{0, 1}, {0, 2}, {1, 2}};
          const double N[3][2] = {{0, -1}, {-1, 0}, {1, 1}};
          for (int c = 0; c < 2; ++c) {
            r0[c] = P[fv[f][0]][c];
            t1[c] = P[fv[f][1]][c] - P[fv[f][0]][c];
            nr[c] = N[f][c];
          }
        } else {
          const int af = f >> 1, sd = f & 1;
          r0[af] = sd;
          nr[af] = sd ? 1.0 : -1.0;
          int b0 = -1, b1 = -1;
          for (int c = 0; c < dim; ++c)
            if (c != af) { if (b0 < 0) b0 = c; else b1 = c; }
          t1[b0] = 1.0;
          if (dim == 3) t2[b1] = 1.0;
        }
        // physical normal J^{-T} nr / |.| and face measure
        double nv[3] = {0, 0, 0};
        for (int c = 0; c < dim; ++c)
          for (int j = 0; j < dim; ++j) nv[c] += Ji[j][c] * nr[j];
        double nn = 0.0;
        for (int c = 0; c < dim; ++c) nn += nv[c] * nv[c];
        nn = sqrt(nn);
        for (int c = 0; c < dim; ++c) nv[c] /= nn;
        double fvol;
        if (dim == 2) {
          const double dx = J[0][0] * t1[0] + J[0][1] * t1[1], dy = J[1][0] * t1[0] + J[1][1] * t1[1];
          fvol = sqrt(dx * dx + dy * dy);
        } else {
          fvol = fabs(det) * nn;   // reference face area 1 (Nanson)
        }
        const double* qs = dir ? &a.qd[0][0] : &a.qn[0][0];
        const int nq = dir ? a.nqd : a.nqn;
        double An[3] = {0, 0, 0}, gamma = 0.0;
        if (dir) {
          double A[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
          if (a.tkind == HDD_TENSOR_ISO_PER_ELEM) {
            for (int c = 0; c < dim; ++c) A[c][c] = a.tper[e];
          } else {
            const int ns = dim == 2 ? 3 : 6;
            double cc[6];
            for (int r = 0; r < ns; ++r) cc[r] = a.tkind == HDD_TENSOR_SYM_PER_ELEM ? a.tper[r * n + e] : a.tc[r];
            if (dim == 2) {
              A[0][0] = cc[0]; A[0][1] = A[1][0] = cc[1]; A[1][1] = cc[2];
            } else {
              A[0][0] = cc[0]; A[0][1] = A[1][0] = cc[1]; A[0][2] = A[2][0] = cc[2];
              A[1][1] = cc[3]; A[1][2] = A[2][1] = cc[4]; A[2][2] = cc[5];
            }
          }
          for (int c = 0; c < dim; ++c)
            for (int j = 0; j < dim; ++j) An[c] += A[c][j] * nv[j];
          for (int c = 0; c < dim; ++c) gamma += nv[c] * An[c];
        }
        const double hpow = dir ? pow(fvol, a.beta) : 1.0;
        for (int q = 0; q < nq; ++q) {
          const double s0 = qs[3 * q], s1 = qs[3 * q + 1], w = qs[3 * q + 2];
          for (int c = 0; c < dim; ++c) xh[c] = r0[c] + s0 * t1[c] + s1 * t2[c];
          for (int c = 0; c < dim; ++c) {
            x[c] = v0[c];
            for (int j = 0; j < dim; ++j) x[c] += J[c][j] * xh[j];
          }
          rhs_basis(a.elem_type, a.degree, i, xh, v, gh);
          const double gv = w * fvol * rhs_fn(dir ? a.dirichlet : a.neumann, e, x, dim);
          if (dir) {
            const double kap = rhs_fn(a.kappa, e, x, dim);
            double gp = 0.0;   // (A grad phi_i) . n = (J^{-1} A n) . grad_ref phi_i
            for (int r = 0; r < dim; ++r) {
              double cr = 0.0;
              for (int j = 0; j < dim; ++j) cr += Ji[r][j] * An[j];
              gp += cr * gh[r];
            }
            acc += gv * (-kap * gp + a.sigma_boundary * kap * gamma / hpow * v);
          } else {
            acc += gv * v;
          }
        }
      }
    }
    a.out[t] = acc;
  }
}

hipError_t launch_rhs(const RhsArgs& a, hipStream_t s)
{
  const int64_t total = (a.own_end - a.own_begin) * a.nb;
  if (total <= 0) return hipSuccess;
  const int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(rhs_kernel, dim3(unsigned(blocks < (1 << 20) ? blocks : (1 << 20))), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hdd
