// dune-hdd_amd/csrc/kernels/swipdg_q1.hip -- Q1 (parallelograms) instantiations of the persistent tile driver:
// closed-form piecewise-constant stiffness (the C1 / C4 kernel), the smooth-kappa quadrature policy, the
// SWIPDG penalty product.
#include "swipdg_device.hh"

namespace hdd {
namespace dev {

#ifdef HDD_ABLATION
// Study (round 3): Q1 own data from element-major 80 B records -- 4 vertices (16 B each) and the
// 4 neighbour ids (16 B) -- instead of 12 SoA rows, and the neighbour's role vertex as one 16-byte gather
// (scripts/microbench/wstream7.hip: the records' read stream costs 28 % less beside the value stream).  The
// launcher builds the records itself (cached per coords pointer): ablation builds only, HDD_DEBUG_FLAGS bit 1024.
template <int TK, int KK, bool PEN = false, bool VX = false>
struct Q1RecPolicy : Q1PwcPolicy<TK, KK, PEN, false> {
  using Base = Q1PwcPolicy<TK, KK, PEN, false>;
  using Own = typename Base::Own;
  using Gat = typename Base::Gat;
  __device__ static void load_own(const AssembleArgs& a, int64_t e, Own& o)
  {
    const dvec2* r = reinterpret_cast<const dvec2*>(a.rec + 10 * e);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const dvec2 v = r[k];
      o.X[k] = v.x;
      o.Y[k] = v.y;
    }
    const ivec4 nb = *reinterpret_cast<const ivec4*>(a.rec + 10 * e + 8);
    o.nbr[0] = nb.x; o.nbr[1] = nb.y; o.nbr[2] = nb.z; o.nbr[3] = nb.w;
    o.finfo = a.finfo[e];
    o.A = tensor_k<TK>(a, e);
    o.ke = kappa_k<KK == HDD_FN_PER_ELEM ? HDD_FN_PER_ELEM : HDD_FN_CONST>(a, e);
  }
  __device__ static void load_gat(const AssembleArgs& a, int64_t e, Own& o, Gat& g)
  {
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int64_t n = o.nbr[f] >= 0 ? int64_t(o.nbr[f]) : e;
      const int c = role_slot<Cube>(o.finfo, f, 2);
      const dvec2 v = reinterpret_cast<const dvec2*>(a.rec + 10 * n)[c];
      g.Cx[f] = v.x;
      g.Cy[f] = v.y;
      g.Ap[f] = tensor_k<TK>(a, n);
      g.kn[f] = kappa_k<KK == HDD_FN_PER_ELEM ? HDD_FN_PER_ELEM : HDD_FN_CONST>(a, n);
    }
  }
};
template <int TK, int KK, bool VX> using Q1Rec = Q1RecPolicy<TK, KK, false, VX>;

__global__ void q1_records_kernel(const double* __restrict__ coords, const int32_t* __restrict__ nbrs, int64_t n,
                                  double* __restrict__ rec)
{
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < n; e += int64_t(gridDim.x) * blockDim.x) {
    for (int k = 0; k < 8; ++k) rec[10 * e + k] = coords[k * n + e];
    int32_t* ri = reinterpret_cast<int32_t*>(rec + 10 * e + 8);
    for (int f = 0; f < 4; ++f) ri[f] = nbrs[f * n + e];
  }
}

hipError_t launch_q1_pwc(const AssembleArgs& a, hipStream_t s)
{
  if (!(a.debug_flags & 1024)) return dispatch_kinds<Q1Pwc>(a, s, false);
  static const double* key = nullptr;
  static int64_t key_n = 0;
  static double* rec = nullptr;
  if (key != a.coords || key_n != a.n_local) {
    if (rec) (void)hipFree(rec);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&rec), size_t(a.n_local) * 80);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(q1_records_kernel, dim3(1024), dim3(256), 0, s, a.coords, a.nbrs, a.n_local, rec);
    key = a.coords;
    key_n = a.n_local;
  }
  AssembleArgs ar = a;
  ar.rec = rec;
  return dispatch_kinds_vx<Q1Rec, false>(ar, s, false);
}
#else
hipError_t launch_q1_pwc(const AssembleArgs& a, hipStream_t s) { return dispatch_kinds<Q1Pwc>(a, s, false); }
#endif
hipError_t launch_q1_smooth(const AssembleArgs& a, hipStream_t s) { return dispatch_kinds<Q1Smooth3>(a, s, true); }

template <int TK, int KK> using Q1Pen = Q1PwcPolicy<TK, KK, true>;
hipError_t launch_q1_penalty(const AssembleArgs& a, hipStream_t s) { return dispatch_pwc<Q1Pen>(a, s); }

}  // namespace dev
}  // namespace hdd
