// include/hdd_discretizations.hh -- header-only C++ operator surface of the MI355X SWIPDG engine.
//
// Mirrors, for the assembly hot path, the reference's discretization classes (header-only C++ like the
// reference itself) on top of the C ABI in hdd.h:
//   Dune::HDD::LinearElliptic::Discretizations::SWIPDG       (discretizations/swipdg.hh:109-520)
//     ctor validation (swipdg.hh:172-176), pattern() (201-204), init() (206-512, LHS part),
//     system_matrix() (base.hh:240-248, an affinely decomposed container: affine part + components with
//     ParameterFunctional coefficients), freeze_parameter(mu) (base.hh:338-341, 357-361)
//   Dune::HDD::LinearElliptic::Discretizations::BlockSWIPDG  (discretizations/block-swipdg.hh:177-846)
//     num_subdomains() (553), neighbouring_subdomains(ss) (558), localize_vector (567),
//     globalize_vectors (583), get_local_operator(ss) (625), get_coupling_operator(ss, nn) (639)
// Errors are thrown as exceptions on this side (DUNE_THROW's role), never across the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "hdd.h"

namespace Dune {
namespace HDD {
namespace LinearElliptic {

namespace internal {
inline void check(int rc, const char* what)
{
  if (rc != HDD_OK) throw std::runtime_error(std::string(what) + ": " + hdd_last_error(nullptr));
}
inline void hip_check(hipError_t e, const char* what)
{
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
// owning device buffer
template <class T>
class DeviceArray {
 public:
  DeviceArray() = default;
  explicit DeviceArray(size_t n) : n_(n) { if (n) hip_check(hipMalloc(&p_, n * sizeof(T)), "hipMalloc"); }
  DeviceArray(const std::vector<T>& h) : DeviceArray(h.size()) { upload(h); }
  DeviceArray(const DeviceArray&) = delete;
  DeviceArray& operator=(const DeviceArray&) = delete;
  DeviceArray(DeviceArray&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
  DeviceArray& operator=(DeviceArray&& o) noexcept
  {
    if (this != &o) {
      if (p_) (void)hipFree(p_);
      p_ = o.p_; n_ = o.n_;
      o.p_ = nullptr; o.n_ = 0;
    }
    return *this;
  }
  ~DeviceArray() { if (p_) (void)hipFree(p_); }
  void upload(const std::vector<T>& h) { hip_check(hipMemcpy(p_, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice), "H2D"); }
  std::vector<T> download() const
  {
    std::vector<T> h(n_);
    if (n_) hip_check(hipMemcpy(h.data(), p_, n_ * sizeof(T), hipMemcpyDeviceToHost), "D2H");
    return h;
  }
  T* get() const { return p_; }
  size_t size() const { return n_; }
 private:
  T* p_ = nullptr;
  size_t n_ = 0;
};
}  // namespace internal

namespace Pymor {
// theta(mu) = scale * mu: the ParameterFunctional forms of the reference's parametric problems
// ("mu", problems/OS2014.hh:74; "-1.0*mu", problems/spe10.hh:167)
class ParameterFunctional {
 public:
  ParameterFunctional(std::string name = "mu", std::string expression = "mu", double scale = 1.0)
    : name_(std::move(name)), expression_(std::move(expression)), scale_(scale) {}
  double evaluate(double mu) const { return scale_ * mu; }
  const std::string& expression() const { return expression_; }
  bool operator==(const ParameterFunctional& o) const { return name_ == o.name_ && scale_ == o.scale_; }
 private:
  std::string name_, expression_;
  double scale_;
};
}  // namespace Pymor

namespace Problems {
// a (localizable) scalar function as the assembly path evaluates it
struct ScalarFunction {
  int kind = HDD_FN_CONST;
  int order = 0;
  double c = 1.0, b = 0.0, kx = 0.0, ky = 0.0;
  std::vector<double> per_element;   // global element order
  static ScalarFunction constant(double v) { ScalarFunction f; f.c = v; return f; }
  static ScalarFunction piecewise_constant(std::vector<double> v)
  {
    ScalarFunction f; f.kind = HDD_FN_PER_ELEM; f.per_element = std::move(v); return f;
  }
  // Stuff::Functions::Expression "a + b*sin(kx*x + ky*y)" with its integration order
  static ScalarFunction sinusoid(double a, double b, double kx, double ky, int order)
  {
    ScalarFunction f; f.kind = HDD_FN_SINUSOID; f.c = a; f.b = b; f.kx = kx; f.ky = ky; f.order = order; return f;
  }
};
struct TensorFunction {
  int kind = HDD_TENSOR_CONST;
  double c[3] = {1.0, 0.0, 1.0};
  std::vector<double> per_element;   // ISO: [ne]; SYM: [3][ne]
  static TensorFunction identity() { return TensorFunction(); }
  static TensorFunction isotropic(std::vector<double> v)
  {
    TensorFunction t; t.kind = HDD_TENSOR_ISO_PER_ELEM; t.per_element = std::move(v); return t;
  }
};
// AffinelyDecomposable diffusion factor: kappa(mu) = kappa_aff + sum_q theta_q(mu) kappa_q
struct DiffusionFactor {
  bool has_affine_part = true;
  ScalarFunction affine_part = ScalarFunction::constant(1.0);
  std::vector<ScalarFunction> components;
  std::vector<Pymor::ParameterFunctional> coefficients;
  int num_components() const { return int(components.size()); }
};
struct Problem {
  DiffusionFactor diffusion_factor;
  TensorFunction diffusion_tensor;
  bool diffusion_tensor_parametric = false;
  bool diffusion_tensor_empty = false;
};
}  // namespace Problems

namespace Discretizations {

// CSR pattern resident on the device (host copy kept for operator extraction)
class Pattern {
 public:
  int64_t rows = 0, cols = 0, nnz = 0;
  std::vector<int64_t> row_ptr, elem_ptr;
  std::vector<int32_t> col;
  internal::DeviceArray<int64_t> d_row_ptr, d_elem_ptr;
  internal::DeviceArray<int32_t> d_col;
  hdd_csr csr() const { return hdd_csr{rows, cols, nnz, d_row_ptr.get(), d_col.get(), d_elem_ptr.get()}; }
};

// AffinelyDecomposedContainer<Matrix>: components on one shared pattern (values on the device)
class AffinelyDecomposedMatrix {
 public:
  std::shared_ptr<const Pattern> pattern;
  std::shared_ptr<internal::DeviceArray<double>> affine;                    // null if no affine part
  std::vector<std::shared_ptr<internal::DeviceArray<double>>> comps;
  std::vector<Pymor::ParameterFunctional> coefficients;
  hdd_ctx* ctx = nullptr;

  bool has_affine_part() const { return bool(affine); }
  int num_components() const { return int(comps.size()); }
  bool parametric() const { return !comps.empty(); }
  std::vector<double> affine_part() const { return affine->download(); }
  std::vector<double> component(int q) const { return comps.at(q)->download(); }
  // A(mu) = A_aff + sum_q theta_q(mu) A_q on the shared pattern (hdd_affine_lincomb)
  std::vector<double> freeze_parameter(double mu) const
  {
    std::vector<const double*> v;
    std::vector<double> theta;
    if (affine) { v.push_back(affine->get()); theta.push_back(1.0); }
    for (size_t q = 0; q < comps.size(); ++q) { v.push_back(comps[q]->get()); theta.push_back(coefficients[q].evaluate(mu)); }
    internal::DeviceArray<double> out(size_t(pattern->nnz) + (pattern->nnz & 1));
    internal::check(hdd_affine_lincomb(ctx, pattern->nnz, v.data(), int32_t(v.size()), theta.data(), 1, out.get(),
                                       int64_t(out.size()), nullptr), "hdd_affine_lincomb");
    internal::hip_check(hipDeviceSynchronize(), "freeze_parameter");
    auto h = out.download();
    h.resize(size_t(pattern->nnz));
    return h;
  }
};

class SWIPDG {
 public:
  // grid: the (multiscale) grid provider; the boundary info is part of the grid (AllDirichlet /
  // AllNeumann); problem: diffusion factor (affinely decomposed) and tensor.
  SWIPDG(const hdd_grid* grid, const Problems::Problem& problem, int hip_device = 0)
    : grid_(grid), problem_(problem)
  {
    // swipdg.hh:172-176
    if (problem.diffusion_tensor_parametric) throw std::logic_error("The diffusion tensor must not be parametric!");
    if (problem.diffusion_tensor_empty) throw std::invalid_argument("The diffusion tensor must not be empty!");
    internal::check(hdd_grid_get_info(grid, &info_), "hdd_grid_get_info");
    internal::check(hdd_ctx_create(hip_device, &ctx_), "hdd_ctx_create");
    internal::check(hdd_local_create(grid, 0, info_.n_subdomains, &local_), "hdd_local_create");
    internal::check(hdd_local_get_info(local_, &linfo_), "hdd_local_get_info");
    build_pattern();
  }
  virtual ~SWIPDG()
  {
    if (local_) hdd_local_destroy(local_);
    if (ctx_) hdd_ctx_destroy(ctx_);
  }
  SWIPDG(const SWIPDG&) = delete;
  SWIPDG& operator=(const SWIPDG&) = delete;

  const Pattern& pattern() const { return *pattern_; }

  // assembles the LHS (every diffusion-factor component + the affine part) on the device; idempotent
  void init()
  {
    if (initialized_) return;
    const int64_t n = linfo_.n_local;
    std::vector<double> coords(size_t(2 * info_.nvpe * n));
    std::vector<int32_t> nbrs(size_t(info_.nfaces * n));
    std::vector<uint32_t> finfo(static_cast<size_t>(n));
    internal::check(hdd_local_fill(local_, coords.data(), nbrs.data(), finfo.data(), nullptr, nullptr), "hdd_local_fill");
    d_coords_ = internal::DeviceArray<double>(coords);
    d_nbrs_ = internal::DeviceArray<int32_t>(nbrs);
    d_finfo_ = internal::DeviceArray<uint32_t>(finfo);
    const auto& T = problem_.diffusion_tensor;
    if (T.kind != HDD_TENSOR_CONST) d_tensor_ = internal::DeviceArray<double>(T.per_element);
    hdd_mesh m{info_.elem_type, 0, n, linfo_.own_begin, linfo_.own_end, d_coords_.get(), d_nbrs_.get(), d_finfo_.get()};
    hdd_tensor_fn A{T.kind, 0, {T.c[0], T.c[1], T.c[2]}, d_tensor_.get()};
    hdd_swipdg_params prm{8.0, 14.0, 1.0 / (2 - 1), -1, -1};   // inner/boundary_sigma(1), default_beta(2)
    const hdd_csr pat = pattern_->csr();
    matrix_.pattern = pattern_;
    matrix_.ctx = ctx_;
    matrix_.coefficients = problem_.diffusion_factor.coefficients;
    auto assemble = [&](const Problems::ScalarFunction& f) {
      auto vals = std::make_shared<internal::DeviceArray<double>>(size_t(pattern_->nnz) + 1);
      std::unique_ptr<internal::DeviceArray<double>> pe;
      if (f.kind == HDD_FN_PER_ELEM) pe.reset(new internal::DeviceArray<double>(f.per_element));
      hdd_scalar_fn k{f.kind, f.order, f.c, f.b, f.kx, f.ky, pe ? pe->get() : nullptr};
      double* v = vals->get();
      internal::check(hdd_swipdg_assemble(ctx_, &m, &k, 1, &A, &prm, &pat, &v, nullptr), "hdd_swipdg_assemble");
      internal::hip_check(hipDeviceSynchronize(), "init");
      return vals;
    };
    for (const auto& c : problem_.diffusion_factor.components) matrix_.comps.push_back(assemble(c));
    if (problem_.diffusion_factor.has_affine_part) matrix_.affine = assemble(problem_.diffusion_factor.affine_part);
    initialized_ = true;
  }

  const AffinelyDecomposedMatrix& system_matrix() const
  {
    if (!initialized_) throw std::logic_error("system_matrix(): call init() first");
    return matrix_;
  }
  int64_t num_dofs() const { return pattern_->rows; }
  hdd_ctx* context() const { return ctx_; }
  const hdd_grid* grid() const { return grid_; }

 protected:
  void build_pattern()
  {
    auto P = std::make_shared<Pattern>();
    const int64_t n = linfo_.n_local;
    std::vector<int32_t> nbrs(size_t(info_.nfaces * n));
    internal::check(hdd_local_fill(local_, nullptr, nbrs.data(), nullptr, nullptr, nullptr), "hdd_local_fill");
    internal::check(hdd_pattern_count(info_.elem_type, n, linfo_.own_begin, linfo_.own_end, nbrs.data(), &P->nnz),
                    "hdd_pattern_count");
    const int64_t own = linfo_.own_end - linfo_.own_begin;
    P->rows = own * info_.nb;
    P->cols = info_.n_elements * info_.nb;
    P->row_ptr.resize(size_t(P->rows + 1));
    P->col.resize(size_t(P->nnz));
    P->elem_ptr.resize(size_t(own + 1));
    internal::check(hdd_pattern_fill(info_.elem_type, n, linfo_.own_begin, linfo_.own_end, nbrs.data(), nullptr,
                                     P->row_ptr.data(), P->col.data(), P->elem_ptr.data()), "hdd_pattern_fill");
    P->d_row_ptr = internal::DeviceArray<int64_t>(P->row_ptr);
    P->d_col = internal::DeviceArray<int32_t>(P->col);
    P->d_elem_ptr = internal::DeviceArray<int64_t>(P->elem_ptr);
    pattern_ = P;
  }

  const hdd_grid* grid_;
  Problems::Problem problem_;
  hdd_grid_info info_{};
  hdd_local_info linfo_{};
  hdd_ctx* ctx_ = nullptr;
  hdd_local* local_ = nullptr;
  std::shared_ptr<Pattern> pattern_;
  internal::DeviceArray<double> d_coords_, d_tensor_;
  internal::DeviceArray<int32_t> d_nbrs_;
  internal::DeviceArray<uint32_t> d_finfo_;
  AffinelyDecomposedMatrix matrix_;
  bool initialized_ = false;
};

// BlockSWIPDG: the grid must carry the subdomain partition (hdd_grid_create_structured with px, py or
// hdd_grid_create_from_connectivity with subdomains); its subdomain-major element order IS the block
// numbering, so the global system matrix is assembled in one pass and the local / coupling operators
// are its diagonal / off-diagonal blocks.
class BlockSWIPDG : public SWIPDG {
 public:
  using SWIPDG::SWIPDG;

  int num_subdomains() const { return info_.n_subdomains; }

  std::vector<int> neighbouring_subdomains(int ss) const
  {
    range_check(ss);
    std::vector<int> out;
    for (int nn = 0; nn < num_subdomains(); ++nn) {
      if (nn == ss) continue;
      int64_t nnz = 0;
      internal::check(hdd_block_operator_map(grid_, ss, nn, pattern_->row_ptr.data(), pattern_->col.data(), nullptr,
                                             nullptr, nullptr, &nnz), "hdd_block_operator_map");
      if (nnz) out.push_back(nn);
    }
    return out;
  }

  AffinelyDecomposedMatrix get_local_operator(int ss) const { return extract(ss, ss); }

  AffinelyDecomposedMatrix get_coupling_operator(int ss, int nn) const
  {
    const auto nb = neighbouring_subdomains(ss);
    if (std::find(nb.begin(), nb.end(), nn) == nb.end())
      throw std::out_of_range("Subdomain " + std::to_string(nn) + " is not a neighbour of subdomain " + std::to_string(ss));
    return extract(ss, nn);
  }

  std::vector<double> localize_vector(const std::vector<double>& global, int ss) const
  {
    range_check(ss);
    if (int64_t(global.size()) != num_dofs()) throw std::out_of_range("localize_vector: wrong global size");
    int64_t a, b;
    internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &b), "hdd_grid_subdomain_range");
    return std::vector<double>(global.begin() + a * info_.nb, global.begin() + b * info_.nb);
  }

  std::vector<double> globalize_vectors(const std::vector<std::vector<double>>& locals) const
  {
    if (int(locals.size()) != num_subdomains()) throw std::invalid_argument("globalize_vectors: wrong number of vectors");
    std::vector<double> out;
    for (int ss = 0; ss < num_subdomains(); ++ss) {
      int64_t a, b;
      internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &b), "hdd_grid_subdomain_range");
      if (int64_t(locals[ss].size()) != (b - a) * info_.nb) throw std::invalid_argument("globalize_vectors: wrong local size");
      out.insert(out.end(), locals[ss].begin(), locals[ss].end());
    }
    return out;
  }

 private:
  void range_check(int ss) const
  {
    if (ss < 0 || ss >= num_subdomains())
      throw std::out_of_range("0 <= ss < num_subdomains() = " + std::to_string(num_subdomains()) + " is not true for ss = " +
                              std::to_string(ss) + "!");
  }

  AffinelyDecomposedMatrix extract(int ss, int nn) const
  {
    range_check(ss);
    range_check(nn);
    const auto& M = system_matrix();
    int64_t nnz = 0;
    internal::check(hdd_block_operator_map(grid_, ss, nn, pattern_->row_ptr.data(), pattern_->col.data(), nullptr,
                                           nullptr, nullptr, &nnz), "hdd_block_operator_map");
    int64_t a, b, c, d;
    internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &b), "range");
    internal::check(hdd_grid_subdomain_range(grid_, nn, nn + 1, &c, &d), "range");
    auto P = std::make_shared<Pattern>();
    P->rows = (b - a) * info_.nb;
    P->cols = (d - c) * info_.nb;
    P->nnz = nnz;
    P->row_ptr.resize(size_t(P->rows + 1));
    P->col.resize(size_t(nnz));
    std::vector<int64_t> src(static_cast<size_t>(nnz));
    internal::check(hdd_block_operator_map(grid_, ss, nn, pattern_->row_ptr.data(), pattern_->col.data(),
                                           P->row_ptr.data(), P->col.data(), src.data(), &nnz), "hdd_block_operator_map");
    P->d_row_ptr = internal::DeviceArray<int64_t>(P->row_ptr);
    P->d_col = internal::DeviceArray<int32_t>(P->col);
    internal::DeviceArray<int64_t> d_src(src);
    AffinelyDecomposedMatrix out;
    out.pattern = P;
    out.ctx = ctx_;
    out.coefficients = M.coefficients;
    auto gather = [&](const internal::DeviceArray<double>& v) {
      auto o = std::make_shared<internal::DeviceArray<double>>(size_t(nnz) + 1);
      internal::check(hdd_gather_values(ctx_, v.get(), d_src.get(), nnz, o->get(), nullptr), "hdd_gather_values");
      return o;
    };
    if (M.affine) out.affine = gather(*M.affine);
    for (const auto& q : M.comps) out.comps.push_back(gather(*q));
    internal::hip_check(hipDeviceSynchronize(), "extract");
    return out;
  }
};

}  // namespace Discretizations
}  // namespace LinearElliptic
}  // namespace HDD
}  // namespace Dune
