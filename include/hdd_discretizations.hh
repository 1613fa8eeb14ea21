// include/hdd_discretizations.hh -- header-only C++ operator surface of the MI355X SWIPDG engine.
//
// Mirrors, for the assembly hot path, the reference's discretization classes (header-only C++ like the
// reference itself) on top of the C ABI in hdd.h:
//   Dune::HDD::LinearElliptic::Discretizations::SWIPDG       (discretizations/swipdg.hh:109-520)
//     ctor validation (swipdg.hh:172-176), pattern() (201-204), init() (206-512: system matrix, right-hand
//     side, products), system_matrix() / rhs() (base.hh:240-258, affinely decomposed containers: affine part
//     + components with ParameterFunctional coefficients), freeze_parameter(mu) (base.hh:338-341, 357-361),
//     available_products() / get_product(id) (base.hh:266-322; "l2", "h1_semi", "elliptic", "boundary_l2",
//     "penalty", "energy" as registered at swipdg.hh:358-508)
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
  // a cos(kx x) cos(ky y) [cos(kz z)]: ESV2007 Testcase1Force (problems/ESV2007.hh:78)
  static ScalarFunction cos_product(double a, double kx, double ky, double kz, int order)
  {
    ScalarFunction f; f.kind = HDD_FN_COS_PRODUCT; f.c = a; f.b = kz; f.kx = kx; f.ky = ky; f.order = order; return f;
  }
  bool is_zero() const { return kind == HDD_FN_CONST && c == 0.0; }
};
struct TensorFunction {
  int kind = HDD_TENSOR_CONST;
  double c[6] = {1.0, 0.0, 1.0, 0.0, 0.0, 0.0};   // 2d a11 a12 a22; 3d a11 a12 a13 a22 a23 a33 (see identity3d)
  std::vector<double> per_element;   // ISO: [ne]; SYM: [3 | 6][ne]
  static TensorFunction identity3d()
  {
    TensorFunction t;
    const double id[6] = {1.0, 0.0, 0.0, 1.0, 0.0, 1.0};
    std::copy(id, id + 6, t.c);
    return t;
  }
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
  // right-hand side data (non-parametric): force, Dirichlet and Neumann values (zero = absent)
  ScalarFunction force = ScalarFunction::constant(0.0);
  ScalarFunction dirichlet = ScalarFunction::constant(0.0);
  ScalarFunction neumann = ScalarFunction::constant(0.0);
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

// AffinelyDecomposedContainer<Vector> (the right-hand side)
class AffinelyDecomposedVector {
 public:
  std::shared_ptr<internal::DeviceArray<double>> affine;
  std::vector<std::shared_ptr<internal::DeviceArray<double>>> comps;
  std::vector<Pymor::ParameterFunctional> coefficients;
  int64_t size = 0;
  bool has_affine_part() const { return bool(affine); }
  int num_components() const { return int(comps.size()); }
  std::vector<double> affine_part() const { auto h = affine->download(); h.resize(size_t(size)); return h; }
  std::vector<double> component(int q) const { auto h = comps.at(q)->download(); h.resize(size_t(size)); return h; }
};

namespace detail {
inline int degree_of(const hdd_grid_info& gi)
{
  if (gi.elem_type != HDD_HEX) return 1;
  int p = 1;
  while ((p + 1) * (p + 1) * (p + 1) < gi.nb) ++p;
  return p;
}
// LocalEvaluation::SWIPDG::internal::{inner,boundary}_sigma(p), default_beta(d)
inline hdd_swipdg_params swipdg_params(int p, int dim)
{
  const double si = p <= 1 ? 8.0 : (p == 2 ? 20.0 : (p == 3 ? 38.0 : 50.0));
  const double sb = p <= 1 ? 14.0 : (p == 2 ? 38.0 : (p == 3 ? 74.0 : 99.0));
  return hdd_swipdg_params{si, sb, 1.0 / (dim - 1), -1, -1};
}
}  // namespace detail

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
    degree_ = detail::degree_of(info_);
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

  // assembles the system matrix (every diffusion-factor component + the affine part), the right-hand side
  // and the requested products on the device; idempotent (container_based_initialized_, swipdg.hh:208)
  void init()
  {
    if (initialized_) return;
    const int64_t n = linfo_.n_local;
    const int dim = info_.dim;
    std::vector<double> coords(size_t(dim * info_.nvpe * n));
    std::vector<int32_t> nbrs(size_t(info_.nfaces * n));
    std::vector<uint32_t> finfo(static_cast<size_t>(n));
    internal::check(hdd_local_fill(local_, coords.data(), nbrs.data(), finfo.data(), nullptr, nullptr), "hdd_local_fill");
    d_coords_ = internal::DeviceArray<double>(coords);
    d_nbrs_ = internal::DeviceArray<int32_t>(nbrs);
    d_finfo_ = internal::DeviceArray<uint32_t>(finfo);
    const auto& T = problem_.diffusion_tensor;
    if (T.kind != HDD_TENSOR_CONST) d_tensor_ = internal::DeviceArray<double>(T.per_element);
    mesh_ = hdd_mesh{info_.elem_type, degree_, n, linfo_.own_begin, linfo_.own_end, d_coords_.get(), d_nbrs_.get(),
                     d_finfo_.get()};
    tensor_ = hdd_tensor_fn{T.kind, 0, {T.c[0], T.c[1], T.c[2], T.c[3], T.c[4], T.c[5]}, d_tensor_.get()};
    prm_ = detail::swipdg_params(degree_, dim);
    const hdd_csr pat = pattern_->csr();
    matrix_.pattern = pattern_;
    matrix_.ctx = ctx_;
    matrix_.coefficients = problem_.diffusion_factor.coefficients;
    auto assemble = [&](const Problems::ScalarFunction& f) {
      auto vals = std::make_shared<internal::DeviceArray<double>>(size_t(pattern_->nnz) + 1);
      Fn k(f);
      double* v = vals->get();
      internal::check(hdd_swipdg_assemble(ctx_, &mesh_, &k.fn, 1, &tensor_, &prm_, &pat, &v, nullptr),
                      "hdd_swipdg_assemble");
      internal::hip_check(hipDeviceSynchronize(), "init");
      return vals;
    };
    for (const auto& c : problem_.diffusion_factor.components) matrix_.comps.push_back(assemble(c));
    if (problem_.diffusion_factor.has_affine_part) matrix_.affine = assemble(problem_.diffusion_factor.affine_part);
    assemble_rhs();
    initialized_ = true;
  }

  const AffinelyDecomposedMatrix& system_matrix() const
  {
    if (!initialized_) throw std::logic_error("system_matrix(): call init() first");
    return matrix_;
  }
  const AffinelyDecomposedVector& rhs() const
  {
    if (!initialized_) throw std::logic_error("rhs(): call init() first");
    return rhs_;
  }

  // base.hh:266-322: "l2", "h1_semi", "elliptic", "boundary_l2", "penalty", "energy"
  std::vector<std::string> available_products() const
  {
    return {"l2", "h1_semi", "elliptic", "boundary_l2", "penalty", "energy"};
  }
  AffinelyDecomposedMatrix get_product(const std::string& id)
  {
    init();
    if (id == "energy") return matrix_;
    int kind;
    if (id == "l2") kind = HDD_PRODUCT_L2;
    else if (id == "h1_semi") kind = HDD_PRODUCT_H1_SEMI;
    else if (id == "elliptic") kind = HDD_PRODUCT_ELLIPTIC;
    else if (id == "boundary_l2") kind = HDD_PRODUCT_BOUNDARY_L2;
    else if (id == "penalty") kind = HDD_PRODUCT_PENALTY;
    else throw std::invalid_argument("Product '" + id + "' not available!");
    const bool volume = kind != HDD_PRODUCT_PENALTY;
    std::shared_ptr<const Pattern> P = volume ? volume_pattern() : std::shared_ptr<const Pattern>(pattern_);
    const hdd_csr pat = P->csr();
    AffinelyDecomposedMatrix out;
    out.pattern = P;
    out.ctx = ctx_;
    auto run = [&](const Problems::ScalarFunction& f) {
      auto vals = std::make_shared<internal::DeviceArray<double>>(size_t(P->nnz) + 1);
      Fn k(f);
      internal::check(hdd_product_assemble(ctx_, &mesh_, kind, &k.fn, &tensor_, &prm_, &pat, vals->get(), nullptr),
                      "hdd_product_assemble");
      internal::hip_check(hipDeviceSynchronize(), "get_product");
      return vals;
    };
    const auto& K = problem_.diffusion_factor;
    if (kind == HDD_PRODUCT_ELLIPTIC || kind == HDD_PRODUCT_PENALTY) {   // affinely decomposed like kappa
      out.coefficients = K.coefficients;
      for (const auto& c : K.components) out.comps.push_back(run(c));
      if (K.has_affine_part) out.affine = run(K.affine_part);
    } else {
      out.affine = run(Problems::ScalarFunction::constant(1.0));
    }
    return out;
  }

  int64_t num_dofs() const { return pattern_->rows; }
  hdd_ctx* context() const { return ctx_; }
  const hdd_grid* grid() const { return grid_; }
  int polynomial_order() const { return degree_; }

 protected:
  // a scalar function bound to the device (per-element values uploaded, kept alive with the descriptor)
  struct Fn {
    hdd_scalar_fn fn;
    std::unique_ptr<internal::DeviceArray<double>> pe;
    explicit Fn(const Problems::ScalarFunction& f)
    {
      if (f.kind == HDD_FN_PER_ELEM) pe.reset(new internal::DeviceArray<double>(f.per_element));
      fn = hdd_scalar_fn{f.kind, f.order, f.c, f.b, f.kx, f.ky, pe ? pe->get() : nullptr};
    }
  };

  // swipdg.hh:251-347: affine part = L2Volume(f) + DirichletBoundarySWIPDG(kappa_aff, A, g_D) + L2Face(g_N);
  // component q = DirichletBoundarySWIPDG(kappa_q, A, g_D) with kappa's coefficient theta_q
  void assemble_rhs()
  {
    const auto& P = problem_;
    const int64_t size = pattern_->rows;
    rhs_.size = size;
    rhs_.coefficients.clear();
    auto run = [&](const Problems::ScalarFunction* force, const Problems::ScalarFunction* kappa) {
      auto b = std::make_shared<internal::DeviceArray<double>>(size_t(size) + 1);
      std::unique_ptr<Fn> f, k, d, nm;
      if (force && !force->is_zero()) f.reset(new Fn(*force));
      if (kappa && !P.dirichlet.is_zero()) { k.reset(new Fn(*kappa)); d.reset(new Fn(P.dirichlet)); }
      if (force && !P.neumann.is_zero()) nm.reset(new Fn(P.neumann));
      internal::check(hdd_swipdg_rhs(ctx_, &mesh_, f ? &f->fn : nullptr, k ? &k->fn : nullptr, &tensor_,
                                     d ? &d->fn : nullptr, nm ? &nm->fn : nullptr, &prm_, b->get(), nullptr),
                      "hdd_swipdg_rhs");
      internal::hip_check(hipDeviceSynchronize(), "rhs");
      return b;
    };
    const auto& K = P.diffusion_factor;
    rhs_.affine = run(&P.force, K.has_affine_part ? &K.affine_part : nullptr);
    if (!P.dirichlet.is_zero())
      for (int q = 0; q < K.num_components(); ++q) {
        rhs_.comps.push_back(run(nullptr, &K.components[q]));
        rhs_.coefficients.push_back(K.coefficients[q]);
      }
  }

  std::shared_ptr<const Pattern> volume_pattern()
  {
    if (volume_pattern_) return volume_pattern_;
    auto P = std::make_shared<Pattern>();
    const int64_t n = linfo_.n_local, own = linfo_.own_end - linfo_.own_begin;
    std::vector<int32_t> nbrs(size_t(info_.nfaces * n));
    internal::check(hdd_local_fill(local_, nullptr, nbrs.data(), nullptr, nullptr, nullptr), "hdd_local_fill");
    internal::check(hdd_dg_pattern_count(0, info_.nb, n, linfo_.own_begin, linfo_.own_end, nbrs.data(), &P->nnz),
                    "hdd_dg_pattern_count");
    P->rows = own * info_.nb;
    P->cols = info_.n_elements * info_.nb;
    P->row_ptr.resize(size_t(P->rows + 1));
    P->col.resize(size_t(P->nnz));
    P->elem_ptr.resize(size_t(own + 1));
    internal::check(hdd_dg_pattern_fill(0, info_.nb, n, linfo_.own_begin, linfo_.own_end, nbrs.data(), nullptr,
                                        P->row_ptr.data(), P->col.data(), P->elem_ptr.data()), "hdd_dg_pattern_fill");
    P->d_row_ptr = internal::DeviceArray<int64_t>(P->row_ptr);
    P->d_col = internal::DeviceArray<int32_t>(P->col);
    P->d_elem_ptr = internal::DeviceArray<int64_t>(P->elem_ptr);
    volume_pattern_ = P;
    return P;
  }

  void build_pattern()
  {
    auto P = std::make_shared<Pattern>();
    const int64_t n = linfo_.n_local;
    std::vector<int32_t> nbrs(size_t(info_.nfaces * n));
    internal::check(hdd_local_fill(local_, nullptr, nbrs.data(), nullptr, nullptr, nullptr), "hdd_local_fill");
    internal::check(hdd_dg_pattern_count(info_.nfaces, info_.nb, n, linfo_.own_begin, linfo_.own_end, nbrs.data(),
                                         &P->nnz), "hdd_dg_pattern_count");
    const int64_t own = linfo_.own_end - linfo_.own_begin;
    P->rows = own * info_.nb;
    P->cols = info_.n_elements * info_.nb;
    P->row_ptr.resize(size_t(P->rows + 1));
    P->col.resize(size_t(P->nnz));
    P->elem_ptr.resize(size_t(own + 1));
    internal::check(hdd_dg_pattern_fill(info_.nfaces, info_.nb, n, linfo_.own_begin, linfo_.own_end, nbrs.data(),
                                        nullptr, P->row_ptr.data(), P->col.data(), P->elem_ptr.data()),
                    "hdd_dg_pattern_fill");
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
  std::shared_ptr<const Pattern> volume_pattern_;
  internal::DeviceArray<double> d_coords_, d_tensor_;
  internal::DeviceArray<int32_t> d_nbrs_;
  internal::DeviceArray<uint32_t> d_finfo_;
  hdd_mesh mesh_{};
  hdd_tensor_fn tensor_{};
  hdd_swipdg_params prm_{};
  int degree_ = 1;
  AffinelyDecomposedMatrix matrix_;
  AffinelyDecomposedVector rhs_;
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
