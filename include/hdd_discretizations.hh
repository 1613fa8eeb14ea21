// include/hdd_discretizations.hh -- header-only C++ operator surface of the MI355X SWIPDG engine.
//
// Mirrors, for the assembly hot path, the reference's discretization classes (header-only C++ like the
// reference itself) on top of the C ABI in hdd.h:
//   Dune::HDD::LinearElliptic::Discretizations::SWIPDG       (discretizations/swipdg.hh:109-520)
//     ctor(grid_provider, boundary_cfg, problem, level_or_subdomain, only_these_products) (swipdg.hh:159-198)
//     with its validation (172-176), pattern() (201-204), init(out, prefix) (206-512: "assembling... done
//     (took Xs)", system matrix, right-hand side with the parametric force / Dirichlet / Neumann component
//     structure of 251-356, the requested products 358-508), system_matrix() / rhs() / get_operator() /
//     get_rhs() (base.hh:240-270), available_products() / get_product(id) (base.hh:272-291),
//     freeze_parameter(mu) (base.hh:338-341, 357-361)
//   Dune::HDD::LinearElliptic::Discretizations::BlockSWIPDG  (discretizations/block-swipdg.hh:177-846)
//     ctor(ms_grid_provider, ignored cfg, problem, products) with the ZeroBoundary / AllDirichlet
//     replacement (172-176, 230-255), init(out, prefix) (262-551), num_subdomains() (553),
//     neighbouring_subdomains(ss) (558), localize_vector (567), globalize_vectors (583),
//     get_local_product(ss, id) (612), get_local_operator(ss) (625), get_coupling_operator(ss, nn) (639),
//     get_local_functional(ss) (678), get_local_discretization(ss) (761)
//   ShardedBlockSWIPDG: BlockSWIPDG with its subdomains distributed over one process / thread per GPU
//     (SURVEY.md 8(e)); each rank owns a contiguous subdomain range and assembles its rows through
//     hdd_block_assemble_sharded, the face halo moved by a Parallel::Communicator (RCCL or host transport).
// Errors are thrown as exceptions on this side (DUNE_THROW's role), never across the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <ostream>
#include <set>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "hdd.h"

namespace Dune {

// DUNE_THROW(NotImplemented, ...) of the reference (swipdg.hh:174)
struct NotImplemented : std::logic_error {
  using std::logic_error::logic_error;
};

namespace Stuff {
namespace Exceptions {   // dune-stuff exception types the reference throws (base.hh:285-289, block-swipdg.hh:560-562)
struct wrong_input_given : std::invalid_argument {
  using std::invalid_argument::invalid_argument;
};
struct you_are_using_this_wrong : std::logic_error {
  using std::logic_error::logic_error;
};
struct index_out_of_range : std::out_of_range {
  using std::out_of_range::out_of_range;
};
struct internal_error : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct requirements_not_met : std::logic_error {
  using std::logic_error::logic_error;
};
}  // namespace Exceptions

namespace Common {
// Stuff::Common::Configuration: the key/value tree the reference passes boundary infos and problems as
class Configuration {
 public:
  Configuration() = default;
  Configuration(std::initializer_list<std::pair<const std::string, std::string>> kv) : m_(kv) {}
  bool has_key(const std::string& k) const { return m_.count(k) > 0; }
  std::string get(const std::string& k, const std::string& def = "") const
  {
    const auto it = m_.find(k);
    return it == m_.end() ? def : it->second;
  }
  std::string& operator[](const std::string& k) { return m_[k]; }

 private:
  std::map<std::string, std::string> m_;
};
// Stuff::Common::Logger().devnull(): the default `out` of init()
inline std::ostream& devnull()
{
  static std::ostream null(nullptr);
  return null;
}
}  // namespace Common

namespace Grid {
namespace BoundaryInfos {
struct AllDirichlet {
  static std::string static_id() { return "stuff.grid.boundaryinfo.alldirichlet"; }
  static Common::Configuration default_config() { return {{"type", static_id()}}; }
};
struct AllNeumann {
  static std::string static_id() { return "stuff.grid.boundaryinfo.allneumann"; }
  static Common::Configuration default_config() { return {{"type", static_id()}}; }
};
// boundary info config -> neighbour code of domain-boundary faces
inline int32_t boundary_code(const Common::Configuration& cfg)
{
  const std::string t = cfg.get("type", AllDirichlet::static_id());
  if (t == AllDirichlet::static_id() || t == "alldirichlet") return HDD_NBR_DIRICHLET;
  if (t == AllNeumann::static_id() || t == "allneumann") return HDD_NBR_NEUMANN;
  throw Exceptions::wrong_input_given("unknown boundary info type '" + t + "' (AllDirichlet / AllNeumann)");
}
}  // namespace BoundaryInfos

namespace Providers {
// Stuff::Grid::Providers::Cube + globalRefine: a structured nx x ny grid of [lower, upper] (quads, or the Kuhn
// triangulation for simplices) and its uniform refinements; level l has nx 2^l x ny 2^l squares
// (testcases/ESV2007.hh:123-129, testcases/spe10.hh:301-307, the refinement ladder of testcases/base.hh:92-103)
class Cube {
 public:
  Cube(int elem_type, std::array<double, 2> lower, std::array<double, 2> upper, std::array<int, 2> num_elements,
       int num_refinements = 0)
  {
    for (int l = 0; l <= num_refinements; ++l) {
      hdd_structured_desc d{elem_type, num_elements[0] << l, num_elements[1] << l, 1, 1, HDD_BOUNDARY_ALL_DIRICHLET, 0,
                            {lower[0], lower[1]}, {upper[0], upper[1]}};
      hdd_grid* g = nullptr;
      if (hdd_grid_create_structured(&d, &g) != HDD_OK)
        throw Exceptions::wrong_input_given(std::string("Providers::Cube: ") + hdd_last_error(nullptr));
      levels_.emplace_back(g, hdd_grid_destroy);
    }
  }
  int num_levels() const { return int(levels_.size()); }
  const hdd_grid* grid(int level) const
  {
    if (level < 0 || level >= num_levels())
      throw Exceptions::index_out_of_range("level " + std::to_string(level) + " not in [0, " +
                                           std::to_string(num_levels()) + ")");
    return levels_[size_t(level)].get();
  }

 private:
  std::vector<std::shared_ptr<hdd_grid>> levels_;
};
}  // namespace Providers
}  // namespace Grid
}  // namespace Stuff

namespace grid {
namespace Multiscale {
namespace Providers {
// grid::Multiscale::Providers::Cube with num_partitions [px py 1] (testcases/base.hh:150-191): one grid whose
// subdomain-major element order is the block numbering
class Cube {
 public:
  // oversampling_layers: the local_oversampled grid part of a subdomain is the subdomain plus this many
  // rings of face-neighbour elements (testcases/base.hh:169, "oversampling_layers", default 0)
  Cube(int elem_type, std::array<double, 2> lower, std::array<double, 2> upper, std::array<int, 2> num_elements,
       std::array<int, 2> num_partitions, int oversampling_layers = 0)
    : layers_(oversampling_layers)
  {
    hdd_structured_desc d{elem_type, num_elements[0], num_elements[1], num_partitions[0], num_partitions[1],
                          HDD_BOUNDARY_ALL_DIRICHLET, 0, {lower[0], lower[1]}, {upper[0], upper[1]}};
    hdd_grid* g = nullptr;
    if (hdd_grid_create_structured(&d, &g) != HDD_OK)
      throw Stuff::Exceptions::wrong_input_given(std::string("Multiscale::Providers::Cube: ") + hdd_last_error(nullptr));
    g_.reset(g, hdd_grid_destroy);
  }
  // 3d: n0 x n1 x n2 axis-aligned hexahedra carrying DG Q_degree, num_partitions [px py pz]
  Cube(std::array<double, 3> lower, std::array<double, 3> upper, std::array<int, 3> num_elements,
       std::array<int, 3> num_partitions, int oversampling_layers = 0, int degree = 1)
    : layers_(oversampling_layers)
  {
    hdd_structured3_desc d{num_elements[0], num_elements[1], num_elements[2], num_partitions[0], num_partitions[1],
                           num_partitions[2], HDD_BOUNDARY_ALL_DIRICHLET, degree,
                           {lower[0], lower[1], lower[2]}, {upper[0], upper[1], upper[2]}};
    hdd_grid* g = nullptr;
    if (hdd_grid_create_structured_3d(&d, &g) != HDD_OK)
      throw Stuff::Exceptions::wrong_input_given(std::string("Multiscale::Providers::Cube: ") + hdd_last_error(nullptr));
    g_.reset(g, hdd_grid_destroy);
  }
  // adopt a grid carrying a subdomain partition (not destroyed)
  explicit Cube(const hdd_grid* g) : g_(const_cast<hdd_grid*>(g), [](hdd_grid*) {}) {}
  const hdd_grid* grid() const { return g_.get(); }
  int num_subdomains() const
  {
    hdd_grid_info gi{};
    hdd_grid_get_info(g_.get(), &gi);
    return gi.n_subdomains;
  }
  int oversampling_layers() const { return layers_; }

 private:
  std::shared_ptr<hdd_grid> g_;
  int layers_ = 0;
};
}  // namespace Providers
}  // namespace Multiscale
}  // namespace grid

namespace HDD {
namespace LinearElliptic {

namespace internal {
inline void check(int rc, const char* what)
{
  if (rc == HDD_OK) return;
  const std::string msg = std::string(what) + ": " + hdd_last_error(nullptr);
  if (rc == HDD_ERR_RANGE) throw Stuff::Exceptions::index_out_of_range(msg);
  if (rc == HDD_ERR_INVALID) throw Stuff::Exceptions::wrong_input_given(msg);
  if (rc == HDD_ERR_UNSUPPORTED) throw NotImplemented(msg);
  throw Stuff::Exceptions::internal_error(msg);
}
inline void hip_check(hipError_t e, const char* what)
{
  if (e != hipSuccess) throw Stuff::Exceptions::internal_error(std::string(what) + ": " + hipGetErrorString(e));
}
// owning device buffer
template <class T>
class DeviceArray {
 public:
  DeviceArray() = default;
  explicit DeviceArray(size_t n) : n_(n) { if (n) hip_check(hipMalloc(&p_, n * sizeof(T)), "hipMalloc"); }
  DeviceArray(const std::vector<T>& h) : DeviceArray(h.size()) { upload(h); }
  // a view of n elements inside an allocation that `owner` keeps alive (batched block operators)
  DeviceArray(T* p, size_t n, std::shared_ptr<const void> owner) : p_(p), n_(n), owner_(std::move(owner)) {}
  DeviceArray(const DeviceArray&) = delete;
  DeviceArray& operator=(const DeviceArray&) = delete;
  DeviceArray(DeviceArray&& o) noexcept : p_(o.p_), n_(o.n_), owner_(std::move(o.owner_)) { o.p_ = nullptr; o.n_ = 0; }
  DeviceArray& operator=(DeviceArray&& o) noexcept
  {
    if (this != &o) {
      release();
      p_ = o.p_; n_ = o.n_; owner_ = std::move(o.owner_);
      o.p_ = nullptr; o.n_ = 0;
    }
    return *this;
  }
  ~DeviceArray() { release(); }
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
  void release()
  {
    if (p_ && !owner_) (void)hipFree(p_);
    owner_.reset();
  }
  T* p_ = nullptr;
  size_t n_ = 0;
  std::shared_ptr<const void> owner_;   // set for views: the allocation is the owner's
};
// a device-to-device copy into an allocation of its own
template <class T>
std::shared_ptr<DeviceArray<T>> device_copy(const DeviceArray<T>& a)
{
  auto o = std::make_shared<DeviceArray<T>>(a.size());
  if (a.size()) hip_check(hipMemcpy(o->get(), a.get(), a.size() * sizeof(T), hipMemcpyDeviceToDevice), "D2D");
  return o;
}
using Timer = std::chrono::steady_clock;
inline double seconds_since(Timer::time_point t0)
{
  return std::chrono::duration<double>(Timer::now() - t0).count();
}
}  // namespace internal

namespace Pymor {
// theta(mu) = scale * mu^power: the ParameterFunctional forms of the reference's parametric problems ("mu",
// problems/OS2014.hh:74; "-1.0*mu", problems/spe10.hh:167) and their products, which SWIPDG registers for
// the kappa_p x g_D,q right-hand-side components ("(" + theta_p + ")*(" + theta_q + ")", swipdg.hh:317-330)
class ParameterFunctional {
 public:
  ParameterFunctional(std::string name = "mu", std::string expression = "mu", double scale = 1.0, int power = 1)
    : name_(std::move(name)), expression_(std::move(expression)), scale_(scale), power_(power) {}
  double evaluate(double mu) const { return scale_ * std::pow(mu, power_); }
  const std::string& expression() const { return expression_; }
  const std::string& name() const { return name_; }
  ParameterFunctional operator*(const ParameterFunctional& o) const
  {
    return ParameterFunctional(name_, "(" + expression_ + ")*(" + o.expression_ + ")", scale_ * o.scale_,
                               power_ + o.power_);
  }
  bool operator==(const ParameterFunctional& o) const
  {
    return name_ == o.name_ && scale_ == o.scale_ && power_ == o.power_;
  }

 private:
  std::string name_, expression_;
  double scale_;
  int power_;
};
}  // namespace Pymor

namespace Problems {
// a (localizable) scalar function as the assembly path evaluates it: analytic kinds are evaluated on the
// device at quadrature points; Checkerboard / Indicator (order 0, entity-centre based) are evaluated at the
// element barycentres on the host and uploaded as per-element values
struct ScalarFunction {
  enum Host { DEVICE = 0, CHECKERBOARD = 1, INDICATOR = 2, INDICATOR_SUM = 3 };
  int kind = HDD_FN_CONST;
  int host = DEVICE;
  int order = 0;
  double c = 1.0, b = 0.0, kx = 0.0, ky = 0.0;
  std::vector<double> per_element;   // PER_ELEM: global element order
  // CHECKERBOARD: cells (x fastest) on [lower, upper]; INDICATOR(_SUM): boxes [5k..5k+4] = lx, ly, ux, uy, value;
  // FLATTOP (device kind): boxes [7k..7k+6] = lx, ly, ux, uy, layer_x, layer_y, value
  std::array<double, 2> lower{{0.0, 0.0}}, upper{{1.0, 1.0}};
  int ncx = 1, ncy = 1;
  std::vector<double> table;

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
  // Stuff::Functions::Checkerboard (the Spe10::Model1 permeability field, problems/spe10.hh:151-156)
  static ScalarFunction checkerboard(std::array<double, 2> lower, std::array<double, 2> upper, int ncx, int ncy,
                                     std::vector<double> cells)
  {
    if (int64_t(cells.size()) != int64_t(ncx) * ncy)
      throw Stuff::Exceptions::wrong_input_given("Checkerboard: need ncx * ncy cell values");
    ScalarFunction f; f.kind = HDD_FN_PER_ELEM; f.host = CHECKERBOARD; f.lower = lower; f.upper = upper;
    f.ncx = ncx; f.ncy = ncy; f.table = std::move(cells); return f;
  }
  // Stuff::Functions::Indicator (problems/spe10.hh:144, 157): value of the first box holding the entity centre
  static ScalarFunction indicator(std::vector<std::array<double, 5>> boxes)
  {
    ScalarFunction f; f.kind = HDD_FN_PER_ELEM; f.host = INDICATOR;
    for (const auto& bx : boxes) f.table.insert(f.table.end(), bx.begin(), bx.end());
    return f;
  }
  // c + b * (sum of one-box Indicators): Stuff::Functions::make_sum of the Spe10 channel's per-box Indicators
  // (problems/spe10.hh:139-148 with channel_boundary_layer == 0), evaluated at the entity centre
  static ScalarFunction indicator_sum(std::vector<std::array<double, 5>> boxes, double c = 0.0, double b = 1.0)
  {
    ScalarFunction f; f.kind = HDD_FN_PER_ELEM; f.host = INDICATOR_SUM; f.c = c; f.b = b;
    for (const auto& bx : boxes) f.table.insert(f.table.end(), bx.begin(), bx.end());
    return f;
  }
  // c + b * (sum of dune-stuff FlatTop functions), the Spe10 channel with channel_boundary_layer != 0
  // (problems/spe10.hh:213-222); evaluated on the device at quadrature points (HDD_FN_FLATTOP).  order: the
  // integration order (restated assumption: 3, the degree of the transitions per coordinate)
  static ScalarFunction flattop_sum(std::vector<std::array<double, 7>> boxes, double c = 0.0, double b = 1.0,
                                    int order = 3)
  {
    ScalarFunction f; f.kind = HDD_FN_FLATTOP; f.c = c; f.b = b; f.order = order;
    for (const auto& bx : boxes) {
      if (!(bx[4] > 0.0 && bx[5] > 0.0))
        throw Stuff::Exceptions::wrong_input_given("FlatTop: the boundary layer must be positive (0: Indicator)");
      f.table.insert(f.table.end(), bx.begin(), bx.end());
    }
    return f;
  }
  bool is_zero() const { return kind == HDD_FN_CONST && host == DEVICE && c == 0.0; }
};

struct TensorFunction {
  enum Host { DEVICE = 0, CHECKERBOARD_ISO = 1 };
  int kind = HDD_TENSOR_CONST;
  int host = DEVICE;
  double c[6] = {1.0, 0.0, 1.0, 0.0, 0.0, 0.0};   // 2d a11 a12 a22; 3d a11 a12 a13 a22 a23 a33 (see identity3d)
  std::vector<double> per_element;   // ISO: [ne]; SYM: [3 | 6][ne] (global element order)
  ScalarFunction field;              // CHECKERBOARD_ISO: A = field(x) I
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
  static TensorFunction symmetric(std::vector<double> v)
  {
    TensorFunction t; t.kind = HDD_TENSOR_SYM_PER_ELEM; t.per_element = std::move(v); return t;
  }
  // Stuff::Functions::Spe10::Model1 (problems/spe10.hh:151-156): checkerboard value times the identity
  static TensorFunction spe10_model1(std::vector<double> cells, std::array<double, 2> lower = {{0.0, 0.0}},
                                     std::array<double, 2> upper = {{5.0, 1.0}}, int ncx = 100, int ncy = 20)
  {
    TensorFunction t; t.kind = HDD_TENSOR_ISO_PER_ELEM; t.host = CHECKERBOARD_ISO;
    t.field = ScalarFunction::checkerboard(lower, upper, ncx, ncy, std::move(cells));
    return t;
  }
};

// Pymor AffinelyDecomposableDefault: f(mu) = f_aff + sum_q theta_q(mu) f_q; a plain ScalarFunction converts
// to the nonparametric form (affine part only)
struct AffinelyDecomposedFunction {
  bool has_affine_part = true;
  ScalarFunction affine_part = ScalarFunction::constant(1.0);
  std::vector<ScalarFunction> components;
  std::vector<Pymor::ParameterFunctional> coefficients;
  AffinelyDecomposedFunction() = default;
  AffinelyDecomposedFunction(const ScalarFunction& f) : affine_part(f) {}   // NOLINT: implicit by design
  int num_components() const { return int(components.size()); }
  bool parametric() const { return !components.empty(); }
  void register_component(ScalarFunction f, Pymor::ParameterFunctional theta)
  {
    components.push_back(std::move(f));
    coefficients.push_back(std::move(theta));
  }
};
using DiffusionFactor = AffinelyDecomposedFunction;

struct Problem {
  DiffusionFactor diffusion_factor;
  TensorFunction diffusion_tensor;
  bool diffusion_tensor_parametric = false;
  bool diffusion_tensor_empty = false;
  AffinelyDecomposedFunction force = ScalarFunction::constant(0.0);
  AffinelyDecomposedFunction dirichlet = ScalarFunction::constant(0.0);
  AffinelyDecomposedFunction neumann = ScalarFunction::constant(0.0);
};

// Problems::ZeroBoundary (problems/zero-boundary.hh:54-60): same data, Dirichlet and Neumann values 0
inline Problem ZeroBoundary(const Problem& p)
{
  Problem z = p;
  z.dirichlet = ScalarFunction::constant(0.0);
  z.neumann = ScalarFunction::constant(0.0);
  return z;
}

// ESV2007 (problems/ESV2007.hh:75-81): kappa = 1, A = I, f = 1/2 pi^2 cos(pi x/2) cos(pi y/2), g_D = g_N = 0
inline Problem ESV2007()
{
  Problem p;
  p.force = ScalarFunction::cos_product(0.5 * M_PI * M_PI, 0.5 * M_PI, 0.5 * M_PI, 0.0, 3);
  return p;
}

// OS2014::ParametricESV2007 (problems/OS2014.hh:63-76, 106-113): kappa(mu) = 1 + 3/4 sin(4 pi (x + y/2))
// - mu 3/4 sin(4 pi (x + y/2)), A = I, f = ESV2007 Testcase1Force 1/2 pi^2 cos(pi x/2) cos(pi y/2)
// (OS2014.hh:48, 110), g_D = g_N = 0; integration order 3 (OS2014.hh:86-96)
inline Problem OS2014()
{
  Problem p;
  const double kx = 4.0 * M_PI, ky = 2.0 * M_PI;
  p.diffusion_factor.affine_part = ScalarFunction::sinusoid(1.0, 0.75, kx, ky, 3);
  p.diffusion_factor.register_component(ScalarFunction::sinusoid(0.0, -0.75, kx, ky, 3),
                                        Pymor::ParameterFunctional("mu", "mu", 1.0));
  p.force = ScalarFunction::cos_product(0.5 * M_PI * M_PI, 0.5 * M_PI, 0.5 * M_PI, 0.0, 3);
  return p;
}

// the FlatTop default boundary layer the Spe10::Model1 default config takes (problems/spe10.hh:86:
// FlatTopFunctionType::default_config()["boundary_layer"]); dune-stuff is absent here, so this is the
// restated default (1e-1 per coordinate), unverifiable
inline std::array<double, 2> flattop_default_boundary_layer() { return {{0.1, 0.1}}; }

// Spe10::Model1 (problems/spe10.hh:131-185): A = permeability checkerboard (100 x 20 cells on [0,5]x[0,1]),
// force = Indicator(force boxes), g_D = g_N = 0; the channel is the sum of one function per channel box
// (139-148): an Indicator when channel_boundary_layer == 0 (the parametric test case, testcases/spe10.hh:257),
// else a FlatTop with that boundary layer (213-222); diffusion factor 1 + 0.9 channel (175-179), or with
// parametric_channel the affine part 1 + channel and the component channel with theta = -1.0*mu (160-172).
// Integration order of a FlatTop channel: flattop_order (restated assumption 3, see ScalarFunction::flattop_sum).
inline Problem Spe10Model1(std::vector<double> permeability, std::vector<std::array<double, 5>> channel,
                           std::vector<std::array<double, 5>> forces, bool parametric_channel,
                           std::array<double, 2> channel_boundary_layer = flattop_default_boundary_layer(),
                           int flattop_order = 3, std::array<double, 2> lower_left = {{0.0, 0.0}},
                           std::array<double, 2> upper_right = {{5.0, 1.0}})
{
  Problem p;
  p.diffusion_tensor = TensorFunction::spe10_model1(std::move(permeability), lower_left, upper_right);
  p.force = ScalarFunction::indicator(std::move(forces));
  if (channel.empty()) return p;   // no channel: diffusion factor 1 + 0.9 * 0 (problems/spe10.hh:141-142)
  const bool indicator = channel_boundary_layer[0] == 0.0 && channel_boundary_layer[1] == 0.0;
  auto channel_fn = [&](double c, double b) {
    if (indicator) return ScalarFunction::indicator_sum(channel, c, b);
    std::vector<std::array<double, 7>> ft;
    for (const auto& bx : channel)
      ft.push_back({{bx[0], bx[1], bx[2], bx[3], channel_boundary_layer[0], channel_boundary_layer[1], bx[4]}});
    return ScalarFunction::flattop_sum(ft, c, b, flattop_order);
  };
  p.diffusion_factor.affine_part = parametric_channel ? channel_fn(1.0, 1.0) : channel_fn(1.0, 0.9);
  if (parametric_channel)
    p.diffusion_factor.register_component(channel_fn(0.0, 1.0), Pymor::ParameterFunctional("mu", "-1.0*mu", -1.0));
  return p;
}

// Spe10::Model1 from its data file, with the reference ctor's arguments in its order (problems/spe10.hh:111-125):
// the permeability checkerboard on [lower_left, upper_right] read by hdd_spe10_model1_read with the Model1
// min / max values (151-156; dune-stuff's reader restated, parity unpinned); the rest as the vector form above
inline Problem Spe10Model1(const std::string& filename, std::array<double, 2> lower_left,
                           std::array<double, 2> upper_right, std::vector<std::array<double, 5>> channel_values,
                           std::vector<std::array<double, 5>> force_values,
                           std::array<double, 2> channel_boundary_layer = flattop_default_boundary_layer(),
                           bool parametric_channel = false, int flattop_order = 3)
{
  std::vector<double> perm(HDD_SPE10_MODEL1_CELLS);
  internal::check(hdd_spe10_model1_read(filename.c_str(), HDD_SPE10_MODEL1_MIN, HDD_SPE10_MODEL1_MAX, perm.data()),
                  "hdd_spe10_model1_read");
  return Spe10Model1(std::move(perm), std::move(channel_values), std::move(force_values), parametric_channel,
                     channel_boundary_layer, flattop_order, lower_left, upper_right);
}
}  // namespace Problems

namespace Parallel {
// the face-halo transport of a ShardedBlockSWIPDG (hdd_comm): RCCL between one process per GPU, an existing
// ncclComm_t, a host callback (MPI, an in-process mailbox, ...), or the in-process device transport (thread
// ranks, RCCL's stream schedule with device copies)
class Communicator {
 public:
  Communicator() = default;   // no peers (a single rank)
  static std::string rccl_unique_id()
  {
    std::string id(HDD_RCCL_ID_BYTES, '\0');
    internal::check(hdd_rccl_get_unique_id(&id[0]), "hdd_rccl_get_unique_id");
    return id;
  }
  static Communicator rccl(const std::string& unique_id, int nranks, int rank, int hip_device)
  {
    if (unique_id.size() != HDD_RCCL_ID_BYTES) throw Stuff::Exceptions::wrong_input_given("RCCL unique id size");
    hdd_comm* c = nullptr;
    internal::check(hdd_comm_create_rccl(unique_id.data(), nranks, rank, hip_device, &c), "hdd_comm_create_rccl");
    return Communicator(c);
  }
  static Communicator wrap_rccl(void* nccl_comm, int hip_device)
  {
    hdd_comm* c = nullptr;
    internal::check(hdd_comm_wrap_rccl(nccl_comm, hip_device, &c), "hdd_comm_wrap_rccl");
    return Communicator(c);
  }
  static Communicator host(hdd_host_exchange_fn fn, void* user, int hip_device)
  {
    hdd_comm* c = nullptr;
    internal::check(hdd_comm_create_host(fn, user, hip_device, &c), "hdd_comm_create_host");
    return Communicator(c);
  }
  // in-process device transport: rank `rank` of the hub's thread ranks (the RCCL stream schedule, device copies)
  static Communicator device(const std::shared_ptr<hdd_device_hub>& hub, int rank, int hip_device)
  {
    hdd_comm* c = nullptr;
    internal::check(hdd_comm_create_device(hub.get(), rank, hip_device, &c), "hdd_comm_create_device");
    return Communicator(c);
  }
  static std::shared_ptr<hdd_device_hub> device_hub(int nranks)
  {
    hdd_device_hub* h = nullptr;
    internal::check(hdd_device_hub_create(nranks, &h), "hdd_device_hub_create");
    return std::shared_ptr<hdd_device_hub>(h, hdd_device_hub_destroy);
  }
  hdd_comm* get() const { return c_.get(); }

 private:
  explicit Communicator(hdd_comm* c) : c_(c, hdd_comm_destroy) {}
  std::shared_ptr<hdd_comm> c_;
};
}  // namespace Parallel

namespace Discretizations {

// CSR pattern resident on the device.  Patterns are built and block operators extracted on the device
// (hdd_pattern_*_device, hdd_block_operator_map_device); host copies of row_ptr / col are downloaded only
// when a caller asks for them (at C5 scale the column array alone is tens of GB).
class Pattern {
 public:
  int64_t rows = 0, cols = 0, nnz = 0;
  internal::DeviceArray<int64_t> d_row_ptr, d_elem_ptr;
  internal::DeviceArray<int32_t> d_col;
  hdd_csr csr() const { return hdd_csr{rows, cols, nnz, d_row_ptr.get(), d_col.get(), d_elem_ptr.get()}; }
  const std::vector<int64_t>& row_ptr() const
  {
    std::lock_guard<std::mutex> lock(m_);
    if (h_row_ptr_.size() != size_t(rows + 1)) {
      h_row_ptr_ = d_row_ptr.download();
      h_row_ptr_.resize(size_t(rows + 1));
    }
    return h_row_ptr_;
  }
  const std::vector<int32_t>& col() const
  {
    std::lock_guard<std::mutex> lock(m_);
    if (h_col_.size() != size_t(nnz)) {
      h_col_ = d_col.download();
      h_col_.resize(size_t(nnz));
    }
    return h_col_;
  }

 private:
  mutable std::mutex m_;
  mutable std::vector<int64_t> h_row_ptr_;
  mutable std::vector<int32_t> h_col_;
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
  std::vector<double> affine_part() const { return trimmed(*affine); }
  std::vector<double> component(int q) const { return trimmed(*comps.at(size_t(q))); }
  const Pymor::ParameterFunctional& coefficient(int q) const { return coefficients.at(size_t(q)); }
  // A copy whose value arrays are its own (device-to-device copies; the immutable pattern is shared).  A plain
  // copy of this class shares the value arrays, as the reference's containers share their backend until a write.
  AffinelyDecomposedMatrix clone() const
  {
    AffinelyDecomposedMatrix c = *this;
    if (affine) c.affine = internal::device_copy(*affine);
    for (auto& q : c.comps) q = internal::device_copy(*q);
    return c;
  }
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

 private:
  std::vector<double> trimmed(const internal::DeviceArray<double>& a) const
  {
    auto h = a.download();
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
  bool parametric() const { return !comps.empty(); }
  std::vector<double> affine_part() const { auto h = affine->download(); h.resize(size_t(size)); return h; }
  std::vector<double> component(int q) const { auto h = comps.at(size_t(q))->download(); h.resize(size_t(size)); return h; }
  const Pymor::ParameterFunctional& coefficient(int q) const { return coefficients.at(size_t(q)); }
  AffinelyDecomposedVector clone() const   // (as AffinelyDecomposedMatrix::clone)
  {
    AffinelyDecomposedVector c = *this;
    if (affine) c.affine = internal::device_copy(*affine);
    for (auto& q : c.comps) q = internal::device_copy(*q);
    return c;
  }
  // b(mu) = b_aff + sum_q theta_q(mu) b_q (host)
  std::vector<double> freeze_parameter(double mu) const
  {
    std::vector<double> out = affine ? affine_part() : std::vector<double>(size_t(size), 0.0);
    for (int q = 0; q < num_components(); ++q) {
      const auto c = component(q);
      const double t = coefficients[size_t(q)].evaluate(mu);
      for (size_t i = 0; i < out.size(); ++i) out[i] += t * c[i];
    }
    return out;
  }
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

// the element columns a function is localized to: n local columns with barycentres and global ids; with
// halo_ghosts the ghost columns are left NaN (a sharded assembly fills them through the face halo)
struct ElementView {
  int64_t n = 0, own_begin = 0, own_end = 0;
  int dim = 2;
  const double* centers = nullptr;    // [dim][n]
  const int64_t* gid = nullptr;       // [n]
  int64_t n_global = 0;
  bool halo_ghosts = false;
};

inline std::vector<double> localize(const Problems::ScalarFunction& f, const ElementView& v)
{
  std::vector<double> h(static_cast<size_t>(v.n));
  if (f.host == Problems::ScalarFunction::CHECKERBOARD || f.host == Problems::ScalarFunction::INDICATOR ||
      f.host == Problems::ScalarFunction::INDICATOR_SUM) {
    if (v.dim != 2) throw NotImplemented("Checkerboard / Indicator functions are 2d");
    if (f.host == Problems::ScalarFunction::CHECKERBOARD)
      internal::check(hdd_checkerboard(v.n, v.centers, f.lower.data(), f.upper.data(), f.ncx, f.ncy, f.table.data(),
                                       h.data()), "hdd_checkerboard");
    else if (f.host == Problems::ScalarFunction::INDICATOR)
      internal::check(hdd_indicator(v.n, v.centers, int32_t(f.table.size() / 5), f.table.data(), h.data()),
                      "hdd_indicator");
    else {   // INDICATOR_SUM: c + b * sum of the boxes' values
      internal::check(hdd_indicator_sum(v.n, v.centers, int32_t(f.table.size() / 5), f.table.data(), h.data()),
                      "hdd_indicator_sum");
      for (auto& x : h) x = f.c + f.b * x;
    }
  } else {
    if (int64_t(f.per_element.size()) != v.n_global)
      throw Stuff::Exceptions::wrong_input_given("per-element function: " + std::to_string(f.per_element.size()) +
                                                 " values for " + std::to_string(v.n_global) + " elements");
    for (int64_t e = 0; e < v.n; ++e) h[size_t(e)] = f.per_element[size_t(v.gid[e])];
  }
  if (v.halo_ghosts)
    for (int64_t e = 0; e < v.n; ++e)
      if (e < v.own_begin || e >= v.own_end) h[size_t(e)] = std::numeric_limits<double>::quiet_NaN();
  return h;
}

// a scalar function bound to the device (per-element values uploaded, kept alive with the descriptor)
struct DeviceFn {
  hdd_scalar_fn fn{};
  std::shared_ptr<internal::DeviceArray<double>> pe, table;
  DeviceFn() = default;
  DeviceFn(const Problems::ScalarFunction& f, const ElementView& v)
  {
    if (f.kind == HDD_FN_PER_ELEM) pe = std::make_shared<internal::DeviceArray<double>>(localize(f, v));
    if (f.kind == HDD_FN_FLATTOP) {
      if (v.dim != 2) throw NotImplemented("FlatTop functions are 2d");
      table = std::make_shared<internal::DeviceArray<double>>(f.table.empty() ? std::vector<double>(1, 0.0) : f.table);
    }
    fn = hdd_scalar_fn{f.kind, f.order, f.c, f.b, f.kx, f.ky, pe ? pe->get() : nullptr,
                       table ? table->get() : nullptr, int32_t(f.table.size() / HDD_FLATTOP_REC), 0};
  }
};

struct DeviceTensor {
  hdd_tensor_fn fn{};
  std::shared_ptr<internal::DeviceArray<double>> pe;
  DeviceTensor() = default;
  DeviceTensor(const Problems::TensorFunction& T, const ElementView& v)
  {
    fn = hdd_tensor_fn{T.kind, 0, {T.c[0], T.c[1], T.c[2], T.c[3], T.c[4], T.c[5]}, nullptr};
    if (T.kind == HDD_TENSOR_CONST) return;
    std::vector<double> h;
    if (T.host == Problems::TensorFunction::CHECKERBOARD_ISO) {
      h = localize(T.field, v);
    } else {
      const int rows = T.kind == HDD_TENSOR_ISO_PER_ELEM ? 1 : (v.dim == 3 ? 6 : 3);
      if (int64_t(T.per_element.size()) != rows * v.n_global)
        throw Stuff::Exceptions::wrong_input_given("per-element tensor: wrong number of values");
      h.resize(size_t(rows * v.n));
      for (int r = 0; r < rows; ++r)
        for (int64_t e = 0; e < v.n; ++e) {
          const bool ghost = e < v.own_begin || e >= v.own_end;
          h[size_t(r * v.n + e)] = (v.halo_ghosts && ghost) ? std::numeric_limits<double>::quiet_NaN()
                                                             : T.per_element[size_t(r * v.n_global + v.gid[e])];
        }
    }
    pe = std::make_shared<internal::DeviceArray<double>>(h);
    fn.per_elem = pe->get();
  }
};

inline const std::vector<std::string>& all_products()
{
  static const std::vector<std::string> p = {"l2", "h1_semi", "elliptic", "boundary_l2", "penalty", "energy"};
  return p;
}
}  // namespace detail

// ------------------------------------------------------------------------------------------------
// SWIPDG (swipdg.hh:109-520)
// ------------------------------------------------------------------------------------------------
class SWIPDG {
 public:
  // which elements the discretization lives on: the whole grid (leaf / level layer) or one subdomain of a
  // multiscale grid (ChooseLayer::local: faces to other subdomains are domain boundary, local numbering)
  enum class Layer { leaf, local };

  // swipdg.hh:159-163: level provider, boundary info config, problem, level, requested products
  SWIPDG(const Stuff::Grid::Providers::Cube& grid_provider, const Stuff::Common::Configuration& bound_inf_cfg,
         const Problems::Problem& prob, int level_or_subdomain = 0,
         const std::vector<std::string>& only_these_products = {}, int hip_device = 0)
    : SWIPDG(grid_provider.grid(level_or_subdomain), bound_inf_cfg, prob, Layer::leaf, 0, only_these_products,
             hip_device) {}

  // swipdg.hh:180-198: multiscale provider -> the (local layer) discretization of subdomain `level_or_subdomain`
  SWIPDG(const grid::Multiscale::Providers::Cube& grid_provider, const Stuff::Common::Configuration& bound_inf_cfg,
         const Problems::Problem& prob, int level_or_subdomain = 0,
         const std::vector<std::string>& only_these_products = {}, int hip_device = 0)
    : SWIPDG(grid_provider.grid(), bound_inf_cfg, prob, Layer::local, level_or_subdomain, only_these_products,
             hip_device) {}

  // convenience: the whole grid with the boundary the grid carries and every product available
  SWIPDG(const hdd_grid* grid, const Problems::Problem& problem, int hip_device = 0)
    : SWIPDG(grid, Stuff::Common::Configuration(), problem, Layer::leaf, 0, detail::all_products(), hip_device,
             /*grid_boundary=*/true) {}

  // a discretization on a grid of its own whose elements are a subset of a parent grid's (parent_ids: parent
  // element id of every element; per-element functions given in the parent's numbering are read through it)
  SWIPDG(std::shared_ptr<hdd_grid> subset_grid, std::vector<int64_t> parent_ids, int64_t n_parent,
         const Stuff::Common::Configuration& bound_inf_cfg, const Problems::Problem& problem,
         const std::vector<std::string>& only_these_products, int hip_device = 0)
    : SWIPDG(subset_grid.get(), bound_inf_cfg, problem, Layer::leaf, 0, only_these_products, hip_device, false,
             &parent_ids, n_parent)
  {
    owned_grid_ = std::move(subset_grid);
  }

  SWIPDG(const hdd_grid* grid, const Stuff::Common::Configuration& bound_inf_cfg, const Problems::Problem& problem,
         Layer layer, int subdomain, const std::vector<std::string>& only_these_products, int hip_device = 0,
         bool grid_boundary = false, const std::vector<int64_t>* parent_ids = nullptr, int64_t n_parent = 0)
    : grid_(grid), problem_(problem), layer_(layer), subdomain_(subdomain), only_these_products_(only_these_products)
  {
    // swipdg.hh:172-176
    if (problem.diffusion_tensor_parametric) throw NotImplemented("The diffusion tensor must not be parametric!");
    if (problem.diffusion_tensor_empty)
      throw Stuff::Exceptions::wrong_input_given("The diffusion tensor must not be empty!");
    for (const auto& id : only_these_products)
      if (std::find(detail::all_products().begin(), detail::all_products().end(), id) == detail::all_products().end())
        throw Stuff::Exceptions::wrong_input_given("unknown product '" + id + "'");
    internal::check(hdd_grid_get_info(grid, &info_), "hdd_grid_get_info");
    boundary_code_ = grid_boundary ? 0 : Stuff::Grid::BoundaryInfos::boundary_code(bound_inf_cfg);
    internal::check(hdd_ctx_create(hip_device, &ctx_), "hdd_ctx_create");
    int32_t s0 = 0, s1 = info_.n_subdomains;
    if (layer == Layer::local) {
      if (subdomain < 0 || subdomain >= info_.n_subdomains)
        throw Stuff::Exceptions::index_out_of_range("Given subdomain " + std::to_string(subdomain) +
                                                    " too large (has to be smaller than " +
                                                    std::to_string(info_.n_subdomains) + "!");
      s0 = subdomain;
      s1 = subdomain + 1;
    }
    internal::check(hdd_local_create(grid, s0, s1, &local_), "hdd_local_create");
    internal::check(hdd_local_get_info(local_, &linfo_), "hdd_local_get_info");
    degree_ = detail::degree_of(info_);
    build_view();
    if (parent_ids) {   // per-element data of the parent grid: look it up through the parent ids
      if (int64_t(parent_ids->size()) != info_.n_elements)
        throw Stuff::Exceptions::wrong_input_given("parent_ids: one id per element expected");
      parent_gid_.resize(gid_.size());
      for (size_t e = 0; e < gid_.size(); ++e) parent_gid_[e] = (*parent_ids)[size_t(gid_[e])];
      view_.gid = parent_gid_.data();
      view_.n_global = n_parent;
    }
    build_pattern();
  }
  virtual ~SWIPDG()
  {
    if (local_) hdd_local_destroy(local_);
    if (ctx_) hdd_ctx_destroy(ctx_);
  }
  SWIPDG(const SWIPDG&) = delete;
  SWIPDG& operator=(const SWIPDG&) = delete;

  static std::string static_id() { return "hdd.linearelliptic.discretizations.containerbased.swipdg"; }

  const Pattern& pattern() const { return *pattern_; }

  // assembles the system matrix (every diffusion-factor component + the affine part), the right-hand side and
  // the requested products on the device; idempotent (container_based_initialized_, swipdg.hh:208, 510)
  void init(std::ostream& out = Stuff::Common::devnull(), const std::string& prefix = "")
  {
    if (initialized_) return;
    out << prefix << "assembling... " << std::flush;
    const auto t0 = internal::Timer::now();
    upload_mesh();
    const hdd_csr pat = pattern_->csr();
    matrix_ = AffinelyDecomposedMatrix();
    matrix_.pattern = pattern_;
    matrix_.ctx = ctx_;
    const auto& K = problem_.diffusion_factor;
    matrix_.coefficients = K.coefficients;
    for (const auto& c : K.components) matrix_.comps.push_back(assemble_lhs(c, pat));
    if (K.has_affine_part) matrix_.affine = assemble_lhs(K.affine_part, pat);
    assemble_rhs();
    products_.clear();
    for (const auto& id : only_these_products_) products_[id] = std::make_shared<AffinelyDecomposedMatrix>(product(id));
    internal::hip_check(hipDeviceSynchronize(), "init");
    out << "done (took " << internal::seconds_since(t0) << "s)" << std::endl;
    initialized_ = true;
  }

  // base.hh:240-270
  const AffinelyDecomposedMatrix& system_matrix() const
  {
    assert_everything_is_ready();
    return matrix_;
  }
  const AffinelyDecomposedMatrix& get_operator() const { return system_matrix(); }
  const AffinelyDecomposedVector& rhs() const
  {
    assert_everything_is_ready();
    return rhs_;
  }
  const AffinelyDecomposedVector& get_rhs() const { return rhs(); }

  // base.hh:272-291: only the products requested in the ctor (only_these_products, swipdg.hh:496-508)
  std::vector<std::string> available_products() const
  {
    std::vector<std::string> ret;
    for (const auto& kv : products_) ret.push_back(kv.first);
    return ret;
  }
  const AffinelyDecomposedMatrix& get_product(const std::string& id) const
  {
    if (products_.empty())
      throw Stuff::Exceptions::you_are_using_this_wrong("Do not call get_product() if available_products() is empty!");
    const auto it = products_.find(id);
    if (it == products_.end()) throw Stuff::Exceptions::wrong_input_given("Product '" + id + "' not available!");
    return *it->second;
  }

  // true if no Dirichlet face was found (DirichletDetector, swipdg.hh:219, 488-489)
  bool purely_neumann() const
  {
    assert_everything_is_ready();
    return purely_neumann_;
  }
  int64_t num_dofs() const { return pattern_->rows; }
  hdd_ctx* context() const { return ctx_; }
  const hdd_grid* grid() const { return grid_; }
  const Problems::Problem& problem() const { return problem_; }
  int polynomial_order() const { return degree_; }
  Layer layer() const { return layer_; }
  int subdomain() const { return subdomain_; }

 protected:
  void assert_everything_is_ready() const
  {
    if (!initialized_)
      throw Stuff::Exceptions::you_are_using_this_wrong("The user has to call init() before calling any other method!");
  }

  // host view of the elements: neighbour codes with the boundary info applied, columns (global / local)
  void build_view()
  {
    const int64_t n = linfo_.n_local;
    coords_.assign(size_t(info_.dim * info_.nvpe * n), 0.0);
    nbrs_.assign(size_t(info_.nfaces * n), 0);
    finfo_.assign(size_t(n), 0u);
    gid_.assign(size_t(n), 0);
    centers_.assign(size_t(info_.dim * n), 0.0);
    internal::check(hdd_local_fill(local_, coords_.data(), nbrs_.data(), finfo_.data(), gid_.data(), nullptr),
                    "hdd_local_fill");
    internal::check(hdd_local_centers(local_, centers_.data()), "hdd_local_centers");
    const int64_t ob = linfo_.own_begin, oe = linfo_.own_end;
    for (int f = 0; f < info_.nfaces; ++f)
      for (int64_t e = ob; e < oe; ++e) {
        int32_t& nb = nbrs_[size_t(f * n + e)];
        // faces to other subdomains are boundary of a local-layer discretization (its grid part ends there)
        if (layer_ == Layer::local && nb >= 0 && (nb < ob || nb >= oe)) nb = HDD_NBR_DIRICHLET;
        if (nb < 0 && boundary_code_ != 0) nb = boundary_code_;
      }
    // local layer: columns in the subdomain's own numbering (mapToGlobal is the block mapper's job)
    cols_.assign(size_t(n), 0);
    for (int64_t e = 0; e < n; ++e) cols_[size_t(e)] = layer_ == Layer::local ? e - ob : gid_[size_t(e)];
    n_cols_ = layer_ == Layer::local ? (oe - ob) * info_.nb : info_.n_elements * info_.nb;
    view_ = detail::ElementView{n, ob, oe, info_.dim, centers_.data(), gid_.data(), info_.n_elements, false};
  }

  // EllipticSWIPDG::pattern (swipdg.hh:169) on the device: hdd_pattern_elem_ptr_device + hdd_pattern_fill_device
  // over the neighbour codes with the boundary info applied, columns through cols_ (global ids, or the
  // subdomain's own numbering for the local layer).  volume: the element-diagonal pattern of the l2 / h1 /
  // elliptic / boundary products (no face neighbours: every neighbour code is a boundary code)
  std::shared_ptr<Pattern> device_pattern(bool volume) const
  {
    auto P = std::make_shared<Pattern>();
    const int64_t n = linfo_.n_local, own = linfo_.own_end - linfo_.own_begin;
    internal::DeviceArray<int32_t> none;
    const int32_t* nb = d_nbrs_.get();
    if (volume) {
      none = internal::DeviceArray<int32_t>(size_t(info_.nfaces * n) + 1);
      internal::hip_check(hipMemset(none.get(), 0xff, none.size() * sizeof(int32_t)), "device_pattern");   // -1
      nb = none.get();
    }
    const hdd_mesh m{info_.elem_type, degree_, n, linfo_.own_begin, linfo_.own_end, nullptr, nb, nullptr, nullptr, nullptr};
    P->rows = own * info_.nb;
    P->cols = n_cols_;
    P->d_elem_ptr = internal::DeviceArray<int64_t>(size_t(own + 1));
    internal::check(hdd_pattern_elem_ptr_device(ctx_, &m, info_.nb, P->d_elem_ptr.get(), &P->nnz, nullptr),
                    "hdd_pattern_elem_ptr_device");
    P->d_row_ptr = internal::DeviceArray<int64_t>(size_t(P->rows + 1));
    P->d_col = internal::DeviceArray<int32_t>(size_t(std::max<int64_t>(P->nnz, 1)));
    internal::check(hdd_pattern_fill_device(ctx_, &m, info_.nb, d_cols_.get(), P->d_elem_ptr.get(), P->d_row_ptr.get(),
                                            P->d_col.get(), nullptr), "hdd_pattern_fill_device");
    internal::hip_check(hipDeviceSynchronize(), "device_pattern");
    return P;
  }

  void build_pattern()
  {
    const auto t0 = internal::Timer::now();
    d_nbrs_ = internal::DeviceArray<int32_t>(nbrs_);
    d_cols_ = internal::DeviceArray<int64_t>(cols_);
    pattern_ = device_pattern(false);
    pattern_seconds_ = internal::seconds_since(t0);
  }

  std::shared_ptr<const Pattern> volume_pattern()
  {
    if (!volume_pattern_) volume_pattern_ = device_pattern(true);
    return volume_pattern_;
  }

  void upload_mesh()
  {
    d_coords_ = internal::DeviceArray<double>(coords_);   // (d_nbrs_: uploaded with the pattern build)
    d_finfo_ = internal::DeviceArray<uint32_t>(finfo_);
    if (info_.dim == 2) {   // vertex-indexed geometry: what the P1 / Q1 stiffness kernels read
      int64_t nv = 0;
      internal::check(hdd_local_vertices(local_, &nv, nullptr, nullptr), "hdd_local_vertices");
      std::vector<int32_t> ev(size_t(info_.nvpe * linfo_.n_local));
      std::vector<double> vxy(size_t(2 * nv));
      internal::check(hdd_local_vertices(local_, &nv, ev.data(), vxy.data()), "hdd_local_vertices");
      d_ev_ = internal::DeviceArray<int32_t>(ev);
      d_vxy_ = internal::DeviceArray<double>(vxy);
    }
    tensor_ = detail::DeviceTensor(problem_.diffusion_tensor, view_);
    mesh_ = hdd_mesh{info_.elem_type, degree_, linfo_.n_local, linfo_.own_begin, linfo_.own_end, d_coords_.get(),
                     d_nbrs_.get(), d_finfo_.get(), d_ev_.get(), d_vxy_.get()};
    prm_ = detail::swipdg_params(degree_, info_.dim);
    purely_neumann_ = true;
    for (int f = 0; f < info_.nfaces; ++f)
      for (int64_t e = linfo_.own_begin; e < linfo_.own_end; ++e)
        if (nbrs_[size_t(f * linfo_.n_local + e)] == HDD_NBR_DIRICHLET) purely_neumann_ = false;
  }

  std::shared_ptr<internal::DeviceArray<double>> assemble_lhs(const Problems::ScalarFunction& f, const hdd_csr& pat)
  {
    auto vals = std::make_shared<internal::DeviceArray<double>>(size_t(pattern_->nnz) + 1);
    detail::DeviceFn k(f, view_);
    double* v = vals->get();
    internal::check(hdd_swipdg_assemble(ctx_, &mesh_, &k.fn, 1, &tensor_.fn, &prm_, &pat, &v, nullptr),
                    "hdd_swipdg_assemble");
    internal::hip_check(hipDeviceSynchronize(), "assemble");
    return vals;
  }

  // one functional evaluation: L2Volume(force) + DirichletBoundarySWIPDG(kappa, A, g_D) + L2Face(g_N), each
  // nullable (hdd_swipdg_rhs)
  std::shared_ptr<internal::DeviceArray<double>> rhs_vector(const Problems::ScalarFunction* force,
                                                            const Problems::ScalarFunction* kappa,
                                                            const Problems::ScalarFunction* dirichlet,
                                                            const Problems::ScalarFunction* neumann)
  {
    const int64_t size = pattern_->rows;
    auto b = std::make_shared<internal::DeviceArray<double>>(size_t(size) + 1);
    detail::DeviceFn f, k, d, nm;
    if (force) f = detail::DeviceFn(*force, view_);
    if (dirichlet) { k = detail::DeviceFn(*kappa, view_); d = detail::DeviceFn(*dirichlet, view_); }
    if (neumann) nm = detail::DeviceFn(*neumann, view_);
    internal::check(hdd_swipdg_rhs(ctx_, &mesh_, force ? &f.fn : nullptr, dirichlet ? &k.fn : nullptr, &tensor_.fn,
                                   dirichlet ? &d.fn : nullptr, neumann ? &nm.fn : nullptr, &prm_, b->get(), nullptr),
                    "hdd_swipdg_rhs");
    internal::hip_check(hipDeviceSynchronize(), "rhs");
    return b;
  }

  // swipdg.hh:251-356: the component structure of the reference's rhs container --
  //   force components (theta_f,q)                      L2Volume(f_q)
  //   affine part                                       L2Volume(f_aff) + Dirichlet(kappa_aff, g_D,aff) + L2Face(g_N,aff)
  //   kappa_aff x g_D components (theta_D,q)            Dirichlet(kappa_aff, g_D,q)
  //   kappa components x g_D,aff (theta_k,q)            Dirichlet(kappa_q, g_D,aff)
  //   kappa_p x g_D,q ((theta_k,p)*(theta_D,q))         Dirichlet(kappa_p, g_D,q)
  //   Neumann components (theta_N,q)                    L2Face(g_N,q)
  void assemble_rhs()
  {
    const auto& P = problem_;
    const auto& K = P.diffusion_factor;
    const auto& F = P.force;
    const auto& D = P.dirichlet;
    const auto& N = P.neumann;
    rhs_ = AffinelyDecomposedVector();
    rhs_.size = pattern_->rows;
    auto add = [&](std::shared_ptr<internal::DeviceArray<double>> v, const Pymor::ParameterFunctional& theta) {
      rhs_.comps.push_back(std::move(v));
      rhs_.coefficients.push_back(theta);
    };
    for (int q = 0; q < F.num_components(); ++q)
      add(rhs_vector(&F.components[size_t(q)], nullptr, nullptr, nullptr), F.coefficients[size_t(q)]);
    const bool dir_aff = K.has_affine_part && D.has_affine_part;
    if (F.has_affine_part || dir_aff || N.has_affine_part)
      rhs_.affine = rhs_vector(F.has_affine_part ? &F.affine_part : nullptr, dir_aff ? &K.affine_part : nullptr,
                               dir_aff ? &D.affine_part : nullptr, N.has_affine_part ? &N.affine_part : nullptr);
    if (K.has_affine_part)
      for (int q = 0; q < D.num_components(); ++q)
        add(rhs_vector(nullptr, &K.affine_part, &D.components[size_t(q)], nullptr), D.coefficients[size_t(q)]);
    if (D.has_affine_part)
      for (int q = 0; q < K.num_components(); ++q)
        add(rhs_vector(nullptr, &K.components[size_t(q)], &D.affine_part, nullptr), K.coefficients[size_t(q)]);
    for (int p = 0; p < K.num_components(); ++p)
      for (int q = 0; q < D.num_components(); ++q)
        add(rhs_vector(nullptr, &K.components[size_t(p)], &D.components[size_t(q)], nullptr),
            K.coefficients[size_t(p)] * D.coefficients[size_t(q)]);
    for (int q = 0; q < N.num_components(); ++q)
      add(rhs_vector(nullptr, nullptr, nullptr, &N.components[size_t(q)]), N.coefficients[size_t(q)]);
  }

  // swipdg.hh:358-508 (over_integrate = 2): "l2", "h1_semi", "boundary_l2" nonparametric; "elliptic" and
  // "penalty" affinely decomposed like kappa; "energy" = a copy of the system matrix
  AffinelyDecomposedMatrix product(const std::string& id)
  {
    if (id == "energy") {
      AffinelyDecomposedMatrix e = matrix_;   // shares the value arrays (read-only copy)
      return e;
    }
    int kind;
    if (id == "l2") kind = HDD_PRODUCT_L2;
    else if (id == "h1_semi") kind = HDD_PRODUCT_H1_SEMI;
    else if (id == "elliptic") kind = HDD_PRODUCT_ELLIPTIC;
    else if (id == "boundary_l2") kind = HDD_PRODUCT_BOUNDARY_L2;
    else if (id == "penalty") kind = HDD_PRODUCT_PENALTY;
    else throw Stuff::Exceptions::wrong_input_given("Product '" + id + "' not available!");
    const bool volume = kind != HDD_PRODUCT_PENALTY;
    std::shared_ptr<const Pattern> P = volume ? volume_pattern() : std::shared_ptr<const Pattern>(pattern_);
    const hdd_csr pat = P->csr();
    AffinelyDecomposedMatrix out;
    out.pattern = P;
    out.ctx = ctx_;
    auto run = [&](const Problems::ScalarFunction& f) {
      auto vals = std::make_shared<internal::DeviceArray<double>>(size_t(P->nnz) + 1);
      detail::DeviceFn k(f, view_);
      internal::check(hdd_product_assemble(ctx_, &mesh_, kind, &k.fn, &tensor_.fn, &prm_, &pat, vals->get(), nullptr),
                      "hdd_product_assemble");
      internal::hip_check(hipDeviceSynchronize(), "product");
      return vals;
    };
    const auto& K = problem_.diffusion_factor;
    if (kind == HDD_PRODUCT_ELLIPTIC || kind == HDD_PRODUCT_PENALTY) {
      out.coefficients = K.coefficients;
      for (const auto& c : K.components) out.comps.push_back(run(c));
      if (K.has_affine_part) out.affine = run(K.affine_part);
    } else {
      out.affine = run(Problems::ScalarFunction::constant(1.0));
    }
    return out;
  }

  const hdd_grid* grid_;
  Problems::Problem problem_;
  Layer layer_ = Layer::leaf;
  int subdomain_ = 0;
  std::vector<std::string> only_these_products_;
  int32_t boundary_code_ = HDD_NBR_DIRICHLET;
  hdd_grid_info info_{};
  hdd_local_info linfo_{};
  hdd_ctx* ctx_ = nullptr;
  hdd_local* local_ = nullptr;
  std::vector<double> coords_, centers_;
  std::vector<int32_t> nbrs_;
  std::vector<uint32_t> finfo_;
  std::vector<int64_t> gid_, cols_, parent_gid_;
  std::shared_ptr<hdd_grid> owned_grid_;   // subset grids (oversampled discretizations)
  int64_t n_cols_ = 0;
  detail::ElementView view_;
  std::shared_ptr<Pattern> pattern_;
  std::shared_ptr<const Pattern> volume_pattern_;
  internal::DeviceArray<double> d_coords_;
  internal::DeviceArray<int32_t> d_ev_;
  internal::DeviceArray<double> d_vxy_;
  internal::DeviceArray<int32_t> d_nbrs_;
  internal::DeviceArray<int64_t> d_cols_;
  internal::DeviceArray<uint32_t> d_finfo_;
  detail::DeviceTensor tensor_;
  hdd_mesh mesh_{};
  hdd_swipdg_params prm_{};
  int degree_ = 1;
  bool purely_neumann_ = false;
  double pattern_seconds_ = 0.0;   // measured time of the pattern build at construction
  AffinelyDecomposedMatrix matrix_;
  AffinelyDecomposedVector rhs_;
  std::map<std::string, std::shared_ptr<AffinelyDecomposedMatrix>> products_;
  bool initialized_ = false;
};

namespace detail {
// face-neighbour subdomains of every subdomain (MsGrid::neighborsOf), one pass over the grid; `pairs`
// (optional) counts the (element of ss, face neighbour in nn) pairs of every subdomain pair -- nb^2 times that
// (plus nb^2 |ss| on the diagonal) is the nnz of the block operator (ss, nn)
inline std::vector<std::set<int>> subdomain_neighbours(const hdd_grid* g, const hdd_grid_info& gi,
                                                       std::map<std::pair<int, int>, int64_t>* pairs = nullptr)
{
  std::vector<std::set<int>> nb(size_t(gi.n_subdomains));
  hdd_local* l = nullptr;
  internal::check(hdd_local_create(g, 0, gi.n_subdomains, &l), "hdd_local_create");
  hdd_local_info li{};
  hdd_local_get_info(l, &li);
  std::vector<int32_t> nbrs(size_t(gi.nfaces * li.n_local)), sd(size_t(li.n_local));
  const int rc = hdd_local_fill(l, nullptr, nbrs.data(), nullptr, nullptr, sd.data());
  hdd_local_destroy(l);
  internal::check(rc, "hdd_local_fill");
  for (int f = 0; f < gi.nfaces; ++f)
    for (int64_t e = 0; e < li.n_local; ++e) {
      const int32_t n = nbrs[size_t(f * li.n_local + e)];
      if (n < 0) continue;
      if (sd[size_t(n)] != sd[size_t(e)]) nb[size_t(sd[size_t(e)])].insert(sd[size_t(n)]);
      if (pairs) ++(*pairs)[{sd[size_t(e)], sd[size_t(n)]}];
    }
  return nb;
}
}  // namespace detail

// ------------------------------------------------------------------------------------------------
// BlockSWIPDG (block-swipdg.hh:177-846): the grid carries the subdomain partition; its subdomain-major
// element order IS the block numbering, so the global system matrix is assembled in one pass and the local /
// coupling operators are its diagonal / off-diagonal blocks.  As in the reference, the problem is replaced
// by ZeroBoundary(problem) and the boundary info by AllDirichlet (block-swipdg.hh:172-176, 230-238).
// ------------------------------------------------------------------------------------------------
class BlockSWIPDG : public SWIPDG {
 public:
  BlockSWIPDG(const grid::Multiscale::Providers::Cube& grid_provider, const Stuff::Common::Configuration& /*ignored*/,
              const Problems::Problem& prob, const std::vector<std::string>& only_these_products = {},
              int hip_device = 0)
    : SWIPDG(grid_provider.grid(), Stuff::Grid::BoundaryInfos::AllDirichlet::default_config(),
             Problems::ZeroBoundary(prob), Layer::leaf, 0, only_these_products, hip_device),
      original_problem_(prob), device_(hip_device), oversampling_layers_(grid_provider.oversampling_layers())
  {
    setup();
  }
  // convenience: raw grid handle, every product available
  BlockSWIPDG(const hdd_grid* grid, const Problems::Problem& prob, int hip_device = 0)
    : SWIPDG(grid, Stuff::Grid::BoundaryInfos::AllDirichlet::default_config(), Problems::ZeroBoundary(prob),
             Layer::leaf, 0, detail::all_products(), hip_device),
      original_problem_(prob), device_(hip_device)
  {
    setup();
  }

  static std::string static_id() { return "hdd.linearelliptic.discretizations.containerbased.block-swipdg"; }

  // block-swipdg.hh:262-551 (the two subdomain walks collapse into the one-pass assembly of SWIPDG::init)
  void init(std::ostream& out = Stuff::Common::devnull(), const std::string& prefix = "")
  {
    if (initialized_) return;
    // the reference's first walk builds the local and coupling patterns (block-swipdg.hh:266-328): here the
    // global block pattern was built once at construction, and its measured time is reported; the second walk
    // (local, boundary and coupling matrices, 330-386) is the one-pass device assembly
    out << prefix << "walking subdomains for the first time (block pattern, built at construction)... done (took "
        << pattern_seconds_ << " sek)" << std::endl;
    out << prefix << "walking subdomains for the second time... " << std::flush;
    const auto t0 = internal::Timer::now();
    SWIPDG::init();
    out << "done (took " << internal::seconds_since(t0) << " sek)" << std::endl;
  }

  int num_subdomains() const { return info_.n_subdomains; }

  // block-swipdg.hh:558-565 (MsGrid::neighborsOf, computed once at construction)
  std::vector<int> neighbouring_subdomains(int ss) const
  {
    range_check(ss);
    return std::vector<int>(neighbours_[size_t(ss)].begin(), neighbours_[size_t(ss)].end());
  }

  AffinelyDecomposedMatrix get_local_operator(int ss) const { return extract(ss, ss); }

  // Every local and coupling operator at once (hdd_block_operators_map_device / _values_device: five
  // launches whatever their number, asynchronous -- the counts come from the face pairs counted at
  // construction).  Their patterns and values are views into one row-pointer, one column and one value array
  // per component (together the size of the system matrix): writing through one of these views changes the
  // shared arrays.  Afterwards get_local_operator / get_coupling_operator hand out clones of them (values of
  // their own, one device copy each) instead of extracting one by one.  The LRBMS consumer (pyMOR's
  // BlockSWIPDG wrapper) asks for all of them.
  const std::map<std::pair<int, int>, AffinelyDecomposedMatrix>& extract_operators() const
  {
    if (!operators_.empty()) return operators_;
    const auto& M = system_matrix();
    const int64_t nb = info_.nb;
    std::vector<std::pair<int, int>> pairs;
    std::vector<hdd_block_range> rng;
    std::vector<int64_t> rows, nnz, noff{0}, roff{0};
    for (int ss = 0; ss < num_subdomains(); ++ss) {
      std::vector<int> nns(neighbours_[size_t(ss)].begin(), neighbours_[size_t(ss)].end());
      nns.push_back(ss);
      std::sort(nns.begin(), nns.end());
      int64_t a, b;
      internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &b), "range");
      for (int nn : nns) {
        int64_t c, d;
        internal::check(hdd_grid_subdomain_range(grid_, nn, nn + 1, &c, &d), "range");
        const auto fp = face_pairs_.find({ss, nn});
        const int64_t n = nb * nb * ((fp == face_pairs_.end() ? 0 : fp->second) + (ss == nn ? b - a : 0));
        pairs.push_back({ss, nn});
        rng.push_back(hdd_block_range{a * nb, b * nb, c * nb, d * nb});
        rows.push_back((b - a) * nb);
        nnz.push_back(n);
        noff.push_back(noff.back() + n + (n & 1));
        roff.push_back(roff.back() + (b - a) * nb + 1);
      }
    }
    const int32_t n_ops = int32_t(pairs.size());
    auto rp = std::make_shared<internal::DeviceArray<int64_t>>(size_t(roff.back()));
    auto col = std::make_shared<internal::DeviceArray<int32_t>>(size_t(noff.back()) + 1);
    const hdd_csr pat = pattern_->csr();
#ifdef NDEBUG
    // release builds stay asynchronous: the counts from the face pairs are trusted (the tests below check them)
    internal::check(hdd_block_operators_map_device(ctx_, &pat, n_ops, rng.data(), rp->get(), col->get(), nullptr,
                                                   nullptr, nullptr), "hdd_block_operators_map_device");
#else
    // debug builds (and the test programs, built without NDEBUG): the device first returns the operators' offsets
    // from the pattern itself (row pointers only, no column writes), which must equal the face-pair counts the
    // column array was sized with -- checked BEFORE any column is written -- then fills the columns
    std::vector<int64_t> dev_off(size_t(n_ops) + 1);
    internal::check(hdd_block_operators_map_device(ctx_, &pat, n_ops, rng.data(), rp->get(), nullptr, nullptr,
                                                   dev_off.data(), nullptr), "hdd_block_operators_map_device (count)");
    for (int32_t k = 0; k <= n_ops; ++k)
      if (dev_off[size_t(k)] != noff[size_t(k)])
        throw std::runtime_error("BlockSWIPDG::extract_operators: the pattern's operator sizes differ from the face-pair "
                                 "counts (operator " + std::to_string(k) + ")");
    internal::check(hdd_block_operators_map_device(ctx_, &pat, n_ops, rng.data(), rp->get(), col->get(), nullptr,
                                                   nullptr, nullptr), "hdd_block_operators_map_device");
#endif
    std::vector<std::shared_ptr<internal::DeviceArray<double>>> all;   // affine first, then the components
    std::vector<const double*> in;
    std::vector<double*> res;
    auto slot = [&](const internal::DeviceArray<double>& v) {
      all.push_back(std::make_shared<internal::DeviceArray<double>>(size_t(noff.back()) + 1));
      in.push_back(v.get());
      res.push_back(all.back()->get());
    };
    if (M.affine) slot(*M.affine);
    for (const auto& q : M.comps) slot(*q);
    for (size_t i0 = 0; i0 < in.size(); i0 += HDD_MAX_COMP) {
      const int32_t k = int32_t(std::min<size_t>(HDD_MAX_COMP, in.size() - i0));
      internal::check(hdd_block_operators_values_device(ctx_, &pat, n_ops, rng.data(), noff.data(), rp->get(),
                                                        in.data() + i0, k, res.data() + i0, nullptr),
                      "hdd_block_operators_values_device");
    }
    for (int32_t k = 0; k < n_ops; ++k) {
      auto P = std::make_shared<Pattern>();
      P->rows = rows[size_t(k)];
      P->cols = rng[size_t(k)].col_end - rng[size_t(k)].col_begin;
      P->nnz = nnz[size_t(k)];
      P->d_row_ptr = internal::DeviceArray<int64_t>(rp->get() + roff[size_t(k)], size_t(P->rows + 1), rp);
      P->d_col = internal::DeviceArray<int32_t>(col->get() + noff[size_t(k)], size_t(P->nnz), col);
      AffinelyDecomposedMatrix out;
      out.pattern = P;
      out.ctx = ctx_;
      out.coefficients = M.coefficients;
      auto view = [&](size_t i) {
        return std::make_shared<internal::DeviceArray<double>>(all[i]->get() + noff[size_t(k)],
                                                               size_t(P->nnz + (P->nnz & 1)), all[i]);
      };
      size_t i = 0;
      if (M.affine) out.affine = view(i++);
      for (; i < all.size(); ++i) out.comps.push_back(view(i));
      operators_.emplace(pairs[size_t(k)], std::move(out));
    }
    return operators_;
  }

  AffinelyDecomposedMatrix get_coupling_operator(int ss, int nn) const
  {
    range_check(ss);
    if (!neighbours_[size_t(ss)].count(nn))
      throw Stuff::Exceptions::index_out_of_range("Subdomain " + std::to_string(nn) + " is not a neighbour of subdomain " +
                                                  std::to_string(ss) + " (call neighbouring_subdomains(" +
                                                  std::to_string(ss) + ") to find out)!");
    return extract(ss, nn);
  }

  // block-swipdg.hh:678-685: the local vector of ss (local discretization rhs + boundary contributions) =
  // the rows of ss of the global rhs, component by component
  AffinelyDecomposedVector get_local_functional(int ss) const
  {
    range_check(ss);
    const auto& b = rhs();
    int64_t a, e;
    internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &e), "hdd_grid_subdomain_range");
    AffinelyDecomposedVector out;
    out.size = (e - a) * info_.nb;
    out.coefficients = b.coefficients;
    auto slice = [&](const internal::DeviceArray<double>& v) {
      auto o = std::make_shared<internal::DeviceArray<double>>(size_t(out.size) + 1);
      internal::hip_check(hipMemcpy(o->get(), v.get() + a * info_.nb, size_t(out.size) * sizeof(double),
                                    hipMemcpyDeviceToDevice), "get_local_functional");
      return o;
    };
    if (b.affine) out.affine = slice(*b.affine);
    for (const auto& c : b.comps) out.comps.push_back(slice(*c));
    return out;
  }

  // block-swipdg.hh:761-768 / LocalDiscretizationsContainer (106-129): SWIPDG on the local grid part of ss,
  // AllNeumann, ZeroBoundary(problem), the requested products; created and initialised on first use
  const SWIPDG& get_local_discretization(int ss) const
  {
    auto& d = local_discretizations_[size_t(subdomain_check(ss))];
    if (!d) d = make_local_discretization(ss);
    return *d;
  }

  // block-swipdg.hh:783-817: SWIPDG on the local_oversampled grid part of ss (the subdomain plus
  // oversampling_layers rings of face neighbours), boundary "dirichlet" or "neumann" on the whole boundary of
  // that grid part, ZeroBoundary(problem), the requested products; created and initialised on first use
  const SWIPDG& get_oversampled_discretization(int ss, const std::string& boundary_value_type) const
  {
    subdomain_check(ss);
    boundary_config(boundary_value_type);
    auto& d = oversampled_[{ss, boundary_value_type}];
    if (!d) d = make_oversampled_discretization(ss, boundary_value_type);
    return *d;
  }

  // The caller-owned variants the reference's Python bindings use (pybindgen caller_owns_return,
  // examples/linearelliptic/cg_bindings_generator.py:57-60): block-swipdg.hh:602-610, 620-623, 634-637, 672-676,
  // 687-690 return `new` copies of the by-value getters; the caller deletes them.  The operator / product /
  // functional copies own their values (clone()), so writing through one changes nothing else.
  std::vector<double>* globalize_vectors_and_return_ptr(const std::vector<std::vector<double>>& locals) const
  {
    return new std::vector<double>(globalize_vectors(locals));
  }
  std::vector<double>* localize_vector_and_return_ptr(const std::vector<double>& global, int ss) const
  {
    return new std::vector<double>(localize_vector(global, ss));
  }
  AffinelyDecomposedMatrix* get_local_product_and_return_ptr(int ss, const std::string& id) const
  {
    return new AffinelyDecomposedMatrix(get_local_product(ss, id).clone());
  }
  AffinelyDecomposedMatrix* get_local_operator_and_return_ptr(int ss) const
  {
    return new AffinelyDecomposedMatrix(get_local_operator(ss));
  }
  AffinelyDecomposedMatrix* get_coupling_operator_and_return_ptr(int ss, int nn) const
  {
    return new AffinelyDecomposedMatrix(get_coupling_operator(ss, nn));
  }
  AffinelyDecomposedVector* get_local_functional_and_return_ptr(int ss) const
  {
    return new AffinelyDecomposedVector(get_local_functional(ss));
  }
  // block-swipdg.hh:770-781 / 819-831: `new` discretizations equal to the cached ones (built and initialised the
  // same way; the reference copy-constructs its discretization, which shares the containers -- SWIPDG owns a
  // context and is not copyable, so this one is built anew).  (The three-argument pb_get_oversampled_discretization
  // of block-swipdg.hh:833-846 calls an overload the reference never defines: not provided.)
  SWIPDG* pb_get_local_discretization(int64_t subdomain) const
  {
    if (subdomain < 0 || subdomain > int64_t(std::numeric_limits<int>::max()))
      throw Stuff::Exceptions::index_out_of_range("There was an error converting " + std::to_string(subdomain) +
                                                  " to size_t");
    const int ss = subdomain_check(int(subdomain));
    return make_local_discretization(ss).release();
  }
  SWIPDG* pb_get_oversampled_discretization(int64_t subdomain, const std::string& boundary_value_type) const
  {
    if (subdomain < 0 || subdomain > int64_t(std::numeric_limits<int>::max()))
      throw Stuff::Exceptions::index_out_of_range("There was an error converting " + std::to_string(subdomain) +
                                                  " to size_t");
    const int ss = subdomain_check(int(subdomain));
    boundary_config(boundary_value_type);
    return make_oversampled_discretization(ss, boundary_value_type).release();
  }
  int oversampling_layers() const { return oversampling_layers_; }
  void set_oversampling_layers(int layers)
  {
    oversampling_layers_ = layers;
    oversampled_.clear();
  }
  // parent element ids of the local_oversampled grid part of ss, ascending
  std::vector<int64_t> oversampled_elements(int ss) const
  {
    int64_t a, b;
    internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &b), "hdd_grid_subdomain_range");
    std::vector<char> in(size_t(info_.n_elements), 0);
    std::vector<int64_t> front;
    for (int64_t e = a; e < b; ++e) { in[size_t(e)] = 1; front.push_back(e); }
    const int64_t n = linfo_.n_local;   // the leaf view holds every element, local == global
    for (int layer = 0; layer < oversampling_layers_; ++layer) {
      std::vector<int64_t> next;
      for (int64_t e : front)
        for (int f = 0; f < info_.nfaces; ++f) {
          const int32_t nb = nbrs_[size_t(f * n + e)];
          if (nb >= 0 && !in[size_t(nb)]) { in[size_t(nb)] = 1; next.push_back(nb); }
        }
      front.swap(next);
    }
    std::vector<int64_t> ids;
    for (int64_t e = 0; e < info_.n_elements; ++e)
      if (in[size_t(e)]) ids.push_back(e);
    return ids;
  }

  // block-swipdg.hh:612-618
  const AffinelyDecomposedMatrix& get_local_product(int ss, const std::string& id) const
  {
    range_check(ss);
    return get_local_discretization(ss).get_product(id);
  }

  std::vector<double> localize_vector(const std::vector<double>& global, int ss) const
  {
    range_check(ss);
    if (int64_t(global.size()) != num_dofs())
      throw Stuff::Exceptions::index_out_of_range("The size() of global_vector does not match the ansatz space!");
    int64_t a, b;
    internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &b), "hdd_grid_subdomain_range");
    return std::vector<double>(global.begin() + a * info_.nb, global.begin() + b * info_.nb);
  }

  std::vector<double> globalize_vectors(const std::vector<std::vector<double>>& locals) const
  {
    if (int(locals.size()) != num_subdomains())
      throw Stuff::Exceptions::wrong_input_given("Given local_vectors has wrong size!");
    std::vector<double> out;
    for (int ss = 0; ss < num_subdomains(); ++ss) {
      int64_t a, b;
      internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &b), "hdd_grid_subdomain_range");
      if (int64_t(locals[size_t(ss)].size()) != (b - a) * info_.nb)
        throw Stuff::Exceptions::wrong_input_given("Given local_vectors[" + std::to_string(ss) + "] has wrong size!");
      out.insert(out.end(), locals[size_t(ss)].begin(), locals[size_t(ss)].end());
    }
    return out;
  }

 private:
  void setup()
  {
    neighbours_ = detail::subdomain_neighbours(grid_, info_, &face_pairs_);
    local_discretizations_.resize(size_t(info_.n_subdomains));
  }

  int subdomain_check(int ss) const   // (the messages of block-swipdg.hh:763-766, 786-789)
  {
    if (ss < 0 || ss >= num_subdomains())
      throw Stuff::Exceptions::index_out_of_range("Given subdomain " + std::to_string(ss) +
                                                  " too large (has to be smaller than " +
                                                  std::to_string(num_subdomains()) + "!");
    return ss;
  }
  static Stuff::Common::Configuration boundary_config(const std::string& boundary_value_type)
  {
    if (boundary_value_type == "dirichlet") return Stuff::Grid::BoundaryInfos::AllDirichlet::default_config();
    if (boundary_value_type == "neumann") return Stuff::Grid::BoundaryInfos::AllNeumann::default_config();
    throw Stuff::Exceptions::wrong_input_given(
        "Unknown boundary_value_type given (has to be dirichlet or neumann): " + boundary_value_type);
  }
  std::unique_ptr<SWIPDG> make_local_discretization(int ss) const
  {
    auto d = std::make_unique<SWIPDG>(grid_, Stuff::Grid::BoundaryInfos::AllNeumann::default_config(),
                                      Problems::ZeroBoundary(original_problem_), Layer::local, ss, only_these_products_,
                                      device_);
    d->init();
    return d;
  }
  std::unique_ptr<SWIPDG> make_oversampled_discretization(int ss, const std::string& boundary_value_type) const
  {
    std::vector<int64_t> ids = oversampled_elements(ss);
    auto d = std::make_unique<SWIPDG>(subset_grid(ids), ids, info_.n_elements, boundary_config(boundary_value_type),
                                      Problems::ZeroBoundary(original_problem_), only_these_products_, device_);
    d->init();
    return d;
  }

  void range_check(int ss) const
  {
    if (ss < 0 || ss >= num_subdomains())
      throw Stuff::Exceptions::index_out_of_range("0 <= ss < num_subdomains() = " + std::to_string(num_subdomains()) +
                                                  " is not true for ss = " + std::to_string(ss) + "!");
  }

  // block-swipdg.hh:625-676: rows of ss, columns of nn, both in local numbering -- extracted on the device from
  // the assembled global matrix (hdd_block_operator_map_device / _values_device); the nnz is known from the
  // face pairs counted at construction, so nothing synchronises until the caller reads the result
  AffinelyDecomposedMatrix extract(int ss, int nn) const
  {
    range_check(ss);
    range_check(nn);
    const auto it = operators_.find({ss, nn});
    if (it != operators_.end()) return it->second.clone();   // extract_operators() ran: a copy of its view
    const auto& M = system_matrix();
    int64_t a, b, c, d;
    internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &b), "range");
    internal::check(hdd_grid_subdomain_range(grid_, nn, nn + 1, &c, &d), "range");
    const int64_t nb = info_.nb;
    const auto fp = face_pairs_.find({ss, nn});
    auto P = std::make_shared<Pattern>();
    P->rows = (b - a) * nb;
    P->cols = (d - c) * nb;
    P->nnz = nb * nb * ((fp == face_pairs_.end() ? 0 : fp->second) + (ss == nn ? b - a : 0));
    P->d_row_ptr = internal::DeviceArray<int64_t>(size_t(P->rows + 1));
    P->d_col = internal::DeviceArray<int32_t>(size_t(P->nnz) + 1);
    const hdd_csr pat = pattern_->csr();
    internal::check(hdd_block_operator_map_device(ctx_, &pat, a * nb, b * nb, c * nb, d * nb, P->d_row_ptr.get(),
                                                  P->d_col.get(), nullptr, nullptr, nullptr),
                    "hdd_block_operator_map_device");
    AffinelyDecomposedMatrix out;
    out.pattern = P;
    out.ctx = ctx_;
    out.coefficients = M.coefficients;
    std::vector<const double*> in;
    std::vector<double*> res;
    auto slot = [&](const internal::DeviceArray<double>& v) {
      auto o = std::make_shared<internal::DeviceArray<double>>(size_t(P->nnz) + 1);
      in.push_back(v.get());
      res.push_back(o->get());
      return o;
    };
    if (M.affine) out.affine = slot(*M.affine);
    for (const auto& q : M.comps) out.comps.push_back(slot(*q));
    for (size_t i0 = 0; i0 < in.size(); i0 += HDD_MAX_COMP) {
      const int32_t k = int32_t(std::min<size_t>(HDD_MAX_COMP, in.size() - i0));
      internal::check(hdd_block_operator_values_device(ctx_, &pat, a * nb, b * nb, c * nb, d * nb, P->d_row_ptr.get(),
                                                       in.data() + i0, k, res.data() + i0, nullptr),
                      "hdd_block_operator_values_device");
    }
    return out;
  }

  // a standalone grid (vertex ids of the parent) of the given parent elements, in their order
  std::shared_ptr<hdd_grid> subset_grid(const std::vector<int64_t>& ids) const
  {
    std::vector<double> vc(size_t(info_.dim) * size_t(info_.n_vertices));
    std::vector<int32_t> ev(size_t(info_.nvpe * info_.n_elements)), sub;
    internal::check(hdd_grid_connectivity(grid_, vc.data(), ev.data(), nullptr), "hdd_grid_connectivity");
    std::vector<int32_t> sev;
    sev.reserve(ids.size() * size_t(info_.nvpe));
    for (int64_t e : ids)
      for (int k = 0; k < info_.nvpe; ++k) sev.push_back(ev[size_t(e * info_.nvpe + k)]);
    hdd_grid* g = nullptr;
    if (info_.elem_type == HDD_HEX) {   // nb = (p+1)^3
      int p = 1;
      while ((p + 1) * (p + 1) * (p + 1) < info_.nb) ++p;
      internal::check(hdd_grid_create_hex_from_connectivity(p, info_.n_vertices, vc.data(), int64_t(ids.size()),
                                                            sev.data(), nullptr, 1, HDD_BOUNDARY_ALL_DIRICHLET, &g),
                      "hdd_grid_create_hex_from_connectivity");
    } else {
      internal::check(hdd_grid_create_from_connectivity(info_.elem_type, info_.n_vertices, vc.data(), int64_t(ids.size()),
                                                        sev.data(), nullptr, 1, HDD_BOUNDARY_ALL_DIRICHLET, &g),
                      "hdd_grid_create_from_connectivity");
    }
    return std::shared_ptr<hdd_grid>(g, hdd_grid_destroy);
  }

  Problems::Problem original_problem_;
  int device_ = 0;
  int oversampling_layers_ = 0;
  std::vector<std::set<int>> neighbours_;
  std::map<std::pair<int, int>, int64_t> face_pairs_;   // (ss, nn) -> element-face pairs (operator nnz / nb^2)
  mutable std::map<std::pair<int, int>, AffinelyDecomposedMatrix> operators_;   // extract_operators()
  mutable std::vector<std::shared_ptr<SWIPDG>> local_discretizations_;
  mutable std::map<std::pair<int, std::string>, std::shared_ptr<SWIPDG>> oversampled_;
};

// ------------------------------------------------------------------------------------------------
// ShardedBlockSWIPDG: BlockSWIPDG over one process / thread per GPU.  Rank r owns the subdomains
// [n_sub r / nranks, n_sub (r+1) / nranks) and assembles their rows (owner-computes: A_ss and A_ss,nn are
// written by the owner of ss, block-swipdg.hh:355-382) through hdd_block_assemble_sharded; the ghost columns
// of the per-element coefficients arrive through the face halo of `comm`.  Host work and memory are
// O(owned + ghost elements): the structured grid is implicit and coefficients are localized per rank.
// ------------------------------------------------------------------------------------------------
class ShardedBlockSWIPDG {
 public:
  ShardedBlockSWIPDG(const grid::Multiscale::Providers::Cube& grid_provider,
                     const Stuff::Common::Configuration& /*ignored*/, const Problems::Problem& prob,
                     Parallel::Communicator comm, int rank, int nranks, int hip_device = 0)
    : ShardedBlockSWIPDG(grid_provider.grid(), prob, std::move(comm), rank, nranks, hip_device) {}

  ShardedBlockSWIPDG(const hdd_grid* grid, const Problems::Problem& prob, Parallel::Communicator comm, int rank,
                     int nranks, int hip_device = 0)
    : grid_(grid), problem_(Problems::ZeroBoundary(prob)), comm_(std::move(comm)), device_(hip_device)
  {
    if (prob.diffusion_tensor_parametric) throw NotImplemented("The diffusion tensor must not be parametric!");
    if (prob.diffusion_tensor_empty) throw Stuff::Exceptions::wrong_input_given("The diffusion tensor must not be empty!");
    internal::check(hdd_grid_get_info(grid, &info_), "hdd_grid_get_info");
    internal::check(hdd_ctx_create(hip_device, &ctx_), "hdd_ctx_create");
    internal::check(hdd_shard_create(ctx_, grid, nranks, rank, nullptr, &shard_), "hdd_shard_create");
    internal::check(hdd_shard_get_info(shard_, &sinfo_), "hdd_shard_get_info");
    internal::check(hdd_shard_mesh(shard_, &mesh_), "hdd_shard_mesh");
    if (sinfo_.n_peers > 0 && !comm_.get())
      throw Stuff::Exceptions::wrong_input_given("ShardedBlockSWIPDG: this rank has halo peers, a Communicator is needed");
  }
  ~ShardedBlockSWIPDG()
  {
    if (shard_) hdd_shard_destroy(shard_);
    if (ctx_) hdd_ctx_destroy(ctx_);
  }
  ShardedBlockSWIPDG(const ShardedBlockSWIPDG&) = delete;
  ShardedBlockSWIPDG& operator=(const ShardedBlockSWIPDG&) = delete;

  // block-swipdg.hh:262-551 for the owned subdomains: pattern of the owned rows (global columns), every
  // diffusion-factor component through the sharded step (one halo exchange per call), the owned rows of the
  // right-hand side (element-local)
  void init(std::ostream& out = Stuff::Common::devnull(), const std::string& prefix = "")
  {
    if (initialized_) return;
    out << prefix << "assembling subdomains [" << sinfo_.s_begin << ", " << sinfo_.s_end << ") of "
        << info_.n_subdomains << " on rank " << sinfo_.rank << "... " << std::flush;
    const auto t0 = internal::Timer::now();
    const int64_t n = sinfo_.n_local;
    centers_.assign(size_t(info_.dim * n), 0.0);
    gid_.assign(size_t(n), 0);
    internal::check(hdd_shard_centers(shard_, centers_.data()), "hdd_shard_centers");
    internal::check(hdd_shard_global_ids(shard_, gid_.data()), "hdd_shard_global_ids");
    view_ = detail::ElementView{n, sinfo_.own_begin, sinfo_.own_end, info_.dim, centers_.data(), gid_.data(),
                                info_.n_elements, /*halo_ghosts=*/true};
    auto P = std::make_shared<Pattern>();
    P->rows = sinfo_.n_rows;
    P->cols = sinfo_.n_cols;
    P->nnz = sinfo_.nnz;
    P->d_row_ptr = internal::DeviceArray<int64_t>(size_t(P->rows + 1));
    P->d_col = internal::DeviceArray<int32_t>(size_t(P->nnz));
    P->d_elem_ptr = internal::DeviceArray<int64_t>(size_t(sinfo_.own_end - sinfo_.own_begin + 1));
    internal::check(hdd_shard_pattern_fill(ctx_, shard_, P->d_row_ptr.get(), P->d_col.get(), P->d_elem_ptr.get(),
                                           nullptr), "hdd_shard_pattern_fill");
    pattern_ = P;
    tensor_ = detail::DeviceTensor(problem_.diffusion_tensor, view_);
    prm_ = detail::swipdg_params(detail::degree_of(info_), info_.dim);
    const auto& K = problem_.diffusion_factor;
    kappas_.clear();
    for (const auto& c : K.components) kappas_.emplace_back(c, view_);
    if (K.has_affine_part) kappas_.emplace_back(K.affine_part, view_);
    matrix_ = AffinelyDecomposedMatrix();
    matrix_.pattern = pattern_;
    matrix_.ctx = ctx_;
    matrix_.coefficients = K.coefficients;
    for (size_t q = 0; q < kappas_.size(); ++q) {
      auto v = std::make_shared<internal::DeviceArray<double>>(size_t(P->nnz) + 1);
      if (q < K.components.size()) matrix_.comps.push_back(v);
      else matrix_.affine = v;
    }
    assemble();   // the halo fills every ghost column (NaN until then)
    assemble_rhs();
    internal::hip_check(hipDeviceSynchronize(), "init");
    out << "done (took " << internal::seconds_since(t0) << "s)" << std::endl;
    initialized_ = true;
  }

  // one sharded LHS step for every component: pack -> exchange -> interior tiles -> unpack -> boundary tiles
  // (hdd_block_assemble_sharded); flags HDD_SHARD_* (NO_HALO once the ghost coefficients are current)
  // One kernel serves diffusion-factor parts of one integration order, so the parts are grouped by order
  // (at most HDD_MAX_COMP per call), one sharded call per group.  The first call exchanges the halo; a later
  // call exchanges again only if it carries per-element parts (their ghost columns are filled by its own
  // unpack), otherwise the ghost tensor columns are current and it runs with HDD_SHARD_NO_HALO.
  void assemble(uint32_t flags = 0, hipStream_t stream = nullptr)
  {
    std::map<int, std::vector<size_t>> by_order;
    for (size_t q = 0; q < kappas_.size(); ++q) {
      const hdd_scalar_fn& f = kappas_[q].fn;
      by_order[f.kind == HDD_FN_CONST || f.kind == HDD_FN_PER_ELEM ? 0 : f.order].push_back(q);
    }
    const hdd_csr pat = pattern_->csr();
    bool exchanged = false;
    for (const auto& g : by_order)
      for (size_t i0 = 0; i0 < g.second.size(); i0 += HDD_MAX_COMP) {
        std::vector<hdd_scalar_fn> k;
        std::vector<double*> v;
        bool per_elem = false;
        for (size_t i = i0; i < std::min(g.second.size(), i0 + HDD_MAX_COMP); ++i) {
          const size_t q = g.second[i];
          k.push_back(kappas_[q].fn);
          per_elem = per_elem || kappas_[q].fn.kind == HDD_FN_PER_ELEM;
          v.push_back(q < matrix_.comps.size() ? matrix_.comps[q]->get() : matrix_.affine->get());
        }
        const uint32_t f = (exchanged && !per_elem) ? (flags | HDD_SHARD_NO_HALO) : flags;
        internal::check(hdd_block_assemble_sharded(ctx_, shard_, comm_.get(), k.data(), int32_t(k.size()), &tensor_.fn,
                                                   &prm_, &pat, v.data(), f, stream), "hdd_block_assemble_sharded");
        exchanged = true;
      }
  }

  const AffinelyDecomposedMatrix& system_matrix() const { ready(); return matrix_; }   // owned rows, global columns
  const AffinelyDecomposedVector& rhs() const { ready(); return rhs_; }                // owned rows
  int num_subdomains() const { return info_.n_subdomains; }
  std::pair<int, int> owned_subdomains() const { return {sinfo_.s_begin, sinfo_.s_end}; }
  int64_t first_owned_dof() const { return sinfo_.global_first * info_.nb; }
  int64_t num_dofs() const { return info_.n_elements * info_.nb; }
  const hdd_shard_info& shard_info() const { return sinfo_; }
  const Pattern& pattern() const { ready(); return *pattern_; }
  hdd_ctx* context() const { return ctx_; }

  // the rows of an owned subdomain ss restricted to the columns of subdomain nn (nn == ss: local operator),
  // as AffinelyDecomposedMatrix in local numbering on both sides (block-swipdg.hh:625-676)
  AffinelyDecomposedMatrix get_operator_block(int ss, int nn) const
  {
    ready();
    if (ss < sinfo_.s_begin || ss >= sinfo_.s_end)
      throw Stuff::Exceptions::index_out_of_range("subdomain " + std::to_string(ss) + " is not owned by this rank");
    if (nn < 0 || nn >= info_.n_subdomains) throw Stuff::Exceptions::index_out_of_range("bad subdomain");
    int64_t a, b, c, d;
    internal::check(hdd_grid_subdomain_range(grid_, ss, ss + 1, &a, &b), "range");
    internal::check(hdd_grid_subdomain_range(grid_, nn, nn + 1, &c, &d), "range");
    const int64_t nb = info_.nb;
    const int64_t r0 = (a - sinfo_.global_first) * nb, r1 = (b - sinfo_.global_first) * nb;
    auto P = std::make_shared<Pattern>();
    P->rows = r1 - r0;
    P->cols = (d - c) * nb;
    P->d_row_ptr = internal::DeviceArray<int64_t>(size_t(P->rows + 1));
    const hdd_csr pat = pattern_->csr();
    // device extraction (hdd_block_operator_map_device): count + scan first (synchronises for the nnz)
    internal::check(hdd_block_operator_map_device(ctx_, &pat, r0, r1, c * nb, d * nb, P->d_row_ptr.get(), nullptr,
                                                  nullptr, &P->nnz, nullptr), "hdd_block_operator_map_device");
    if (P->nnz == 0 && nn != ss)
      throw Stuff::Exceptions::index_out_of_range("Subdomain " + std::to_string(nn) + " is not a neighbour of subdomain " +
                                                  std::to_string(ss));
    P->d_col = internal::DeviceArray<int32_t>(size_t(P->nnz) + 1);
    internal::check(hdd_block_operator_map_device(ctx_, &pat, r0, r1, c * nb, d * nb, P->d_row_ptr.get(), P->d_col.get(),
                                                  nullptr, nullptr, nullptr), "hdd_block_operator_map_device");
    AffinelyDecomposedMatrix out;
    out.pattern = P;
    out.ctx = ctx_;
    out.coefficients = matrix_.coefficients;
    auto extract = [&](const internal::DeviceArray<double>& v) {
      auto o = std::make_shared<internal::DeviceArray<double>>(size_t(P->nnz) + 1);
      const double* in = v.get();
      double* res = o->get();
      internal::check(hdd_block_operator_values_device(ctx_, &pat, r0, r1, c * nb, d * nb, P->d_row_ptr.get(), &in, 1,
                                                       &res, nullptr), "hdd_block_operator_values_device");
      return o;
    };
    if (matrix_.affine) out.affine = extract(*matrix_.affine);
    for (const auto& q : matrix_.comps) out.comps.push_back(extract(*q));
    internal::hip_check(hipDeviceSynchronize(), "get_operator_block");
    return out;
  }
  AffinelyDecomposedMatrix get_local_operator(int ss) const { return get_operator_block(ss, ss); }
  AffinelyDecomposedMatrix get_coupling_operator(int ss, int nn) const
  {
    if (nn == ss) throw Stuff::Exceptions::index_out_of_range("a subdomain is not its own neighbour");
    return get_operator_block(ss, nn);
  }

 private:
  void ready() const
  {
    if (!initialized_)
      throw Stuff::Exceptions::you_are_using_this_wrong("The user has to call init() before calling any other method!");
  }

  // owned rows of the block right-hand side (ZeroBoundary: L2Volume(force) only; element-local, no halo)
  void assemble_rhs()
  {
    const auto& F = problem_.force;
    rhs_ = AffinelyDecomposedVector();
    rhs_.size = sinfo_.n_rows;
    auto run = [&](const Problems::ScalarFunction* f, const Problems::ScalarFunction* kappa) {
      auto b = std::make_shared<internal::DeviceArray<double>>(size_t(rhs_.size) + 1);
      detail::DeviceFn fd, kd, dd;
      if (f) fd = detail::DeviceFn(*f, view_);
      const Problems::ScalarFunction zero = Problems::ScalarFunction::constant(0.0);
      if (kappa) { kd = detail::DeviceFn(*kappa, view_); dd = detail::DeviceFn(zero, view_); }
      internal::check(hdd_swipdg_rhs(ctx_, &mesh_, f ? &fd.fn : nullptr, kappa ? &kd.fn : nullptr, &tensor_.fn,
                                     kappa ? &dd.fn : nullptr, nullptr, &prm_, b->get(), nullptr), "hdd_swipdg_rhs");
      return b;
    };
    const auto& K = problem_.diffusion_factor;
    for (int q = 0; q < F.num_components(); ++q) {
      rhs_.comps.push_back(run(&F.components[size_t(q)], nullptr));
      rhs_.coefficients.push_back(F.coefficients[size_t(q)]);
    }
    rhs_.affine = run(F.has_affine_part ? &F.affine_part : nullptr, K.has_affine_part ? &K.affine_part : nullptr);
    for (int q = 0; q < K.num_components(); ++q) {   // kappa_q x (g_D = 0): registered as in swipdg.hh:300-311
      rhs_.comps.push_back(run(nullptr, &K.components[size_t(q)]));
      rhs_.coefficients.push_back(K.coefficients[size_t(q)]);
    }
  }

  const hdd_grid* grid_;
  Problems::Problem problem_;
  Parallel::Communicator comm_;
  int device_ = 0;
  hdd_grid_info info_{};
  hdd_ctx* ctx_ = nullptr;
  hdd_shard* shard_ = nullptr;
  hdd_shard_info sinfo_{};
  hdd_mesh mesh_{};
  std::vector<double> centers_;
  std::vector<int64_t> gid_;
  detail::ElementView view_;
  std::shared_ptr<Pattern> pattern_;
  detail::DeviceTensor tensor_;
  std::vector<detail::DeviceFn> kappas_;
  hdd_swipdg_params prm_{};
  AffinelyDecomposedMatrix matrix_;
  AffinelyDecomposedVector rhs_;
  bool initialized_ = false;
};

}  // namespace Discretizations
}  // namespace LinearElliptic
}  // namespace HDD
}  // namespace Dune
