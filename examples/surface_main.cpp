// examples/surface_main.cpp -- the C++ operator surface (include/hdd_discretizations.hh) used the way the
// reference's examples/tests use Discretizations::SWIPDG / BlockSWIPDG (examples/linearelliptic/
// block-swipdg_main.cc:21-92, test/linearelliptic-block-swipdg.hh): construct on a (multiscale) grid,
// init(), query the affinely decomposed system matrix, local and coupling operators, freeze a parameter.
// Writes raw arrays to <outdir> for tests/test_gpu_surface.py to compare with the CPU oracle.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "hdd_discretizations.hh"

using namespace Dune::HDD::LinearElliptic;

template <class T>
static void dump(const std::string& path, const std::vector<T>& v)
{
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(v.data()), std::streamsize(v.size() * sizeof(T)));
}

int main(int argc, char** argv)
{
  const std::string out = argc > 1 ? argv[1] : ".";
  // 1. ESV2007 on a multiscale cube grid: 16x16 Kuhn triangles of [-1,1]^2, partitions [2 2 1]
  hdd_structured_desc d{HDD_SIMPLEX, 16, 16, 2, 2, HDD_BOUNDARY_ALL_DIRICHLET, 0, {-1.0, -1.0}, {1.0, 1.0}};
  hdd_grid* g = nullptr;
  if (hdd_grid_create_structured(&d, &g) != HDD_OK) return 1;
  Problems::Problem esv;   // kappa = 1 (affine part), A = I, Testcase1Force, g_D = g_N = 0
  esv.force = Problems::ScalarFunction::cos_product(0.5 * M_PI * M_PI, 0.5 * M_PI, 0.5 * M_PI, 0.0, 3);
  {
    Discretizations::BlockSWIPDG block(g, esv);
    block.init();
    dump(out + "/block_rhs.bin", block.rhs().affine_part());
    std::printf("rhs components %d\n", block.rhs().num_components());
    for (const char* id : {"l2", "penalty"}) {
      const auto P = block.get_product(id);
      dump(out + "/product_" + std::string(id) + "_row_ptr.bin", P.pattern->row_ptr);
      auto pv = P.affine_part();
      pv.resize(size_t(P.pattern->nnz));
      dump(out + "/product_" + std::string(id) + ".bin", pv);
    }
    try {
      block.get_product("h2");
      std::printf("unknown product accepted\n");
    } catch (const std::invalid_argument& e) {
      std::printf("product rejected: %s\n", e.what());
    }
    const auto& A = block.system_matrix();
    dump(out + "/block_row_ptr.bin", A.pattern->row_ptr);
    dump(out + "/block_col.bin", A.pattern->col);
    auto v = A.affine_part();
    v.resize(size_t(A.pattern->nnz));
    dump(out + "/block_affine.bin", v);
    const auto nbs = block.neighbouring_subdomains(0);
    dump(out + "/neighbours0.bin", std::vector<int32_t>(nbs.begin(), nbs.end()));
    const auto L = block.get_local_operator(0);
    dump(out + "/local0_row_ptr.bin", L.pattern->row_ptr);
    dump(out + "/local0_col.bin", L.pattern->col);
    auto lv = L.affine_part();
    lv.resize(size_t(L.pattern->nnz));
    dump(out + "/local0_affine.bin", lv);
    const auto C = block.get_coupling_operator(0, nbs.at(0));
    dump(out + "/coupling0_row_ptr.bin", C.pattern->row_ptr);
    dump(out + "/coupling0_col.bin", C.pattern->col);
    auto cv = C.affine_part();
    cv.resize(size_t(C.pattern->nnz));
    dump(out + "/coupling0_affine.bin", cv);
    // localize / globalize round trip
    std::vector<double> x(size_t(block.num_dofs()));
    for (size_t i = 0; i < x.size(); ++i) x[i] = double(i);
    std::vector<std::vector<double>> locals;
    for (int ss = 0; ss < block.num_subdomains(); ++ss) locals.push_back(block.localize_vector(x, ss));
    std::printf("roundtrip %d\n", int(block.globalize_vectors(locals) == x));
    try {
      block.get_coupling_operator(0, 3);   // diagonal subdomain: not a face neighbour
      std::printf("coupling(0,3) unexpectedly allowed\n");
    } catch (const std::out_of_range& e) {
      std::printf("coupling(0,3) rejected: %s\n", e.what());
    }
  }
  hdd_grid_destroy(g);

  // 2. OS2014: kappa(mu) = (1 + 3/4 sin(4 pi (x + y/2))) - mu 3/4 sin(...), A = I, 8x8 Kuhn, monolithic
  hdd_structured_desc d2{HDD_SIMPLEX, 8, 8, 1, 1, HDD_BOUNDARY_ALL_DIRICHLET, 0, {-1.0, -1.0}, {1.0, 1.0}};
  if (hdd_grid_create_structured(&d2, &g) != HDD_OK) return 1;
  Problems::Problem os;
  const double kx = 4.0 * M_PI, ky = 2.0 * M_PI;
  os.diffusion_factor.affine_part = Problems::ScalarFunction::sinusoid(1.0, 0.75, kx, ky, 3);
  os.diffusion_factor.components.push_back(Problems::ScalarFunction::sinusoid(0.0, -0.75, kx, ky, 3));
  os.diffusion_factor.coefficients.emplace_back("mu", "mu", 1.0);
  {
    Discretizations::SWIPDG sw(g, os);
    sw.init();
    const auto& A = sw.system_matrix();
    std::printf("os2014 parametric %d components %d\n", int(A.parametric()), A.num_components());
    auto a = A.affine_part(); a.resize(size_t(A.pattern->nnz));
    auto c = A.component(0); c.resize(size_t(A.pattern->nnz));
    dump(out + "/os_affine.bin", a);
    dump(out + "/os_comp0.bin", c);
    dump(out + "/os_frozen_0.3.bin", A.freeze_parameter(0.3));
  }
  // 3. the reference's ctor validation (swipdg.hh:173-176)
  Problems::Problem bad;
  bad.diffusion_tensor_parametric = true;
  try {
    Discretizations::SWIPDG sw(g, bad);
    std::printf("parametric tensor unexpectedly accepted\n");
  } catch (const std::logic_error& e) {
    std::printf("rejected: %s\n", e.what());
  }
  hdd_grid_destroy(g);

  // 4. C5 through the same surface: ESV2007 3d, Q3 on a 3x3x3 hexahedral grid of [-1,1]^3
  hdd_structured3_desc d3{3, 3, 3, 1, 1, 1, HDD_BOUNDARY_ALL_DIRICHLET, 3, {-1.0, -1.0, -1.0}, {1.0, 1.0, 1.0}};
  if (hdd_grid_create_structured_3d(&d3, &g) != HDD_OK) return 1;
  Problems::Problem esv3;
  esv3.diffusion_tensor = Problems::TensorFunction::identity3d();
  esv3.force = Problems::ScalarFunction::cos_product(0.75 * M_PI * M_PI, 0.5 * M_PI, 0.5 * M_PI, 0.5 * M_PI, 3);
  {
    Discretizations::SWIPDG sw(g, esv3);
    sw.init();
    const auto& A = sw.system_matrix();
    std::printf("hex order %d dofs %lld\n", sw.polynomial_order(), (long long)sw.num_dofs());
    auto a = A.affine_part(); a.resize(size_t(A.pattern->nnz));
    dump(out + "/hex_row_ptr.bin", A.pattern->row_ptr);
    dump(out + "/hex_col.bin", A.pattern->col);
    dump(out + "/hex_affine.bin", a);
    dump(out + "/hex_rhs.bin", sw.rhs().affine_part());
  }
  hdd_grid_destroy(g);
  std::printf("surface ok\n");
  return 0;
}
