// examples/surface_main.cpp -- the C++ operator surface (include/hdd_discretizations.hh) used the way the
// reference's examples/tests use Discretizations::SWIPDG / BlockSWIPDG (examples/linearelliptic/
// block-swipdg_main.cc:21-92, test/linearelliptic-block-swipdg.hh): construct on a (multiscale) grid,
// init(), query the affinely decomposed system matrix, local and coupling operators, freeze a parameter.
// Writes raw arrays to <outdir> for tests/test_gpu_surface.py to compare with the CPU oracle.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "hdd_discretizations.hh"

using namespace Dune::HDD::LinearElliptic;
namespace S = Dune::Stuff;
template <class T>
using internal_array_t = Dune::HDD::LinearElliptic::internal::DeviceArray<T>;

template <class T>
static void dump(const std::string& path, const std::vector<T>& v)
{
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(v.data()), std::streamsize(v.size() * sizeof(T)));
}

// position-weighted 64-bit checksum of a device array's bit patterns: sum_k bits[k] * (2k + 1) mod 2^64 (the
// Python front-end computes the same on its own assembly: tests/test_gpu_surface.py::test_cpp_full_size_*)
template <class T>
uint64_t checksum(const internal_array_t<T>& a, int64_t n)
{
  uint64_t h = 0;
  const int64_t chunk = int64_t(1) << 26;
  std::vector<T> buf;
  for (int64_t k0 = 0; k0 < n; k0 += chunk) {
    const int64_t m = std::min(chunk, n - k0);
    buf.resize(size_t(m));
    if (hipMemcpy(buf.data(), a.get() + k0, size_t(m) * sizeof(T), hipMemcpyDeviceToHost) != hipSuccess)
      throw std::runtime_error("checksum: D2H");
    for (int64_t k = 0; k < m; ++k) {
      uint64_t bits = 0;
      std::memcpy(&bits, &buf[size_t(k)], sizeof(T));
      h += bits * uint64_t(2 * (k0 + k) + 1);
    }
  }
  return h;
}

// full-size runs of the reference-signature SWIPDG (device pattern, no host copy of it): C2 (SPE10 P1,
// 3200 x 640 Kuhn) and ESV2007 3d Q3 on n^3 hexahedra
int run_big(const std::string& which, int n)
{
  if (which == "c4ops") {   // BASELINE's 8-GPU decomposition: every block operator, one by one and batched
    hdd_structured_desc d{HDD_CUBE, 3520, 1200, 8, 8, HDD_BOUNDARY_ALL_DIRICHLET, 0, {0.0, 0.0}, {5.0, 1.0}};
    hdd_grid* g = nullptr;
    if (hdd_grid_create_structured(&d, &g) != HDD_OK) return 1;
    std::vector<double> perm(2000);
    for (int i = 0; i < 2000; ++i) perm[size_t(i)] = std::pow(10.0, -3.0 + 6.0 * std::fmod(0.618033988749895 * i, 1.0));
    {
      Discretizations::BlockSWIPDG block(g, Problems::Spe10Model1(perm, {}, {}, false));
      block.init();
      (void)hipDeviceSynchronize();
      std::vector<std::pair<int, int>> pairs;
      for (int ss = 0; ss < block.num_subdomains(); ++ss) {
        pairs.push_back({ss, ss});
        for (int nn : block.neighbouring_subdomains(ss)) pairs.push_back({ss, nn});
      }
      std::vector<Discretizations::AffinelyDecomposedMatrix> one;
      for (int rep = 0; rep < 2; ++rep) {   // (the second pass: allocator warm)
        one.clear();
        const auto t0 = std::chrono::steady_clock::now();
        for (const auto& p : pairs)
          one.push_back(p.first == p.second ? block.get_local_operator(p.first) : block.get_coupling_operator(p.first, p.second));
        (void)hipDeviceSynchronize();
        std::printf("c4 ops one-by-one: %zu operators %.2f ms\n", pairs.size(),
                    1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      }
      const auto t0 = std::chrono::steady_clock::now();
      const auto& all = block.extract_operators();
      (void)hipDeviceSynchronize();
      const double ms = 1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      int64_t nnz = 0;
      bool same = all.size() == pairs.size();
      for (size_t k = 0; k < pairs.size() && same; ++k) {
        const auto& b = all.at(pairs[k]);
        const auto& a = one[k];
        nnz += b.pattern->nnz;
        same = a.pattern->nnz == b.pattern->nnz &&
               checksum(a.pattern->d_row_ptr, a.pattern->rows + 1) == checksum(b.pattern->d_row_ptr, b.pattern->rows + 1) &&
               checksum(a.pattern->d_col, a.pattern->nnz) == checksum(b.pattern->d_col, b.pattern->nnz) &&
               checksum(*a.affine, a.pattern->nnz) == checksum(*b.affine, b.pattern->nnz);
      }
      std::printf("c4 ops batched: %zu operators nnz %lld %.2f ms equal %d\n", all.size(), (long long)nnz, ms, int(same));
    }
    hdd_grid_destroy(g);
    return 0;
  }
  if (which == "c2") {
    S::Grid::Providers::Cube provider(HDD_SIMPLEX, {0.0, 0.0}, {5.0, 1.0}, {3200, 640});
    std::vector<double> perm(2000);
    for (int i = 0; i < 2000; ++i) perm[size_t(i)] = std::pow(10.0, -3.0 + 6.0 * std::fmod(0.618033988749895 * i, 1.0));
    Discretizations::SWIPDG sw(provider, S::Grid::BoundaryInfos::AllDirichlet::default_config(),
                               Problems::Spe10Model1(perm, {}, {}, false), 0, {});
    sw.init();
    const auto& A = sw.system_matrix();
    std::printf("big c2: rows %lld nnz %lld col_hash %llu val_hash %llu\n", (long long)A.pattern->rows,
                (long long)A.pattern->nnz, (unsigned long long)checksum(A.pattern->d_col, A.pattern->nnz),
                (unsigned long long)checksum(*A.affine, A.pattern->nnz));
    return 0;
  }
  hdd_structured3_desc d3{n, n, n, 1, 1, 1, HDD_BOUNDARY_ALL_DIRICHLET, 3, {-1.0, -1.0, -1.0}, {1.0, 1.0, 1.0}};
  hdd_grid* g = nullptr;
  if (hdd_grid_create_structured_3d(&d3, &g) != HDD_OK) return 1;
  Problems::Problem esv3;
  esv3.diffusion_tensor = Problems::TensorFunction::identity3d();
  esv3.force = Problems::ScalarFunction::cos_product(0.75 * M_PI * M_PI, 0.5 * M_PI, 0.5 * M_PI, 0.5 * M_PI, 3);
  {
    Discretizations::SWIPDG sw(g, S::Common::Configuration(), esv3, Discretizations::SWIPDG::Layer::leaf, 0, {}, 0,
                               /*grid_boundary=*/true);
    sw.init();
    const auto& A = sw.system_matrix();
    std::printf("big hex%d: order %d rows %lld nnz %lld col_hash %llu val_hash %llu\n", n, sw.polynomial_order(),
                (long long)A.pattern->rows, (long long)A.pattern->nnz,
                (unsigned long long)checksum(A.pattern->d_col, A.pattern->nnz),
                (unsigned long long)checksum(*A.affine, A.pattern->nnz));
  }
  hdd_grid_destroy(g);
  return 0;
}

int main(int argc, char** argv)
{
  if (argc > 2 && std::string(argv[1]) == "big") return run_big(argv[2], argc > 3 ? std::atoi(argv[3]) : 32);
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
      dump(out + "/product_" + std::string(id) + "_row_ptr.bin", P.pattern->row_ptr());
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
    dump(out + "/block_row_ptr.bin", A.pattern->row_ptr());
    dump(out + "/block_col.bin", A.pattern->col());
    auto v = A.affine_part();
    v.resize(size_t(A.pattern->nnz));
    dump(out + "/block_affine.bin", v);
    const auto nbs = block.neighbouring_subdomains(0);
    dump(out + "/neighbours0.bin", std::vector<int32_t>(nbs.begin(), nbs.end()));
    const auto L = block.get_local_operator(0);
    dump(out + "/local0_row_ptr.bin", L.pattern->row_ptr());
    dump(out + "/local0_col.bin", L.pattern->col());
    auto lv = L.affine_part();
    lv.resize(size_t(L.pattern->nnz));
    dump(out + "/local0_affine.bin", lv);
    const auto C = block.get_coupling_operator(0, nbs.at(0));
    dump(out + "/coupling0_row_ptr.bin", C.pattern->row_ptr());
    dump(out + "/coupling0_col.bin", C.pattern->col());
    auto cv = C.affine_part();
    cv.resize(size_t(C.pattern->nnz));
    dump(out + "/coupling0_affine.bin", cv);
    // localize / globalize round trip
    std::vector<double> x(size_t(block.num_dofs()));
    for (size_t i = 0; i < x.size(); ++i) x[i] = double(i);
    std::vector<std::vector<double>> locals;
    for (int ss = 0; ss < block.num_subdomains(); ++ss) locals.push_back(block.localize_vector(x, ss));
    std::printf("roundtrip %d\n", int(block.globalize_vectors(locals) == x));
    // every operator at once (extract_operators): the same arrays as the one-by-one extraction above
    {
      const auto& all = block.extract_operators();
      const auto& L2 = all.at({0, 0});
      const auto& C2 = all.at({0, nbs.at(0)});
      auto l2v = L2.affine_part();
      auto c2v = C2.affine_part();
      const bool same = L2.pattern->row_ptr() == L.pattern->row_ptr() && L2.pattern->col() == L.pattern->col() &&
                        l2v == lv && C2.pattern->row_ptr() == C.pattern->row_ptr() &&
                        C2.pattern->col() == C.pattern->col() && c2v == cv &&
                        L2.freeze_parameter(0.5) == L.freeze_parameter(0.5) &&
                        block.get_coupling_operator(0, nbs.at(0)).pattern == C2.pattern;
      std::printf("batched operators %zu same %d\n", all.size(), int(same));
    }
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
    dump(out + "/hex_row_ptr.bin", A.pattern->row_ptr());
    dump(out + "/hex_col.bin", A.pattern->col());
    dump(out + "/hex_affine.bin", a);
    dump(out + "/hex_rhs.bin", sw.rhs().affine_part());
  }
  hdd_grid_destroy(g);

  // 5. the reference's constructor / init surface (swipdg.hh:159-163, 206, 216-217, 486; base.hh:272-291)
  {
    S::Grid::Providers::Cube provider(HDD_SIMPLEX, {-1.0, -1.0}, {1.0, 1.0}, {8, 8}, 1);   // levels 8^2, 16^2
    Discretizations::SWIPDG sw(provider, S::Grid::BoundaryInfos::AllDirichlet::default_config(), Problems::ESV2007(),
                               1, {"l2", "penalty"});
    sw.init(std::cout, "  [swipdg] ");
    std::string avail;
    for (const auto& id : sw.available_products()) avail += id + " ";
    std::printf("available products: %s\n", avail.c_str());
    try {
      sw.get_product("h1_semi");
    } catch (const S::Exceptions::wrong_input_given& e) {
      std::printf("not requested: %s\n", e.what());
    }
    dump(out + "/lvl1_row_ptr.bin", sw.pattern().row_ptr());
    dump(out + "/lvl1_affine.bin", sw.system_matrix().affine_part());
    dump(out + "/lvl1_rhs.bin", sw.rhs().affine_part());
    Discretizations::SWIPDG bare(provider, S::Grid::BoundaryInfos::AllDirichlet::default_config(), Problems::ESV2007());
    try {
      bare.system_matrix();
    } catch (const S::Exceptions::you_are_using_this_wrong& e) {
      std::printf("before init: %s\n", e.what());
    }
    bare.init();
    try {
      bare.get_product("l2");
    } catch (const S::Exceptions::you_are_using_this_wrong& e) {
      std::printf("no products: %s\n", e.what());
    }
    try {
      Discretizations::SWIPDG bad_level(provider, S::Grid::BoundaryInfos::AllDirichlet::default_config(),
                                        Problems::ESV2007(), 5);
    } catch (const S::Exceptions::index_out_of_range& e) {
      std::printf("bad level: %s\n", e.what());
    }
  }

  // 6. BlockSWIPDG on a multiscale provider: local discretization / product / functional (block-swipdg.hh:612-685, 761)
  {
    Dune::grid::Multiscale::Providers::Cube ms(HDD_SIMPLEX, {-1.0, -1.0}, {1.0, 1.0}, {16, 16}, {2, 2},
                                               /*oversampling_layers=*/1);
    Discretizations::BlockSWIPDG block(ms, S::Common::Configuration(), Problems::ESV2007(), {"l2", "h1_semi"});
    block.init(std::cout, "  [block] ");
    const auto& L0 = block.get_local_discretization(0);
    std::printf("local discretization 0: layer local %d, dofs %lld, purely neumann %d\n",
                int(L0.layer() == Discretizations::SWIPDG::Layer::local), (long long)L0.num_dofs(),
                int(L0.purely_neumann()));
    dump(out + "/ld0_row_ptr.bin", L0.pattern().row_ptr());
    dump(out + "/ld0_col.bin", L0.pattern().col());
    dump(out + "/ld0_affine.bin", L0.system_matrix().affine_part());
    const auto& P0 = block.get_local_product(0, "l2");
    dump(out + "/lp0_row_ptr.bin", P0.pattern->row_ptr());
    dump(out + "/lp0_l2.bin", P0.affine_part());
    const auto F0 = block.get_local_functional(0);
    dump(out + "/lf0.bin", F0.affine_part());
    dump(out + "/lf0_from_ld.bin", L0.rhs().affine_part());
    std::printf("local functional 0: size %lld components %d\n", (long long)F0.size, F0.num_components());
    try {
      block.get_local_discretization(4);
    } catch (const S::Exceptions::index_out_of_range& e) {
      std::printf("local discretization 4 rejected\n");
    }
    // block-swipdg.hh:783-817: subdomain 0 + one ring of face neighbours, Dirichlet / Neumann boundary
    for (const char* bt : {"dirichlet", "neumann"}) {
      const auto& O = block.get_oversampled_discretization(0, bt);
      dump(out + "/os0_" + std::string(bt) + "_row_ptr.bin", O.pattern().row_ptr());
      dump(out + "/os0_" + std::string(bt) + "_col.bin", O.pattern().col());
      dump(out + "/os0_" + std::string(bt) + "_affine.bin", O.system_matrix().affine_part());
      dump(out + "/os0_" + std::string(bt) + "_rhs.bin", O.rhs().affine_part());
    }
    const auto ids = block.oversampled_elements(0);
    dump(out + "/os0_ids.bin", ids);
    std::printf("oversampled 0: %zu elements (layers %d)\n", ids.size(), block.oversampling_layers());
    try {
      block.get_oversampled_discretization(0, "robin");
    } catch (const S::Exceptions::wrong_input_given& e) {
      std::printf("oversampled robin rejected\n");
    }
    // the caller-owned variants of the reference's Python bindings (block-swipdg.hh:602-690, 770-831): each `new`
    // object equals its by-value getter, owns its values (zeroing them changes nothing else) and is deleted here
    {
      int ok = 1;
      using M = Discretizations::AffinelyDecomposedMatrix;
      auto same = [](const M& a, const M& b) {
        return a.pattern->row_ptr() == b.pattern->row_ptr() && a.pattern->col() == b.pattern->col() &&
               a.affine_part() == b.affine_part() && a.num_components() == b.num_components();
      };
      auto zero = [](const M& a) {
        (void)hipMemset(a.affine->get(), 0, size_t(a.pattern->nnz) * sizeof(double));
        (void)hipDeviceSynchronize();
      };
      std::vector<double> x(size_t(block.num_dofs()));
      for (size_t i = 0; i < x.size(); ++i) x[i] = 0.5 * double(i);
      std::vector<std::vector<double>> locals;
      for (int ss = 0; ss < block.num_subdomains(); ++ss) {
        std::vector<double>* lv = block.localize_vector_and_return_ptr(x, ss);
        ok &= *lv == block.localize_vector(x, ss);
        locals.push_back(*lv);
        delete lv;
      }
      std::vector<double>* gv = block.globalize_vectors_and_return_ptr(locals);
      ok &= *gv == x;
      delete gv;
      const int nb0 = block.neighbouring_subdomains(0).at(0);
      for (int pass = 0; pass < 2; ++pass) {   // extraction one by one, then from the batched views
        if (pass == 1) block.extract_operators();
        const M lo_ref = block.get_local_operator(0), co_ref = block.get_coupling_operator(0, nb0);
        M* lo = block.get_local_operator_and_return_ptr(0);
        M* co = block.get_coupling_operator_and_return_ptr(0, nb0);
        ok &= same(*lo, lo_ref) && same(*co, co_ref);
        zero(*lo);
        zero(*co);
        ok &= same(block.get_local_operator(0), lo_ref) && same(block.get_coupling_operator(0, nb0), co_ref);
        if (pass == 1)   // the batched view itself is untouched too
          ok &= block.extract_operators().at({0, nb0}).affine_part() == co_ref.affine_part();
        delete lo;
        delete co;
      }
      M* lp = block.get_local_product_and_return_ptr(0, "l2");
      const M lp_ref = block.get_local_product(0, "l2");
      const auto lp_vals = lp_ref.affine_part();
      ok &= same(*lp, lp_ref);
      zero(*lp);
      ok &= block.get_local_product(0, "l2").affine_part() == lp_vals;
      delete lp;
      Discretizations::AffinelyDecomposedVector* lf = block.get_local_functional_and_return_ptr(0);
      ok &= lf->affine_part() == block.get_local_functional(0).affine_part() && lf->size == block.get_local_functional(0).size;
      delete lf;
      Discretizations::SWIPDG* ld = block.pb_get_local_discretization(0);
      ok &= ld->system_matrix().affine_part() == L0.system_matrix().affine_part() &&
            ld->rhs().affine_part() == L0.rhs().affine_part() && ld->pattern().col() == L0.pattern().col() &&
            ld->available_products() == L0.available_products() && ld != &L0;
      delete ld;
      for (const char* bt : {"dirichlet", "neumann"}) {
        Discretizations::SWIPDG* od = block.pb_get_oversampled_discretization(0, bt);
        const auto& O = block.get_oversampled_discretization(0, bt);
        ok &= od->system_matrix().affine_part() == O.system_matrix().affine_part() &&
              od->rhs().affine_part() == O.rhs().affine_part() && od->num_dofs() == O.num_dofs();
        delete od;
      }
      try {
        delete block.pb_get_local_discretization(-1);
        ok = 0;
      } catch (const S::Exceptions::index_out_of_range&) {
      }
      try {
        delete block.pb_get_oversampled_discretization(0, "robin");
        ok = 0;
      } catch (const S::Exceptions::wrong_input_given&) {
      }
      std::printf("caller-owned copies %d\n", ok);
    }
  }

  // 6b. the same in 3d (block-swipdg.hh:783-817 is dimension-generic): ESV2007 3d on 4 x 3 x 3 hexahedra, Q2,
  //     2 x 1 x 1 subdomains, one oversampling layer -- subdomain 0 plus the next x-slab of elements (a box)
  {
    Dune::grid::Multiscale::Providers::Cube ms({-1.0, -1.0, -1.0}, {1.0, 1.0, 1.0}, {4, 3, 3}, {2, 1, 1},
                                               /*oversampling_layers=*/1, /*degree=*/2);
    Discretizations::BlockSWIPDG block(ms, S::Common::Configuration(), esv3, {});
    block.init();
    for (const char* bt : {"dirichlet", "neumann"}) {
      const auto& O = block.get_oversampled_discretization(0, bt);
      dump(out + "/os3_" + std::string(bt) + "_row_ptr.bin", O.pattern().row_ptr());
      dump(out + "/os3_" + std::string(bt) + "_col.bin", O.pattern().col());
      dump(out + "/os3_" + std::string(bt) + "_affine.bin", O.system_matrix().affine_part());
      dump(out + "/os3_" + std::string(bt) + "_rhs.bin", O.rhs().affine_part());
    }
    const auto ids = block.oversampled_elements(0);
    dump(out + "/os3_ids.bin", ids);
    std::printf("oversampled 3d 0: %zu elements (layers %d)\n", ids.size(), block.oversampling_layers());
  }

  // 7. parametric SPE10 Model1 (problems/spe10.hh:160-172): A = checkerboard, kappa = (1 + channel) - mu channel,
  //    force = Indicator; channel / force boxes read from <outdir>/spe10_boxes.bin when present
  {
    std::vector<double> perm(2000);
    for (int i = 0; i < 2000; ++i) perm[size_t(i)] = std::pow(10.0, -3.0 + 6.0 * std::fmod(0.618033988749895 * i, 1.0));
    std::vector<std::array<double, 5>> channel, forces;
    std::ifstream bf(out + "/spe10_boxes.bin", std::ios::binary);
    if (bf) {
      double hdr[2];
      bf.read(reinterpret_cast<char*>(hdr), sizeof(hdr));
      for (int k = 0; k < int(hdr[0]) + int(hdr[1]); ++k) {
        std::array<double, 5> b;
        bf.read(reinterpret_cast<char*>(b.data()), sizeof(b));
        (k < int(hdr[0]) ? channel : forces).push_back(b);
      }
    }
    dump(out + "/spe10_perm.bin", perm);
    S::Grid::Providers::Cube provider(HDD_SIMPLEX, {0.0, 0.0}, {5.0, 1.0}, {100, 20});
    Discretizations::SWIPDG sw(provider, S::Grid::BoundaryInfos::AllDirichlet::default_config(),
                               Problems::Spe10Model1(perm, channel, forces, true, {{0.0, 0.0}}), 0, {"elliptic"});
    sw.init();
    const auto& A = sw.system_matrix();
    std::printf("spe10 parametric %d components %d coefficient %s rhs components %d coefficient %s\n",
                int(A.parametric()), A.num_components(), A.coefficient(0).expression().c_str(),
                sw.rhs().num_components(), sw.rhs().coefficient(0).expression().c_str());
    dump(out + "/spe10_affine.bin", A.affine_part());
    dump(out + "/spe10_comp0.bin", A.component(0));
    dump(out + "/spe10_frozen_0.5.bin", A.freeze_parameter(0.5));
    dump(out + "/spe10_rhs.bin", sw.rhs().affine_part());
    dump(out + "/spe10_rhs_comp0.bin", sw.rhs().component(0));
    const auto& E = sw.get_product("elliptic");
    dump(out + "/spe10_elliptic_comp0.bin", E.component(0));
    // the reference's default channel_boundary_layer (problems/spe10.hh:86, FlatTop's default): the channel is a
    // sum of FlatTop functions (213-222), evaluated at quadrature points; non-parametric 1 + 0.9 channel and
    // the parametric split
    // (on 97 x 21 squares: the 0.05-aligned channel boxes are narrower than two layers, so the FlatTop sum is
    // discontinuous on lines y, x = 0.05 k; a mesh whose lines avoid them keeps every quadrature point off those)
    S::Grid::Providers::Cube provider97(HDD_SIMPLEX, {0.0, 0.0}, {5.0, 1.0}, {97, 21});
    Discretizations::SWIPDG ft(provider97, S::Grid::BoundaryInfos::AllDirichlet::default_config(),
                               Problems::Spe10Model1(perm, channel, forces, false));
    ft.init();
    dump(out + "/spe10ft_affine.bin", ft.system_matrix().affine_part());
    Discretizations::SWIPDG ftp(provider97, S::Grid::BoundaryInfos::AllDirichlet::default_config(),
                                Problems::Spe10Model1(perm, channel, forces, true));
    ftp.init();
    std::printf("spe10 flattop channel: components %d order %d\n", ftp.system_matrix().num_components(),
                ftp.problem().diffusion_factor.components.at(0).order);
    dump(out + "/spe10ftp_affine.bin", ftp.system_matrix().affine_part());
    dump(out + "/spe10ftp_comp0.bin", ftp.system_matrix().component(0));
  }

  // 8. parametric right-hand side with kappa_p x g_D,q cross terms (swipdg.hh:257-330): OS2014 kappa, g_D(mu) =
  //    sin(..) + mu cos(..) cos(..), g_N = 0, f = ESV2007 force on 8x8 Kuhn with AllDirichlet
  {
    S::Grid::Providers::Cube provider(HDD_SIMPLEX, {-1.0, -1.0}, {1.0, 1.0}, {8, 8});
    auto p = Problems::OS2014();
    p.dirichlet = Problems::ScalarFunction::sinusoid(0.25, 0.5, 1.0, 2.0, 3);
    p.dirichlet.register_component(Problems::ScalarFunction::cos_product(0.7, 1.5, 0.5, 0.0, 3),
                                   Dune::HDD::LinearElliptic::Pymor::ParameterFunctional("mu", "mu", 1.0));
    Discretizations::SWIPDG sw(provider, S::Grid::BoundaryInfos::AllDirichlet::default_config(), p);
    sw.init();
    const auto& b = sw.rhs();
    std::string coefs;
    for (int q = 0; q < b.num_components(); ++q) coefs += b.coefficient(q).expression() + ";";
    std::printf("parametric rhs components %d coefficients %s\n", b.num_components(), coefs.c_str());
    dump(out + "/prhs_affine.bin", b.affine_part());
    for (int q = 0; q < b.num_components(); ++q) dump(out + "/prhs_comp" + std::to_string(q) + ".bin", b.component(q));
    dump(out + "/prhs_frozen_0.7.bin", b.freeze_parameter(0.7));
  }
  std::printf("surface ok\n");
  return 0;
}
