// Host-side sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer) for the product's host code: the
// grid providers, rank-local views, halo plans, coefficient lookups, CSR pattern builders and block-operator maps
// of csrc/host/grid.cpp, called through the C ABI (include/hdd.h) over a sweep of sizes, partitions, element types,
// boundary kinds and the documented error paths.  GPU code is out of reach of the sanitizers on this pool; this
// covers everything the library runs on the host.  Built and run by tests/test_host_sanitizers.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

#include "hdd.h"

static int failures = 0;
#define CHECK(cond)                                                            \
  do {                                                                         \
    if (!(cond)) {                                                             \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                              \
    }                                                                          \
  } while (0)

// a rank-local view end to end: info, SoA fill, centres, vertices, pattern (both builders), halo plan, send lists
static void exercise_local(const hdd_grid* g, int32_t s0, int32_t s1, int32_t world)
{
  hdd_grid_info gi;
  CHECK(hdd_grid_get_info(g, &gi) == HDD_OK);
  hdd_local* l = nullptr;
  CHECK(hdd_local_create(g, s0, s1, &l) == HDD_OK);
  if (!l) return;
  hdd_local_info li;
  CHECK(hdd_local_get_info(l, &li) == HDD_OK);
  const int64_t n = li.n_local, no = li.own_end - li.own_begin;
  CHECK(no >= 0 && li.own_begin >= 0 && li.own_end <= n);
  std::vector<double> coords(size_t(gi.dim * gi.nvpe) * n), centers(size_t(gi.dim) * n);
  std::vector<int32_t> nbrs(size_t(gi.nfaces) * n), sub(n);
  std::vector<uint32_t> finfo(n);
  std::vector<int64_t> gid(n);
  CHECK(hdd_local_fill(l, coords.data(), nbrs.data(), finfo.data(), gid.data(), sub.data()) == HDD_OK);
  CHECK(hdd_local_fill(l, nullptr, nullptr, nullptr, nullptr, nullptr) == HDD_OK);
  CHECK(hdd_local_centers(l, centers.data()) == HDD_OK);
  for (int64_t e = 1; e < n; ++e) CHECK(gid[e] > gid[e - 1]);   // local order == global order
  int64_t nv = 0;
  if (gi.dim == 2) {
    CHECK(hdd_local_vertices(l, &nv, nullptr, nullptr) == HDD_OK);
    std::vector<int32_t> ev(size_t(gi.nvpe) * n);
    std::vector<double> vxy(size_t(nv) * gi.dim);
    CHECK(hdd_local_vertices(l, &nv, ev.data(), vxy.data()) == HDD_OK);
    for (int32_t v : ev) CHECK(v >= 0 && v < nv);
    // coefficient lookups at the barycentres
    std::vector<double> cells(100 * 20), out(n);
    std::iota(cells.begin(), cells.end(), 1.0);
    const double lo[2] = {-1.0, -1.0}, up[2] = {1.0, 1.0};
    CHECK(hdd_checkerboard(n, centers.data(), lo, up, 100, 20, cells.data(), out.data()) == HDD_OK);
    const double boxes[10] = {-0.5, -0.5, 0.5, 0.5, 2.0, 0.0, 0.0, 1.0, 1.0, 3.0};
    CHECK(hdd_indicator(n, centers.data(), 2, boxes, out.data()) == HDD_OK);
    CHECK(hdd_indicator_sum(n, centers.data(), 2, boxes, out.data()) == HDD_OK);
  }
  // patterns: the element-type builder (2d) and the DG builder (faces + volume-only)
  for (int nf : {gi.nfaces, 0}) {
    int64_t nnz = -1;
    CHECK(hdd_dg_pattern_count(nf, gi.nb, n, li.own_begin, li.own_end, nbrs.data(), &nnz) == HDD_OK);
    CHECK(nnz >= int64_t(gi.nb) * gi.nb * no);
    std::vector<int64_t> rp(size_t(gi.nb) * no + 1), ep(no + 1);
    std::vector<int32_t> col(nnz > 0 ? nnz : 1);
    CHECK(hdd_dg_pattern_fill(nf, gi.nb, n, li.own_begin, li.own_end, nbrs.data(), gid.data(), rp.data(), col.data(),
                              ep.data()) == HDD_OK);
    CHECK(rp[0] == 0 && rp.back() == nnz);
    for (size_t r = 0; r + 1 < rp.size(); ++r) {
      CHECK(rp[r + 1] > rp[r]);
      for (int64_t q = rp[r] + 1; q < rp[r + 1]; ++q) CHECK(col[q] > col[q - 1]);   // sorted, no duplicates
    }
    if (gi.dim == 2 && nf == gi.nfaces) {
      int64_t nnz2 = -1;
      CHECK(hdd_pattern_count(gi.elem_type, n, li.own_begin, li.own_end, nbrs.data(), &nnz2) == HDD_OK);
      CHECK(nnz2 == nnz);
      std::vector<int64_t> rp2(rp.size()), ep2(ep.size());
      std::vector<int32_t> col2(col.size());
      CHECK(hdd_pattern_fill(gi.elem_type, n, li.own_begin, li.own_end, nbrs.data(), gid.data(), rp2.data(),
                             col2.data(), ep2.data()) == HDD_OK);
      CHECK(rp2 == rp && col2 == col && ep2 == ep);
    }
  }
  // halo plan of `world` ranks owning contiguous subdomain ranges; this view is rank r's when [s0, s1) is its range
  std::vector<int32_t> owner(gi.n_subdomains);
  for (int32_t r = 0; r < world; ++r)
    for (int32_t s = int32_t(int64_t(r) * gi.n_subdomains / world); s < int32_t(int64_t(r + 1) * gi.n_subdomains / world); ++s)
      owner[s] = r;
  const int32_t me = owner[s0];
  int32_t np = -1;
  if (hdd_local_halo_plan(l, owner.data(), me, &np, nullptr, nullptr, nullptr, nullptr) == HDD_OK && np >= 0) {
    std::vector<int32_t> peers(np > 0 ? np : 1);
    std::vector<int64_t> sc(peers.size()), ro(peers.size()), rc(peers.size());
    CHECK(hdd_local_halo_plan(l, owner.data(), me, &np, peers.data(), sc.data(), ro.data(), rc.data()) == HDD_OK);
    int64_t ghosts = 0;
    for (int32_t p = 0; p < np; ++p) {
      ghosts += rc[p];
      CHECK(ro[p] >= 0 && ro[p] + rc[p] <= n);
      std::vector<int32_t> ids(sc[p] > 0 ? sc[p] : 1);
      CHECK(hdd_local_send_list(l, owner.data(), me, p, ids.data()) == HDD_OK);
      for (int64_t k = 0; k < sc[p]; ++k) CHECK(ids[k] >= li.own_begin && ids[k] < li.own_end);
    }
    CHECK(ghosts == li.n_ghost);
    CHECK(hdd_local_send_list(l, owner.data(), me, np, nullptr) != HDD_OK);   // peer index out of range
  }
  hdd_local_destroy(l);
}

static void exercise_grid(hdd_grid* g, int32_t world)
{
  hdd_grid_info gi;
  CHECK(hdd_grid_get_info(g, &gi) == HDD_OK);
  int64_t a = -1, b = -1;
  CHECK(hdd_grid_subdomain_range(g, 0, gi.n_subdomains, &a, &b) == HDD_OK && a == 0 && b == gi.n_elements);
  CHECK(hdd_grid_subdomain_range(g, 0, gi.n_subdomains + 1, &a, &b) != HDD_OK);
  if (gi.dim == 2) {
    std::vector<double> vc(size_t(gi.n_vertices) * gi.dim);
    std::vector<int32_t> ev(size_t(gi.n_elements) * gi.nvpe), sd(gi.n_elements);
    CHECK(hdd_grid_connectivity(g, vc.data(), ev.data(), sd.data()) == HDD_OK);
  }
  // the whole grid, every single subdomain, and each rank's range
  exercise_local(g, 0, gi.n_subdomains, 1);
  for (int32_t s = 0; s < gi.n_subdomains; ++s) exercise_local(g, s, s + 1, gi.n_subdomains);
  for (int32_t r = 0; r < world && world <= gi.n_subdomains; ++r)
    exercise_local(g, int32_t(int64_t(r) * gi.n_subdomains / world), int32_t(int64_t(r + 1) * gi.n_subdomains / world),
                   world);
  CHECK(hdd_local_create(g, 0, gi.n_subdomains + 1, nullptr) != HDD_OK);
  // block operator maps on the monolithic pattern
  if (gi.dim == 2 && gi.n_subdomains <= 16) {
    hdd_local* l = nullptr;
    CHECK(hdd_local_create(g, 0, gi.n_subdomains, &l) == HDD_OK);
    hdd_local_info li;
    hdd_local_get_info(l, &li);
    std::vector<int32_t> nbrs(size_t(gi.nfaces) * li.n_local);
    hdd_local_fill(l, nullptr, nbrs.data(), nullptr, nullptr, nullptr);
    int64_t nnz = 0;
    hdd_pattern_count(gi.elem_type, li.n_local, 0, li.n_local, nbrs.data(), &nnz);
    std::vector<int64_t> rp(size_t(gi.nb) * li.n_local + 1), ep(li.n_local + 1);
    std::vector<int32_t> col(nnz);
    hdd_pattern_fill(gi.elem_type, li.n_local, 0, li.n_local, nbrs.data(), nullptr, rp.data(), col.data(), ep.data());
    int64_t total = 0;
    for (int32_t ss = 0; ss < gi.n_subdomains; ++ss)
      for (int32_t nn = 0; nn < gi.n_subdomains; ++nn) {
        int64_t k = -1;
        CHECK(hdd_block_operator_map(g, ss, nn, rp.data(), col.data(), nullptr, nullptr, nullptr, &k) == HDD_OK);
        int64_t r0, r1;
        hdd_grid_subdomain_range(g, ss, ss + 1, &r0, &r1);
        std::vector<int64_t> orp(size_t(r1 - r0) * gi.nb + 1), src(k > 0 ? k : 1);
        std::vector<int32_t> ocol(k > 0 ? k : 1);
        int64_t k2 = -1;
        CHECK(hdd_block_operator_map(g, ss, nn, rp.data(), col.data(), orp.data(), ocol.data(), src.data(), &k2) ==
              HDD_OK);
        CHECK(k2 == k && orp.back() == k);
        total += k;
      }
    CHECK(total == nnz);   // the blocks partition the monolithic pattern
    CHECK(hdd_block_operator_map(g, gi.n_subdomains, 0, rp.data(), col.data(), nullptr, nullptr, nullptr, &total) !=
          HDD_OK);
    hdd_local_destroy(l);
  }
}

int main()
{
  // 2d structured: element types, ragged sizes, partitions, boundary kinds
  const int sizes[][4] = {{1, 1, 1, 1}, {9, 1, 1, 1}, {1, 9, 1, 1}, {16, 16, 1, 1}, {33, 17, 2, 2},
                          {65, 2, 4, 1},  {12, 8, 3, 1}, {24, 16, 4, 4}, {7, 5, 7, 5}};
  for (int et : {HDD_SIMPLEX, HDD_CUBE})
    for (const auto& s : sizes)
      for (int bnd : {HDD_BOUNDARY_ALL_DIRICHLET, HDD_BOUNDARY_ALL_NEUMANN}) {
        hdd_structured_desc d = {};
        d.elem_type = et;
        d.nx = s[0]; d.ny = s[1]; d.px = s[2]; d.py = s[3];
        d.boundary = bnd;
        d.lower[0] = d.lower[1] = -1.0;
        d.upper[0] = d.upper[1] = 1.0;
        hdd_grid* g = nullptr;
        CHECK(hdd_grid_create_structured(&d, &g) == HDD_OK);
        if (g) {
          exercise_grid(g, 2);
          hdd_grid_destroy(g);
        }
      }
  // 3d structured hexahedra, Q1..Q3
  for (int p = 1; p <= 3; ++p) {
    hdd_structured3_desc d = {};
    d.nx = 5; d.ny = 4; d.nz = 3; d.px = 2; d.py = 1; d.pz = 1;
    d.degree = p;
    d.upper[0] = d.upper[1] = d.upper[2] = 1.0;
    hdd_grid* g = nullptr;
    CHECK(hdd_grid_create_structured_3d(&d, &g) == HDD_OK);
    if (g) {
      exercise_grid(g, 2);
      hdd_grid_destroy(g);
    }
  }
  // 2d from connectivity: a Kuhn mesh with every triangle's vertices rotated, subdomains by column
  {
    const int nx = 6, ny = 5;
    std::vector<double> vc;
    for (int j = 0; j <= ny; ++j)
      for (int i = 0; i <= nx; ++i) {
        vc.push_back(i / double(nx));
        vc.push_back(j / double(ny));
      }
    std::vector<int32_t> ev, sd;
    for (int j = 0; j < ny; ++j)
      for (int i = 0; i < nx; ++i) {
        const int v00 = j * (nx + 1) + i, v10 = v00 + 1, v01 = v00 + nx + 1, v11 = v01 + 1;
        const int t[2][3] = {{v00, v10, v11}, {v00, v11, v01}};
        for (int k = 0; k < 2; ++k) {
          const int r = (i + j + k) % 3;
          for (int q = 0; q < 3; ++q) ev.push_back(t[k][(q + r) % 3]);
          sd.push_back(i * 3 / nx);
        }
      }
    hdd_grid* g = nullptr;
    CHECK(hdd_grid_create_from_connectivity(HDD_SIMPLEX, (nx + 1) * (ny + 1), vc.data(), int64_t(sd.size()), ev.data(),
                                            sd.data(), 3, HDD_BOUNDARY_ALL_DIRICHLET, &g) == HDD_OK);
    if (g) {
      exercise_grid(g, 3);
      hdd_grid_destroy(g);
    }
    // rejections: a vertex id out of range, a subdomain id out of range
    std::vector<int32_t> bad = ev;
    bad[4] = (nx + 1) * (ny + 1);
    CHECK(hdd_grid_create_from_connectivity(HDD_SIMPLEX, (nx + 1) * (ny + 1), vc.data(), int64_t(sd.size()),
                                            bad.data(), nullptr, 1, 0, &g) != HDD_OK);
    std::vector<int32_t> bsd = sd;
    bsd[3] = 3;
    CHECK(hdd_grid_create_from_connectivity(HDD_SIMPLEX, (nx + 1) * (ny + 1), vc.data(), int64_t(sd.size()),
                                            ev.data(), bsd.data(), 3, 0, &g) != HDD_OK);
  }
  // 3d hexahedra from connectivity (a 3 x 2 x 2 box)
  {
    const int nx = 3, ny = 2, nz = 2;
    std::vector<double> vc;
    for (int k = 0; k <= nz; ++k)
      for (int j = 0; j <= ny; ++j)
        for (int i = 0; i <= nx; ++i) {
          vc.push_back(i);
          vc.push_back(j);
          vc.push_back(k);
        }
    std::vector<int32_t> ev;
    for (int k = 0; k < nz; ++k)
      for (int j = 0; j < ny; ++j)
        for (int i = 0; i < nx; ++i)
          for (int q = 0; q < 8; ++q)
            ev.push_back(((k + (q >> 2)) * (ny + 1) + j + ((q >> 1) & 1)) * (nx + 1) + i + (q & 1));
    hdd_grid* g = nullptr;
    CHECK(hdd_grid_create_hex_from_connectivity(2, int64_t(vc.size() / 3), vc.data(), int64_t(ev.size() / 8), ev.data(),
                                                nullptr, 1, HDD_BOUNDARY_ALL_DIRICHLET, &g) == HDD_OK);
    if (g) {
      exercise_grid(g, 1);
      hdd_grid_destroy(g);
    }
  }
  // invalid arguments
  {
    hdd_structured_desc d = {};
    d.elem_type = HDD_SIMPLEX;
    d.nx = 0; d.ny = 4; d.px = d.py = 1;
    d.upper[0] = d.upper[1] = 1.0;
    hdd_grid* g = nullptr;
    CHECK(hdd_grid_create_structured(&d, &g) != HDD_OK);
    d.nx = 4; d.px = 5;   // more subdomains than squares
    CHECK(hdd_grid_create_structured(&d, &g) != HDD_OK);
    CHECK(hdd_grid_create_structured(nullptr, &g) != HDD_OK);
    double cells[HDD_SPE10_MODEL1_CELLS];
    CHECK(hdd_spe10_model1_read("/nonexistent/spe10.dat", 0.001, 998.915, cells) != HDD_OK);
    CHECK(hdd_last_error(nullptr)[0] != '\0');
  }
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("host sanitizer run: all checks passed\n");
  return 0;
}
