// dune-hdd_amd/csrc/host/grid.cpp
//
// Host-side grids, rank-local views, halo plans and the sparsity pattern of the SWIPDG operator.
//
// Replaces, for the assembly hot path, the grid providers and patterns the reference builds on:
//   - Stuff::Grid::Providers::Cube + globalRefine            (testcases/ESV2007.hh:123-129, spe10.hh:301-307)
//   - grid::Multiscale::Providers::Cube with num_partitions   (testcases/base.hh:150-191)
//   - EllipticSWIPDG::pattern(test, ansatz)                    (discretizations/swipdg.hh:169)
//   - BlockSWIPDG add_local_to_global_pattern / compute_face_pattern (block-swipdg.hh:304-325, 1036-1049)
//
// Element numbering is subdomain-major (Spaces::Block::mapToGlobal(ss, ii) = offset(ss) + ii), subdomain
// id = sx*py + sy so that vertical strips of subdomains are contiguous element ranges (one per rank).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "hdd.h"
#include "hdd_internal.hh"

namespace hdd {

// Dune reference elements: simplex faces 0:(0,1) 1:(0,2) 2:(1,2); cube faces 0:(0,2) 1:(1,3) 2:(0,1) 3:(2,3)
static const int kSimplexFV[3][2] = {{0, 1}, {0, 2}, {1, 2}};
static const int kCubeFV[4][2] = {{0, 2}, {1, 3}, {0, 1}, {2, 3}};

static inline const int (*face_table(int et))[2] { return et == HDD_SIMPLEX ? kSimplexFV : kCubeFV; }
static inline int nvpe_of(int et) { return et == HDD_SIMPLEX ? 3 : 4; }

// numpy.linspace-compatible node coordinate (i*step + start, last node = stop)
static inline double linspace_node(double a, double b, int64_t n, int64_t i)
{
  if (i == n) return b;
  const double step = (b - a) / double(n);
  return double(i) * step + a;
}

struct Grid {
  virtual ~Grid() = default;
  int elem_type = HDD_SIMPLEX, nvpe = 3, nf = 3, nb = 3, dim = 2;
  int64_t ne = 0, nv = 0;
  int32_t n_sub = 1;
  std::vector<int64_t> sub_first;   // [n_sub+1] element ranges of the subdomains
  virtual void vertices(int64_t g, int64_t* v) const = 0;
  virtual void vertex_coord(int64_t v, double* xy) const = 0;   // dim values
  virtual int64_t neighbor(int64_t g, int f) const = 0;      // >= 0 element, else HDD_NBR_*
  virtual uint32_t face_info(int64_t g) const = 0;
  int32_t subdomain(int64_t g) const
  {
    return int32_t(std::upper_bound(sub_first.begin(), sub_first.end(), g) - sub_first.begin()) - 1;
  }
};

// ------------------------------------------------------------------------------------------------
// structured nx x ny squares (Kuhn split for simplices), px x py subdomains, implicit formulas
// ------------------------------------------------------------------------------------------------
struct StructuredGrid final : Grid {
  hdd_structured_desc d{};
  int ec = 1;                          // elements per square
  std::vector<int64_t> cs, rs;         // first column / row of each subdomain column / row  [p+1]
  std::vector<int64_t> sq_first;       // first square of each subdomain [n_sub+1]
  int32_t bcode = HDD_NBR_DIRICHLET;

  explicit StructuredGrid(const hdd_structured_desc& desc) : d(desc)
  {
    elem_type = d.elem_type;
    nvpe = nvpe_of(elem_type);
    nf = nvpe;
    nb = nvpe;
    ec = elem_type == HDD_SIMPLEX ? 2 : 1;
    nv = int64_t(d.nx + 1) * (d.ny + 1);
    ne = int64_t(d.nx) * d.ny * ec;
    bcode = d.boundary == HDD_BOUNDARY_ALL_NEUMANN ? HDD_NBR_NEUMANN : HDD_NBR_DIRICHLET;
    // square column i belongs to subdomain column floor(i*px/nx): first column of sx = ceil(sx*nx/px)
    cs.resize(d.px + 1);
    rs.resize(d.py + 1);
    for (int s = 0; s <= d.px; ++s) cs[s] = (int64_t(s) * d.nx + d.px - 1) / d.px;
    for (int s = 0; s <= d.py; ++s) rs[s] = (int64_t(s) * d.ny + d.py - 1) / d.py;
    n_sub = d.px * d.py;
    sq_first.assign(n_sub + 1, 0);
    for (int sx = 0; sx < d.px; ++sx)
      for (int sy = 0; sy < d.py; ++sy) {
        const int s = sx * d.py + sy;
        sq_first[s + 1] = (cs[sx + 1] - cs[sx]) * (rs[sy + 1] - rs[sy]);
      }
    for (int s = 0; s < n_sub; ++s) sq_first[s + 1] += sq_first[s];
    sub_first.resize(n_sub + 1);
    for (int s = 0; s <= n_sub; ++s) sub_first[s] = sq_first[s] * ec;
  }

  int64_t square_id(int64_t i, int64_t j) const
  {
    const int64_t sx = (i * d.px) / d.nx, sy = (j * d.py) / d.ny;
    const int64_t s = sx * d.py + sy;
    const int64_t w = cs[sx + 1] - cs[sx];
    return sq_first[s] + (j - rs[sy]) * w + (i - cs[sx]);
  }

  void square_of(int64_t sq, int64_t* i, int64_t* j) const
  {
    const int64_t s = int64_t(std::upper_bound(sq_first.begin(), sq_first.end(), sq) - sq_first.begin()) - 1;
    const int64_t sx = s / d.py, sy = s % d.py;
    const int64_t w = cs[sx + 1] - cs[sx];
    const int64_t loc = sq - sq_first[s];
    *i = cs[sx] + loc % w;
    *j = rs[sy] + loc / w;
  }

  void vertices(int64_t g, int64_t* v) const override
  {
    int64_t i, j;
    square_of(g / ec, &i, &j);
    const int64_t v00 = j * (d.nx + 1) + i, v10 = v00 + 1, v01 = v00 + d.nx + 1, v11 = v01 + 1;
    if (elem_type == HDD_CUBE) {
      v[0] = v00; v[1] = v10; v[2] = v01; v[3] = v11;
    } else if (g % 2 == 0) {   // createSimplexGrid permutation (x, y): v00, v10, v11
      v[0] = v00; v[1] = v10; v[2] = v11;
    } else {                   // permutation (y, x): v00, v01, v11
      v[0] = v00; v[1] = v01; v[2] = v11;
    }
  }

  void vertex_coord(int64_t v, double* xy) const override
  {
    const int64_t i = v % (d.nx + 1), j = v / (d.nx + 1);
    xy[0] = linspace_node(d.lower[0], d.upper[0], d.nx, i);
    xy[1] = linspace_node(d.lower[1], d.upper[1], d.ny, j);
  }

  int64_t elem_at(int64_t i, int64_t j, int t) const
  {
    if (i < 0 || j < 0 || i >= d.nx || j >= d.ny) return bcode;
    return square_id(i, j) * ec + t;
  }

  int64_t neighbor(int64_t g, int f) const override
  {
    int64_t i, j;
    square_of(g / ec, &i, &j);
    if (elem_type == HDD_CUBE) {
      switch (f) {
        case 0: return elem_at(i - 1, j, 0);
        case 1: return elem_at(i + 1, j, 0);
        case 2: return elem_at(i, j - 1, 0);
        default: return elem_at(i, j + 1, 0);
      }
    }
    if (g % 2 == 0) {          // (v00, v10, v11): bottom, diagonal, right
      switch (f) {
        case 0: return elem_at(i, j - 1, 1);
        case 1: return elem_at(i, j, 1);
        default: return elem_at(i + 1, j, 1);
      }
    }
    switch (f) {               // (v00, v01, v11): left, diagonal, top
      case 0: return elem_at(i - 1, j, 0);
      case 1: return elem_at(i, j, 0);
      default: return elem_at(i, j + 1, 0);
    }
  }

  uint32_t face_info(int64_t g) const override
  {
    // twin faces (no reversed orientation on structured grids)
    if (elem_type == HDD_CUBE) return (1u << 0) | (0u << 4) | (3u << 8) | (2u << 12);
    if (g % 2 == 0) return (2u << 0) | (1u << 4) | (0u << 8);
    return (2u << 0) | (1u << 4) | (0u << 8);
  }
};

// ------------------------------------------------------------------------------------------------
// structured nx x ny x nz axis-aligned hexahedra (3d), px x py x pz subdomains, implicit formulas
// ------------------------------------------------------------------------------------------------
struct StructuredGrid3 final : Grid {
  hdd_structured3_desc d{};
  int64_t n[3] = {1, 1, 1}, p[3] = {1, 1, 1};
  std::vector<int64_t> cut[3];         // first layer of each subdomain slab per axis [p+1]
  std::vector<int64_t> blk_first;      // first element of each subdomain [n_sub+1]
  int32_t bcode = HDD_NBR_DIRICHLET;

  explicit StructuredGrid3(const hdd_structured3_desc& desc) : d(desc)
  {
    elem_type = HDD_HEX;
    dim = 3;
    nvpe = 8;
    nf = 6;
    nb = (d.degree + 1) * (d.degree + 1) * (d.degree + 1);
    n[0] = d.nx; n[1] = d.ny; n[2] = d.nz;
    p[0] = d.px; p[1] = d.py; p[2] = d.pz;
    nv = (n[0] + 1) * (n[1] + 1) * (n[2] + 1);
    ne = n[0] * n[1] * n[2];
    bcode = d.boundary == HDD_BOUNDARY_ALL_NEUMANN ? HDD_NBR_NEUMANN : HDD_NBR_DIRICHLET;
    for (int a = 0; a < 3; ++a) {
      cut[a].resize(p[a] + 1);
      for (int64_t s = 0; s <= p[a]; ++s) cut[a][s] = (s * n[a] + p[a] - 1) / p[a];
    }
    n_sub = int32_t(p[0] * p[1] * p[2]);
    blk_first.assign(n_sub + 1, 0);
    for (int64_t sx = 0; sx < p[0]; ++sx)
      for (int64_t sy = 0; sy < p[1]; ++sy)
        for (int64_t sz = 0; sz < p[2]; ++sz) {
          const int64_t s = (sx * p[1] + sy) * p[2] + sz;
          blk_first[s + 1] = (cut[0][sx + 1] - cut[0][sx]) * (cut[1][sy + 1] - cut[1][sy]) * (cut[2][sz + 1] - cut[2][sz]);
        }
    for (int s = 0; s < n_sub; ++s) blk_first[s + 1] += blk_first[s];
    sub_first = blk_first;
  }

  int64_t elem_id(const int64_t* c) const
  {
    int64_t sc[3], w[3];
    for (int a = 0; a < 3; ++a) {
      sc[a] = (c[a] * p[a]) / n[a];
      w[a] = cut[a][sc[a] + 1] - cut[a][sc[a]];
    }
    const int64_t s = (sc[0] * p[1] + sc[1]) * p[2] + sc[2];
    const int64_t l0 = c[0] - cut[0][sc[0]], l1 = c[1] - cut[1][sc[1]], l2 = c[2] - cut[2][sc[2]];
    return blk_first[s] + l0 + w[0] * (l1 + w[1] * l2);
  }

  void cell_of(int64_t g, int64_t* c) const
  {
    const int64_t s = int64_t(std::upper_bound(blk_first.begin(), blk_first.end(), g) - blk_first.begin()) - 1;
    const int64_t sz = s % p[2], sy = (s / p[2]) % p[1], sx = s / (p[1] * p[2]);
    const int64_t sc[3] = {sx, sy, sz};
    int64_t w[3];
    for (int a = 0; a < 3; ++a) w[a] = cut[a][sc[a] + 1] - cut[a][sc[a]];
    int64_t loc = g - blk_first[s];
    for (int a = 0; a < 3; ++a) {
      c[a] = cut[a][sc[a]] + loc % w[a];
      loc /= w[a];
    }
  }

  void vertices(int64_t g, int64_t* v) const override
  {
    int64_t c[3];
    cell_of(g, c);
    for (int k = 0; k < 8; ++k)   // Dune cube vertex k = (k&1, (k>>1)&1, k>>2)
      v[k] = (c[0] + (k & 1)) + (n[0] + 1) * ((c[1] + ((k >> 1) & 1)) + (n[1] + 1) * (c[2] + (k >> 2)));
  }

  void vertex_coord(int64_t v, double* xyz) const override
  {
    const int64_t i = v % (n[0] + 1), j = (v / (n[0] + 1)) % (n[1] + 1), k = v / ((n[0] + 1) * (n[1] + 1));
    xyz[0] = linspace_node(d.lower[0], d.upper[0], n[0], i);
    xyz[1] = linspace_node(d.lower[1], d.upper[1], n[1], j);
    xyz[2] = linspace_node(d.lower[2], d.upper[2], n[2], k);
  }

  int64_t neighbor(int64_t g, int f) const override
  {
    int64_t c[3];
    cell_of(g, c);
    const int a = f / 2;
    c[a] += (f & 1) ? 1 : -1;
    if (c[a] < 0 || c[a] >= n[a]) return bcode;
    return elem_id(c);
  }

  uint32_t face_info(int64_t) const override
  {
    uint32_t fi = 0;   // twin of face f is f^1, never reversed (aligned structured faces)
    for (uint32_t f = 0; f < 6; ++f) fi |= (f ^ 1u) << (4 * f);
    return fi;
  }
};

// ------------------------------------------------------------------------------------------------
// general conforming mesh from connectivity
// ------------------------------------------------------------------------------------------------
struct ExplicitGrid final : Grid {
  std::vector<double> vc;       // [nv][dim]
  std::vector<int64_t> ev;      // [ne][nvpe] (renumbered elements)
  std::vector<int64_t> nbr;     // [ne][nf]
  std::vector<uint32_t> finfo;  // [ne]

  void vertices(int64_t g, int64_t* v) const override
  {
    for (int k = 0; k < nvpe; ++k) v[k] = ev[g * nvpe + k];
  }
  void vertex_coord(int64_t v, double* xy) const override
  {
    for (int c = 0; c < dim; ++c) xy[c] = vc[dim * v + c];
  }
  int64_t neighbor(int64_t g, int f) const override { return nbr[g * nf + f]; }
  uint32_t face_info(int64_t g) const override { return finfo[g]; }
};

// ------------------------------------------------------------------------------------------------
// rank-local view
// ------------------------------------------------------------------------------------------------
struct Local {
  const Grid* g = nullptr;
  int32_t s_begin = 0, s_end = 0;
  int64_t g0 = 0, g1 = 0;               // owned global range
  std::vector<int64_t> ghost_lo, ghost_hi;  // sorted global ids of ghosts below g0 / above g1
  int64_t n_local() const { return int64_t(ghost_lo.size()) + (g1 - g0) + int64_t(ghost_hi.size()); }
  int64_t own_begin() const { return int64_t(ghost_lo.size()); }
  int64_t own_end() const { return own_begin() + (g1 - g0); }
  int64_t global_of(int64_t l) const
  {
    const int64_t nlo = int64_t(ghost_lo.size());
    if (l < nlo) return ghost_lo[l];
    if (l < nlo + (g1 - g0)) return g0 + (l - nlo);
    return ghost_hi[l - nlo - (g1 - g0)];
  }
  int64_t local_of(int64_t gid) const
  {
    if (gid >= g0 && gid < g1) return own_begin() + (gid - g0);
    if (gid < g0) {
      auto it = std::lower_bound(ghost_lo.begin(), ghost_lo.end(), gid);
      return (it != ghost_lo.end() && *it == gid) ? int64_t(it - ghost_lo.begin()) : -1;
    }
    auto it = std::lower_bound(ghost_hi.begin(), ghost_hi.end(), gid);
    return (it != ghost_hi.end() && *it == gid) ? own_end() + int64_t(it - ghost_hi.begin()) : -1;
  }
};

}  // namespace hdd

struct hdd_grid {
  std::unique_ptr<hdd::Grid> impl;
};
struct hdd_local {
  hdd::Local impl;
};

using namespace hdd;

// vertices (local indices, ascending) of face f: 2d from the reference-element tables, hex face f = the
// four vertices k with bit f/2 of k equal to f&1 (Dune cube: faces 2a / 2a+1 at x_a = 0 / 1)
static int face_vertices(int elem_type, int f, int* k)
{
  if (elem_type == HDD_HEX) {
    int n = 0;
    for (int v = 0; v < 8; ++v)
      if (((v >> (f / 2)) & 1) == (f & 1)) k[n++] = v;
    return 4;
  }
  const auto FV = face_table(elem_type);
  k[0] = FV[f][0];
  k[1] = FV[f][1];
  return 2;
}

// shared tail of the connectivity constructors: subdomain-major renumbering (stable), face matching by the
// sorted vertex ids of each face, twin face / orientation bits
static int finish_explicit(std::unique_ptr<ExplicitGrid> G, int64_t n_vertices, const double* vertex_coords,
                           int64_t n_elements, const int32_t* elem_vert, const int32_t* subdomain,
                           int32_t n_subdomains, int32_t boundary, hdd_grid** out, const std::string& fn)
{
  G->nv = n_vertices;
  G->ne = n_elements;
  G->n_sub = subdomain ? n_subdomains : 1;
  if (G->n_sub < 1) return set_error(HDD_ERR_INVALID, fn + ": n_subdomains < 1");
  const int nvpe = G->nvpe, nf = G->nf, dim = G->dim;
  std::vector<int64_t> order(n_elements);
  G->sub_first.assign(G->n_sub + 1, 0);
  for (int64_t e = 0; e < n_elements; ++e) {
    const int32_t s = subdomain ? subdomain[e] : 0;
    if (s < 0 || s >= G->n_sub) return set_error(HDD_ERR_RANGE, fn + ": bad subdomain");
    G->sub_first[s + 1]++;
  }
  for (int s = 0; s < G->n_sub; ++s) G->sub_first[s + 1] += G->sub_first[s];
  {
    std::vector<int64_t> pos(G->sub_first.begin(), G->sub_first.end() - 1);
    for (int64_t e = 0; e < n_elements; ++e) order[pos[subdomain ? subdomain[e] : 0]++] = e;  // new -> old
  }
  G->vc.assign(vertex_coords, vertex_coords + dim * n_vertices);
  G->ev.resize(n_elements * nvpe);
  for (int64_t n = 0; n < n_elements; ++n)
    for (int k = 0; k < nvpe; ++k) {
      const int32_t v = elem_vert[order[n] * nvpe + k];
      if (v < 0 || v >= n_vertices) return set_error(HDD_ERR_RANGE, fn + ": bad vertex");
      G->ev[n * nvpe + k] = v;
    }
  struct Rec { int64_t key[4]; int64_t ef; };
  std::vector<Rec> rec(n_elements * nf);
  int fvk[8][4] = {};
  int nfv = 0;
  for (int f = 0; f < nf; ++f) nfv = face_vertices(G->elem_type, f, fvk[f]);
  for (int64_t e = 0; e < n_elements; ++e)
    for (int f = 0; f < nf; ++f) {
      Rec r{{-1, -1, -1, -1}, e * nf + f};
      for (int i = 0; i < nfv; ++i) r.key[i] = G->ev[e * nvpe + fvk[f][i]];
      std::sort(r.key, r.key + nfv);
      rec[e * nf + f] = r;
    }
  auto same = [](const Rec& x, const Rec& y) {
    return x.key[0] == y.key[0] && x.key[1] == y.key[1] && x.key[2] == y.key[2] && x.key[3] == y.key[3];
  };
  std::sort(rec.begin(), rec.end(), [](const Rec& x, const Rec& y) {
    for (int i = 0; i < 4; ++i)
      if (x.key[i] != y.key[i]) return x.key[i] < y.key[i];
    return x.ef < y.ef;
  });
  const int64_t bcode = boundary == HDD_BOUNDARY_ALL_NEUMANN ? HDD_NBR_NEUMANN : HDD_NBR_DIRICHLET;
  G->nbr.assign(n_elements * nf, bcode);
  uint32_t fi0 = 0;   // hex: twin f^1 on every face, boundary faces included (as StructuredGrid3::face_info)
  if (G->elem_type == HDD_HEX)
    for (uint32_t f = 0; f < 6; ++f) fi0 |= (f ^ 1u) << (4 * f);
  G->finfo.assign(n_elements, fi0);
  for (size_t i = 0; i < rec.size();) {
    size_t j = i + 1;
    while (j < rec.size() && same(rec[j], rec[i])) ++j;
    if (j - i > 2) return set_error(HDD_ERR_INVALID, fn + ": non-manifold face");
    if (j - i == 2) {
      const int64_t p = rec[i].ef, q = rec[i + 1].ef;
      const int64_t ep = p / nf, eq = q / nf;
      const int fp = int(p % nf), fq = int(q % nf);
      const bool rev = G->ev[ep * nvpe + fvk[fp][0]] != G->ev[eq * nvpe + fvk[fq][0]];
      if (G->elem_type == HDD_HEX && (fq != (fp ^ 1) || rev))
        return set_error(HDD_ERR_UNSUPPORTED, fn + ": hexahedra " + std::to_string(ep) + " / " + std::to_string(eq) +
                                                  " do not share an aligned face (twin f^1)");
      G->nbr[p] = eq;
      G->nbr[q] = ep;
      if (G->elem_type != HDD_HEX) {
        G->finfo[ep] |= (uint32_t(fq) | (rev ? 8u : 0u)) << (4 * fp);
        G->finfo[eq] |= (uint32_t(fp) | (rev ? 8u : 0u)) << (4 * fq);
      }
    }
    i = j;
  }
  auto* g = new hdd_grid;
  g->impl = std::move(G);
  *out = g;
  return HDD_OK;
}

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" int hdd_grid_create_structured(const hdd_structured_desc* desc, hdd_grid** out)
{
  if (!desc || !out) return set_error(HDD_ERR_INVALID, "hdd_grid_create_structured: null argument");
  if (desc->elem_type != HDD_SIMPLEX && desc->elem_type != HDD_CUBE)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_grid_create_structured: unknown element type");
  if (desc->nx < 1 || desc->ny < 1 || desc->px < 1 || desc->py < 1 || desc->px > desc->nx || desc->py > desc->ny)
    return set_error(HDD_ERR_INVALID, "hdd_grid_create_structured: need 1 <= px <= nx and 1 <= py <= ny");
  if (!(desc->upper[0] > desc->lower[0]) || !(desc->upper[1] > desc->lower[1]))
    return set_error(HDD_ERR_INVALID, "hdd_grid_create_structured: empty domain");
  const int64_t ne = int64_t(desc->nx) * desc->ny * (desc->elem_type == HDD_SIMPLEX ? 2 : 1);
  if (ne > int64_t(INT32_MAX) / 4)
    return set_error(HDD_ERR_RANGE, "hdd_grid_create_structured: too many elements for int32 DoF columns");
  auto* g = new hdd_grid;
  g->impl.reset(new StructuredGrid(*desc));
  *out = g;
  return HDD_OK;
}

extern "C" int hdd_grid_create_structured_3d(const hdd_structured3_desc* desc, hdd_grid** out)
{
  if (!desc || !out) return set_error(HDD_ERR_INVALID, "hdd_grid_create_structured_3d: null argument");
  if (desc->nx < 1 || desc->ny < 1 || desc->nz < 1 || desc->px < 1 || desc->py < 1 || desc->pz < 1 ||
      desc->px > desc->nx || desc->py > desc->ny || desc->pz > desc->nz)
    return set_error(HDD_ERR_INVALID, "hdd_grid_create_structured_3d: need 1 <= p_a <= n_a");
  if (desc->degree < 1 || desc->degree > 3)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_grid_create_structured_3d: degree must be 1, 2 or 3");
  for (int a = 0; a < 3; ++a)
    if (!(desc->upper[a] > desc->lower[a]))
      return set_error(HDD_ERR_INVALID, "hdd_grid_create_structured_3d: empty domain");
  const int64_t nb = int64_t(desc->degree + 1) * (desc->degree + 1) * (desc->degree + 1);
  const int64_t ne = int64_t(desc->nx) * desc->ny * desc->nz;
  if (ne * nb > int64_t(INT32_MAX))
    return set_error(HDD_ERR_RANGE, "hdd_grid_create_structured_3d: too many DoFs for int32 columns");
  auto* g = new hdd_grid;
  g->impl.reset(new StructuredGrid3(*desc));
  *out = g;
  return HDD_OK;
}

extern "C" int hdd_grid_create_from_connectivity(int32_t elem_type, int64_t n_vertices, const double* vertex_coords,
                                                 int64_t n_elements, const int32_t* elem_vert,
                                                 const int32_t* subdomain, int32_t n_subdomains, int32_t boundary,
                                                 hdd_grid** out)
{
  if (!vertex_coords || !elem_vert || !out || n_vertices <= 0 || n_elements <= 0)
    return set_error(HDD_ERR_INVALID, "hdd_grid_create_from_connectivity: invalid argument");
  if (elem_type != HDD_SIMPLEX && elem_type != HDD_CUBE)
    return set_error(HDD_ERR_UNSUPPORTED, "hdd_grid_create_from_connectivity: unknown element type");
  // DoF columns (element * nb + i) and neighbour ids are int32 on the device
  if (n_elements > int64_t(INT32_MAX) / nvpe_of(elem_type))
    return set_error(HDD_ERR_RANGE, "hdd_grid_create_from_connectivity: too many elements for int32 DoF columns");
  if (elem_type == HDD_CUBE) {
    // the Q1 kernels (and the oracle) take the geometry from vertices 0, 1, 2 (affine map): every
    // quadrilateral must be a parallelogram, x0 + x3 == x1 + x2 (Dune cube vertex order)
    for (int64_t e = 0; e < n_elements; ++e) {
      const int32_t* v = elem_vert + 4 * e;
      for (int k = 0; k < 4; ++k)
        if (v[k] < 0 || v[k] >= n_vertices) return set_error(HDD_ERR_RANGE, "hdd_grid_create_from_connectivity: bad vertex");
      for (int c = 0; c < 2; ++c) {
        const double x0 = vertex_coords[2 * v[0] + c], x1 = vertex_coords[2 * v[1] + c];
        const double x2 = vertex_coords[2 * v[2] + c], x3 = vertex_coords[2 * v[3] + c];
        const double scale = std::max(std::max(std::fabs(x1 - x0), std::fabs(x2 - x0)), std::fabs(x3 - x0));
        if (std::fabs((x0 + x3) - (x1 + x2)) > 1e-10 * std::max(scale, 1e-300))
          return set_error(HDD_ERR_UNSUPPORTED, "hdd_grid_create_from_connectivity: element " + std::to_string(e) +
                                                    " is not a parallelogram (bilinear quadrilaterals are not supported)");
      }
    }
  }
  auto G = std::make_unique<ExplicitGrid>();
  G->elem_type = elem_type;
  G->nvpe = nvpe_of(elem_type);
  G->nf = G->nvpe;
  G->nb = G->nvpe;
  return finish_explicit(std::move(G), n_vertices, vertex_coords, n_elements, elem_vert, subdomain, n_subdomains,
                         boundary, out, "hdd_grid_create_from_connectivity");
}

extern "C" int hdd_grid_create_hex_from_connectivity(int32_t degree, int64_t n_vertices, const double* vertex_coords,
                                                     int64_t n_elements, const int32_t* elem_vert,
                                                     const int32_t* subdomain, int32_t n_subdomains, int32_t boundary,
                                                     hdd_grid** out)
{
  const char* fn = "hdd_grid_create_hex_from_connectivity";
  if (!vertex_coords || !elem_vert || !out || n_vertices <= 0 || n_elements <= 0)
    return set_error(HDD_ERR_INVALID, std::string(fn) + ": invalid argument");
  if (degree < 1 || degree > 3) return set_error(HDD_ERR_UNSUPPORTED, std::string(fn) + ": degree must be 1, 2 or 3");
  const int64_t nb = int64_t(degree + 1) * (degree + 1) * (degree + 1);
  if (n_elements * nb > int64_t(INT32_MAX)) return set_error(HDD_ERR_RANGE, std::string(fn) + ": too many DoFs for int32 columns");
  // the Q_p hex kernels take an affine, axis-aligned box per element (diagonal Jacobian from vertices 0, 1, 2, 4)
  // with aligned twin faces: every element must be lower + (k&1, (k>>1)&1, k>>2) * h in Dune cube vertex order
  for (int64_t e = 0; e < n_elements; ++e) {
    const int32_t* v = elem_vert + 8 * e;
    for (int k = 0; k < 8; ++k)
      if (v[k] < 0 || v[k] >= n_vertices) return set_error(HDD_ERR_RANGE, std::string(fn) + ": bad vertex");
    for (int c = 0; c < 3; ++c) {
      const double lo = vertex_coords[3 * v[0] + c], hi = vertex_coords[3 * v[1 << c] + c];
      if (!(hi > lo)) return set_error(HDD_ERR_UNSUPPORTED, std::string(fn) + ": element " + std::to_string(e) +
                                                             " is not an axis-aligned box in Dune vertex order");
      for (int k = 0; k < 8; ++k) {
        const double want = ((k >> c) & 1) ? hi : lo, x = vertex_coords[3 * v[k] + c];
        if (std::fabs(x - want) > 1e-12 * std::max(std::fabs(hi - lo), std::fabs(want)))
          return set_error(HDD_ERR_UNSUPPORTED, std::string(fn) + ": element " + std::to_string(e) +
                                                    " is not an axis-aligned box in Dune vertex order");
      }
    }
  }
  auto G = std::make_unique<ExplicitGrid>();
  G->elem_type = HDD_HEX;
  G->dim = 3;
  G->nvpe = 8;
  G->nf = 6;
  G->nb = int(nb);
  return finish_explicit(std::move(G), n_vertices, vertex_coords, n_elements, elem_vert, subdomain, n_subdomains,
                         boundary, out, fn);
}

extern "C" void hdd_grid_destroy(hdd_grid* g) { delete g; }

extern "C" int hdd_grid_get_info(const hdd_grid* g, hdd_grid_info* out)
{
  if (!g || !out) return set_error(HDD_ERR_INVALID, "hdd_grid_get_info: null argument");
  const Grid& G = *g->impl;
  out->elem_type = G.elem_type;
  out->nb = G.nb;
  out->nfaces = G.nf;
  out->nvpe = G.nvpe;
  out->n_elements = G.ne;
  out->n_vertices = G.nv;
  out->n_subdomains = G.n_sub;
  out->dim = G.dim;
  return HDD_OK;
}

extern "C" int hdd_grid_subdomain_range(const hdd_grid* g, int32_t s_begin, int32_t s_end, int64_t* first,
                                        int64_t* last)
{
  if (!g || !first || !last) return set_error(HDD_ERR_INVALID, "hdd_grid_subdomain_range: null argument");
  const Grid& G = *g->impl;
  if (s_begin < 0 || s_end > G.n_sub || s_begin >= s_end)
    return set_error(HDD_ERR_RANGE, "hdd_grid_subdomain_range: 0 <= s_begin < s_end <= num_subdomains violated");
  *first = G.sub_first[s_begin];
  *last = G.sub_first[s_end];
  return HDD_OK;
}

extern "C" int hdd_grid_connectivity(const hdd_grid* g, double* vertex_coords, int32_t* elem_vert, int32_t* subdomain)
{
  if (!g) return set_error(HDD_ERR_INVALID, "hdd_grid_connectivity: null grid");
  const Grid& G = *g->impl;
  if (vertex_coords)
    for (int64_t v = 0; v < G.nv; ++v) G.vertex_coord(v, vertex_coords + G.dim * v);
  int64_t vv[8];
  for (int64_t e = 0; e < G.ne; ++e) {
    if (elem_vert) {
      G.vertices(e, vv);
      for (int k = 0; k < G.nvpe; ++k) elem_vert[e * G.nvpe + k] = int32_t(vv[k]);
    }
    if (subdomain) subdomain[e] = G.subdomain(e);
  }
  return HDD_OK;
}

extern "C" int hdd_local_create(const hdd_grid* g, int32_t s_begin, int32_t s_end, hdd_local** out)
{
  if (!g || !out) return set_error(HDD_ERR_INVALID, "hdd_local_create: null argument");
  const Grid& G = *g->impl;
  if (s_begin < 0 || s_end > G.n_sub || s_begin >= s_end)
    return set_error(HDD_ERR_RANGE, "hdd_local_create: 0 <= s_begin < s_end <= num_subdomains violated");
  auto* l = new hdd_local;
  Local& L = l->impl;
  L.g = &G;
  L.s_begin = s_begin;
  L.s_end = s_end;
  L.g0 = G.sub_first[s_begin];
  L.g1 = G.sub_first[s_end];
  for (int64_t e = L.g0; e < L.g1; ++e)
    for (int f = 0; f < G.nf; ++f) {
      const int64_t n = G.neighbor(e, f);
      if (n < 0) continue;
      if (n < L.g0) L.ghost_lo.push_back(n);
      else if (n >= L.g1) L.ghost_hi.push_back(n);
    }
  for (auto* v : {&L.ghost_lo, &L.ghost_hi}) {
    std::sort(v->begin(), v->end());
    v->erase(std::unique(v->begin(), v->end()), v->end());
  }
  *out = l;
  return HDD_OK;
}

extern "C" void hdd_local_destroy(hdd_local* l) { delete l; }

extern "C" int hdd_local_get_info(const hdd_local* l, hdd_local_info* out)
{
  if (!l || !out) return set_error(HDD_ERR_INVALID, "hdd_local_get_info: null argument");
  const Local& L = l->impl;
  out->n_local = L.n_local();
  out->own_begin = L.own_begin();
  out->own_end = L.own_end();
  out->n_ghost = int64_t(L.ghost_lo.size() + L.ghost_hi.size());
  out->global_first = L.g0;
  return HDD_OK;
}

extern "C" int hdd_local_fill(const hdd_local* l, double* coords, int32_t* neighbors, uint32_t* face_info,
                              int64_t* global_id, int32_t* subdomain)
{
  if (!l) return set_error(HDD_ERR_INVALID, "hdd_local_fill: null local");
  const Local& L = l->impl;
  const Grid& G = *L.g;
  const int64_t nl = L.n_local();
  const int dim = G.dim;
  int64_t vv[8];
  double xy[3];
  for (int64_t e = 0; e < nl; ++e) {
    const int64_t gid = L.global_of(e);
    const bool owned = e >= L.own_begin() && e < L.own_end();
    if (coords) {
      G.vertices(gid, vv);
      for (int k = 0; k < G.nvpe; ++k) {
        G.vertex_coord(vv[k], xy);
        for (int c = 0; c < dim; ++c) coords[(dim * k + c) * nl + e] = xy[c];
      }
    }
    if (neighbors)
      for (int f = 0; f < G.nf; ++f) {
        int64_t v = -3;
        if (owned) {
          const int64_t n = G.neighbor(gid, f);
          v = n >= 0 ? L.local_of(n) : n;
          if (n >= 0 && v < 0) return set_error(HDD_ERR_INVALID, "hdd_local_fill: ghost missing (internal)");
        }
        neighbors[f * nl + e] = int32_t(v);
      }
    if (face_info) face_info[e] = owned ? G.face_info(gid) : 0u;
    if (global_id) global_id[e] = gid;
    if (subdomain) subdomain[e] = G.subdomain(gid);
  }
  return HDD_OK;
}

extern "C" int hdd_local_centers(const hdd_local* l, double* centers)
{
  if (!l || !centers) return set_error(HDD_ERR_INVALID, "hdd_local_centers: null argument");
  const Local& L = l->impl;
  const Grid& G = *L.g;
  const int64_t nl = L.n_local();
  int64_t vv[8];
  double xy[3];
  for (int64_t e = 0; e < nl; ++e) {
    G.vertices(L.global_of(e), vv);
    double sum[3] = {0.0, 0.0, 0.0};
    for (int k = 0; k < G.nvpe; ++k) {
      G.vertex_coord(vv[k], xy);
      for (int c = 0; c < G.dim; ++c) sum[c] += xy[c];
    }
    for (int c = 0; c < G.dim; ++c) centers[c * nl + e] = sum[c] / G.nvpe;
  }
  return HDD_OK;
}

extern "C" int hdd_local_vertices(const hdd_local* l, int64_t* n_vertices, int32_t* elem_vertices,
                                  double* vertex_coords)
{
  if (!l || !n_vertices) return set_error(HDD_ERR_INVALID, "hdd_local_vertices: null argument");
  const Local& L = l->impl;
  const Grid& G = *L.g;
  const int64_t nl = L.n_local();
  const int nv = G.nvpe;
  // local vertex set = sorted distinct global ids of the local elements' vertices (elements in local
  // order = global order, so neighbouring elements get neighbouring vertex ids)
  std::vector<int64_t> ids(size_t(nl) * nv);
  int64_t vv[8];
  for (int64_t e = 0; e < nl; ++e) {
    G.vertices(L.global_of(e), vv);
    for (int k = 0; k < nv; ++k) ids[size_t(e) * nv + k] = vv[k];
  }
  std::vector<int64_t> uniq(ids);
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  if (int64_t(uniq.size()) > int64_t(INT32_MAX))
    return set_error(HDD_ERR_RANGE, "hdd_local_vertices: too many local vertices for int32 ids");
  *n_vertices = int64_t(uniq.size());
  if (elem_vertices)
    for (int64_t e = 0; e < nl; ++e)
      for (int k = 0; k < nv; ++k) {
        const int64_t g = ids[size_t(e) * nv + k];
        elem_vertices[k * nl + e] = int32_t(std::lower_bound(uniq.begin(), uniq.end(), g) - uniq.begin());
      }
  if (vertex_coords)
    for (size_t v = 0; v < uniq.size(); ++v) G.vertex_coord(uniq[v], vertex_coords + G.dim * v);
  return HDD_OK;
}

static int ghost_owner(const Local& L, const int32_t* owner, int64_t gid)
{
  return owner[L.g->subdomain(gid)];
}

extern "C" int hdd_local_halo_plan(const hdd_local* l, const int32_t* owner, int32_t my_rank, int32_t* n_peers,
                                   int32_t* peers, int64_t* send_count, int64_t* recv_offset, int64_t* recv_count)
{
  if (!l || !owner || !n_peers) return set_error(HDD_ERR_INVALID, "hdd_local_halo_plan: null argument");
  const Local& L = l->impl;
  const Grid& G = *L.g;
  for (int32_t s = L.s_begin; s < L.s_end; ++s)
    if (owner[s] != my_rank) return set_error(HDD_ERR_INVALID, "hdd_local_halo_plan: owned subdomain not mine");
  // receive side: ghosts grouped by owner (contiguous because owners hold contiguous subdomain ranges)
  std::vector<int32_t> pr;
  std::vector<int64_t> roff, rcnt;
  const int64_t nl = L.n_local();
  for (int64_t e = 0; e < nl; ++e) {
    if (e >= L.own_begin() && e < L.own_end()) continue;
    const int r = ghost_owner(L, owner, L.global_of(e));
    if (r == my_rank) return set_error(HDD_ERR_INVALID, "hdd_local_halo_plan: ghost owned by this rank");
    if (!pr.empty() && pr.back() == r && roff.back() + rcnt.back() == e) {
      rcnt.back()++;
      continue;
    }
    if (std::find(pr.begin(), pr.end(), r) != pr.end())
      return set_error(HDD_ERR_UNSUPPORTED, "hdd_local_halo_plan: ghosts of one owner are not contiguous");
    pr.push_back(r);
    roff.push_back(e);
    rcnt.push_back(1);
  }
  // send side: owned elements with a face neighbour owned by the peer (the peer's ghosts, same order)
  std::vector<int64_t> scnt(pr.size(), 0);
  for (int64_t e = L.g0; e < L.g1; ++e) {
    std::vector<int> seen;
    for (int f = 0; f < G.nf; ++f) {
      const int64_t n = G.neighbor(e, f);
      if (n < 0 || (n >= L.g0 && n < L.g1)) continue;
      const int r = ghost_owner(L, owner, n);
      if (std::find(seen.begin(), seen.end(), r) != seen.end()) continue;
      seen.push_back(r);
      const auto it = std::find(pr.begin(), pr.end(), r);
      scnt[it - pr.begin()]++;
    }
  }
  // sort peers ascending (ghost groups already ascend with owner rank when ranks ascend with subdomains)
  std::vector<size_t> idx(pr.size());
  std::iota(idx.begin(), idx.end(), 0);
  std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return pr[a] < pr[b]; });
  *n_peers = int32_t(pr.size());
  if (peers)
    for (size_t k = 0; k < idx.size(); ++k) {
      peers[k] = pr[idx[k]];
      if (send_count) send_count[k] = scnt[idx[k]];
      if (recv_offset) recv_offset[k] = roff[idx[k]];
      if (recv_count) recv_count[k] = rcnt[idx[k]];
    }
  return HDD_OK;
}

extern "C" int hdd_local_send_list(const hdd_local* l, const int32_t* owner, int32_t my_rank, int32_t peer_index,
                                   int32_t* local_ids)
{
  if (!l || !owner || !local_ids) return set_error(HDD_ERR_INVALID, "hdd_local_send_list: null argument");
  int32_t np = 0;
  int rc = hdd_local_halo_plan(l, owner, my_rank, &np, nullptr, nullptr, nullptr, nullptr);
  if (rc) return rc;
  if (peer_index < 0 || peer_index >= np) return set_error(HDD_ERR_RANGE, "hdd_local_send_list: bad peer index");
  std::vector<int32_t> peers(np);
  std::vector<int64_t> sc(np), ro(np), rcv(np);
  rc = hdd_local_halo_plan(l, owner, my_rank, &np, peers.data(), sc.data(), ro.data(), rcv.data());
  if (rc) return rc;
  const int32_t peer = peers[peer_index];
  const Local& L = l->impl;
  const Grid& G = *L.g;
  int64_t k = 0;
  for (int64_t e = L.g0; e < L.g1; ++e)
    for (int f = 0; f < G.nf; ++f) {
      const int64_t n = G.neighbor(e, f);
      if (n < 0 || (n >= L.g0 && n < L.g1)) continue;
      if (ghost_owner(L, owner, n) == peer) {
        local_ids[k++] = int32_t(L.local_of(e));
        break;
      }
    }
  return HDD_OK;
}

extern "C" int hdd_checkerboard(int64_t n, const double* centers, const double lower[2], const double upper[2],
                                int32_t ncx, int32_t ncy, const double* cell_values, double* out)
{
  if (!centers || !lower || !upper || !cell_values || !out || ncx < 1 || ncy < 1)
    return set_error(HDD_ERR_INVALID, "hdd_checkerboard: invalid argument");
  for (int64_t e = 0; e < n; ++e) {
    int64_t cx = int64_t((centers[e] - lower[0]) / (upper[0] - lower[0]) * ncx);
    int64_t cy = int64_t((centers[n + e] - lower[1]) / (upper[1] - lower[1]) * ncy);
    cx = std::min<int64_t>(std::max<int64_t>(cx, 0), ncx - 1);
    cy = std::min<int64_t>(std::max<int64_t>(cy, 0), ncy - 1);
    out[e] = cell_values[cy * ncx + cx];
  }
  return HDD_OK;
}

extern "C" int hdd_spe10_model1_read(const char* filename, double min_value, double max_value, double* cells)
{
  if (!filename || !cells) return set_error(HDD_ERR_INVALID, "hdd_spe10_model1_read: null argument");
  if (!(max_value > min_value))
    return set_error(HDD_ERR_INVALID, "hdd_spe10_model1_read: max (is " + std::to_string(max_value) +
                                          ") has to be larger than min (is " + std::to_string(min_value) + ")!");
  std::ifstream in(filename);
  if (!in.is_open()) return set_error(HDD_ERR_INVALID, std::string("hdd_spe10_model1_read: could not open '") + filename + "'!");
  const double scale = (max_value - min_value) / (HDD_SPE10_MODEL1_MAX - HDD_SPE10_MODEL1_MIN);
  const double shift = min_value - scale * HDD_SPE10_MODEL1_MIN;
  int64_t k = 0;
  double v = 0.0;
  while (k < HDD_SPE10_MODEL1_CELLS && in >> v) cells[k++] = v * scale + shift;
  if (k != HDD_SPE10_MODEL1_CELLS)
    return set_error(HDD_ERR_INVALID, std::string("hdd_spe10_model1_read: '") + filename + "' holds " +
                                          std::to_string(k) + " values, " + std::to_string(HDD_SPE10_MODEL1_CELLS) +
                                          " expected");
  return HDD_OK;
}

extern "C" int hdd_indicator(int64_t n, const double* centers, int32_t n_boxes, const double* boxes, double* out)
{
  if (!centers || !out || n_boxes < 0 || (n_boxes && !boxes))
    return set_error(HDD_ERR_INVALID, "hdd_indicator: invalid argument");
  for (int64_t e = 0; e < n; ++e) {
    const double x = centers[e], y = centers[n + e];
    double v = 0.0;
    for (int32_t k = 0; k < n_boxes; ++k) {
      const double* b = boxes + 5 * k;
      if (b[0] <= x && x <= b[2] && b[1] <= y && y <= b[3]) {
        v = b[4];
        break;
      }
    }
    out[e] = v;
  }
  return HDD_OK;
}

extern "C" int hdd_indicator_sum(int64_t n, const double* centers, int32_t n_boxes, const double* boxes, double* out)
{
  if (!centers || !out || n_boxes < 0 || (n_boxes && !boxes))
    return set_error(HDD_ERR_INVALID, "hdd_indicator_sum: invalid argument");
  for (int64_t e = 0; e < n; ++e) {
    const double x = centers[e], y = centers[n + e];
    double v = 0.0;
    for (int32_t k = 0; k < n_boxes; ++k) {
      const double* b = boxes + 5 * k;
      if (b[0] <= x && x <= b[2] && b[1] <= y && y <= b[3]) v += b[4];
    }
    out[e] = v;
  }
  return HDD_OK;
}

// ------------------------------------------------------------------------------------------------
// pattern
// ------------------------------------------------------------------------------------------------
static int nb_of(int32_t et) { return et == HDD_SIMPLEX ? 3 : (et == HDD_CUBE ? 4 : 0); }

extern "C" int hdd_dg_pattern_count(int32_t nf, int32_t nb, int64_t n_local, int64_t own_begin, int64_t own_end,
                                    const int32_t* neighbors, int64_t* nnz)
{
  if (nf < 0 || nf > 6 || nb < 1) return set_error(HDD_ERR_INVALID, "hdd_dg_pattern_count: need 0 <= n_faces <= 6, nb >= 1");
  if (!neighbors || !nnz || own_begin < 0 || own_end > n_local || own_begin > own_end)
    return set_error(HDD_ERR_INVALID, "hdd_dg_pattern_count: invalid argument");
  int64_t total = 0;
  for (int64_t e = own_begin; e < own_end; ++e) {
    int blocks = 1;
    for (int f = 0; f < nf; ++f) blocks += neighbors[f * n_local + e] >= 0;
    total += int64_t(nb) * nb * blocks;
  }
  *nnz = total;
  return HDD_OK;
}

extern "C" int hdd_dg_pattern_fill(int32_t nf, int32_t nb, int64_t n_local, int64_t own_begin, int64_t own_end,
                                   const int32_t* neighbors, const int64_t* global_id, int64_t* row_ptr,
                                   int32_t* col, int64_t* elem_ptr)
{
  if (nf < 0 || nf > 6 || nb < 1) return set_error(HDD_ERR_INVALID, "hdd_dg_pattern_fill: need 0 <= n_faces <= 6, nb >= 1");
  if (!neighbors || !row_ptr || !col || own_begin < 0 || own_end > n_local || own_begin > own_end)
    return set_error(HDD_ERR_INVALID, "hdd_dg_pattern_fill: invalid argument");
  int64_t off = 0;
  row_ptr[0] = 0;
  for (int64_t e = own_begin; e < own_end; ++e) {
    const int64_t k = e - own_begin;
    int64_t blk[7];
    int nblk = 0;
    blk[nblk++] = global_id ? global_id[e] : e;
    for (int f = 0; f < nf; ++f) {
      const int32_t n = neighbors[f * n_local + e];
      if (n >= 0) {
        if (n >= n_local) return set_error(HDD_ERR_RANGE, "hdd_dg_pattern_fill: neighbour out of range");
        blk[nblk++] = global_id ? global_id[n] : n;
      }
    }
    std::sort(blk, blk + nblk);
    if (elem_ptr) elem_ptr[k] = off;
    for (int i = 0; i < nb; ++i) {
      for (int b = 0; b < nblk; ++b)
        for (int j = 0; j < nb; ++j) col[off++] = int32_t(blk[b] * nb + j);
      row_ptr[k * nb + i + 1] = off;
    }
  }
  if (elem_ptr) elem_ptr[own_end - own_begin] = off;
  return HDD_OK;
}

extern "C" int hdd_pattern_count(int32_t elem_type, int64_t n_local, int64_t own_begin, int64_t own_end,
                                 const int32_t* neighbors, int64_t* nnz)
{
  const int nb = nb_of(elem_type);
  if (!nb) return set_error(HDD_ERR_UNSUPPORTED, "hdd_pattern_count: 2d element type expected (use hdd_dg_pattern_count)");
  return hdd_dg_pattern_count(nb, nb, n_local, own_begin, own_end, neighbors, nnz);
}

extern "C" int hdd_pattern_fill(int32_t elem_type, int64_t n_local, int64_t own_begin, int64_t own_end,
                                const int32_t* neighbors, const int64_t* global_id, int64_t* row_ptr, int32_t* col,
                                int64_t* elem_ptr)
{
  const int nb = nb_of(elem_type);
  if (!nb) return set_error(HDD_ERR_UNSUPPORTED, "hdd_pattern_fill: 2d element type expected (use hdd_dg_pattern_fill)");
  return hdd_dg_pattern_fill(nb, nb, n_local, own_begin, own_end, neighbors, global_id, row_ptr, col, elem_ptr);
}

// ------------------------------------------------------------------------------------------------
// block operator maps (local / coupling operators of BlockSWIPDG)
// ------------------------------------------------------------------------------------------------
extern "C" int hdd_block_operator_map(const hdd_grid* g, int32_t ss, int32_t nn, const int64_t* row_ptr,
                                      const int32_t* col, int64_t* out_row_ptr, int32_t* out_col, int64_t* out_src,
                                      int64_t* nnz)
{
  if (!g || !row_ptr || !col || !nnz) return set_error(HDD_ERR_INVALID, "hdd_block_operator_map: null argument");
  const Grid& G = *g->impl;
  if (ss < 0 || nn < 0 || ss >= G.n_sub || nn >= G.n_sub)
    return set_error(HDD_ERR_RANGE, "hdd_block_operator_map: 0 <= ss, nn < num_subdomains violated");
  const int nb = G.nb;
  const int64_t r0 = G.sub_first[ss] * nb, r1 = G.sub_first[ss + 1] * nb;
  const int64_t c0 = G.sub_first[nn] * nb, c1 = G.sub_first[nn + 1] * nb;
  int64_t k = 0;
  if (out_row_ptr) out_row_ptr[0] = 0;
  for (int64_t r = r0; r < r1; ++r) {
    for (int64_t q = row_ptr[r]; q < row_ptr[r + 1]; ++q) {
      const int64_t c = col[q];
      if (c < c0 || c >= c1) continue;
      if (out_col) {
        out_col[k] = int32_t(c - c0);
        if (out_src) out_src[k] = q;
      }
      ++k;
    }
    if (out_row_ptr) out_row_ptr[r - r0 + 1] = k;
  }
  *nnz = k;
  return HDD_OK;
}
