// examples/problems_main.cpp -- host-only checks of the problem definitions behind the C++ surface (no GPU call).
//
//   problems_main spe10 <data_file> <cells.bin>
//       Problems::Spe10Model1 built from the SPE10 Model1 data file (the reference ctor, problems/spe10.hh:111-125)
//       must equal the vector form built from the cells the caller expects the file to hold (cells.bin: 2000
//       doubles), for the plain and the parametric channel, on the default and on a shifted domain.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "hdd_discretizations.hh"

using namespace Dune::HDD::LinearElliptic;

namespace {

bool same_fn(const Problems::ScalarFunction& a, const Problems::ScalarFunction& b)
{
  return a.kind == b.kind && a.host == b.host && a.order == b.order && a.c == b.c && a.b == b.b && a.lower == b.lower &&
         a.upper == b.upper && a.ncx == b.ncx && a.ncy == b.ncy && a.table == b.table && a.per_element == b.per_element;
}

bool same_problem(const Problems::Problem& a, const Problems::Problem& b)
{
  const auto& ka = a.diffusion_factor;
  const auto& kb = b.diffusion_factor;
  bool ok = a.diffusion_tensor.kind == b.diffusion_tensor.kind && a.diffusion_tensor.host == b.diffusion_tensor.host &&
            same_fn(a.diffusion_tensor.field, b.diffusion_tensor.field) && same_fn(a.force.affine_part, b.force.affine_part) &&
            ka.has_affine_part == kb.has_affine_part && same_fn(ka.affine_part, kb.affine_part) &&
            ka.components.size() == kb.components.size();
  for (size_t q = 0; ok && q < ka.components.size(); ++q)
    ok = same_fn(ka.components[q], kb.components[q]) &&
         ka.coefficients[q].expression() == kb.coefficients[q].expression();
  return ok;
}

int run_spe10(const std::string& file, const std::string& cells_bin)
{
  std::vector<double> cells(HDD_SPE10_MODEL1_CELLS);
  {
    std::ifstream f(cells_bin, std::ios::binary);
    f.read(reinterpret_cast<char*>(cells.data()), std::streamsize(cells.size() * sizeof(double)));
    if (!f) { std::fprintf(stderr, "cannot read %s\n", cells_bin.c_str()); return 2; }
  }
  // the reference default config's forces (problems/spe10.hh:74-80) and a two-box channel
  const std::vector<std::array<double, 5>> forces = {{0.95, 0.30, 1.10, 0.45, 2000.0},
                                                      {3.00, 0.75, 3.15, 0.90, -1000.0},
                                                      {4.25, 0.25, 4.40, 0.40, -1000.0}};
  const std::vector<std::array<double, 5>> channel = {{1.7, 0.35, 1.75, 0.40, -1.0}, {1.75, 0.35, 1.80, 0.40, -1.1}};
  int ok = 1;
  for (bool parametric : {false, true})
    for (const auto& dom : {std::array<std::array<double, 2>, 2>{{{0.0, 0.0}, {5.0, 1.0}}},
                            std::array<std::array<double, 2>, 2>{{{-1.0, 2.0}, {4.0, 3.5}}}}) {
      const auto from_file = Problems::Spe10Model1(file, dom[0], dom[1], channel, forces, {{0.0, 0.0}}, parametric);
      const auto from_cells = Problems::Spe10Model1(cells, channel, forces, parametric, {{0.0, 0.0}}, 3, dom[0], dom[1]);
      ok &= same_problem(from_file, from_cells) && from_file.diffusion_tensor.field.lower == dom[0] &&
            from_file.diffusion_tensor.field.upper == dom[1] && from_file.diffusion_tensor.field.ncx == 100 &&
            from_file.diffusion_tensor.field.ncy == 20;
    }
  // the default channel_boundary_layer (FlatTop channel) and the non-parametric default
  ok &= same_problem(Problems::Spe10Model1(file, {{0.0, 0.0}}, {{5.0, 1.0}}, channel, forces),
                     Problems::Spe10Model1(cells, channel, forces, false));
  std::printf("spe10 file == vector: %d\n", ok);
  try {
    Problems::Spe10Model1(file + ".missing", {{0.0, 0.0}}, {{5.0, 1.0}}, {}, forces);
    std::printf("missing file accepted\n");
    ok = 0;
  } catch (const std::exception& e) {
    std::printf("missing file rejected: %s\n", e.what());
  }
  return ok ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv)
{
  try {
    if (argc == 4 && std::string(argv[1]) == "spe10") return run_spe10(argv[2], argv[3]);
    std::fprintf(stderr, "usage: problems_main spe10 <data_file> <cells.bin>\n");
    return 2;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
