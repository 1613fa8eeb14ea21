// examples/sharded_main.cpp -- the sharded BlockSWIPDG driven from C++.
//
// Each rank owns a contiguous range of subdomains (block-swipdg.hh:355-382: the owner of ss writes A_ss and
// A_ss,nn) and assembles its rows with ShardedBlockSWIPDG -> hdd_block_assemble_sharded; the face halo (the
// per-element tensor / diffusion-factor records of the ghost elements) goes through a hdd_comm.
//
//   sharded_main threads <n> [outdir]
//       n ranks as threads on GPU 0 with an in-process mailbox as the host transport (RCCL refuses two ranks
//       on one device); every rank's rows must equal, bit for bit, the rows of the single-GPU BlockSWIPDG.
//   sharded_main device <n> [outdir]
//       the same n thread ranks with the in-process device transport (hdd_comm_create_device): the halo moves by
//       device copies on each rank's transfer stream with RCCL's event schedule, so the step takes its RCCL branch
//       (pack, exchange and ghost-adjacent elements on the transfer stream, joined by an event).
//   sharded_main rccl <id_file> <rank> <nranks> <hip_device> [outdir]
//       one process per GPU over RCCL: rank 0 writes its ncclUniqueId to id_file, the others read it; the
//       rows are written to outdir/rank<r>.bin for the caller to compare.
// Problem: the parametric SPE10 Model1 structure (problems/spe10.hh:160-172): A = checkerboard permeability,
// kappa(mu) = (1 + channel) - mu channel with an Indicator channel, force = Indicator of three boxes.
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <iostream>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hdd_discretizations.hh"

using namespace Dune::HDD::LinearElliptic;
namespace D = Dune::HDD::LinearElliptic::Discretizations;

namespace {

// in-process host transport: a mailbox of FIFO queues per (from, to) pair
struct Mailbox {
  std::mutex m;
  std::condition_variable cv;
  std::map<std::pair<int, int>, std::deque<std::vector<double>>> box;
};
struct Endpoint {
  Mailbox* mb;
  int rank;
};

int mailbox_exchange(void* user, int32_t n_peers, const int32_t* peers, const double* const* send,
                     const int64_t* send_count, double* const* recv, const int64_t* recv_count)
{
  auto* ep = static_cast<Endpoint*>(user);
  Mailbox& mb = *ep->mb;
  {
    std::lock_guard<std::mutex> lk(mb.m);
    for (int k = 0; k < n_peers; ++k)
      mb.box[{ep->rank, peers[k]}].emplace_back(send[k], send[k] + send_count[k]);
  }
  mb.cv.notify_all();
  for (int k = 0; k < n_peers; ++k) {
    std::unique_lock<std::mutex> lk(mb.m);
    auto& q = mb.box[{peers[k], ep->rank}];
    if (!mb.cv.wait_for(lk, std::chrono::seconds(60), [&] { return !q.empty(); })) return HDD_ERR_INVALID;
    std::vector<double> msg = std::move(q.front());
    q.pop_front();
    if (int64_t(msg.size()) != recv_count[k]) return HDD_ERR_INVALID;
    std::memcpy(recv[k], msg.data(), msg.size() * sizeof(double));
  }
  return HDD_OK;
}

Problems::Problem spe10_parametric()
{
  std::vector<double> perm(100 * 20);
  uint64_t s = 88172645463325252ull;   // xorshift: log10 k ~ U(-3, 3)
  for (auto& v : perm) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    v = std::pow(10.0, -3.0 + 6.0 * double(s >> 11) / double(1ull << 53));
  }
  std::vector<std::array<double, 5>> channel;   // a staircase channel of 0.05 x 0.05 boxes (testcases/spe10.hh style)
  for (int i = 0; i < 40; ++i) {
    const double x = 1.7 + 0.05 * i, y = 0.35 + 0.05 * ((i / 10) % 3);
    channel.push_back({x, y, x + 0.05, y + 0.05, -1.0 - 0.002 * i});
  }
  std::vector<std::array<double, 5>> forces = {{0.95, 0.30, 1.10, 0.45, 2000.0},
                                               {3.00, 0.75, 3.15, 0.90, -1000.0},
                                               {4.25, 0.25, 4.40, 0.40, -1000.0}};
  return Problems::Spe10Model1(perm, channel, forces, /*parametric_channel=*/true, /*channel_boundary_layer=*/{{0.0, 0.0}});
}

template <class T>
void dump(const std::string& path, const std::vector<T>& v)
{
  std::ofstream f(path, std::ios::binary);
  f.write(reinterpret_cast<const char*>(v.data()), std::streamsize(v.size() * sizeof(T)));
}

// rows of the owned subdomains of one rank, all components: [affine][comp 0] ...
std::vector<double> rank_values(const D::ShardedBlockSWIPDG& sh)
{
  const auto& A = sh.system_matrix();
  std::vector<double> out = A.affine_part();
  for (int q = 0; q < A.num_components(); ++q) {
    const auto c = A.component(q);
    out.insert(out.end(), c.begin(), c.end());
  }
  return out;
}

// diffusion-factor parts of different integration orders (affine part: the per-element Indicator channel,
// order 0; component: a sinusoid of order 3): ShardedBlockSWIPDG makes one sharded call per order
Problems::Problem mixed_orders()
{
  auto p = spe10_parametric();
  p.diffusion_factor.components.clear();
  p.diffusion_factor.coefficients.clear();
  p.diffusion_factor.register_component(Problems::ScalarFunction::sinusoid(0.0, 0.5, 3.0, 2.0, 3),
                                        Pymor::ParameterFunctional("mu", "mu", 1.0));
  return p;
}

int run_threads(int n, const std::string& outdir, bool device)
{
  int fails = 0;
  for (int pi = 0; pi < 2; ++pi)
  for (int et : {HDD_SIMPLEX, HDD_CUBE}) {
    const auto problem = pi == 0 ? spe10_parametric() : mixed_orders();
    Dune::grid::Multiscale::Providers::Cube ms(et, {0.0, 0.0}, {5.0, 1.0}, {40 * n, 24}, {2 * n, 2});
    // the reference: single-GPU BlockSWIPDG of the whole multiscale grid
    D::BlockSWIPDG block(ms, Dune::Stuff::Common::Configuration(), problem);
    block.init(std::cout, "  [block] ");
    const auto& G = block.system_matrix();
    const auto ga = G.affine_part(), gc = G.component(0);
    const auto& gp = block.pattern();
    const auto& grp = gp.row_ptr();
    const auto& gcol = gp.col();

    Mailbox mb;
    const auto hub = Parallel::Communicator::device_hub(n);   // (device transport)
    std::vector<std::vector<double>> vals(static_cast<size_t>(n)), rhs(static_cast<size_t>(n));
    std::vector<std::vector<int32_t>> cols(static_cast<size_t>(n));
    std::vector<int64_t> first(static_cast<size_t>(n)), rows(static_cast<size_t>(n));
    std::vector<std::string> err(static_cast<size_t>(n));
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
      th.emplace_back([&, r] {
        try {
          Endpoint ep{&mb, r};
          auto comm = device ? Parallel::Communicator::device(hub, r, 0)
                             : Parallel::Communicator::host(mailbox_exchange, &ep, 0);
          D::ShardedBlockSWIPDG sh(ms, Dune::Stuff::Common::Configuration(), problem, comm, r, n, 0);
          sh.init();
          sh.assemble();   // more steps: the halo again, through the same transport
          if (device) sh.assemble();
          (void)hipDeviceSynchronize();
          const auto& A = sh.system_matrix();
          vals[size_t(r)] = A.affine_part();
          const auto c = A.component(0);
          vals[size_t(r)].insert(vals[size_t(r)].end(), c.begin(), c.end());
          rhs[size_t(r)] = sh.rhs().affine_part();
          cols[size_t(r)] = sh.pattern().col();
          first[size_t(r)] = sh.first_owned_dof();
          rows[size_t(r)] = sh.pattern().rows;
          if (!outdir.empty() && pi == 0) dump(outdir + "/thread_rank" + std::to_string(r) + ".bin", vals[size_t(r)]);
        } catch (const std::exception& e) {
          err[size_t(r)] = e.what();
        }
      });
    for (auto& t : th) t.join();
    const auto grhs = block.rhs().affine_part();
    int64_t mismatches = 0;
    for (int r = 0; r < n; ++r) {
      if (!err[size_t(r)].empty()) {
        std::printf("rank %d failed: %s\n", r, err[size_t(r)].c_str());
        ++fails;
        continue;
      }
      const int64_t r0 = first[size_t(r)], q0 = grp[size_t(r0)], q1 = grp[size_t(r0 + rows[size_t(r)])];
      const int64_t nnz = q1 - q0;
      if (int64_t(cols[size_t(r)].size()) != nnz) { ++mismatches; continue; }
      // equal values: bit for bit up to the sign of zero (the device build's -fno-signed-zeros lets the branch-free
      // full-tile path fold a zero product of a vanishing kappa component to +0 where the element pass keeps -0)
      auto same = [](double x, double y) { return x == y || (std::isnan(x) && std::isnan(y)); };
      auto report = [&](const char* what, int64_t k, double got, double want) {   // the first few, for diagnosis
        if (++mismatches <= 6)
          std::printf("  rank %d %s [%lld]: %.17g vs %.17g\n", r, what, (long long)k, got, want);
      };
      for (int64_t k = 0; k < nnz; ++k) {
        if (cols[size_t(r)][size_t(k)] != gcol[size_t(q0 + k)]) report("col", k, cols[size_t(r)][size_t(k)], gcol[size_t(q0 + k)]);
        if (!same(vals[size_t(r)][size_t(k)], ga[size_t(q0 + k)]))
          report("affine", k, vals[size_t(r)][size_t(k)], ga[size_t(q0 + k)]);
        if (!same(vals[size_t(r)][size_t(nnz + k)], gc[size_t(q0 + k)]))
          report("component", k, vals[size_t(r)][size_t(nnz + k)], gc[size_t(q0 + k)]);
      }
      for (int64_t i = 0; i < rows[size_t(r)]; ++i)
        if (!same(rhs[size_t(r)][size_t(i)], grhs[size_t(r0 + i)]))
          report("rhs", i, rhs[size_t(r)][size_t(i)], grhs[size_t(r0 + i)]);
    }
    std::printf("%s, %s: %d thread ranks, %lld nnz, mismatches vs single-GPU BlockSWIPDG: %lld\n",
                pi == 0 ? "parametric SPE10" : "mixed-order kappa parts", et == HDD_SIMPLEX ? "P1 Kuhn" : "Q1 quads", n,
                (long long)gp.nnz, (long long)mismatches);
    fails += mismatches != 0;
  }
  if (!fails) std::printf("sharded %s ok\n", device ? "device-transport threads" : "threads");
  return fails ? 1 : 0;
}

int run_rccl(const std::string& id_file, int rank, int nranks, int device, const std::string& outdir)
{
  std::string id;
  if (rank == 0) {
    id = Parallel::Communicator::rccl_unique_id();
    const std::string tmp = id_file + ".tmp";
    { std::ofstream f(tmp, std::ios::binary); f.write(id.data(), std::streamsize(id.size())); }
    std::rename(tmp.c_str(), id_file.c_str());
  } else {
    for (int t = 0; t < 6000; ++t) {   // up to 60 s
      std::ifstream f(id_file, std::ios::binary);
      if (f) {
        id.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
        if (id.size() == HDD_RCCL_ID_BYTES) break;
      }
      usleep(10000);
    }
  }
  auto comm = Parallel::Communicator::rccl(id, nranks, rank, device);
  Dune::grid::Multiscale::Providers::Cube ms(HDD_SIMPLEX, {0.0, 0.0}, {5.0, 1.0}, {40 * nranks, 24}, {2 * nranks, 2});
  D::ShardedBlockSWIPDG sh(ms, Dune::Stuff::Common::Configuration(), spe10_parametric(), comm, rank, nranks, device);
  sh.init(std::cout, "  [rank " + std::to_string(rank) + "] ");
  for (int k = 0; k < 3; ++k) sh.assemble();   // more halo steps over RCCL
  (void)hipDeviceSynchronize();
  const auto v = rank_values(sh);
  double sum = 0.0;
  for (double x : v) sum += std::fabs(x);
  if (!outdir.empty()) dump(outdir + "/rccl_rank" + std::to_string(rank) + ".bin", v);
  std::printf("rccl rank %d/%d: %lld values, peers %d, sum|a| %.17g%s\n", rank, nranks, (long long)v.size(),
              sh.shard_info().n_peers, sum, std::isfinite(sum) ? "" : " (NON-FINITE)");
  return std::isfinite(sum) ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv)
{
  try {
    const std::string mode = argc > 1 ? argv[1] : "threads";
    if (mode == "threads" || mode == "device")
      return run_threads(argc > 2 ? std::atoi(argv[2]) : 3, argc > 3 ? argv[3] : "", mode == "device");
    if (mode == "rccl" && argc >= 6)
      return run_rccl(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), std::atoi(argv[5]), argc > 6 ? argv[6] : "");
    std::fprintf(stderr, "usage: sharded_main threads|device <n> [outdir] | rccl <id_file> <rank> <nranks> <device> [outdir]\n");
    return 2;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
