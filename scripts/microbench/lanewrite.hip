#pragma clang diagnostic ignored "-Wunused-result"
// per-lane contiguous block stores (each lane writes its own L/64 doubles with 16-byte stores) vs
// tile-coalesced stores, persistent single-wave workgroups
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef int ivec4 __attribute__((ext_vector_type(4)));
template <int L, int MODE>   // MODE 0 coalesced plain, 1 coalesced nt, 2 lane plain, 3 lane nt
__global__ void __launch_bounds__(64) tw(double* out, long ntiles)
{
  constexpr int PER = L / 64, ST = PER / 2;
  const long G = gridDim.x, b = blockIdx.x;
  const long x = b & 7, w = b >> 3, gx = G >> 3;
  long t = (ntiles * x) / 8 + w;
  const long t_end = (ntiles * (x + 1)) / 8;
  const int lane = threadIdx.x;
  for (; t < t_end; t += gx) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + t * L, (short)0, L * 8, 0x00020000);
#pragma unroll
    for (int k = 0; k < ST; ++k) {
      dvec2 v = {double(k), double(lane)};
      const int idx = MODE < 2 ? 2 * (lane + 64 * k) : lane * PER + 2 * k;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ivec4, v), r, idx * 8, 0, (MODE & 1) ? 2 : 0);
    }
  }
}
template <int L, int MODE>
static void run(double* out, long n, int cus)
{
  const long ntiles = n / L;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int wgcu : {2, 4, 8, 12}) {
    std::vector<float> ts;
    for (int r = 0; r < 9; ++r) {
      hipEventRecord(e0);
      tw<L, MODE><<<cus * wgcu, 64>>>(out, ntiles);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("L=%5d mode=%s wg/cu=%2d median %.4f ms  %6.0f GB/s\n", L,
           MODE == 0 ? "coal-plain" : MODE == 1 ? "coal-nt   " : MODE == 2 ? "lane-plain" : "lane-nt   ", wgcu, ts[4],
           double(ntiles) * L * 8 / (ts[4] * 1e-3) / 1e9);
  }
}
int main()
{
  const long bytes = 2700L << 20, n = bytes / 8;
  double* out;
  hipMalloc(&out, bytes);
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  run<2304, 0>(out, n, cus); run<2304, 1>(out, n, cus); run<2304, 2>(out, n, cus); run<2304, 3>(out, n, cus);
  run<5120, 0>(out, n, cus); run<5120, 1>(out, n, cus); run<5120, 2>(out, n, cus); run<5120, 3>(out, n, cus);
  return 0;
}
